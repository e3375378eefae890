"""fp64 / VALU issue fractions per kernel from a scripts/pmc_dwt.sh summary.

    python scripts/pmc_fp64_frac.py gpurun_out/pmc_c3_enc/summary.txt [kernel-regex]

Per dispatch: GRBM_GUI_ACTIVE sums the 8 XCDs' busy cycles, so the kernel's
cycles are GRBM/8; a wave64 VALU instruction holds one SIMD for 4 cycles
(16 lanes per clock, float64 included on gfx950: the 34 T lane-op/s peak);
issue fraction = 4 x instructions / (SIMDs x cycles), SIMDs = 4 x 256."""
import ast
import json
import re
import sys

SIMDS = 4 * 256


def main():
    rows = []
    for line in open(sys.argv[1]):
        if " {" not in line:
            continue
        name, d = line.split(" {", 1)
        if len(sys.argv) > 2 and not re.search(sys.argv[2], name):
            continue
        c = ast.literal_eval("{" + d.strip())
        cyc = c["GRBM_GUI_ACTIVE"] / 8
        f64 = c["SQ_INSTS_VALU_ADD_F64"] + c["SQ_INSTS_VALU_MUL_F64"] + c["SQ_INSTS_VALU_FMA_F64"]
        rows.append({"kernel": name.split(" grid=")[0], "cycles": int(cyc),
                     "fp64_insts": int(f64), "valu_insts": int(c["SQ_INSTS_VALU"]),
                     "fp64_issue_frac": round(4 * f64 / (SIMDS * cyc), 3),
                     "valu_issue_frac": round(4 * c["SQ_INSTS_VALU"] / (SIMDS * cyc), 3),
                     "wait_frac": round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 3)})
    tot = {k: sum(r[k] for r in rows) for k in ("cycles", "fp64_insts", "valu_insts")}
    tot["fp64_issue_frac"] = round(4 * tot["fp64_insts"] / (SIMDS * tot["cycles"]), 3)
    tot["valu_issue_frac"] = round(4 * tot["valu_insts"] / (SIMDS * tot["cycles"]), 3)
    print(json.dumps({"source": sys.argv[1], "filter": sys.argv[2] if len(sys.argv) > 2 else None,
                      "kernels": rows, "call": tot}, indent=1))


if __name__ == "__main__":
    main()

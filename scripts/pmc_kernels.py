"""Per-kernel summary of rocprofv3 --pmc passes (one directory per pass) plus
the kernel trace's resource columns, keyed by the kernel's full template name
(zlib_parse_kernel<true> and <false> stay apart).

    python scripts/pmc_kernels.py RAW_DIR [kernel-regex] > summary.json

RAW_DIR holds p*/ (counter passes) and optionally trace/ (--kernel-trace).
Derived per kernel (averages over dispatches):
  cycles          GRBM_GUI_ACTIVE / 8 (the counter sums the 8 XCDs)
  valu_issue_frac 4 x SQ_INSTS_VALU / (1024 SIMDs x cycles)
  fp64_issue_frac 4 x (ADD + MUL + FMA _F64) / (1024 x cycles)
  wait_frac       SQ_WAIT_ANY / SQ_WAVE_CYCLES
  salu_per_valu   SQ_INSTS_SALU / SQ_INSTS_VALU
  hbm_bytes       2 x FETCH_SIZE + WRITE_SIZE, KiB -> bytes (gfx950 FETCH_SIZE
                  reports half of wide streaming reads: MI355X_MICROARCH.md)
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

SIMDS = 4 * 256


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"^void\s+", "", name)
    name = re.sub(r"\b(vcf|dfl|lift)::", "", name)
    name = re.sub(r"\(.*$", "", name)            # drop the argument list
    return name[:120]


def main():
    raw = sys.argv[1]
    pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(raw, "p*", "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row.get("Kernel_Name", "?"))
                if pat and not pat.search(k):
                    continue
                acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    res = {}
    for k, d in acc.items():
        c = {n: sum(v) / len(v) for n, v in d.items()}
        r = {"counters": {n: round(v) for n, v in sorted(c.items())},
             "dispatches": max(len(v) for v in d.values())}
        if "GRBM_GUI_ACTIVE" in c:
            cyc = c["GRBM_GUI_ACTIVE"] / 8
            r["cycles"] = round(cyc)
            if "SQ_INSTS_VALU" in c:
                r["valu_issue_frac"] = round(4 * c["SQ_INSTS_VALU"] / (SIMDS * cyc), 4)
            f64 = sum(c.get(x, 0.0) for x in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64"))
            if f64:
                r["fp64_issue_frac"] = round(4 * f64 / (SIMDS * cyc), 4)
        if c.get("SQ_WAVE_CYCLES"):
            r["wait_frac"] = round(c.get("SQ_WAIT_ANY", 0.0) / c["SQ_WAVE_CYCLES"], 4)
            if "SQ_ACTIVE_INST_ANY" in c:
                r["active_inst_frac"] = round(c["SQ_ACTIVE_INST_ANY"] / c["SQ_WAVE_CYCLES"], 4)
        if c.get("SQ_INSTS_VALU") and "SQ_INSTS_SALU" in c:
            r["salu_per_valu"] = round(c["SQ_INSTS_SALU"] / c["SQ_INSTS_VALU"], 3)
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            r["hbm_bytes"] = round(1024 * (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]))
        if c.get("SQ_WAVES") and c.get("SQ_INSTS_VALU"):
            r["valu_per_wave"] = round(c["SQ_INSTS_VALU"] / c["SQ_WAVES"], 1)
        res[k] = r
    # resources and durations from the kernel trace
    for f in glob.glob(os.path.join(raw, "trace", "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            dur = defaultdict(list)
            rsrc = {}
            for row in csv.DictReader(fh):
                k = short(row.get("Kernel_Name", "?"))
                if pat and not pat.search(k):
                    continue
                dur[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6)
                rsrc[k] = {x: row.get(x) for x in ("Arch_VGPR_Count", "Accum_VGPR_Count", "SGPR_Count",
                                                    "LDS_Block_Size", "Scratch_Size", "Workgroup_Size")
                           if row.get(x) is not None}
        for k, v in dur.items():
            e = res.setdefault(k, {})
            e["trace_ms_avg"] = round(sum(v) / len(v), 4)
            e["trace_dispatches"] = len(v)
            e["resources"] = rsrc[k]
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()

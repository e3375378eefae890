"""Turn a scripts/pmc.sh summary into profiles/pmc_encode_4k.json (bench.py's `traffic`).

    python scripts/pmc_to_traffic.py <summary.json> <source note> > profiles/pmc_encode_4k.json

HBM bytes per launch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024 (MI355X_MICROARCH.md, HBM
section: FETCH_SIZE is KiB and tallies 128-B read requests at 64 B on gfx950, so it is doubled;
WRITE_SIZE is exact).  Cross-check: TCC_EA0_RDREQ * 64 == FETCH_SIZE * 1024.
"""
import json
import sys

s = json.load(open(sys.argv[1]))["dct_dz_encode_kernel"]
disp = s.pop("_dispatches_per_counter")
rd = 2 * s["FETCH_SIZE"] * 1024
wr = s["WRITE_SIZE"] * 1024
alg = 64 * 2160 * 3840 * 3 * 2
out = {
    "workload": ("dct_dz_encode 2160x3840x3 u8 RGB frames (4K), B=8, YCoCg, deadzone Q=32, subband layout, "
                 "64 frames/step/GPU resident in HBM"),
    "kernel": "dct_dz_encode_kernel",
    "source": sys.argv[2],
    "method": ("hbm = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (MI355X_MICROARCH.md, HBM section: FETCH_SIZE is KiB "
               "and tallies 128-B read requests at 64 B on gfx950, so it is doubled; WRITE_SIZE is exact). "
               "Cross-check TCC_EA0_RDREQ*64 == FETCH_SIZE*1024"),
    "counters": dict(s, _dispatches_per_counter=disp),
    "hbm_read_bytes_per_launch": int(rd),
    "hbm_write_bytes_per_launch": int(wr),
    "hbm_bytes_per_launch": int(rd + wr),
    "alg_bytes_per_launch": alg,
    "traffic_over_alg": round((rd + wr) / alg, 5),
    "cross_check_rdreq_x64_bytes": s["TCC_EA0_RDREQ_sum"] * 64,
}
print(json.dumps(out, indent=1))

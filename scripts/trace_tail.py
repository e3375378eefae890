"""Per-launch statistics of the LAST n dispatches of one kernel in a rocprofv3
kernel trace (the timed launches of a bench run come last).

    python scripts/trace_tail.py <run_kernel_trace.csv> <kernel-regex> <n> [alg_bytes]

Prints one JSON object: average / min / max / std of the n launches' durations
(End - Start, ms) and, with alg_bytes, the achieved GB/s and fraction of the
8 TB/s HBM peak -- the same quantities bench.py's roofline block reports from
its HIP events.
"""
import csv
import json
import re
import sys

import numpy as np


def main():
    path, pat, n = sys.argv[1], re.compile(sys.argv[2]), int(sys.argv[3])
    alg = float(sys.argv[4]) if len(sys.argv) > 4 else None
    rows = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            if pat.search(r["Kernel_Name"]):
                rows.append((int(r["Dispatch_Id"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                             r["Kernel_Name"]))
    rows.sort()
    sel = rows[-n:]
    d = np.array([(e - s) * 1e-6 for _, s, e, _ in sel])
    out = {"trace": path, "kernel": sel[-1][3] if sel else None, "launches_in_trace": len(rows),
           "launches": len(sel), "avg_ms": round(float(d.mean()), 5), "min_ms": round(float(d.min()), 5),
           "max_ms": round(float(d.max()), 5), "std_ms": round(float(d.std()), 5),
           "span_ms": round((sel[-1][2] - sel[0][1]) * 1e-6, 4)}
    if alg:
        out["alg_bytes_per_launch"] = int(alg)
        out["achieved_GBps"] = round(alg / (d.mean() * 1e-3) / 1e9, 1)
        out["frac_of_8TBps"] = round(alg / (d.mean() * 1e-3) / 8e12, 4)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

#!/bin/bash
# Round 6 batch 30: band counts of the inverse line kernels (levels 3..5) in the C3 decode.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
WHAT=decode_line timeout -k 10 300 python3 -u scripts/dwt_bands_scan.py 40 6 0 1 2 3 4 6 8 12 16 > gpurun_out/r06_dwt_bands_line.json 2> gpurun_out/r06_dwt_bands_line.err
rc=$?; echo "line rc=$rc"; cat gpurun_out/r06_dwt_bands_line.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_dwt_bands_line.err; exit $rc; }

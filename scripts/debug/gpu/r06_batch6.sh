#!/bin/bash
# Round 6 batch 6: band21 with the split row pass (4 waves / SIMD) vs without, ABBA (library variants).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
WHAT=dwtdec timeout -k 10 300 python3 -u scripts/lib_ab_encode.py 12 b21s0 b21s1 > gpurun_out/r06_b21split_ab.json 2> gpurun_out/r06_b21split_ab.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/r06_b21split_ab.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_b21split_ab.err; exit $rc; }

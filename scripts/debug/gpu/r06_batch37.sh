#!/bin/bash
# Round 6 batch 37: the lazy parse capped at 5 waves / SIMD (96 VGPRs, 12 spilled), two strips per workgroup, a 7 424-byte
# window (20 strips per CU) vs 4 waves and 9 216 bytes (16 per CU), ABBA on C4.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python3 -u scripts/debug/zvar_ab.py 256 6 base w5 > gpurun_out/r06_zab_w5.json 2> gpurun_out/r06_zab_w5.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/r06_zab_w5.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_zab_w5.err; exit $rc; }

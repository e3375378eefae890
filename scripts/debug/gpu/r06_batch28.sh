#!/bin/bash
# Round 6 batch 28: K1 rank masks from per-digit rounds (then bit-sliced) vs bit-sliced only, ABBA on
# C4 with a copy of each library (the load-to-load spread), then raw RGB through both.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python3 -u scripts/debug/zvar_ab.py 256 6 dloop dbits dloop2 dbits2 > gpurun_out/r06_zab_dloop.json 2> gpurun_out/r06_zab_dloop.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/r06_zab_dloop.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_zab_dloop.err; exit $rc; }

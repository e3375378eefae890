#!/bin/bash
# Round 6 batch 13: K1 as a two-pass LSD radix sort vs the owner-wave scatters, ABBA on C4.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u scripts/debug/zvar_ab.py 256 8 dflt k1old v3mix > gpurun_out/r06_zab_k1sort.json 2> gpurun_out/r06_zab_k1sort.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/r06_zab_k1sort.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_zab_k1sort.err; exit $rc; }

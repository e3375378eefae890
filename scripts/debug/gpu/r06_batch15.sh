#!/bin/bash
# Round 6 batch 15: radix-sort K1 with batched loads: ABBA on C4 and its kernel times.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u scripts/debug/zvar_ab.py 256 8 dflt k1old v3mix > gpurun_out/r06_zab_k1sort2.json 2> gpurun_out/r06_zab_k1sort2.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/r06_zab_k1sort2.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_zab_k1sort2.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06_k1sort2_prof -o k -- python3 scripts/debug/zvar_once.py dflt 256 3 > gpurun_out/r06_k1sort2_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r06_k1sort2_prof.log; exit $rc; }

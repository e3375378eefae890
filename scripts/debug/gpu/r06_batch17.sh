#!/bin/bash
# Round 6 batch 17: radix-sort K1 v2 (pass-2 counts at placement, hd[] in pass 2): ABBA + phase clocks.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u scripts/debug/zvar_ab.py 256 8 dflt k1old > gpurun_out/r06_zab_k1sort3.json 2> gpurun_out/r06_zab_k1sort3.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/r06_zab_k1sort3.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_zab_k1sort3.err; exit $rc; }
timeout -k 10 240 python3 -u scripts/debug/zprof_run.py 256 > gpurun_out/r06_zprof_sort2.json 2> gpurun_out/r06_zprof_sort2.err
rc=$?; echo "zprof rc=$rc"; python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print({k:v for k,v in d.items() if k.startswith('sort') or k=='ms'})" gpurun_out/r06_zprof_sort2.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_zprof_sort2.err; exit $rc; }

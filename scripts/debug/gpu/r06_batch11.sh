#!/bin/bash
# Round 6 batch 11: K1 v3 (sequential rank loops, cursor reads, one-hash groups), ABBA and clocks.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u scripts/debug/zvar_ab.py 256 8 dflt k1old v3mix > gpurun_out/r06_zab_k1v3.json 2> gpurun_out/r06_zab_k1v3.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/r06_zab_k1v3.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_zab_k1v3.err; exit $rc; }
for L in libvcf_zprof.so libvcf_zprof_mix.so; do
ZPROF_LIB=$L timeout -k 10 240 python3 -u scripts/debug/zprof_run.py 256 > gpurun_out/r06_zprof3_$L.json 2> gpurun_out/r06_zprof3_$L.err
rc=$?; echo "zprof $L rc=$rc"; python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print({k:v for k,v in d.items() if k.startswith('k1') or k=='ms'})" gpurun_out/r06_zprof3_$L.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_zprof3_$L.err; exit $rc; }
done

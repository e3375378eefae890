#!/bin/bash
# Round 6 batch 12: K1 with the shared top bucket, ABBA and clocks.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u scripts/debug/zvar_ab.py 256 8 dflt k1old v3mix topmix > gpurun_out/r06_zab_k1top.json 2> gpurun_out/r06_zab_k1top.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/r06_zab_k1top.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_zab_k1top.err; exit $rc; }
for L in libvcf_zprof.so libvcf_zprof_topmix.so; do
ZPROF_LIB=$L timeout -k 10 240 python3 -u scripts/debug/zprof_run.py 256 > gpurun_out/r06_zprof4_$L.json 2> gpurun_out/r06_zprof4_$L.err
rc=$?; echo "zprof $L rc=$rc"; python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print({k:v for k,v in d.items() if k.startswith('k1') or k=='ms'})" gpurun_out/r06_zprof4_$L.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_zprof4_$L.err; exit $rc; }
done

#!/bin/bash
# Round 6 batch 10: K1 phase clocks of the v2 scatter (h >> 12 and folded owners).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for L in libvcf_zprof.so libvcf_zprof_mix.so; do
ZPROF_LIB=$L timeout -k 10 240 python3 -u scripts/debug/zprof_run.py 256 > gpurun_out/r06_zprof_$L.json 2> gpurun_out/r06_zprof_$L.err
rc=$?; echo "zprof $L rc=$rc"; python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print({k:v for k,v in d.items() if k.startswith('k1') or k=='ms'})" gpurun_out/r06_zprof_$L.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_zprof_$L.err; exit $rc; }
done

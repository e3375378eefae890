#!/bin/bash
# Round 6 batch 2: deflate prefetch prediction variants (ABBA) and their per-phase counters.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u scripts/debug/zvar_ab.py 256 6 base p1 p2 > gpurun_out/r06_zab_v3.json 2> gpurun_out/r06_zab_v3.err
rc=$?; echo "zab rc=$rc"; cat gpurun_out/r06_zab_v3.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_zab_v3.err; exit $rc; }
for L in libvcf_zprof.so libvcf_zprof_p1.so; do
  ZPROF_LIB=$L timeout -k 10 300 python3 -u scripts/debug/zprof_run.py 256 >> gpurun_out/r06_zprof3.jsonl 2>> gpurun_out/r06_zprof3.err
  rc=$?; echo "zprof $L rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cat gpurun_out/r06_zprof3.jsonl

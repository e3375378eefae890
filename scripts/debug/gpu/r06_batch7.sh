#!/bin/bash
# Round 6 batch 7: K1 phase clocks (diagnostic build) and the product C4 call's kernel stats.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 240 python3 -u scripts/debug/zprof_run.py 256 > gpurun_out/r06_zprof_k1b.json 2> gpurun_out/r06_zprof_k1b.err
rc=$?; echo "zprof rc=$rc"; cat gpurun_out/r06_zprof_k1b.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_zprof_k1b.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06_c4prof2 -o c4 -- python3 scripts/zlib_once.py 256 3 > gpurun_out/r06_c4prof2.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r06_c4prof2.log; exit $rc; }
find gpurun_out/r06_c4prof2 -name '*kernel_stats.csv' -exec head -8 {} \;

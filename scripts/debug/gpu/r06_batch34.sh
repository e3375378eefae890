#!/bin/bash
# Round 6 batch 34: the final deflate's kernel times on one C4 call and its per-phase clocks.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06_c4prof_final -o c4 -- python3 scripts/zlib_once.py 256 3 > gpurun_out/r06_c4prof_final.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r06_c4prof_final.log; exit $rc; }
timeout -k 10 240 python3 -u scripts/debug/zprof_run.py 256 > gpurun_out/r06_zprof_final.json 2> gpurun_out/r06_zprof_final.err
rc=$?; echo "zprof rc=$rc"; cat gpurun_out/r06_zprof_final.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_zprof_final.err; exit $rc; }

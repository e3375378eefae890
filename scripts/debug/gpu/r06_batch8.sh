#!/bin/bash
# Round 6 batch 8: K1 scatter sub-phase clocks (diagnostic build).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 240 python3 -u scripts/debug/zprof_run.py 256 > gpurun_out/r06_zprof_k1c.json 2> gpurun_out/r06_zprof_k1c.err
rc=$?; echo "zprof rc=$rc"; cat gpurun_out/r06_zprof_k1c.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_zprof_k1c.err; exit $rc; }

#!/bin/bash
# Round 6: lifting tolerance tests + measurement, then the zlib counters again (per kernel).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/lift_tolerance.py > gpurun_out/r06_lift_tolerance.json 2> gpurun_out/r06_lift_tolerance.err
rc=$?; echo "lift tolerance rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_dwt_lift_gpu.py -k "float64 or within" > gpurun_out/r06_t2.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r06_t2.log; [ $rc -eq 0 ] || exit $rc
bash scripts/pmc_r06.sh zlib_c4 python3 scripts/zlib_once.py 256 1 || exit $?
echo done

#!/bin/bash
# Round 6: the fused inverse 2 + 1 (band21): DWT + lifting GPU tests, ABBA on vs off, kernel trace,
# then the zlib counters.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_dwt_gpu.py tests/test_dwt_lift_gpu.py > gpurun_out/r06_t3.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r06_t3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/dwt_toggle_ab.py vcf_dwt_set_inverse_band21 decode 12 > gpurun_out/r06_band21_ab.json
rc=$?; echo "ab rc=$rc"; cat gpurun_out/r06_band21_ab.json; [ $rc -eq 0 ] || exit $rc
bash scripts/pmc_r06.sh c3_dec python3 scripts/dwt_once.py 0 3 || exit $?
bash scripts/pmc_r06.sh zlib_c4 python3 scripts/zlib_once.py 256 1 || exit $?

timeout -k 10 300 python3 -u scripts/debug/zprof_run.py 256 > gpurun_out/r06_zprof.json 2> gpurun_out/r06_zprof.err
rc=$?; echo "zprof rc=$rc"; cat gpurun_out/r06_zprof.json

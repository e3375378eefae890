#!/bin/bash
# Round 6: zlib diagnostics (per-phase counters) + ABBA of deflate variants; band21 ABBA again.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u scripts/debug/zprof_run.py 256 > gpurun_out/r06_zprof2.json 2> gpurun_out/r06_zprof2.err
rc=$?; echo "zprof rc=$rc"; cat gpurun_out/r06_zprof2.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u scripts/debug/zvar_ab.py 256 6 ${ZVARS:-late0} > gpurun_out/r06_zab.json 2> gpurun_out/r06_zab.err
rc=$?; echo "zab rc=$rc"; cat gpurun_out/r06_zab.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_dwt_gpu.py -k "band21 or line_decode" > gpurun_out/r06_t4.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r06_t4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/dwt_toggle_ab.py vcf_dwt_set_inverse_band21 decode 12

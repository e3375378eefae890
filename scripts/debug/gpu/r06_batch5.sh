#!/bin/bash
# Round 6 batch 5: deflate/inflate tests on the product library (256-position windows), then
# ABBA of the K1 third pass (hd[] without the head kernel).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu \
    tests/test_deflate_gpu.py tests/test_inflate_gpu.py tests/test_codec_gpu.py tests/test_ipp_gpu.py > gpurun_out/r06_t5.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r06_t5.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u scripts/debug/zvar_ab.py 256 6 lwdef h1 > gpurun_out/r06_zab_v6.json 2> gpurun_out/r06_zab_v6.err
rc=$?; echo "zab rc=$rc"; cat gpurun_out/r06_zab_v6.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_zab_v6.err; exit $rc; }

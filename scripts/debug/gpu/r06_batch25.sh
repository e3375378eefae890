#!/bin/bash
# Round 6 batch 25: side kernels over K1's list of non-lazy strips: deflate/inflate/codec/IPP GPU
# tests on the product library, then ABBA against the side-kernel-free bound (library copies).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu \
    tests/test_deflate_gpu.py tests/test_inflate_gpu.py tests/test_codec_gpu.py tests/test_ipp_gpu.py > gpurun_out/r06_t25.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r06_t25.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u scripts/debug/zvar_ab.py 256 6 list lcopy noside pcopy > gpurun_out/r06_zab_list.json 2> gpurun_out/r06_zab_list.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/r06_zab_list.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_zab_list.err; exit $rc; }

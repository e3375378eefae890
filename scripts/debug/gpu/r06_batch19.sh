#!/bin/bash
# Round 6 batch 19: K1 as the radix sort in the product library: deflate/inflate/codec/IPP GPU
# tests, then the C4 call's kernel times.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu \
    tests/test_deflate_gpu.py tests/test_inflate_gpu.py tests/test_codec_gpu.py tests/test_ipp_gpu.py > gpurun_out/r06_t19.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r06_t19.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06_c4prof3 -o c4 -- python3 scripts/zlib_once.py 256 3 > gpurun_out/r06_c4prof3.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r06_c4prof3.log; exit $rc; }

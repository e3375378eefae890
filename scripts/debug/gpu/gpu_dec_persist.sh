#!/bin/bash
# Persistent DCT decode: decode tests, then product (variant 0) vs round 4's kernel (A/B library
# decode variant 10) on dense and smooth 4K content, ABBA in one process.
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-dp}
timeout -k 10 900 python -u -m pytest tests/test_dct_gpu.py tests/test_codec_gpu.py tests/test_configs_gpu.py tests/test_ipp_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
DECODE=1 DENSE=1 timeout -k 10 300 python -u scripts/bench_variants.py 0,10 > gpurun_out/dec_${TAG}_dense.log 2>&1 || exit $?
tail -3 gpurun_out/dec_${TAG}_dense.log
DECODE=1 timeout -k 10 300 python -u scripts/bench_variants.py 0,10 > gpurun_out/dec_${TAG}_smooth.log 2>&1 || exit $?
tail -3 gpurun_out/dec_${TAG}_smooth.log

#!/bin/bash
# Round 6, first GPU call: changed-area tests, then counters of the GPU deflate (C4
# content) and of the DCT decode (dense and smooth 64 x 4K).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_abi.py tests/test_dwt_lift_gpu.py tests/test_deflate_gpu.py tests/test_tcbaac_gpu.py tests/test_codec_gpu.py > gpurun_out/r06_t1.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r06_t1.log; [ $rc -eq 0 ] || exit $rc
bash scripts/pmc_r06.sh zlib_c4 python3 scripts/zlib_once.py 256 1 || exit $?
DENSE=1 bash scripts/pmc_r06.sh dct_dec_dense python3 scripts/dct_dec_once.py 2 || exit $?
bash scripts/pmc_r06.sh dct_dec_smooth python3 scripts/dct_dec_once.py 2 || exit $?
echo done

#!/bin/bash
# Round 6 batch 35: the lazy window laid over the flush-only LDS (9 216-byte window at 16 strips per
# CU) vs the 3 840-byte window: ABBA on C4 (library copies; prev = the last committed product),
# then the deflate/inflate/codec/IPP GPU tests on the product library (which has it).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python3 -u scripts/debug/zvar_ab.py 256 6 alias noalias alias2 noalias2 prev > gpurun_out/r06_zab_alias.json 2> gpurun_out/r06_zab_alias.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/r06_zab_alias.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_zab_alias.err; exit $rc; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu \
    tests/test_deflate_gpu.py tests/test_inflate_gpu.py tests/test_codec_gpu.py tests/test_ipp_gpu.py > gpurun_out/r06_t35.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r06_t35.log; exit $rc

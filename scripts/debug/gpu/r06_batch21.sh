#!/bin/bash
# Round 6 batch 21: product library with K1 sort + longest-first parse dispatch + DPP run heads:
# deflate/inflate/codec/IPP GPU tests, ABBA of the DPP change.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu \
    tests/test_deflate_gpu.py tests/test_inflate_gpu.py tests/test_codec_gpu.py tests/test_ipp_gpu.py > gpurun_out/r06_t21.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r06_t21.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u scripts/debug/zvar_ab.py 256 8 dflt dpp > gpurun_out/r06_zab_dpp.json 2> gpurun_out/r06_zab_dpp.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/r06_zab_dpp.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_zab_dpp.err; exit $rc; }

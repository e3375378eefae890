#!/bin/bash
# Round 6 batch 32: the C3 decode as a two-chunk frame pipeline (levels 5..3 beside the other
# chunk's fused 2 + 1 band) vs one stream; then the DWT GPU tests on the product library.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
WHAT=decode_pipe timeout -k 10 300 python3 -u scripts/dwt_bands_scan.py 40 8 0 1 > gpurun_out/r06_dwt_dec_pipe.json 2> gpurun_out/r06_dwt_dec_pipe.err
rc=$?; echo "pipe rc=$rc"; cat gpurun_out/r06_dwt_dec_pipe.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_dwt_dec_pipe.err; exit $rc; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_dwt_gpu.py tests/test_dwt_lift_gpu.py tests/test_configs_gpu.py > gpurun_out/r06_t32.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r06_t32.log; exit $rc

#!/bin/bash
# The lifting DWT path: its GPU tests, then kernel stats of 200 encodes / decodes.
set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dwt_lift_gpu.py \
    > gpurun_out/lift_tests.log 2>&1
rc=$?; tail -5 gpurun_out/lift_tests.log; [ $rc -eq 0 ] || exit $rc
LIFT=1 bash scripts/debug/gpu/gpu_c3_prof.sh lift

#!/bin/bash
# codec GPU tests (the staged pipeline now deflates TIFF strips on the GPU), then the III end-to-end bench
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_codec_gpu.py tests/test_configs_gpu.py tests/test_tcbaac_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_e2e.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_e2e.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/bench_e2e.py --frames 64 > gpurun_out/e2e.jsonl 2> gpurun_out/e2e.err
rc=$?; echo "e2e rc=$rc"; cat gpurun_out/e2e.jsonl | cut -c1-900; tail -3 gpurun_out/e2e.err; exit $rc

#!/bin/bash
# Strip-kernel DWT: parity vs oracle, A/B against the fused kernels, f64 issue rate.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 60 ./scripts/micro/f64_rate > "$OUT/f64_rate.log" 2>&1; echo "f64 rc=$?"; cat "$OUT/f64_rate.log"
timeout -k 10 600 python -u -m pytest tests/test_dwt_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_dwt.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/pytest_dwt.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/ab_dwt.py ${AB:-1,6,7} > "$OUT/ab_dwt.log" 2>&1; rc=$?; echo "ab rc=$rc"; cat "$OUT/ab_dwt.log"

#!/bin/bash
# 2D-DWT frame pipeline: DWT GPU tests, then ABBA encode/decode A/B of the stream counts.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_dwt_gpu.py > "$OUT/pytest_dwt.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_dwt.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/ab_dwt.py ${ENC:-0,23,20} > "$OUT/ab_dwt_pipe_enc.log" 2>&1
rc=$?; echo "ab enc rc=$rc"; cat "$OUT/ab_dwt_pipe_enc.log"; [ $rc -eq 0 ] || exit $rc
DECODE=1 timeout -k 10 200 python -u scripts/ab_dwt.py ${DEC:-0,9} > "$OUT/ab_dwt_pipe_dec.log" 2>&1
rc=$?; echo "ab dec rc=$rc"; cat "$OUT/ab_dwt_pipe_dec.log"; exit $rc

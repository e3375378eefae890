#!/bin/bash
# GPU deflate: parity tests, then the throughput comparison (bounded steps).
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
OUT=$(pwd)/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_deflate_gpu.py -m gpu -x -v --timeout 180 --timeout-method thread > "$OUT/pytest_zlib.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" "$OUT/pytest_zlib.log" | tail -30
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/bench_zlib.py ${ZARGS:-} > "$OUT/bench_zlib.jsonl" 2> "$OUT/bench_zlib.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench_zlib.jsonl"; tail -5 "$OUT/bench_zlib.err"; exit $rc

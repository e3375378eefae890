#!/bin/bash
# GPU deflate: parity tests, the throughput comparison, and rocprofv3 kernel
# stats of the C4 workload (256 x 1080p shifted frames), each step bounded.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
TAG=${TAG:-z}
timeout -k 10 400 python -u -m pytest tests/test_deflate_gpu.py ${EXTRA_TESTS:-} -m gpu -x -v --timeout 180 --timeout-method thread > "$OUT/pytest_$TAG.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR|passed|failed" "$OUT/pytest_$TAG.log" | tail -15
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/bench_zlib.py ${ZARGS:-} > "$OUT/bench_$TAG.jsonl" 2> "$OUT/bench_$TAG.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench_$TAG.jsonl"; tail -3 "$OUT/bench_$TAG.err"
[ $rc -ne 0 ] && exit $rc
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/zprof_$TAG" -o run \
    -- python3 "$ROOT/scripts/bench_zlib.py" --only dct_c4_1080p --frames 256 --reps 1 > "$OUT/zprof_$TAG.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; grep -h workload "$OUT/zprof_$TAG.log" | cut -c1-240
f=$(find "$OUT/zprof_$TAG" -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | cut -c1-160 | head -12
exit $rc

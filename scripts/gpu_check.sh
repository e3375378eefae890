#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Stops at the first fault/abort/timeout (exit codes other than 0/1 from pytest).
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }

timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest_gpu rc=$rc"; tail -3 "$OUT/pytest_gpu.log"
if fatal $rc; then echo "fatal pytest rc=$rc"; exit $rc; fi

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 "$OUT/smoke.log"
if [ $rc -ne 0 ]; then exit $rc; fi

timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"; tail -3 "$OUT/bench.err"
if [ $rc -ne 0 ]; then exit $rc; fi

if [ "${NO_PROF:-0}" != "1" ]; then
  cd /tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run \
      -- python3 "$ROOT/bench.py" --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/prof_bench.log" 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -2 "$OUT/prof_bench.log"
  ls "$OUT/prof"
fi

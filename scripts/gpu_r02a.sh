#!/bin/bash
# Round 2, first GPU session: parity tests, smoke, bench with the driver's
# arguments (fixed warm-up + settle phase), rocprofv3 kernel stats of it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest_gpu rc=$rc"; tail -3 "$OUT/pytest_gpu.log"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_drv.json" 2> "$OUT/bench_drv.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench_drv.json"; tail -3 "$OUT/bench_drv.err"; [ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_drv" -o run \
    -- python3 "$ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/prof_drv.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -1 "$OUT/prof_drv.log"

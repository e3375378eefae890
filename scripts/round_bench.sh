#!/bin/bash
# bench.py line + rocprofv3 kernel stats of the same command + secondary paths.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; TAG=${1:-r01}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench_$TAG.json"; [ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run \
    -- python3 "$ROOT/bench.py" > "$OUT/prof_$TAG.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -1 "$OUT/prof_$TAG.log"; [ $rc -eq 0 ] || exit $rc
cd "$ROOT"
timeout -k 10 600 python scripts/bench_paths.py ${PATHS:+--only $PATHS} > "$OUT/paths_$TAG.log" 2> "$OUT/paths_$TAG.err"
rc=$?; echo "paths rc=$rc"; cat "$OUT/paths_$TAG.log"; tail -3 "$OUT/paths_$TAG.err"
exit $rc

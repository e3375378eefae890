#!/bin/bash
# The headline alone (no C4/C5 blocks, no CPU leg): bench.py line, then the same
# command under rocprofv3 --kernel-trace --stats, and the timed launches' stats
# from the trace (the last --steps dispatches of the encode kernel).
# Usage: scripts/gpu_headline_prof.sh <tag> [extra bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; TAG=${1:-r05}; shift || true
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--c4-frames 0 --c5-frames 0 --c3-steps 0 --c2-reps 0 --no-cpu-baseline --steps 100 $*"
timeout -k 10 300 python3 bench.py $ARGS > "$OUT/hl_$TAG.json" 2> "$OUT/hl_$TAG.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/hl_$TAG.json"; [ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/hlprof_$TAG" -o run \
    -- python3 "$ROOT/bench.py" $ARGS > "$OUT/hlprof_$TAG.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -1 "$OUT/hlprof_$TAG.log"; [ $rc -eq 0 ] || exit $rc
cd "$ROOT"
T=$(find "$OUT/hlprof_$TAG" -name "*kernel_trace.csv" | head -1)
S=$(find "$OUT/hlprof_$TAG" -name "*kernel_stats.csv" | head -1)
python3 scripts/trace_tail.py "$T" dct_dz_encode 100 3185049600 > "$OUT/hlprof_${TAG}_timed.json"
cat "$OUT/hlprof_${TAG}_timed.json"
cp "$S" "$OUT/hlprof_${TAG}_kernel_stats.csv"

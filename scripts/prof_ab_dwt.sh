#!/bin/bash
# rocprofv3 kernel stats of the DWT A/B script (per-level kernel times per variant)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_ab_dwt" -o run -- python3 "$ROOT/scripts/ab_dwt.py" ${AB:-1,6} > "$OUT/prof_ab_dwt.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -4 "$OUT/prof_ab_dwt.log"; exit $rc

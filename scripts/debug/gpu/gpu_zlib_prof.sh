#!/bin/bash
# rocprofv3 kernel stats of the GPU deflate bench (per-kernel times of K1/K2/K3)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/zprof" -o run \
    -- python3 "$ROOT/scripts/bench_zlib.py" ${ZARGS:-} > "$OUT/zprof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; grep -h workload "$OUT/zprof.log" | cut -c1-200
f=$(find "$OUT/zprof" -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | cut -c1-160 | head -12
exit $rc

#!/bin/bash
# GPU deflate check: the deflate tests, scripts/bench_zlib.py on C4 content (BUDGETS:
# workspace budgets to A/B, default the device-sized one), and a rocprofv3 kernel trace.
# Usage: scripts/debug/gpu/gpu_zab.sh TAG
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-z}
timeout -k 10 600 python -u -m pytest tests/test_deflate_gpu.py tests/test_inflate_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
for B in ${BUDGETS:-0}; do
  if [ "$B" = 0 ]; then unset VCF_ZX_BUDGET; else export VCF_ZX_BUDGET=$B; fi
  timeout -k 10 300 python -u scripts/bench_zlib.py --only ${ZW:-dct_c4_1080p} --frames 256 --reps 3 > gpurun_out/zab_${TAG}_$B.jsonl 2>&1 || exit $?
  echo "budget $B"; grep "^{" gpurun_out/zab_${TAG}_$B.jsonl | cut -c1-200
done
unset VCF_ZX_BUDGET
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/zprof_$TAG" -o run \
    -- python3 "$GRAFT_REPO_ROOT/scripts/bench_zlib.py" --only dct_c4_1080p --frames 256 --reps 2 > "$GRAFT_REPO_ROOT/gpurun_out/zprof_$TAG.log" 2>&1
echo "rocprof rc=$?"
cut -c1-160 $(find "$GRAFT_REPO_ROOT/gpurun_out/zprof_$TAG" -name "*kernel_stats.csv")

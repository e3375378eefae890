#!/bin/bash
# C3 per-kernel time: rocprofv3 kernel stats of 200 encodes and of 200 decodes
# (8 x 4K, l=5 bior4.4, Q=32) through scripts/dwt_once.py.  Usage: scripts/debug/gpu/gpu_c3_prof.sh TAG [VARIANT]
# (LIFT=1 in the environment: the lifting entry points)
set -u
cd "$GRAFT_REPO_ROOT"; ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp; cd /tmp
TAG=${1:-c3}; V=${2:-0}
for D in 0 1; do
  DECODE=$D timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/c3prof_${TAG}_d$D" -o run \
      -- python3 "$ROOT/scripts/dwt_once.py" $V 200 > "$ROOT/gpurun_out/c3prof_${TAG}_d$D.log" 2>&1
  rc=$?; echo "decode=$D rc=$rc"; [ $rc -eq 0 ] || exit $rc
  cat $(find "$ROOT/gpurun_out/c3prof_${TAG}_d$D" -name "*kernel_stats.csv") | cut -c1-220
done

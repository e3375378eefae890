#!/bin/bash
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for F in 1 4 16 64; do
  timeout -k 10 200 python -u scripts/bench_zlib.py --reps 2 --frames $F --only dct_1080p,rgb_1080p > gpurun_out/zs_$F.jsonl 2>/dev/null || exit $?
  python -c "
import json
for l in open('gpurun_out/zs_$F.jsonl'): d=json.loads(l); print($F, d['workload'][:12], d['gpu_ms'], round(d['gpu_ms']/$F,3), 'ms/frame')"
done

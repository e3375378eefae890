#!/bin/bash
# Band kernel schedule A/B: the DWT tests, then bench.py's C3 block with VCF_DWT_BAL=1 / 0 (ABBA).
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-bal}
timeout -k 10 900 python -u -m pytest tests/test_dwt_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
for V in 1 0 0 1; do
  VCF_DWT_BAL=$V timeout -k 10 200 python -u bench.py --steps 10 --c4-frames 0 --c5-frames 0 --c2-reps 0 --no-cpu-baseline > gpurun_out/c3_${TAG}_$V.json 2>/dev/null || exit $?
  echo "bal=$V $(python3 -c "import json; d=json.load(open('gpurun_out/c3_${TAG}_$V.json'))['c3_dwt']; print(d['encode']['launch_ms_events'], d['decode']['launch_ms_events'], d.get('error'))")"
done

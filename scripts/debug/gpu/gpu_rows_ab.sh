#!/bin/bash
# Block-row encode kernel: DCT/codec/deflate tests, then the headline with the block-row
# kernel (VCF_DCT_ROWS=1) and the raster-tile kernel (0) in ABBA order, then C4 deflate.
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-rows}
timeout -k 10 900 python -u -m pytest tests/test_dct_gpu.py tests/test_configs_gpu.py tests/test_codec_gpu.py tests/test_deflate_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
for V in 1 0 0 1 1 0; do
  VCF_DCT_ROWS=$V timeout -k 10 200 python -u bench.py --c4-frames 0 --c5-frames 0 --c3-steps 0 --c2-reps 0 --no-cpu-baseline > gpurun_out/hl_${TAG}_$V.json 2>/dev/null || exit $?
  echo "rows=$V $(python3 -c "import json; d=json.load(open('gpurun_out/hl_${TAG}_$V.json')); print(d['roofline']['kernel_ms_per_launch'], d['ms_per_step'], d['roofline']['frac'])")"
done
timeout -k 10 300 python -u scripts/bench_zlib.py --only dct_c4_1080p --frames 256 --reps 3 > gpurun_out/zab_$TAG.jsonl 2>&1 || exit $?
grep "^{" gpurun_out/zab_$TAG.jsonl | cut -c1-120

#!/bin/bash
# A/B of GPU deflate library variants (scripts/build_variant.sh) on C4 content, ABBA-ish order.
# Usage: scripts/debug/gpu/gpu_zwin.sh TAG VARIANT...   (VARIANT "0" = the product library)
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; shift
for V in "$@" 0; do
  if [ "$V" = 0 ]; then unset VCF_AMD_LIB; else export VCF_AMD_LIB=$PWD/vcf_amd/libvcf_amd_$V.so; fi
  timeout -k 10 300 python -u scripts/bench_zlib.py --only ${ZW:-dct_c4_1080p} --frames 256 --reps 3 > gpurun_out/zwin_${TAG}_$V.jsonl 2>&1 || exit $?
  echo "variant $V: $(grep '^{' gpurun_out/zwin_${TAG}_$V.jsonl | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["gpu_ms"], d["bytes_equal_zlib"])')"
done

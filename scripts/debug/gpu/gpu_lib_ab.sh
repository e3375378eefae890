#!/bin/bash
# A/B of the C3 DWT timing between the product library and vcf_amd/libvcf_amd_$1.so
# (ABBA, scripts/dwt_time.py), after the DWT GPU tests on the product library.
set -u
cd "$GRAFT_REPO_ROOT"
V=${1:-old}
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dwt_gpu.py \
    > gpurun_out/lib_ab_tests.log 2>&1
rc=$?; tail -2 gpurun_out/lib_ab_tests.log; [ $rc -eq 0 ] || exit $rc
for X in prod $V $V prod; do
  if [ $X = prod ]; then timeout -k 10 120 python3 scripts/dwt_time.py 50 5 || exit 1
  else VCF_AMD_LIB=vcf_amd/libvcf_amd_$X.so timeout -k 10 120 python3 scripts/dwt_time.py 50 5 || exit 1; fi
done

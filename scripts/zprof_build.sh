#!/bin/bash
# Diagnostic build of the GPU deflate with per-phase clock counters (VCF_ZLIB_PROF):
# build/zprof/libvcf_zprof.so = the product sources with vcf_deflate.hip instrumented.
# Run in the build container; scripts/zprof_run.py loads it on the GPU box.
set -eu
cd "$(dirname "$0")/.."
mkdir -p build/zprof
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -I include -I vcf_amd/csrc"
$H -DVCF_ZLIB_PROF=1 -c vcf_amd/csrc/vcf_deflate.hip -o build/zprof/vcf_deflate.o
$H -c vcf_amd/csrc/vcf_runtime.hip -o build/zprof/vcf_runtime.o
$H --offload-arch=gfx950 -shared build/zprof/vcf_deflate.o build/zprof/vcf_runtime.o -o scripts/libvcf_zprof.so
echo built scripts/libvcf_zprof.so

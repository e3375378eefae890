#!/bin/bash
# Diagnostic builds of the GPU deflate with per-phase clock counters (VCF_ZLIB_PROF):
# scripts/debug/libvcf_zprof.so = the product sources with vcf_deflate.hip instrumented;
# with arguments NAME DEFINES..., scripts/debug/libvcf_zprof_NAME.so with those -D options
# (A/B of the diagnostic switches).  Run in the build container; scripts/debug/zprof_run.py
# loads it on the GPU box (ZPROF_LIB=libvcf_zprof_NAME.so).
set -eu
cd "$(dirname "$0")/../.."
name="${1:-}"; shift || true
defs=""; for d in "$@"; do defs="$defs -D$d"; done
mkdir -p build/zprof
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -I include -I vcf_amd/csrc"
$H -DVCF_ZLIB_PROF=1 $defs -c vcf_amd/csrc/vcf_deflate.hip -o build/zprof/vcf_deflate$name.o
$H -c vcf_amd/csrc/vcf_runtime.hip -o build/zprof/vcf_runtime.o
out=scripts/debug/libvcf_zprof${name:+_$name}.so
$H --offload-arch=gfx950 -shared build/zprof/vcf_deflate$name.o build/zprof/vcf_runtime.o -o $out
echo built $out

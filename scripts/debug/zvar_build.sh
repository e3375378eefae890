#!/bin/bash
# A/B builds of the GPU deflate without instrumentation: scripts/debug/libvcf_zvar_NAME.so
# from vcf_deflate.hip with the given -D switches (VCF_ZX_*); scripts/debug/zdbg.py loads
# one with ZLIB_SO=libvcf_zvar_NAME.so.
set -eu
cd "$(dirname "$0")/../.."
name="$1"; shift
defs=""; for d in "$@"; do defs="$defs -D$d"; done
mkdir -p build/zprof
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -I include -I vcf_amd/csrc"
$H $defs -c vcf_amd/csrc/vcf_deflate.hip -o build/zprof/vcf_deflate_v$name.o
$H -c vcf_amd/csrc/vcf_runtime.hip -o build/zprof/vcf_runtime.o
$H --offload-arch=gfx950 -shared build/zprof/vcf_deflate_v$name.o build/zprof/vcf_runtime.o -o scripts/debug/libvcf_zvar_$name.so
echo built scripts/debug/libvcf_zvar_$name.so

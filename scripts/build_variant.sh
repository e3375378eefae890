#!/bin/bash
# Build an A/B variant of the product library: one source recompiled with extra
# -D switches, linked with the other product objects (build/obj, from
# python -m vcf_amd._build) into vcf_amd/libvcf_amd_<NAME>.so; run against it
# with VCF_AMD_LIB=vcf_amd/libvcf_amd_<NAME>.so.  Build container only.
# Usage: scripts/build_variant.sh NAME SOURCE.hip "-DX=1 -DY=2"
set -eu
cd "$(dirname "$0")/.."
NAME=$1; SRC=$2; DEFS=${3:-}
H=/opt/rocm/bin/hipcc
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -I include -I vcf_amd/csrc"
mkdir -p build/variant
$H $FLAGS $DEFS -c vcf_amd/csrc/$SRC -o build/variant/${SRC%.hip}_$NAME.o
OBJS=$(python3 -c "
import vcf_amd._build as B
print(' '.join('build/obj/' + s.rsplit('.', 1)[0] + '.o' for s in B.SOURCES if s != '$SRC'))")
$H --offload-arch=gfx950 -shared -fPIC $OBJS build/variant/${SRC%.hip}_$NAME.o -lz -ldl -o vcf_amd/libvcf_amd_$NAME.so
echo built vcf_amd/libvcf_amd_$NAME.so

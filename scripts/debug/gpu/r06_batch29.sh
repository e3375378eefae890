#!/bin/bash
# Round 6 batch 29: K1 rank masks (per-digit rounds vs bit-sliced, with library copies), then the
# band cuts of the bit-exact DWT's fused kernels.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python3 -u scripts/debug/zvar_ab.py 256 6 dloop dbits dloop2 dbits2 > gpurun_out/r06_zab_dloop.json 2> gpurun_out/r06_zab_dloop.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/r06_zab_dloop.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_zab_dloop.err; exit $rc; }
timeout -k 10 300 python3 -u scripts/dwt_bands_scan.py 40 6 0 1 2 3 4 5 6 8 12 > gpurun_out/r06_dwt_bands_enc.json 2> gpurun_out/r06_dwt_bands_enc.err
rc=$?; echo "enc rc=$rc"; cat gpurun_out/r06_dwt_bands_enc.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_dwt_bands_enc.err; exit $rc; }
WHAT=decode timeout -k 10 300 python3 -u scripts/dwt_bands_scan.py 40 6 0 60 90 108 136 180 216 270 360 540 > gpurun_out/r06_dwt_bands_dec.json 2> gpurun_out/r06_dwt_bands_dec.err
rc=$?; echo "dec rc=$rc"; cat gpurun_out/r06_dwt_bands_dec.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_dwt_bands_dec.err; exit $rc; }

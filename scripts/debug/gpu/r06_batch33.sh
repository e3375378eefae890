#!/bin/bash
# Round 6 batch 33: the C3 encode as a two-chunk frame pipeline with the band kernel (whole-call band
# cut) vs one stream.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
WHAT=encode_pipe timeout -k 10 300 python3 -u scripts/dwt_bands_scan.py 40 8 0 1 > gpurun_out/r06_dwt_enc_pipe.json 2> gpurun_out/r06_dwt_enc_pipe.err
rc=$?; echo "pipe rc=$rc"; cat gpurun_out/r06_dwt_enc_pipe.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_dwt_enc_pipe.err; exit $rc; }

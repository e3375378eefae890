#!/bin/bash
# Round 6 batch 23: the noise floor of library A/B: the product library and a byte-identical copy
# (a second load), the variant build of the same source and its copy, and the quad-count variant.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python3 -u scripts/debug/zvar_ab.py 256 8 pcopy dflt dcopy quad > gpurun_out/r06_zab_copies.json 2> gpurun_out/r06_zab_copies.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/r06_zab_copies.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_zab_copies.err; exit $rc; }

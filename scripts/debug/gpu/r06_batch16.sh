#!/bin/bash
# Round 6 batch 16: phase clocks of the radix-sort K1 (diagnostic build).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 240 python3 -u scripts/debug/zprof_run.py 256 > gpurun_out/r06_zprof_sort.json 2> gpurun_out/r06_zprof_sort.err
rc=$?; echo "zprof rc=$rc"; python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print({k:v for k,v in d.items() if k.startswith('sort') or k=='ms'})" gpurun_out/r06_zprof_sort.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_zprof_sort.err; exit $rc; }

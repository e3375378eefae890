#!/bin/bash
# Round 6 batch 26: GPU deflate on raw RGB / DCT index workloads (the non-lazy path's speed after
# the side-kernel list), then the counters of one C4 call (K1 radix sort, lazy parse).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u scripts/bench_zlib.py --frames 64 --reps 3 > gpurun_out/r06_bench_zlib.jsonl 2> gpurun_out/r06_bench_zlib.err
rc=$?; echo "bench_zlib rc=$rc"; cut -c1-400 gpurun_out/r06_bench_zlib.jsonl; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_bench_zlib.err; exit $rc; }
bash scripts/pmc_r06.sh zlib_c4_r06b python3 scripts/zlib_once.py 256 1

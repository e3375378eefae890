set -u -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/bench_zlib.py --only dct_c4_1080p,dct_1080p,dct_4k,rgb_1080p --frames 256 --reps 3 > gpurun_out/bz.jsonl 2> gpurun_out/bz.err; rc=$?
cut -c1-700 gpurun_out/bz.jsonl; grep -i "differ\|error\|Trace" gpurun_out/bz.err; exit $rc

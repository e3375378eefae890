set -u -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for L in libvcf_zprof.so libvcf_zprof_noprio.so libvcf_zprof_serial.so libvcf_zprof.so libvcf_zprof_noprio.so libvcf_zprof_serial.so; do
  ZPROF_LIB=$L timeout -k 10 200 python -u scripts/zprof_run.py 256 || exit $?
done
timeout -k 10 400 python -u -m pytest tests/test_deflate_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/zt.log 2>&1; rc=$?; echo "deflate tests rc=$rc"; tail -2 gpurun_out/zt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_zlib.py --only dct_c4_1080p,dct_1080p,rgb_1080p --frames 256 --reps 3 > gpurun_out/bz.jsonl 2> gpurun_out/bz.err || exit $?
cut -c1-400 gpurun_out/bz.jsonl; grep differ gpurun_out/bz.err
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/zprof_w7" -o run \
    -- python3 "$GRAFT_REPO_ROOT/scripts/bench_zlib.py" --only dct_c4_1080p --frames 256 --reps 1 > "$GRAFT_REPO_ROOT/gpurun_out/zprof_w7.log" 2>&1; echo "rocprof rc=$?"

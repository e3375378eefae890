set -u -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_dct_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "decode_variants" > gpurun_out/dec_t.log 2>&1; rc=$?; echo "decode tests rc=$rc"; tail -3 gpurun_out/dec_t.log; [ $rc -eq 0 ] || exit $rc
DECODE=1 DENSE=1 timeout -k 10 200 python -u scripts/bench_variants.py 0,8,9,10,11,12,13 > gpurun_out/dec_ab_dense.log 2>&1 || exit $?
cat gpurun_out/dec_ab_dense.log
DECODE=1 timeout -k 10 200 python -u scripts/bench_variants.py 0,8,9,10,11,12,13 > gpurun_out/dec_ab_smooth.log 2>&1 || exit $?
cat gpurun_out/dec_ab_smooth.log
timeout -k 10 400 python -u -m pytest tests/test_deflate_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/zt.log 2>&1; rc=$?; echo "deflate tests rc=$rc"; tail -2 gpurun_out/zt.log; [ $rc -eq 0 ] || exit $rc
for L in libvcf_zprof.so libvcf_zprof_nocap.so libvcf_zprof_serial.so libvcf_zprof.so libvcf_zprof_nocap.so libvcf_zprof_serial.so; do
  ZPROF_LIB=$L timeout -k 10 200 python -u scripts/debug/zprof_run.py 256 || exit $?
done
timeout -k 10 300 python -u scripts/bench_zlib.py --only dct_c4_1080p --frames 256 --reps 3 > gpurun_out/bz.jsonl 2>/dev/null || exit $?
cut -c1-300 gpurun_out/bz.jsonl
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/zprof_w6" -o run \
    -- python3 "$GRAFT_REPO_ROOT/scripts/bench_zlib.py" --only dct_c4_1080p --frames 256 --reps 1 > "$GRAFT_REPO_ROOT/gpurun_out/zprof_w6.log" 2>&1; echo "rocprof rc=$?"

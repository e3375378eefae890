set -u -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_inflate_gpu.py tests/test_deflate_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/zt.log 2>&1; rc=$?; echo "inflate/deflate tests rc=$rc"; tail -15 gpurun_out/zt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/zprof_run.py 256 > gpurun_out/zp256.json || exit $?
cat gpurun_out/zp256.json
timeout -k 10 300 python -u scripts/bench_zlib.py --only dct_c4_1080p,dct_1080p,rgb_1080p --frames 256 --reps 2 2>/dev/null | cut -c1-220 || exit $?
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/zprof_w5" -o run \
    -- python3 "$GRAFT_REPO_ROOT/scripts/bench_zlib.py" --only dct_c4_1080p --frames 256 --reps 1 > "$GRAFT_REPO_ROOT/gpurun_out/zprof_w5.log" 2>&1; echo "rocprof rc=$?"
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_codec_gpu.py tests/test_standalone_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/codec.log 2>&1; rc=$?; echo "codec tests rc=$rc"; tail -3 gpurun_out/codec.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_e2e.py --frames 64 > gpurun_out/e2e.jsonl 2> gpurun_out/e2e.err; echo "e2e rc=$?"; cut -c1-600 gpurun_out/e2e.jsonl

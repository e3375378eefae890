set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for L in sl1 sl2 sl1 sl2; do
  ZLIB_SO=libvcf_zvar_$L.so timeout -k 10 300 python -u scripts/zdbg.py 256 gpurun_out/zs_${L}.npz 2>&1 | grep -v "^  strip" | cut -c1-200 || exit $?
done
timeout -k 10 400 python -u -m pytest tests/test_deflate_gpu.py tests/test_ipp_gpu.py tests/test_codec_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/zt.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/zt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_zlib.py --only dct_c4_1080p,dct_1080p,rgb_1080p --frames 256 --reps 3 > gpurun_out/bz.jsonl 2> gpurun_out/bz.err || exit $?
cut -c1-400 gpurun_out/bz.jsonl; grep differ gpurun_out/bz.err
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/zk_sl2" -o run \
    -- python3 "$GRAFT_REPO_ROOT/scripts/bench_zlib.py" --only dct_c4_1080p --frames 256 --reps 1 > /dev/null 2>&1; echo "rocprof rc=$?"

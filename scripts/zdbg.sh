set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_deflate_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/zt.log 2>&1; echo "deflate tests rc=$?"; tail -2 gpurun_out/zt.log
VCF_ZLIB_SLOTS=1 timeout -k 10 200 python -u scripts/zprof_run.py 256 > gpurun_out/zp256.json || exit $?
cat gpurun_out/zp256.json
VCF_ZLIB_SLOTS=3 timeout -k 10 300 python -u scripts/zdbg.py 256 gpurun_out/zd3.npz || exit $?
VCF_ZLIB_SLOTS=3 timeout -k 10 300 python -u scripts/zdbg.py 256 gpurun_out/zd3b.npz || exit $?
for S in 1 3; do
VCF_ZLIB_SLOTS=$S timeout -k 10 300 python -u scripts/bench_zlib.py --only dct_c4_1080p,dct_1080p,rgb_1080p --frames 256 --reps 2 2>/dev/null | cut -c1-200; done

set -u -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_dct_gpu.py tests/test_configs_gpu.py tests/test_codec_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/dec_t.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/dec_t.log; [ $rc -eq 0 ] || exit $rc
DECODE=1 DENSE=1 timeout -k 10 200 python -u scripts/bench_variants.py 0,9,10 > gpurun_out/dec_ab_dense2.log 2>&1 || exit $?
cat gpurun_out/dec_ab_dense2.log
DECODE=1 timeout -k 10 200 python -u scripts/bench_variants.py 0,9,10 > gpurun_out/dec_ab_smooth2.log 2>&1 || exit $?
cat gpurun_out/dec_ab_smooth2.log

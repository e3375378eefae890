set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_dct_gpu.py tests/test_codec_gpu.py tests/test_configs_gpu.py tests/test_dct_any_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_dec.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_dec.log; [ $rc -eq 0 ] || exit $rc
DECODE=1 ROUNDS=16 timeout -k 10 300 python -u scripts/bench_variants.py 2,0 > gpurun_out/ab_dec.log 2>&1
rc=$?; echo "ab rc=$rc"; tail -3 gpurun_out/ab_dec.log

set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_dct_any_gpu.py tests/test_abi.py tests/test_codec_gpu.py tests/test_dct_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_any.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_any.log

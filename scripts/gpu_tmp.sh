set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests/test_plugins_gpu.py tests/test_dwt_gpu.py tests/test_dct_any_gpu.py tests/test_abi.py tests/test_codec_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_plug.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_plug.log

set -u -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_deflate_gpu.py tests/test_inflate_gpu.py tests/test_codec_gpu.py tests/test_ipp_gpu.py tests/test_dist_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/zt.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/zt.log; exit $rc

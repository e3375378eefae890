set -u -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for L in e0 e1 e0 e1; do
  ZLIB_SO=libvcf_zvar_$L.so timeout -k 10 300 python -u scripts/zdbg.py 256 gpurun_out/zs_${L}.npz > gpurun_out/zs_$L.log 2>&1; rc=$?
  grep -v "^  strip" gpurun_out/zs_$L.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 400 python -u -m pytest tests/test_deflate_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/zt.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/zt.log; exit $rc

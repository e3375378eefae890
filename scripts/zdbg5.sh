set -u -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for L in pp0 pp3 pp0 pp3; do
  ZLIB_SO=libvcf_zvar_$L.so timeout -k 10 300 python -u scripts/zdbg.py 256 gpurun_out/zs_${L}.npz > gpurun_out/zs_$L.log 2>&1; rc=$?
  grep -v "^  strip" gpurun_out/zs_$L.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done

set -u -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2; do
  ZLIB_SO=libvcf_zvar_wcheck.so timeout -k 10 300 python -u scripts/zdbg.py 256 gpurun_out/zw_$r.npz 2>&1 | grep -v "^  strip" | cut -c1-200 || exit $?
done
for r in 1 2 3 4 5; do
  timeout -k 10 300 python -u scripts/zdbg.py 256 gpurun_out/zp_$r.npz 2>&1 | grep -v "^  strip" | cut -c1-200 || exit $?
  ZLIB_SO=libvcf_zvar_serial.so timeout -k 10 300 python -u scripts/zdbg.py 256 gpurun_out/zs_$r.npz 2>&1 | grep -v "^  strip" | cut -c1-200 || exit $?
done

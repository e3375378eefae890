#!/bin/bash
# Round-6 counters: a kernel trace + five --pmc passes over one command, summarised
# per kernel with full template names (scripts/pmc_kernels.py).
#   scripts/pmc_r06.sh NAME CMD...      -> gpurun_out/pmc_NAME/{summary.json,trace.log}
# e.g. scripts/pmc_r06.sh zlib_c4 python3 scripts/zlib_once.py 256 1
#      DENSE=1 scripts/pmc_r06.sh dct_dec_dense python3 scripts/dct_dec_once.py 2
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); NAME=$1; shift
OUT=$ROOT/gpurun_out/pmc_$NAME; RAW=/tmp/pmc_$NAME
rm -rf "$OUT" "$RAW"; mkdir -p "$OUT" "$RAW"; export TMPDIR=/tmp
cd /tmp
# the command's relative paths are the repo's: run it from there through an absolute path
ARGS=()
for a in "$@"; do if [ -e "$ROOT/$a" ]; then ARGS+=("$ROOT/$a"); else ARGS+=("$a"); fi; done
timeout -k 10 -s KILL ${PMC_TIMEOUT:-240} rocprofv3 --kernel-trace --stats --output-format csv -d "$RAW/trace" -o run \
    -- "${ARGS[@]}" > "$OUT/trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/trace.log"; exit $rc; }
find "$RAW/trace" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 -s KILL ${PMC_TIMEOUT:-240} rocprofv3 --pmc $grp --output-format csv -d "$RAW/p$i" -o pmc \
      -- "${ARGS[@]}" > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || { tail -5 "$OUT/p$i.log"; exit $rc; }
done
python3 "$ROOT/scripts/pmc_kernels.py" "$RAW" > "$OUT/summary.json"
# the raw counter CSVs travel back too (small: one row per dispatch and counter)
for d in "$RAW"/p* "$RAW"/trace; do mkdir -p "$OUT/raw/$(basename "$d")"; find "$d" -name "*.csv" -exec cp {} "$OUT/raw/$(basename "$d")/" \; ; done
echo "summary: $OUT/summary.json"

#!/bin/bash
# PMC passes + a kernel trace over the C3 DWT encode (scripts/dwt_once.py VARIANT):
#   VARIANT=17 scripts/pmc_dwt.sh   -> gpurun_out/pmc_dwt_v$VARIANT/{summary.txt,trace}
#   DECODE=1 VARIANT=0 scripts/pmc_dwt.sh -> the decode, gpurun_out/pmc_dwt_v0_dec/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); V=${VARIANT:-0}; SUF=""; if [ "${DECODE:-0}" = 1 ]; then SUF=_dec; fi
OUT=$ROOT/gpurun_out/pmc_dwt_v$V$SUF; RAW=/tmp/pmc_dwt_v$V$SUF
rm -rf "$OUT" "$RAW"; mkdir -p "$OUT" "$RAW"; export TMPDIR=/tmp; cd /tmp   # raw counters stay on the box
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$RAW/trace" -o run \
    -- python3 "$ROOT/scripts/dwt_once.py" "$V" 20 > "$OUT/trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
find "$RAW/trace" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
i=0
for grp in "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES" \
           "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F64 GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$RAW/p$i" -o pmc \
      -- python3 "$ROOT/scripts/dwt_once.py" "$V" 2 > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done
python3 - "$RAW" > "$OUT/summary.txt" << 'PY'
import csv, glob, sys, collections, re
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r.get("Kernel_Name", "")
        m = re.search(r"(\w+_kernel)<([^>]*)>", n) or re.search(r"(\w+_kernel)\(", n)
        if not m: continue
        key = m.group(0)[:70] + " grid=" + r.get("Grid_Size", r.get("Grid_Size_X", "?"))
        acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(acc.items()):
    print(k, {c: round(sum(v) / len(v)) for c, v in sorted(d.items())})
PY
cat "$OUT/summary.txt"

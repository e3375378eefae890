#!/bin/bash
# PMC passes over one DWT encode variant: VARIANT=6 scripts/pmc_strip.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc_strip_${VARIANT:-6}; mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o pmc \
      -- python3 "$ROOT/scripts/dwt_once.py" ${VARIANT:-6} 2 > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 - "$OUT" << 'PY' > "$OUT/summary.txt"
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
echo summary rc=$?; cat "$OUT/summary.txt"

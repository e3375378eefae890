#!/bin/bash
# PMC passes over the DWT bench (fused level kernels): scripts/pmc_dwt.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=/tmp/pmc_dwt; rm -rf "$OUT"; mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp   # raw counters stay on the box
i=0
for grp in "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES" \
           "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F64 GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o pmc \
      -- python3 "$ROOT/scripts/bench_paths.py" --only dwt --dwt-variants 0 --steps 1 > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  case $rc in 0) ;; 124|134|137|139) exit $rc;; *) tail -3 "$OUT/p$i.log";; esac
done
python3 - "$OUT" << 'PY'
import csv, glob, sys, collections, re
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r.get("Kernel_Name", "")
        m = re.search(r"(\w+_kernel)<([^>]*)>", n) or re.search(r"(\w+_kernel)\(", n)
        if not m: continue
        key = m.group(0)[:60] + " grid=" + r.get("Grid_Size", r.get("Grid_Size_X", "?"))
        acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(acc.items()):
    print(k, {c: round(sum(v) / len(v)) for c, v in sorted(d.items())})
PY

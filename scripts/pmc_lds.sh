#!/bin/bash
# LDS / VALU / memory-instruction counters per encode variant: scripts/pmc_lds.sh "1 3"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc_lds; mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
for v in ${1:-1 3}; do
  for grp in "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_MEM_VIOLATIONS" \
             "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES" \
             "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"; do
    tag=$(echo $grp | cut -c1-12 | tr ' ' '_')
    timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/v${v}_$tag" -o pmc \
        -- python3 "$ROOT/bench.py" --no-cpu-baseline --steps 3 --warmup 1 --variant $v > "$OUT/v${v}_$tag.log" 2>&1
    rc=$?; echo "v$v [$grp] rc=$rc"
    case $rc in 0) ;; 124|134|137|139) exit $rc;; *) tail -3 "$OUT/v${v}_$tag.log";; esac
  done
done
python3 - "$OUT" << 'PY'
import csv, glob, os, sys, collections
out = sys.argv[1]
for v in sorted({os.path.basename(d).split('_')[0] for d in glob.glob(out + '/v*_*') if os.path.isdir(d)}):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"{out}/{v}_*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "encode" in r.get("Kernel_Name", ""):
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(v, {k: round(sum(x) / len(x)) for k, x in sorted(acc.items())})
PY

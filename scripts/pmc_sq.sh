#!/bin/bash
# SQ stall-breakdown counters per encode variant: scripts/pmc_sq.sh "1 2 4"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc_sq; mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
for v in ${1:-1 2}; do
  for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES" \
             "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS" \
             "GRBM_GUI_ACTIVE GRBM_COUNT"; do
    tag=$(echo $grp | cut -c1-12 | tr ' ' '_')
    timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/v${v}_$tag" -o pmc \
        -- python3 "$ROOT/bench.py" --no-cpu-baseline --steps 3 --warmup 1 --variant $v > "$OUT/v${v}_$tag.log" 2>&1
    rc=$?; echo "v$v [$grp] rc=$rc"
    case $rc in 0) ;; 124|134|137|139) exit $rc;; *) tail -3 "$OUT/v${v}_$tag.log";; esac
  done
  python3 "$ROOT/scripts/pmc_summary.py" "$OUT" > /dev/null
done
python3 - "$OUT" << 'PY'
import csv, glob, os, sys, collections
out = sys.argv[1]
for v in sorted({os.path.basename(d).split('_')[0] for d in glob.glob(out + '/v*_*') if os.path.isdir(d)}):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"{out}/{v}_*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(v, {k: round(sum(x) / len(x)) for k, x in sorted(acc.items())})
PY

#!/bin/bash
# SQ counters for one configuration's kernels (default RS(200,55) 256 KiB), one pass per group.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
ARGS=${SWEEP_ARGS:---k 200 --m 55 --shard-bytes 262144 --stripes 64 --erase 0,2,4,6 --nv 2 --rounds 1 --reps 1}
mkdir -p gpurun_out/sqw
i=0
# PMC_GROUPS: counter groups separated by ';' (one rocprofv3 pass each)
G=${PMC_GROUPS:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD;SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_INSTS_VMEM_WR"}
IFS=';' read -ra GRPS <<< "$G"
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d "$R/gpurun_out/sqw/g$i" -o run -- \
    python3 "$R/tools/kernel_sweep.py" $ARGS > gpurun_out/sqw/g$i.log 2>&1 || { echo "group $i failed"; tail -5 gpurun_out/sqw/g$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(dict)
for f in glob.glob("gpurun_out/sqw/g*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:70]
        agg[k].setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k, d in agg.items():
    if "at::" in k: continue
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:24s} {sum(v)/len(v):.4g}  (n={len(v)})")
PY

#!/bin/bash
# Instruction / scalar cache counters (SQC) of the low-rate block-form decode kernels
# (RS(300,1000) 1 MiB x 4), one rocprofv3 --pmc pass per pair.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
OUT=gpurun_out/r5/sqc; mkdir -p $OUT
ARGS="--k 300 --m 1000 --shard-bytes 1048576 --stripes 4 --erase 100:0:3 --nv 4 --rounds 1 --reps 1"
i=0
for grp in "SQC_ICACHE_HITS SQC_ICACHE_MISSES" "SQC_DCACHE_HITS SQC_DCACHE_MISSES" "SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$R/$OUT/g$i" -o run -- \
    python3 "$R/tools/kernel_sweep.py" $ARGS > $OUT/g$i.log 2>&1 || { echo "group $i failed"; tail -5 $OUT/g$i.log; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, collections, sys
agg = collections.defaultdict(dict)
for f in glob.glob(sys.argv[1] + "/g*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:70]
        agg[k].setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k, d in agg.items():
    if "at::" in k: continue
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {sum(v)/len(v):.6g}  (n={len(v)})")
PY

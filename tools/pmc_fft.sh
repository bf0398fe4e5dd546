#!/bin/bash
# SQ counters + HBM traffic of one configuration's kernels (default: RS(200,55) 256 KiB
# encode on the FFT kernel), one rocprofv3 --pmc pass per counter group.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
ARGS=${SWEEP_ARGS:---k 200 --m 55 --shard-bytes 262144 --stripes 64 --erase 0 --nv 4 --rounds 1 --reps 1}
OUT=${PMC_OUT:-gpurun_out/pmcfft}
mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_WR SQ_IFETCH" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$R/$OUT/g$i" -o run -- \
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
        print(f"   {c:24s} {sum(v)/len(v):.6g}  (n={len(v)})")
PY

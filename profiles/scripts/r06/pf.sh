#!/bin/bash
# Round 6: (1) deeper next-position prefetch in the c4 pattern-compiled reconstruct, spilled builds
# allowed, interleaved A/B in one process (256 stripes); (2) where the per-stripe chunk-16/32 fused
# reconstruct's time goes (RS_AMD_FFT_DEBUG bits: 1 no loads, 2 no stores, 4 no tail, 8 no runtime
# multiplies); (3) the per-stripe call's kernel split under rocprofv3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r6pf; mkdir -p $O
FORM=pattern ROUNDS=3 REPS=3 timeout -k 10 500 python -u tools/fft_decompose.py 200 55 262144 256 55 \
  RS_AMD_FFT_ALLOW_SPILL=1 RS_AMD_FFT_PREFETCH=3,4,5,6 > $O/pf_pattern.log 2>&1 || { tail -5 $O/pf_pattern.log; exit 1; }
grep '^{' $O/pf_pattern.log | cut -c1-260
for shp in "k=16 m=16 loss=16 max_e=16" "k=40 m=12 loss=12 max_e=12"; do
  f=$O/dbg_$(echo $shp | tr ' =' '__').log
  timeout -k 10 300 python -u tools/patterns_bench.py 256 $shp sb=1048576 RS_AMD_FFT_DEBUG=0,1,2,3,4,8,12 > $f 2>&1 || { tail -5 $f; exit 1; }
  grep DEBUG $f | cut -c1-300
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof16 -o run -- python3 tools/patterns_bench.py 256 k=16 m=16 loss=16 max_e=16 sb=1048576 > $O/prof16.log 2>&1 || { tail -5 $O/prof16.log; exit 1; }
find $O/prof16 -name '*kernel_stats.csv' -exec cut -d, -f1-8 {} \; | head -12
# (4) SQ / SQC counters of the per-stripe RS(16,16) call, one --pmc pass per group
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT" \
           "SQC_DCACHE_HITS SQC_DCACHE_MISSES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$(pwd)/$O/sq$i" -o run -- \
    python3 tools/patterns_bench.py 256 k=16 m=16 loss=16 max_e=16 sb=1048576 > $O/sq$i.log 2>&1 || { echo "group $i failed"; tail -5 $O/sq$i.log; exit 1; }
done
python3 - "$O" <<'PY'
import csv, glob, collections, sys
agg = collections.defaultdict(dict)
for f in glob.glob(sys.argv[1] + "/sq*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:70]
        agg[k].setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k, d in agg.items():
    if "at::" in k or "rs_fft_decode" not in k: continue
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {sum(v)/len(v):.6g}  (n={len(v)})")
PY

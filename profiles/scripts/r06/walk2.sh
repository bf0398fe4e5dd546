#!/bin/bash
# Round 6: CU-grouped unit walk (RS_AMD_FFT_WALK=2) for the per-stripe chunk-16 / chunk-32 fused
# reconstruct: the 4 (2) workgroups a CU holds take consecutive units of one stripe, so the rmul
# masks of that stripe's decode block are shared in the scalar cache. Rates A/B and SQC hit rates.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r6w2; mkdir -p $O
for shp in "k=16 m=16 loss=16 max_e=16" "k=40 m=12 loss=12 max_e=12" "k=64 m=32 loss=32 max_e=32"; do
  f=$O/w_$(echo $shp | tr ' =' '__').log
  timeout -k 10 300 python -u tools/patterns_bench.py 256 $shp sb=1048576 RS_AMD_FFT_WALK=0,2,0,2 > $f 2>&1 || { tail -5 $f; exit 1; }
  grep WALK $f | cut -c1-300
done
for wk in 0 2; do
  RS_AMD_FFT_WALK=$wk timeout -s KILL 120 rocprofv3 --pmc SQC_DCACHE_HITS SQC_DCACHE_MISSES --output-format csv -d "$(pwd)/$O/sqc$wk" -o run -- \
    python3 tools/patterns_bench.py 256 k=16 m=16 loss=16 max_e=16 sb=1048576 > $O/sqc$wk.log 2>&1 || { echo "sqc $wk failed"; tail -5 $O/sqc$wk.log; exit 1; }
done
python3 - "$O" <<'PY'
import csv, glob, collections, sys
for f in sorted(glob.glob(sys.argv[1] + "/sqc*/run_counter_collection.csv")):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "rs_fft_decode" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f.split("/")[-2], {k: round(sum(v) / len(v)) for k, v in agg.items()})
PY

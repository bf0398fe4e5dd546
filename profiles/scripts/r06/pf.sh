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

#!/bin/bash
# Round 4: runtime-multiply variants of the per-stripe fused reconstruct (mid-band codes)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp; export RS_AMD_JIT_SYNC=1
: > gpurun_out/r4_mb_ab.log
for a in "256 k=16 m=16 sb=1048576 loss=16 max_e=16" "256 k=40 m=12 sb=1048576 loss=12 max_e=12" "256 k=200 m=55 sb=262144 loss=55 max_e=55"; do
  for v in "RS_AMD_FFT_RMULG=1,2,4,8" "RS_AMD_FFT_RMULV=0,1"; do
    timeout -k 10 300 python -u tools/patterns_bench.py $a $v > gpurun_out/pb_ab.log 2>&1 || { echo FAILED $a $v; tail gpurun_out/pb_ab.log; exit 1; }
    echo "== $a $v" >> gpurun_out/r4_mb_ab.log; grep -E '^\{' gpurun_out/pb_ab.log | grep -v '"RS_AMD_PATTERNS"' >> gpurun_out/r4_mb_ab.log
  done
done
cut -c1-160 gpurun_out/r4_mb_ab.log

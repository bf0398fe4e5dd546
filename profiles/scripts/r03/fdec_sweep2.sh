#!/bin/bash
# Round-3 sweep that set the per-stripe fused threshold (max_e >= 0.6 m) and measured the
# blocked walk for batch-wide blocks (profiles/r03/fdec/patterns_threshold_sweep.log).
# RS_AMD_FDEC_SHARED_BLOCKED was a temporary switch, removed once measured (neutral).
mkdir -p gpurun_out; export TMPDIR=/tmp
for a in "256 k=200 m=55 sb=262144 loss=20 max_e=20" "256 k=200 m=55 sb=262144 loss=30 max_e=30" "256 k=200 m=55 sb=262144 loss=40 max_e=40" "256 k=64 m=64 sb=262144 loss=20 max_e=20" "256 k=100 m=20 sb=262144 loss=20 max_e=20" "256 k=40 m=12 sb=1048576 loss=12 max_e=12" "256 k=16 m=16 sb=1048576 loss=16 max_e=16"; do
  timeout -k 10 300 python -u tools/patterns_bench.py $a RS_AMD_FDEC=0,1 > gpurun_out/pb12.log 2>&1 || exit $?
  echo "$a"; tail -4 gpurun_out/pb12.log | cut -c1-200
done
timeout -k 10 300 python -u tools/kernel_sweep.py --k 200 --m 55 --shard-bytes 262144 --stripes 256 --erase 55:1:3 --nv 4 --rounds 2 --reps 3 --var RS_AMD_FDEC=1 --var RS_AMD_FDEC_SHARED_BLOCKED=0,1 > gpurun_out/ks12.log 2>&1 || exit $?
cut -c1-330 gpurun_out/ks12.log | grep nv

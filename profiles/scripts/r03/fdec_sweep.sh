#!/bin/bash
# Round-3 A/B that chose the blocked unit walk for per-stripe fused decode blocks
# (profiles/r03/fdec/blocked_and_shared_sweep.log). RS_AMD_FDEC_BLOCKED was a temporary
# switch, removed once measured: re-running this needs it back in rs_patterns.cpp.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_fdec.py -q --timeout 200 --timeout-method thread > gpurun_out/t11.log 2>&1; tail -2 gpurun_out/t11.log || exit 1
export RS_AMD_FDEC=1
for a in "256 k=64 m=64 sb=262144 loss=40 max_e=40" "256 k=200 m=55 sb=262144 loss=55 max_e=55"; do
  timeout -k 10 300 python -u tools/patterns_bench.py $a RS_AMD_FDEC_BLOCKED=0,1 > gpurun_out/pb11.log 2>&1 || exit $?
  tail -4 gpurun_out/pb11.log | cut -c1-200
done
unset RS_AMD_FDEC
for km in "64 64 40:0:1" "100 20 20:0:1" "33 17 17:0:2" "128 32 32:0:4" "16 16 16:0:1"; do
  set -- $km
  timeout -k 10 300 python -u tools/kernel_sweep.py --k $1 --m $2 --shard-bytes 262144 --stripes 256 --erase $3 --nv 4 --rounds 2 --reps 3 --wait --var RS_AMD_FDEC=0,1 > gpurun_out/ks11.log 2>&1 || exit $?
  cut -c1-330 gpurun_out/ks11.log | grep nv
done

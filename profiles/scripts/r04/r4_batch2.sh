#!/bin/bash
# Round 4: the launch-sequence reconstruct's kernels (rocprofv3 per-phase durations), its
# scratch slicing (RS_AMD_SCRATCH_CAP_MB: whole batch vs slices that stay in the 256 MiB
# Infinity Cache), and the mid-band per-stripe kernels with / without VGPR transpose masks.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
L=gpurun_out/r4b2.log
: > $L
ks() { timeout -k 10 300 python -u tools/kernel_sweep.py --nv 4 --rounds 2 --reps 3 --wait "$@" >> $L 2>&1; }
ks --k 300 --m 1000 --shard-bytes 65536 --stripes 8 --erase 100:0:3 --var RS_AMD_SCRATCH_CAP_MB=96,160,320,1024 || { echo SWEEP1 FAILED; tail $L; exit 1; }
ks --k 1000 --m 4000 --shard-bytes 4096 --stripes 64 --erase 300:0:3 --var RS_AMD_SCRATCH_CAP_MB=96,160,320,1024 || { echo SWEEP2 FAILED; tail $L; exit 1; }
grep -E '^\{' $L | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_low" -o run -- \
  python -u tools/kernel_sweep.py --k 300 --m 1000 --shard-bytes 65536 --stripes 8 --erase 100:0:3 --nv 4 --rounds 1 --reps 2 > gpurun_out/prof_low.log 2>&1 || { echo PROF FAILED; tail gpurun_out/prof_low.log; exit 1; }
find gpurun_out/prof_low -name '*kernel_stats.csv' -exec head -20 {} \; | cut -c1-220
export RS_AMD_JIT_SYNC=1
for a in "512 k=32 m=8 sb=1048576 loss=8 max_e=8" "512 k=100 m=4 sb=1048576 loss=4 max_e=4" "2048 k=10 m=4 sb=1048576 loss=4 max_e=4"; do
  timeout -k 10 400 python -u tools/patterns_bench.py $a RS_AMD_NET_VMASK=0,1 > gpurun_out/pbv.log 2>&1 || { echo PB FAILED; tail gpurun_out/pbv.log; exit 1; }
  echo "== $a" >> gpurun_out/r4b2_pb.log; grep -E '^\{' gpurun_out/pbv.log >> gpurun_out/r4b2_pb.log
done
cut -c1-200 gpurun_out/r4b2_pb.log

#!/bin/bash
# Round-3 final-tree snapshot of the other configs: encode / reconstruct
# times of representative codes, per-stripe patterns, low rate. HIP events, bit-exact checks
# inside the tools.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
run() { local t=$1; shift; timeout -k 10 $t "$@" >> gpurun_out/final_sweep.log 2>&1 || { echo "FAILED: $*"; tail -3 gpurun_out/final_sweep.log; exit 1; }; }
: > gpurun_out/final_sweep.log
for km in "16 16 1048576 512 16:0:1" "32 8 1048576 256 8:0:1" "64 64 262144 256 40:0:1" "100 20 262144 256 20:0:1" \
          "33 17 1048576 64 17:0:1" "200 55 262144 256 20:0:3"; do
  set -- $km
  run 300 python -u tools/kernel_sweep.py --k $1 --m $2 --shard-bytes $3 --stripes $4 --erase $5 --nv 4 --rounds 3 --reps 3 --wait
done
run 300 python -u tools/patterns_bench.py 2048
run 300 python -u tools/patterns_bench.py 256 k=200 m=55 sb=262144 loss=55 max_e=55
run 300 python -u tools/kernel_sweep.py --k 300 --m 1000 --shard-bytes 65536 --stripes 8 --erase 100:0:3 --nv 4 --rounds 2 --reps 2 --wait
grep -E '^\{' gpurun_out/final_sweep.log | cut -c1-330

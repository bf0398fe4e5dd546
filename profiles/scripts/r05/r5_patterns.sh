#!/bin/bash
# Round 5 final: per-stripe erasure-pattern rates (rs_reconstruct_batch_dev_patterns) at the
# verdict's shapes, the same tool and shapes as profiles/r04/patterns/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r5pat; export TMPDIR=/tmp
for a in "256 k=200 m=55 sb=262144 loss=55 max_e=55" "256 k=16 m=16 sb=1048576 loss=16 max_e=16" \
         "256 k=40 m=12 sb=1048576 loss=12 max_e=12" "512 k=32 m=8 sb=1048576 loss=8 max_e=8"; do
  n=$(echo $a | tr ' =' '__')
  timeout -k 10 300 python -u tools/patterns_bench.py $a > gpurun_out/r5pat/pb_$n.log 2>&1 || { echo "FAILED $a"; tail -5 gpurun_out/r5pat/pb_$n.log; exit 1; }
  echo "== $a"; grep -E '^\{' gpurun_out/r5pat/pb_$n.log | tail -3 | cut -c1-260
done

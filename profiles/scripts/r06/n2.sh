#!/bin/bash
# Round 6: the N > 1 bench path (torchrun env, barrier, MAX of rank times, aggregate value) on the
# final tree, two ranks sharing the one card over gloo (the 8-GPU RCCL runs are the driver's).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r6n2; mkdir -p $O
RS_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --stripes 2048 > $O/n2.log 2>&1 \
  || { tail -20 $O/n2.log; exit 1; }
grep '^{' $O/n2.log | cut -c1-400

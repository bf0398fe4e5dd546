#!/bin/bash
# Round 6: the low-rate block form against the W-point decode (RS_AMD_LOW_BLOCK=0) where
# the rows read sit in late blocks: C = 128, leading recovery rows lost.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r6lm; mkdir -p $O
timeout -k 10 300 python -u tools/kernel_sweep.py --k 128 --m 65408 --shard-bytes 64 --stripes 1 --erase 128:0:1 \
  --rec-erase 60000:0 --nv 4 --rounds 3 --reps 3 --wait --var RS_AMD_LOW_BLOCK=1,0 > $O/c128_w65536.log 2>&1 || { tail -5 $O/c128_w65536.log; exit 1; }
grep '^{' $O/c128_w65536.log | cut -c1-300
timeout -k 10 300 python -u tools/kernel_sweep.py --k 128 --m 1900 --shard-bytes 65536 --stripes 16 --erase 64:0:1 \
  --rec-erase 1000:0 --nv 4 --rounds 3 --reps 3 --wait --var RS_AMD_LOW_BLOCK=1,0 > $O/c128_m1900.log 2>&1 || { tail -5 $O/c128_m1900.log; exit 1; }
grep '^{' $O/c128_m1900.log | cut -c1-300

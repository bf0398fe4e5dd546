#!/bin/bash
# Round 5: the low-rate generic encode, phase launches (k_ephase) against the per-lane column
# walk (k_encode_low_coef / k_encode_low_generic) after the phase kernels' spill fix,
# interleaved in one process (RS_AMD_LOW_ENC_PHASES=1 / 0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r5; export TMPDIR=/tmp
: > gpurun_out/r5/encph.log
for a in "300 1000 1048576 16 100:0:3" "300 1000 65536 8 100:0:3" "200 1000 65536 8 100:0:2" "100 600 65536 16 50:0:2" "1000 4000 4096 64 300:0:3"; do
  set -- $a
  timeout -k 10 300 python -u tools/kernel_sweep.py --k $1 --m $2 --shard-bytes $3 --stripes $4 --erase $5 --nv 4 \
    --rounds 3 --reps 3 --wait --var RS_AMD_LOW_ENC_PHASES=1,0 >> gpurun_out/r5/encph.log 2>&1 || { echo "SWEEP FAILED: $a"; tail -5 gpurun_out/r5/encph.log; exit 1; }
done
grep -E '^\{' gpurun_out/r5/encph.log | cut -c1-200

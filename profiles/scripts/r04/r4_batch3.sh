#!/bin/bash
# Round 4: phase kernels with / without per-group scheduling barriers (RS_AMD_DPH_SB)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
L=gpurun_out/r4b3.log
: > $L
ks() { timeout -k 10 300 python -u tools/kernel_sweep.py --nv 4 --rounds 3 --reps 3 --wait "$@" >> $L 2>&1; }
ks --k 300 --m 1000 --shard-bytes 65536 --stripes 8 --erase 100:0:3 --var RS_AMD_DPH_SB=0,1 || { echo SWEEP1 FAILED; tail $L; exit 1; }
ks --k 1000 --m 4000 --shard-bytes 4096 --stripes 64 --erase 300:0:3 --var RS_AMD_DPH_SB=0,1 || { echo SWEEP2 FAILED; tail $L; exit 1; }
ks --k 200 --m 1000 --shard-bytes 65536 --stripes 8 --erase 100:0:2 --var RS_AMD_DPH_SB=0,1 || { echo SWEEP3 FAILED; tail $L; exit 1; }
grep -E '^\{' $L | cut -c1-330
RS_AMD_DPH_SB=1 timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests/test_lowrate.py > gpurun_out/r4b3_tests.log 2>&1; tail -2 gpurun_out/r4b3_tests.log

#!/bin/bash
# Round 4: branch-free gather / scatter in the phase kernels: parity, then rates and per-phase times
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
L=gpurun_out/r4b8.log
: > $L
timeout -k 10 900 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_lowrate.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py >> $L 2>&1 || { echo "TESTS FAILED"; tail -30 $L; exit 1; }
tail -2 $L
for a in "200 1000 65536 8 100:0:2" "300 1000 65536 8 100:0:3" "1000 4000 4096 64 300:0:3" "300 1000 1048576 16 100:0:3"; do
  set -- $a
  timeout -k 10 300 python -u tools/kernel_sweep.py --k $1 --m $2 --shard-bytes $3 --stripes $4 --erase $5 --nv 4 --rounds 3 --reps 3 --wait >> $L 2>&1 || { echo "SWEEP FAILED: $a"; tail -5 $L; exit 1; }
done
grep -E '^\{' $L | cut -c1-330
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_low8" -o run -- \
  python -u tools/kernel_sweep.py --k 300 --m 1000 --shard-bytes 65536 --stripes 8 --erase 100:0:3 --nv 4 --rounds 1 --reps 2 > gpurun_out/prof_low8.log 2>&1 || { echo PROF FAILED; tail gpurun_out/prof_low8.log; exit 1; }
grep dphase gpurun_out/prof_low8/run_kernel_stats.csv | cut -c1-200

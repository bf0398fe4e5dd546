#!/bin/bash
# Round 5: the low-rate reconstruct in block form (C-point transforms, launch_low_blocks):
# parity (low-rate tests, fuzz), rates against RS_AMD_LOW_BLOCK=0 (the W-point decode)
# interleaved in one process, and a kernel trace of the RS(300,1000) 1 MiB x 16 case.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r5; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_lowrate.py tests/test_gpu_fuzz.py > gpurun_out/r5/lowblk_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/r5/lowblk_tests.log; exit 1; }
tail -2 gpurun_out/r5/lowblk_tests.log
: > gpurun_out/r5/lowblk_rates.log
for a in "200 1000 65536 8 100:0:2" "300 1000 65536 8 100:0:3" "1000 4000 4096 64 300:0:3" "300 1000 1048576 16 100:0:3" "100 600 65536 16 50:0:2"; do
  set -- $a
  timeout -k 10 300 python -u tools/kernel_sweep.py --k $1 --m $2 --shard-bytes $3 --stripes $4 --erase $5 --nv 4 \
    --rounds 3 --reps 3 --wait --var RS_AMD_LOW_BLOCK=1,0 >> gpurun_out/r5/lowblk_rates.log 2>&1 || { echo "SWEEP FAILED: $a"; tail -5 gpurun_out/r5/lowblk_rates.log; exit 1; }
done
grep -E '^\{' gpurun_out/r5/lowblk_rates.log | cut -c1-330
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r5/lbprof" -o lb -- \
  python3 "$GRAFT_REPO_ROOT/tools/kernel_sweep.py" --k 300 --m 1000 --shard-bytes 1048576 --stripes 16 --erase 100:0:3 --nv 4 \
  --rounds 1 --reps 3 --wait > "$GRAFT_REPO_ROOT/gpurun_out/r5/lbprof.log" 2>&1 || { echo PROF FAILED; tail -5 "$GRAFT_REPO_ROOT/gpurun_out/r5/lbprof.log"; exit 1; }
echo done

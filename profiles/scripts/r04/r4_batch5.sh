#!/bin/bash
# Round 4: fused reconstruct with 4-plane runtime-multiply steps by default: parity, rates
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fdec.py tests/test_gpu_warm.py tests/test_gpu_parity.py > gpurun_out/r4b9_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r4b9_tests.log; exit 1; }
tail -2 gpurun_out/r4b9_tests.log
timeout -k 10 300 python -u tools/kernel_sweep.py --k 200 --m 55 --shard-bytes 262144 --stripes 256 --erase 55:1:3 --nv 4 --rounds 3 --reps 3 --var RS_AMD_FDEC=1 > gpurun_out/r4b9.log 2>&1 || exit 1
export RS_AMD_JIT_SYNC=1
for a in "256 k=200 m=55 sb=262144 loss=55 max_e=55" "256 k=16 m=16 sb=1048576 loss=16 max_e=16" "256 k=40 m=12 sb=1048576 loss=12 max_e=12" "256 k=64 m=64 sb=262144 loss=40 max_e=40"; do
  timeout -k 10 300 python -u tools/patterns_bench.py $a >> gpurun_out/r4b9.log 2>&1 || exit 1
done
grep -E '^\{' gpurun_out/r4b9.log | grep -v '"fft"\|"matrix"' | cut -c1-250

#!/bin/bash
# Phased column walk (rs_kernels.hip xform_ph) on the GPU: the engine KATs / oracle
# comparisons, the generic and low-rate parity tests, then the low-rate rates of
# DESIGN.md §3.4 (HIP events, bit-exact checks inside kernel_sweep.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
L=gpurun_out/phased.log
: > $L
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_lowrate.py tests/test_gpu_fuzz.py >> $L 2>&1 || { echo "TESTS FAILED"; tail -30 $L; exit 1; }
tail -3 $L
for a in "200 1000 65536 8 100:0:2" "300 1000 65536 8 100:0:3" "1000 4000 4096 64 300:0:3" "300 1000 1048576 16 100:0:3"; do
  set -- $a
  timeout -k 10 300 python -u tools/kernel_sweep.py --k $1 --m $2 --shard-bytes $3 --stripes $4 --erase $5 --nv 4 --rounds 2 --reps 3 --wait >> $L 2>&1 || { echo "SWEEP FAILED: $a"; tail -5 $L; exit 1; }
done
grep -E '^\{' $L | cut -c1-330

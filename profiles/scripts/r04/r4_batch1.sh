#!/bin/bash
# Round 4: the launch-sequence generic reconstruct (parity + low-rate rates) and the VGPR-mask
# A/B of the FFT kernels (RS_AMD_FFT_VMASK) on the c4 shape, one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
L=gpurun_out/r4b1.log
: > $L
timeout -k 10 900 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_lowrate.py tests/test_gpu_fuzz.py >> $L 2>&1 || { echo "TESTS FAILED"; tail -30 $L; exit 1; }
tail -3 $L
for a in "200 1000 65536 8 100:0:2" "300 1000 65536 8 100:0:3" "1000 4000 4096 64 300:0:3" "300 1000 1048576 16 100:0:3"; do
  set -- $a
  timeout -k 10 300 python -u tools/kernel_sweep.py --k $1 --m $2 --shard-bytes $3 --stripes $4 --erase $5 --nv 4 --rounds 2 --reps 3 --wait >> $L 2>&1 || { echo "SWEEP FAILED: $a"; tail -5 $L; exit 1; }
done
grep -E '^\{' $L | cut -c1-330
FORM=pattern timeout -k 10 400 python -u tools/fft_decompose.py 200 55 262144 256 55 RS_AMD_FFT_VMASK=0,1 > gpurun_out/vmask_p.log 2>&1 || { echo "VMASK P FAILED"; tail -5 gpurun_out/vmask_p.log; exit 1; }
FORM=dyn timeout -k 10 400 python -u tools/fft_decompose.py 200 55 262144 256 55 RS_AMD_FFT_VMASK=0,1 > gpurun_out/vmask_d.log 2>&1 || { echo "VMASK D FAILED"; tail -5 gpurun_out/vmask_d.log; exit 1; }
tail -n 6 gpurun_out/vmask_p.log gpurun_out/vmask_d.log | cut -c1-250

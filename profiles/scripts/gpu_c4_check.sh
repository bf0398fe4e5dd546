#!/bin/bash
# c4 (RS(200,55) 256 KiB) on one GPU box: FFT / syndrome parity tests, then encode knobs
# and the 55-erasure reconstruct timed after the background compiles finish.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_gpu_fft.py tests/test_gpu_syndrome.py -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/c4_tests.log 2>&1
rc=$?; tail -5 gpurun_out/c4_tests.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u tools/kernel_sweep.py --k 200 --m 55 --shard-bytes 262144 --stripes 256 --erase 0 --nv 4 --rounds 3 \
  ${SWEEP_VARS:---var RS_AMD_FFT_LDS128=0,1 --var RS_AMD_FFT_XUNIT=1,0 --var RS_AMD_FFT_PREFETCH=4,6 --var RS_AMD_FFT_NT=3} 2>&1 | grep -v amdgpu.ids > gpurun_out/c4_enc_sweep.log
rc2=$?; cut -c1-300 gpurun_out/c4_enc_sweep.log | tail -9
[ $rc2 -ne 0 ] && exit $rc2
timeout -k 10 400 python -u tools/kernel_sweep.py --k 200 --m 55 --shard-bytes 262144 --stripes 256 --erase 55:1:3 --nv 4 --rounds 3 --wait \
  --var RS_AMD_FFT=1,0 2>&1 | grep -v amdgpu.ids > gpurun_out/c4_rec.log
rc3=$?; tail -3 gpurun_out/c4_rec.log; exit $rc3

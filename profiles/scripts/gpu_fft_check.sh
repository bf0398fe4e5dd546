#!/bin/bash
# FFT encode kernels on one GPU box: parity tests, then an A/B sweep on the c4 shape.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export RS_AMD_JIT_VERBOSE=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_fft.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/fft_tests.log 2>&1
rc=$?; tail -8 gpurun_out/fft_tests.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u tools/kernel_sweep.py --k 200 --m 55 --shard-bytes 262144 --stripes 256 --erase 0 --nv 4 --rounds 3 \
  ${SWEEP_VARS:---var RS_AMD_FFT_PREFETCH=4,2,0 --var RS_AMD_FFT_NT=0,1,3} > gpurun_out/fft_sweep.log 2>&1
rc2=$?; grep -v amdgpu.ids gpurun_out/fft_sweep.log | grep -v "jit\]" | tail -12; exit $rc2

#!/bin/bash
# Round 4: fused-decode parity + allocation-failure tests, then the FFT kernels' decomposition.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fdec.py tests/test_gpu_alloc_fail.py tests/test_gpu_warm.py -m gpu -x -v \
    -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r4_decomp_tests.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r4_decomp_tests.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/r4_decomp_tests.log | head -20; exit $rc; }
timeout -k 10 700 python -u tools/fft_decompose.py 200 55 262144 256 55 ${DBG:-RS_AMD_FFT_DEBUG=16,0,17,19,20,24,3,28} \
    > gpurun_out/r4_decomp.log 2>&1 || { tail -5 gpurun_out/r4_decomp.log; exit 4; }
cut -c1-260 gpurun_out/r4_decomp.log

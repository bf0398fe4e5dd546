#!/bin/bash
# Round 4: phase timelines of the c4 FFT kernels (measurement builds) + the tests touched since.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_lowrate.py tests/test_gpu_syndrome.py -m gpu -x -q \
    -p no:cacheprovider --timeout 300 --timeout-method thread -k "scratch_cap or background_compile or large_codes" \
    > gpurun_out/r4_misc_tests.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r4_misc_tests.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/r4_misc_tests.log | head -20; exit $rc; }
: > gpurun_out/r4_stamps.log
for form in encode fused pattern; do
  timeout -k 10 300 python -u tools/fft_stamps.py 200 55 262144 256 55 $form >> gpurun_out/r4_stamps.log 2>&1 || { tail -5 gpurun_out/r4_stamps.log; exit 3; }
done
grep -v amdgpu.ids gpurun_out/r4_stamps.log | cut -c1-250

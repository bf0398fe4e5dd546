#!/bin/bash
# Round 5 session 1: the changed paths' GPU tests (pdecode policy, exit with the upgrade in
# flight, allocation failure, low-rate generic reconstruct with A in place), then the baseline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
timeout -k 10 900 python -u -m pytest tests/test_gpu_warm.py tests/test_gpu_exit.py tests/test_gpu_alloc_fail.py \
    tests/test_lowrate.py tests/test_gpu_fdec.py -m gpu -x -v -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/r5/tests_s1.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r5/tests_s1.log | tail -2
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/r5/tests_s1.log | head -30; exit $rc; fi
bash tools/r5_base.sh

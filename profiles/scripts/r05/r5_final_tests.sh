#!/bin/bash
# Round 5 final, part 1: the whole GPU test suite and the driver's smoke on the final tree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5final
timeout -k 10 1050 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread \
    > gpurun_out/r5final/gpu_tests.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r5final/gpu_tests.log | tail -2
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/r5final/gpu_tests.log | head -20; exit $rc; fi
timeout -k 10 120 python __graft_entry__.py smoke > gpurun_out/r5final/smoke.log 2>&1 || { tail -5 gpurun_out/r5final/smoke.log; exit 3; }
tail -1 gpurun_out/r5final/smoke.log

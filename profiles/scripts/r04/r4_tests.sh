#!/bin/bash
# Round 4: full GPU test suite + smoke on the current tree, each step under its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/r4_gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r4_gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python __graft_entry__.py smoke > gpurun_out/r4_smoke.log 2>&1 || { tail -5 gpurun_out/r4_smoke.log; exit 3; }
tail -2 gpurun_out/r4_smoke.log
exit $rc

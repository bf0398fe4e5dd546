#!/bin/bash
# Round 4: targeted GPU tests (files in $1, -k expression in $KEXPR) then an optional bench run ($2 = 1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 240 --timeout-method thread \
    $1 ${KEXPR:+-k "$KEXPR"} > gpurun_out/r4_quick_tests.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/r4_quick_tests.log | tail -3
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/r4_quick_tests.log | head -20; exit $rc; }
if [ "$2" = "1" ]; then
  timeout -k 10 500 python -u bench.py > gpurun_out/r4_bench.log 2>&1 || { tail -5 gpurun_out/r4_bench.log; exit 5; }
  tail -c 3000 gpurun_out/r4_bench.log
fi
exit 0

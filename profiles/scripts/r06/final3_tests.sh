#!/bin/bash
# Round 6 final (third pass, after the host ring copy and staging changes), part 1: the whole GPU test suite and the driver's smoke on the final tree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r6final3; mkdir -p $O
timeout -k 10 1050 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread \
    > $O/gpu_tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/gpu_tests.log | tail -2
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" $O/gpu_tests.log | head -20; exit $rc; fi
timeout -k 10 120 python __graft_entry__.py smoke > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 3; }
tail -1 $O/smoke.log

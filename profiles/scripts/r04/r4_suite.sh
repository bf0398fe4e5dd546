#!/bin/bash
# Round 4: the full GPU suite on HEAD (log kept under profiles/r04/), then the low-rate rates
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1120 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread --durations=40 > gpurun_out/r4_suite.log 2>&1
rc=$?; tail -4 gpurun_out/r4_suite.log; [ $rc -le 1 ] || exit $rc
exit $rc

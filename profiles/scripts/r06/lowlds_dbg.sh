#!/bin/bash
# Round 6: which cases of the on-chip low-rate kernels fail (no -x)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r6lds; mkdir -p $O
timeout -k 10 300 python -u -m pytest -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu \
  tests/test_lowrate.py -k "lds_paths or large_codes or block_form" > $O/dbg.log 2>&1
grep -E "passed|failed|FAILED" $O/dbg.log | cut -c1-200 | tail -30
exit 0

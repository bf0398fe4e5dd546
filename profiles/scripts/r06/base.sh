#!/bin/bash
# Round 6 start: the driver's bench on HEAD (c4 leg included), each step under its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r6base; mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench.log 2>&1; rc=$?
tail -c 3000 $O/bench.log
exit $rc

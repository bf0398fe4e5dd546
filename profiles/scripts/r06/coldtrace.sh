#!/bin/bash
# Round 6: where a new wide pattern's first call spends its host time: HIP API + kernel trace of
# tools/cold_patterns.py (no counters).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
R=$(pwd); export TMPDIR=/tmp
O=gpurun_out/r6cold; mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --output-format csv -d "$R/$O/trace" -o run -- \
  python3 "$R/tools/cold_patterns.py" > "$R/$O/cold.log" 2>&1 || { tail -5 "$R/$O/cold.log"; exit 1; }
grep '^{' "$R/$O/cold.log" | cut -c1-200
ls "$R/$O/trace"

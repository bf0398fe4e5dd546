#!/bin/bash
# Round 6: c4 pattern-compiled reconstruct, where each wave's rows of R are loaded
# (RS_AMD_PDEC_RLOAD 0 / 1 / 3) x prefetch 3 / 4, interleaved A/B in one process.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r6rl; mkdir -p $O
FORM=pattern ROUNDS=4 REPS=3 timeout -k 10 500 python tools/fft_decompose.py 200 55 262144 256 55 \
  RS_AMD_PDEC_RLOAD=0,1,3 RS_AMD_FFT_PREFETCH=3,4 > $O/rload.log 2>&1; rc=$?
grep -v "^round" $O/rload.log | grep -v amdgpu.ids | cut -c1-300
exit $rc

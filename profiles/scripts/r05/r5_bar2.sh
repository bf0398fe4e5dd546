#!/bin/bash
# Round 5: the exchanges' second barrier as an LDS read-done counter (RS_AMD_FFT_BAR2=0) against
# the barrier, at prefetch 3 and 4 (a spilling build falls back to less prefetch on its own).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
A="200 55 262144 256 55"
for form in dyn pattern; do
  FORM=$form timeout -k 10 500 python -u tools/fft_decompose.py $A RS_AMD_FFT_BAR2=1,0 RS_AMD_FFT_PREFETCH=3,4 \
    > gpurun_out/r5/bar2_$form.log 2>&1 || { tail -5 gpurun_out/r5/bar2_$form.log; exit 1; }
  grep '^{' gpurun_out/r5/bar2_$form.log | cut -c1-300
done

#!/bin/bash
# Round 4: pattern-compiled fused decode — parity tests, then steady-state timing of c4 forms.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_fdec.py tests/test_gpu_warm.py -m gpu -x -v \
    -p no:cacheprovider --timeout 400 --timeout-method thread > gpurun_out/r4_pdec_tests.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r4_pdec_tests.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/r4_pdec_tests.log | head -20; exit $rc; }
timeout -k 10 600 python -u tools/kernel_sweep.py --k 200 --m 55 --shard-bytes 262144 --stripes 256 --erase 55:1:3 \
    --nv 4 --rounds 3 --reps 3 --wait --var RS_AMD_PDEC=1,0 > gpurun_out/r4_pdec_sweep.log 2>&1 || { tail -5 gpurun_out/r4_pdec_sweep.log; exit 4; }
grep '^{' gpurun_out/r4_pdec_sweep.log | cut -c1-300

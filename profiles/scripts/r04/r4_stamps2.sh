#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r4_stamps2.log
timeout -k 10 300 python -u tools/fft_stamps.py 200 55 262144 256 55 encode >> gpurun_out/r4_stamps2.log 2>&1 &&
timeout -k 10 300 python -u tools/fft_stamps.py 200 55 262144 256 55 encode RS_AMD_FFT_DEBUG=3 >> gpurun_out/r4_stamps2.log 2>&1 &&
timeout -k 10 300 python -u tools/fft_stamps.py 200 55 262144 256 55 pattern >> gpurun_out/r4_stamps2.log 2>&1 || { tail -5 gpurun_out/r4_stamps2.log; exit 3; }
grep -v amdgpu.ids gpurun_out/r4_stamps2.log | cut -c1-300

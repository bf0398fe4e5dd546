#!/bin/bash
# Round 5: a chunk's non-prefetched positions loaded by LDS-DMA into the wave's own exchange
# slots right after the previous exchange (RS_AMD_FFT_DMA=1; RS_AMD_FFT_DMAPF positions stay in
# the VGPR prefetch) against the VGPR loads, c4 encode + both fused reconstructs, bit-exact check.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
A="200 55 262144 256 55"
for form in pattern dyn; do
  FORM=$form timeout -k 10 600 python -u tools/fft_decompose.py $A RS_AMD_FFT_DMA=0,1 RS_AMD_FFT_DMAPF=0,3 \
    > gpurun_out/r5/dma_$form.log 2>&1 || { tail -5 gpurun_out/r5/dma_$form.log; exit 1; }
  grep '^{' gpurun_out/r5/dma_$form.log | cut -c1-300
done

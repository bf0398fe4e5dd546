# FFT kernel: blocked unit assignment A/B (RS_AMD_FFT_BLOCKED), parity under it
set -o pipefail
mkdir -p gpurun_out
RS_AMD_FFT_BLOCKED=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_fft.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "oracle and not c4 or 1k or inverse or strided" > gpurun_out/r2e_fft.log 2>&1
rc=$?; tail -3 gpurun_out/r2e_fft.log; grep -E "^FAILED" gpurun_out/r2e_fft.log | head; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
for c in "32 32 1048576 64" "200 55 262144 256" "100 20 262144 256" "64 64 262144 256" "32 32 1024 65536"; do
  set -- $c
  timeout -k 10 300 python -u tools/kernel_sweep.py --k $1 --m $2 --shard-bytes $3 --stripes $4 --erase 0 --nv 4 --rounds 3 --var RS_AMD_FFT_BLOCKED=0,1 2>&1 | grep -v amdgpu.ids | grep '^{' | cut -c1-250 || exit 1
done

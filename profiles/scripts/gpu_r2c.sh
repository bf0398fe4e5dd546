# FFT kernel at 1 KiB shards (two-stripe units): parity + harness-shape sweeps
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fft.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r2c_fft.log 2>&1
rc=$?; tail -3 gpurun_out/r2c_fft.log; grep -E "^FAILED" gpurun_out/r2c_fft.log | head; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
for km in "32 32 65536" "64 64 32768"; do
  set -- $km
  timeout -k 10 300 python -u tools/kernel_sweep.py --k $1 --m $2 --shard-bytes 1024 --stripes $3 --erase 0 --nv 4 --rounds 3 --var RS_AMD_FFT=1,0 2>&1 | grep -v amdgpu.ids | grep '^{' | cut -c1-330 || exit 1
done
timeout -k 10 300 python -u tools/kernel_sweep.py --k 200 --m 55 --shard-bytes 1024 --stripes 65536 --erase 0 --nv 4 --rounds 3 --var RS_AMD_FFT=1,0 2>&1 | grep -v amdgpu.ids | grep '^{' | cut -c1-330 || exit 1

# inverse FFT reconstruct (every original lost, RS(k,k)), shard-size probe of the FFT encode
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fft.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "inverse or 1k" > gpurun_out/r2d_fft.log 2>&1
rc=$?; tail -3 gpurun_out/r2d_fft.log; grep -E "^FAILED" gpurun_out/r2d_fft.log | head; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
for km in "32 32 65536" "64 64 32768"; do
  set -- $km
  timeout -k 10 300 python -u tools/kernel_sweep.py --k $1 --m $2 --shard-bytes 1024 --stripes $3 --erase $1:0:1 --nv 4 --rounds 3 --wait --var RS_AMD_FFT=1,0 2>&1 | grep -v amdgpu.ids | grep '^{' | cut -c1-330 || exit 1
done
for sbn in "65536 1024" "1048576 64" "16384 4096"; do
  set -- $sbn
  timeout -k 10 300 python -u tools/kernel_sweep.py --k 32 --m 32 --shard-bytes $1 --stripes $2 --erase 32:0:1 --nv 4 --rounds 3 --wait 2>&1 | grep -v amdgpu.ids | grep '^{' | cut -c1-330 || exit 1
done

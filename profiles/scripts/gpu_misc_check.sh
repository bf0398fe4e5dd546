set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_distributed.py -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread -k "multi_device or error_drains or small_shard or world_size_2 or baseline_shapes" > gpurun_out/g3_tests.log 2>&1
rc=$?; tail -5 gpurun_out/g3_tests.log; grep -E "^FAILED|Error" gpurun_out/g3_tests.log | head; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for km in "100 20 262144 256" "64 64 262144 256" "32 32 1048576 64" "33 17 1048576 64"; do
  set -- $km
  timeout -k 10 300 python -u tools/kernel_sweep.py --k $1 --m $2 --shard-bytes $3 --stripes $4 --erase 0 --nv 4 --rounds 3 --var RS_AMD_FFT=1,0 2>&1 | grep -v amdgpu.ids | grep '^{' | cut -c1-330 || exit 1
done

# round-2 follow-up: low-rate maps past 64 recovery shards, reference harness shapes at 1 KiB
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_lowrate.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r2b_lowrate.log 2>&1
rc=$?; tail -3 gpurun_out/r2b_lowrate.log; grep -E "^FAILED" gpurun_out/r2b_lowrate.log | head; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for km in "32 32 65536" "64 64 32768"; do
  set -- $km
  timeout -k 10 300 python -u tools/kernel_sweep.py --k $1 --m $2 --shard-bytes 1024 --stripes $3 --erase 0 --nv 4 --rounds 3 --var RS_AMD_NET_SMALL_ENCODE=1,0 2>&1 | grep -v amdgpu.ids | grep '^{' | cut -c1-330 || exit 1
  timeout -k 10 300 python -u tools/kernel_sweep.py --k $1 --m $2 --shard-bytes 1024 --stripes $3 --erase $1:0:1 --nv 4 --rounds 3 --wait 2>&1 | grep -v amdgpu.ids | grep '^{' | cut -c1-330 || exit 1
done

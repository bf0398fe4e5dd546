# background-compiled encode networks: tests + RS(100,20) generic vs network
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r7
timeout -k 10 300 python -u -m pytest tests/test_gpu_syndrome.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k background > gpurun_out/r7/t.log 2>&1 || { tail -30 gpurun_out/r7/t.log; exit 1; }
tail -1 gpurun_out/r7/t.log
RS_AMD_JIT_SYNC=1 RS_AMD_JIT_VERBOSE=1 timeout -k 10 400 python3 tools/kernel_sweep.py --k 100 --m 20 --shard-bytes 262144 --stripes 256 \
  --erase 0,1,2,3 --nv 1 --rounds 2 --reps 2 --var RS_AMD_NET_ASYNC_BLOCKS=0,1024 > gpurun_out/r7/rs100.jsonl 2>gpurun_out/r7/err.log
cat gpurun_out/r7/rs100.jsonl; grep compiled gpurun_out/r7/err.log | cut -c1-150

# full suite + direct background networks: RS(200,55) losing 8, RS(100,20) losing 4
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r8
s=$(date +%s)
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider --durations=5 > gpurun_out/r8/suite.log 2>&1 || { tail -40 gpurun_out/r8/suite.log; exit 1; }
echo "suite wall $(( $(date +%s) - s )) s"; tail -8 gpurun_out/r8/suite.log
RS_AMD_JIT_SYNC=1 RS_AMD_JIT_VERBOSE=1 timeout -k 10 400 python3 tools/kernel_sweep.py --k 200 --m 55 --shard-bytes 262144 --stripes 256 \
  --erase 0,9,33,47,101,150,177,199 --nv 1 --rounds 2 --reps 2 --var RS_AMD_NET_ASYNC_BLOCKS=0,1024 > gpurun_out/r8/rs200_e8.jsonl 2>gpurun_out/r8/err.log || exit 1
RS_AMD_JIT_SYNC=1 RS_AMD_JIT_VERBOSE=1 timeout -k 10 400 python3 tools/kernel_sweep.py --k 100 --m 20 --shard-bytes 262144 --stripes 256 \
  --erase 0,1,2,3 --nv 1 --rounds 2 --reps 2 --var RS_AMD_NET_ASYNC_BLOCKS=0,1024 > gpurun_out/r8/rs100.jsonl 2>>gpurun_out/r8/err.log
cat gpurun_out/r8/rs200_e8.jsonl gpurun_out/r8/rs100.jsonl; grep compiled gpurun_out/r8/err.log | cut -c1-150

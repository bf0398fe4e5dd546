# full GPU suite (timed) + RS(200,55) with the syndrome network compiled synchronously
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4
s=$(date +%s)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider --durations=8 > gpurun_out/r4/suite.log 2>&1 || { tail -40 gpurun_out/r4/suite.log; exit 1; }
echo "suite wall $(( $(date +%s) - s )) s"; tail -14 gpurun_out/r4/suite.log
RS_AMD_JIT_SYNC=1 RS_AMD_JIT_VERBOSE=1 timeout -k 10 300 python3 tools/kernel_sweep.py --k 200 --m 55 --shard-bytes 262144 --stripes 256 \
  --erase $(python3 -c "print(','.join(str(i) for i in range(0,110,2)))") --nv 1 --rounds 3 --reps 2 > gpurun_out/r4/rs200.jsonl 2>gpurun_out/r4/rs200.err
cat gpurun_out/r4/rs200.jsonl; grep compiled gpurun_out/r4/rs200.err | cut -c1-160

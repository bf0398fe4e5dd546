# ws64 next-chunk prefetch A/B on RS(200,55) + the parity tests that cover ws64
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "200 or ws64 or syndrome or wide or 64" > gpurun_out/r2/suite.log 2>&1 || { tail -30 gpurun_out/r2/suite.log; exit 1; }
tail -1 gpurun_out/r2/suite.log
timeout -k 10 400 python3 tools/kernel_sweep.py --k 200 --m 55 --shard-bytes 262144 --stripes 256 \
  --erase $(python3 -c "print(','.join(str(i) for i in range(0,110,2)))") --nv 1,2 --rounds 3 --reps 2 \
  --var RS_AMD_WS64_PF=0,1 > gpurun_out/r2/rs200_pf.jsonl 2>gpurun_out/r2/rs200.err
cat gpurun_out/r2/rs200_pf.jsonl

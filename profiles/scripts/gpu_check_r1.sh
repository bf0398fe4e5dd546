set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r1/suite.log 2>&1 || { tail -30 gpurun_out/r1/suite.log; exit 1; }
tail -2 gpurun_out/r1/suite.log
timeout -k 10 300 python3 tools/kernel_sweep.py --k 200 --m 55 --shard-bytes 262144 --stripes 256 \
  --erase $(python3 -c "print(','.join(str(i) for i in range(0,110,2)))") --nv 1,2 --rounds 2 --reps 2 > gpurun_out/r1/rs200.jsonl 2>gpurun_out/r1/rs200.err
cat gpurun_out/r1/rs200.jsonl
timeout -k 10 200 python3 tools/kernel_sweep.py --k 10 --m 4 --shard-bytes 1048576 --stripes 2048 --nv 4 --rounds 2 --reps 3 --var RS_AMD_JIT=0,1 > gpurun_out/r1/rs10.jsonl 2>gpurun_out/r1/rs10.err
cat gpurun_out/r1/rs10.jsonl

#!/bin/bash
# Round profile: PMC HBM traffic of the bench kernels (separate passes), kernel-trace
# stats of the bench, and kernel sweeps of the other BASELINE configs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
mkdir -p gpurun_out/round
bash tools/pmc.sh || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/round/prof" -o run -- \
  python3 "$R/bench.py" --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/round/bench_prof.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/kernel_sweep.py --k 4 --m 2 --shard-bytes 65536 --stripes 16384 --erase 1,3 --nv 4 \
  --rounds 3 --reps 3 --var RS_AMD_JIT=0,1 > gpurun_out/round/sweep_rs4_2.jsonl 2> gpurun_out/round/sweep_rs4_2.err || exit 1
timeout -k 10 400 python3 tools/kernel_sweep.py --k 200 --m 55 --shard-bytes 262144 --stripes 256 \
  --erase $(python3 -c "print(','.join(str(i) for i in range(0,110,2)))") --nv 1 --rounds 2 --reps 2 \
  > gpurun_out/round/sweep_rs200_55.jsonl 2> gpurun_out/round/sweep_rs200_55.err || exit 1
cat gpurun_out/round/sweep_rs4_2.jsonl gpurun_out/round/sweep_rs200_55.jsonl

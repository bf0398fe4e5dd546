# syndrome e x e map as a network (RS_AMD_NET_MAX_BLOCKS lifts the size cap) vs the table kernel
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r3
RS_AMD_JIT_VERBOSE=1 timeout -k 10 500 python3 tools/kernel_sweep.py --k 200 --m 55 --shard-bytes 262144 --stripes 256 \
  --erase $(python3 -c "print(','.join(str(i) for i in range(0,110,2)))") --nv 1 --rounds 2 --reps 2 \
  --var RS_AMD_NET_MAX_BLOCKS=64,1000 > gpurun_out/r3/rs200_synnet.jsonl 2>gpurun_out/r3/rs200.err
cat gpurun_out/r3/rs200_synnet.jsonl; grep -i "compiled" gpurun_out/r3/rs200.err | cut -c1-200

# network output tiles of 4 vs 8 (RS_AMD_NET_TILE) on multi-tile maps and the 55 x 55 syndrome map
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r5
for cfg in "16 16 1048576 512 0,1,2,3" "32 8 1048576 256 0,1,2,3,4,5,6,7"; do
  set -- $cfg
  timeout -k 10 240 python3 tools/kernel_sweep.py --k $1 --m $2 --shard-bytes $3 --stripes $4 --erase $5 --nv 4 \
    --rounds 2 --reps 3 --var RS_AMD_NET_TILE=4,8 >> gpurun_out/r5/tiles.jsonl 2>>gpurun_out/r5/err.log || exit 1
done
RS_AMD_JIT_SYNC=1 RS_AMD_JIT_VERBOSE=1 timeout -k 10 400 python3 tools/kernel_sweep.py --k 200 --m 55 --shard-bytes 262144 --stripes 256 \
  --erase $(python3 -c "print(','.join(str(i) for i in range(0,110,2)))") --nv 1 --rounds 2 --reps 2 \
  --var RS_AMD_NET_TILE=4,8 >> gpurun_out/r5/tiles.jsonl 2>>gpurun_out/r5/err.log
cat gpurun_out/r5/tiles.jsonl; grep compiled gpurun_out/r5/err.log | cut -c1-150

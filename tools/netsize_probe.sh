# Network kernel speed vs size (output tiles, nt loads): tools/netsize_probe.sh [NT values]
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ns
NTS=${1:-2,3}
for cfg in "16 16 1048576 512 0,1,2,3" "32 8 1048576 256 0,1,2,3,4,5,6,7" "16 12 1048576 512 0,1,2,3,4,5,6,7"; do
  set -- $cfg
  timeout -k 10 240 python3 tools/kernel_sweep.py --k $1 --m $2 --shard-bytes $3 --stripes $4 --erase $5 --nv 4 \
    --rounds 2 --reps 3 --var RS_AMD_NET_NT=$NTS >> gpurun_out/ns/netsize.jsonl 2>>gpurun_out/ns/err.log
done
cat gpurun_out/ns/netsize.jsonl

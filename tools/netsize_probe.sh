set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ns
for cfg in "16 16 1048576 512 0,1,2,3" "32 8 1048576 256 0,1,2,3" "64 4 524288 256 0,1,2,3" "48 4 524288 256 0,1,2,3"; do
  set -- $cfg
  timeout -k 10 240 python3 tools/kernel_sweep.py --k $1 --m $2 --shard-bytes $3 --stripes $4 --erase $5 --nv 4 --rounds 2 --reps 3 --var RS_AMD_JIT=0,1 >> gpurun_out/ns/netsize.jsonl 2>>gpurun_out/ns/err.log
done
cat gpurun_out/ns/netsize.jsonl

set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/patterns_bench.py 2048 RS_AMD_PSYN_PF=1,2,3,4 RS_AMD_PSYN_WAVES=3,4 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r2g_patterns.jsonl

set -o pipefail
mkdir -p gpurun_out/r2h
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
RS_AMD_PATTERNS=auto timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r2h/prof" -o run -- python -u "$R/tools/patterns_bench.py" 2048 > "$R/gpurun_out/r2h/prof.log" 2>&1
f=$(find "$R/gpurun_out/r2h/prof" -name "*kernel_stats.csv" | head -1); cut -c1-160 "$f" | head -12

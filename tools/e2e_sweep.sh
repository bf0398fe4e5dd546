# host pipeline shape sweep: RS_AMD_HOST_SLOTS x RS_AMD_HOST_SLICE_MB (pinned, RS(10,4) 1 MiB x 512)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/e2e
IFS=, read -ra VS <<< "${SHAPES:-3 256,4 128,6 64,3 512,2 256,8 32}"
for v in "${VS[@]}"; do
  set -- $v
  RS_AMD_HOST_SLOTS=$1 RS_AMD_HOST_SLICE_MB=$2 timeout -k 10 200 python3 tools/e2e_bench.py --stripes 512 --pageable-stripes 8 \
    > gpurun_out/e2e/s$1_m$2.log 2>&1 || { tail -5 gpurun_out/e2e/s$1_m$2.log; exit 1; }
  echo "slots=$1 slice=$2 $(tail -1 gpurun_out/e2e/s$1_m$2.log | python3 -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["pinned"])')"
done

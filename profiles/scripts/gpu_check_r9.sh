# LDS-table matrix kernel: tests, per-stripe patterns bench, table-path RS(10,4) reconstruct A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r9
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r9/suite.log 2>&1 || { tail -40 gpurun_out/r9/suite.log; exit 1; }
tail -1 gpurun_out/r9/suite.log
for v in 0 1; do
  RS_AMD_MATRIX_LDS=$v timeout -k 10 200 python3 tools/patterns_bench.py 2048 > gpurun_out/r9/patterns_lds$v.log 2>&1 || { tail -5 gpurun_out/r9/patterns_lds$v.log; exit 1; }
  echo "lds=$v $(tail -1 gpurun_out/r9/patterns_lds$v.log | cut -c1-300)"
done
RS_AMD_JIT=0 timeout -k 10 300 python3 tools/kernel_sweep.py --k 10 --m 4 --shard-bytes 1048576 --stripes 2048 --nv 4 --rounds 2 --reps 3 \
  --var RS_AMD_MATRIX_LDS=0,1 > gpurun_out/r9/rs10_tab.jsonl 2>&1; cat gpurun_out/r9/rs10_tab.jsonl | cut -c1-300

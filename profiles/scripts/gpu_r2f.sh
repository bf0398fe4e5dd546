# per-stripe patterns on the syndrome network (rs_psyn.hpp): parity + timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "per_stripe" > gpurun_out/r2f_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r2f_tests.log; grep -E "^FAILED" gpurun_out/r2f_tests.log | head; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/patterns_bench.py 2048 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r2f_patterns.jsonl

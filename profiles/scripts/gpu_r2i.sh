# wide-code per-stripe patterns: parity + timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "per_stripe" > gpurun_out/r2i_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r2i_tests.log; grep -E "^FAILED|Error" gpurun_out/r2i_tests.log | head; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/patterns_bench.py 256 k=200 m=55 sb=262144 loss=8 max_e=8 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r2i_wide.jsonl
timeout -k 10 300 python -u tools/patterns_bench.py 256 k=100 m=20 sb=262144 loss=4 max_e=4 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r2i_wide.jsonl

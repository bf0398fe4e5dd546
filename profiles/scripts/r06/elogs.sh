#!/bin/bash
# Round 6: erasure locators summed point by point (host plans and the per-stripe k_erasure_logs):
# per-stripe / low-rate / fuzz GPU tests, per-stripe rates, bench (c4 cold first calls).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r6el; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fdec.py tests/test_lowrate.py tests/test_gpu_fuzz.py \
  tests/test_gpu_syndrome.py tests/test_gpu_warm.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 \
  || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for shp in "k=16 m=16 loss=16 max_e=16" "k=40 m=12 loss=12 max_e=12"; do
  f=$O/pb_$(echo $shp | tr ' =' '__').log
  timeout -k 10 300 python -u tools/patterns_bench.py 256 $shp sb=1048576 > $f 2>&1 || { tail -5 $f; exit 1; }
  grep '"auto"' $f | cut -c1-250
done
f=$O/pb_k_200_m_55.log
timeout -k 10 300 python -u tools/patterns_bench.py 256 k=200 m=55 loss=55 max_e=55 sb=262144 > $f 2>&1 || { tail -5 $f; exit 1; }
grep '"auto"' $f | cut -c1-250
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], json.dumps(d['c4_gpu']['reconstruct_cold'])[:400])"

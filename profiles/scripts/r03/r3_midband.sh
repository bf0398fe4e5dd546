cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "mid_band or per_stripe" > gpurun_out/midband_tests.log 2>&1; rc=$?; tail -3 gpurun_out/midband_tests.log; [ $rc -le 1 ] || exit $rc
export RS_AMD_JIT_SYNC=1
for a in "512 k=32 m=8 sb=1048576 loss=8 max_e=8" "512 k=100 m=4 sb=1048576 loss=4 max_e=4" "256 k=40 m=12 sb=1048576 loss=12 max_e=12" "2048 k=10 m=4 sb=1048576 loss=4 max_e=4" "256 k=16 m=16 sb=1048576 loss=16 max_e=16"; do
  timeout -k 10 300 python -u tools/patterns_bench.py $a > gpurun_out/pb_$(echo $a | tr ' =' '__').log 2>&1 || exit $?
  tail -5 gpurun_out/pb_$(echo $a | tr ' =' '__').log | cut -c1-300
done

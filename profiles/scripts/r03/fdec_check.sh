#!/bin/bash
# Fused FFT reconstruct: GPU parity tests, then the c4 reconstruct
# (RS(200,55) 256 KiB x 256, 55 erased) with the fused kernel against the syndrome network.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name limit cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -v amdgpu.ids "gpurun_out/$name.log" | tail -n 6 | cut -c1-600
  echo "== $name rc=$rc"
  return $rc
}
for step in ${STEPS:-tests c4}; do
  case $step in
    tests) run fdec_tests 500 python -u -m pytest tests/test_gpu_fdec.py -x -v --timeout 200 --timeout-method thread ${PYK:+-k "$PYK"} || exit $? ;;
    c4) run fdec_c4 500 python -u tools/kernel_sweep.py --k 200 --m 55 --shard-bytes 262144 --stripes 256 \
          --erase 55:1:3 --nv 4 --rounds 3 --reps 3 --wait --var RS_AMD_FDEC=0,1 || exit $? ;;
    prof) run fdec_prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$(pwd)/gpurun_out/fdec_prof" -o run -- \
            python3 tools/kernel_sweep.py --k 200 --m 55 --shard-bytes 262144 --stripes 256 \
            --erase 55:1:3 --nv 4 --rounds 2 --reps 3 --wait --var RS_AMD_FDEC=0,1 || exit $? ;;
    sq) run fdec_sq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM \
            --output-format csv -d "$(pwd)/gpurun_out/fdec_sq" -o run -- \
            python3 tools/kernel_sweep.py --k 200 --m 55 --shard-bytes 262144 --stripes 256 \
            --erase 55:1:3 --nv 4 --rounds 1 --reps 1 --var RS_AMD_FDEC=1 || exit $? ;;
    cold) run fdec_cold 300 python3 -u tools/cold_patterns.py || exit $? ;;
  esac
done
exit 0

#!/bin/bash
# Round GPU session: full GPU test suite, smoke, bench, rocprofv3 kernel stats of the
# bench, PMC traffic at the bench config, and the c4 (RS(200,55)) FFT kernels' traffic.
# Each step has its own limit; stop at the first crash / timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -v amdgpu.ids "gpurun_out/$name.log" | tail -n ${TAIL:-6}
  echo "== $name rc=$rc"
  return $rc
}
if [ -z "$SKIP_TESTS" ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread
  rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
step smoke 200 python __graft_entry__.py smoke || exit $?
TAIL=1 step bench 400 python bench.py || exit $?
step rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- \
    python3 "$R/bench.py" --steps 5 --warmup 2 --cpu-seconds 0 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  step pmc_$c 300 rocprofv3 --pmc $c --output-format csv -d "$R/gpurun_out/pmc/$c" -o run -- \
      python3 "$R/bench.py" --steps 2 --warmup 1 --cpu-seconds 0 --no-verify || exit $?
  step pmc4_$c 300 rocprofv3 --pmc $c --output-format csv -d "$R/gpurun_out/pmc4/$c" -o run -- \
      python3 "$R/tools/kernel_sweep.py" --k 200 --m 55 --shard-bytes 262144 --stripes 256 --erase 55:1:3 --nv 4 \
      --rounds 1 --reps 1 --wait || exit $?
  # the fused FFT reconstruct of the same pattern (RS_AMD_FDEC=1: no syndrome scratch)
  step pmc4f_$c 300 rocprofv3 --pmc $c --output-format csv -d "$R/gpurun_out/pmc4f/$c" -o run -- \
      python3 "$R/tools/kernel_sweep.py" --k 200 --m 55 --shard-bytes 262144 --stripes 256 --erase 55:1:3 --nv 4 \
      --rounds 1 --reps 1 --var RS_AMD_FDEC=1 || exit $?
done
# SQ / LDS counters of the c4 FFT kernels (encode, fused reconstruct), one pass per group
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM"; do
  i=$((i+1))
  step sq4_$i 200 rocprofv3 --pmc $grp --output-format csv -d "$R/gpurun_out/sq4/g$i" -o run -- \
      python3 "$R/tools/kernel_sweep.py" --k 200 --m 55 --shard-bytes 262144 --stripes 256 --erase 55:1:3 --nv 4 \
      --rounds 1 --reps 1 --var RS_AMD_FDEC=1 || exit $?
done
exit 0

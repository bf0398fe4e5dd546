#!/bin/bash
# Round 6 final (third pass), part 2: bench (driver contract), rocprofv3 kernel stats of the same command,
# PMC traffic at the bench config and of the c4 kernels, each step under its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
R=$(pwd); export TMPDIR=/tmp
O=gpurun_out/r6final3; mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  grep -v amdgpu.ids "$O/$name.log" | grep -v '^round' | grep -v "^W2026\|^E2026" | tail -n ${TAIL:-3} | cut -c1-400
  echo "== $name rc=$rc"
  return $rc
}
TAIL=1 step bench 400 python bench.py || exit $?
step rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof" -o run -- \
    python3 "$R/bench.py" --steps 5 --warmup 2 --cpu-seconds 0 || exit $?
A="200 55 262144 256 55"
for c in FETCH_SIZE WRITE_SIZE; do
  step pmc_$c 300 rocprofv3 --pmc $c --output-format csv -d "$R/$O/pmc/$c" -o run -- \
      python3 "$R/bench.py" --steps 2 --warmup 1 --cpu-seconds 0 --c4-reps 0 --no-verify || exit $?
  FORM=pattern ROUNDS=1 REPS=1 step pmc4p_$c 300 rocprofv3 --pmc $c --output-format csv -d "$R/$O/pmc4p/$c" -o run -- \
      python3 "$R/tools/fft_decompose.py" $A RS_AMD_FFT_DEBUG=0 || exit $?
  FORM=dyn ROUNDS=1 REPS=1 step pmc4d_$c 300 rocprofv3 --pmc $c --output-format csv -d "$R/$O/pmc4d/$c" -o run -- \
      python3 "$R/tools/fft_decompose.py" $A RS_AMD_FFT_DEBUG=0 || exit $?
done
exit 0

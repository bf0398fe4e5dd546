#!/bin/bash
# Round-3 fused FFT reconstruct session: full GPU suite, cold patterns, per-stripe wide
# patterns (fused vs FFT syndromes + solve). Each step under its own limit; stop at the
# first crash / timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name limit cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -v amdgpu.ids "gpurun_out/$name.log" | tail -n ${TAIL:-4} | cut -c1-400
  echo "== $name rc=$rc"
  return $rc
}
for step in ${STEPS:-suite cold pat}; do
  case $step in
    suite) run gpu_suite 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread --durations=25
           rc=$?; [ $rc -le 1 ] || exit $rc ;;
    cold) run cold_patterns 300 python3 -u tools/cold_patterns.py || exit $? ;;
    pat) for a in "256 k=200 m=55 sb=262144 loss=55 max_e=55" "256 k=200 m=55 sb=262144 loss=20 max_e=20" \
                  "256 k=16 m=16 sb=1048576 loss=16 max_e=16" "256 k=40 m=12 sb=1048576 loss=12 max_e=12" \
                  "256 k=64 m=64 sb=262144 loss=40 max_e=40"; do
           TAIL=8 run "pat_$(echo $a | tr ' =' '__')" 300 python -u tools/patterns_bench.py $a RS_AMD_FDEC=0,1 || exit $?
         done ;;
  esac
done
exit 0

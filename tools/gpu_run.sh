#!/bin/bash
# One parametrised GPU session (gpurun): steps separated by "--", run in order, each
# under its own time limit; the session stops at the first step that crashes, times
# out or fails (pytest's "tests failed" status 1 stops it too). Output under gpurun_out/.
#   bash tools/gpu_run.sh tests -k per_stripe -- sweep --k 32 --m 32 --shard-bytes 1024 \
#        --stripes 65536 --erase 0 --var RS_AMD_FFT=1,0 -- patterns 2048 -- prof patterns tools/patterns_bench.py 1024
# steps:
#   tests [pytest args]       python -m pytest -m gpu [paths, default tests/] (900 s)
#   sweep [kernel_sweep args] tools/kernel_sweep.py, JSON lines (300 s)
#   patterns [args]           tools/patterns_bench.py (300 s)
#   prof TAG script [args]    rocprofv3 --kernel-trace --stats of a python script (300 s)
#   pmc TAG COUNTER script [args]  one rocprofv3 --pmc pass (300 s)
#   round                     tools/gpu_round.sh (full suite, smoke, bench, rocprof, PMC)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
mkdir -p gpurun_out
n=0
run_step() {
  n=$((n + 1))
  local kind=$1; shift
  local log="gpurun_out/step${n}_${kind}.log" rc
  echo "== step $n: $kind $*"
  case $kind in
    tests) [ $# -eq 0 ] && set -- tests  # test paths / -k expressions, default the whole suite
           timeout -k 10 900 python -u -m pytest -m gpu -q -p no:cacheprovider --timeout 300 \
             --timeout-method thread "$@" > "$log" 2>&1 ;;
    sweep) timeout -k 10 300 python -u tools/kernel_sweep.py "$@" > "$log" 2>&1 ;;
    patterns) timeout -k 10 300 python -u tools/patterns_bench.py "$@" > "$log" 2>&1 ;;
    prof) local tag=$1 script=$2; shift 2
          timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$tag" -o run \
            -- python3 "$R/$script" "$@" > "$log" 2>&1 ;;
    pmc) local tag=$1 ctr=$2 script=$3; shift 3
         timeout -s KILL 300 rocprofv3 --pmc "$ctr" --output-format csv -d "$R/gpurun_out/pmc_$tag/$ctr" -o run \
           -- python3 "$R/$script" "$@" > "$log" 2>&1 ;;
    round) bash tools/gpu_round.sh > "$log" 2>&1 ;;
    *) echo "unknown step $kind"; return 2 ;;
  esac
  rc=$?
  grep -v amdgpu.ids "$log" | grep -E '^\{|passed|failed|FAILED|Error|== ' | cut -c1-300 | tail -n 40
  echo "== step $n rc=$rc"
  return $rc
}
args=()
for a in "$@" --; do
  if [ "$a" = "--" ]; then
    [ ${#args[@]} -gt 0 ] && { run_step "${args[@]}" || exit $?; }
    args=()
  else
    args+=("$a")
  fi
done
exit 0

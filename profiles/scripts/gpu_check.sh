#!/bin/bash
# One GPU session: parity tests -> smoke -> short bench. Each GPU step has its
# own time limit; stop at the first crash/fault/timeout (exit codes other than
# pytest's "tests failed" = 1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PYTEST_ARGS=${PYTEST_ARGS:-"-m gpu -q -p no:cacheprovider --timeout 300"}
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -n 25 "gpurun_out/$name.log"
  echo "== $name exit $rc"
  return $rc
}
run pytest_gpu 420 python -m pytest tests $PYTEST_ARGS
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop: pytest rc=$rc"; exit $rc; fi
run smoke 200 python __graft_entry__.py smoke || exit $?
run bench 300 python bench.py ${BENCH_ARGS:---steps 5 --warmup 2 --cpu-seconds 8} || exit $?
if [ -n "$PROFILE" ]; then
  R=$(pwd)
  export TMPDIR=/tmp
  run rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- \
      python3 "$R/bench.py" ${PROF_ARGS:---steps 5 --warmup 2 --cpu-seconds 0} || exit $?
fi
exit $rc

#!/bin/bash
# Round-3 measurement session (gpurun): bench (c4 leg at 512 stripes + cold pattern),
# the c4 syndrome path's forms, and low-rate codec rates. Each step under its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name limit cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -v amdgpu.ids "gpurun_out/$name.log" | tail -n 4 | cut -c1-400
  echo "== $name rc=$rc"
  return $rc
}
for step in ${STEPS:-bench synform low}; do
  case $step in
    bench) run bench 500 python -u bench.py || exit $? ;;
    synform) run synform 400 python -u tools/kernel_sweep.py --k 200 --m 55 --shard-bytes 262144 --stripes 256 \
               --erase 55:1:3 --nv 4 --rounds 3 --reps 3 --wait --var RS_AMD_FDEC=0,1 || exit $? ;;  # (round 3 first compared RS_AMD_SYN_FORM forms, since removed)
    low) for shape in "300 1000 65536 8 100:0:3" "200 1000 65536 8 100:0:2" "1000 4000 4096 64 300:0:3" \
                      "32 1000 65536 16 20:0:1" "16 4000 16384 16 8:0:2" "10 60 1048576 64 8:0:1"; do
           set -- $shape
           run "low_$1_$2" 300 python -u tools/kernel_sweep.py --k $1 --m $2 --shard-bytes $3 --stripes $4 \
             --erase $5 --nv 4 --rounds 2 --reps 2 --wait || exit $?
         done ;;
  esac
done
exit 0

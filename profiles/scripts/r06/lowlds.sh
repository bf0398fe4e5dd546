#!/bin/bash
# Round 6: the LDS-resident low-rate encode (k_encode_low_lds, C = 512): parity against the
# oracle (low-rate GPU tests), then rates against the phase launches (RS_AMD_LOW_LDS=0),
# interleaved in one process, and its PMC traffic.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
R=$(pwd); export TMPDIR=/tmp
O=gpurun_out/r6lds; mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  grep -v amdgpu.ids "$O/$name.log" | grep -v '^round' | tail -n ${TAIL:-4} | cut -c1-330
  echo "== $name rc=$rc"
  return $rc
}
TAIL=3 step tests 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_lowrate.py || exit $?
for a in "300 1000 1048576 16 100:0:3" "300 1000 65536 8 100:0:3" "500 700 262144 16 100:0:5" "260 3000 65536 8 100:0:2"; do
  set -- $a
  TAIL=2 step rates_$1_$2_$3 300 python -u tools/kernel_sweep.py --k $1 --m $2 --shard-bytes $3 --stripes $4 --erase $5 \
    --nv 4 --rounds 3 --reps 3 --wait --var RS_AMD_LOW_LDS=1,0 || exit $?
done
for c in FETCH_SIZE WRITE_SIZE; do
  cd /tmp
  timeout -k 10 -s KILL 200 rocprofv3 --pmc $c --output-format csv -d "$R/$O/pmc/$c" -o run -- \
    python3 "$R/tools/kernel_sweep.py" --k 300 --m 1000 --shard-bytes 1048576 --stripes 16 --erase 100:0:3 --nv 4 \
    --rounds 1 --reps 1 > "$R/$O/pmc_$c.log" 2>&1 || { echo "PMC $c FAILED"; tail -5 "$R/$O/pmc_$c.log"; exit 1; }
  cd "$R"; echo "== pmc $c ok"
done
exit 0

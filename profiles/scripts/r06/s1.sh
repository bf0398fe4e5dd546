#!/bin/bash
# Round 6 session 1: GPU tests of what changed (low-rate block skip, plan gate, pdecode tail
# merge), the c4 traffic-shape sweep (tools/c4_probe.hip), the end-to-end host path on HEAD
# (tools/e2e_bench.py + tools/pcie_probe.py). Each step under its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
R=$(pwd); export TMPDIR=/tmp
O=gpurun_out/r6s1; mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  grep -v amdgpu.ids "$O/$name.log" | grep -v '^round' | tail -n ${TAIL:-4} | cut -c1-400
  echo "== $name rc=$rc"
  return $rc
}
TAIL=3 step tests 480 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_lowrate.py tests/test_gpu_warm.py tests/test_gpu_fdec.py || exit $?
hipcc -O3 --offload-arch=gfx950 tools/c4_probe.hip -o tools/c4_probe || exit 1
TAIL=60 step probe 300 tools/c4_probe 512 || exit $?
TAIL=5 step pcie 120 python -u tools/pcie_probe.py || exit $?
TAIL=3 step e2e_rs10_4 300 python -u tools/e2e_bench.py --stripes 512 --pageable-stripes 128 || exit $?
TAIL=3 step e2e_c4 300 python -u tools/e2e_bench.py --k 200 --m 55 --shard-bytes 262144 --stripes 64 \
  --pageable-stripes 16 --erase $(python3 -c "print(','.join(map(str, list(range(1, 200, 3))[:55])))") || exit $?
exit 0

#!/bin/bash
# Round 6: pinned staging (copy-out and copy-in in one host pass) for pageable host buffers (RS_AMD_HOST_STAGE, default on) — host GPU tests,
# then A/B in one process against the runtime's pageable path (=0), RS(10,4) and c4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r6stage2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "host or oneshot or concurrency or exit" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 \
  || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python -u tools/e2e_bench.py --stripes 256 --pageable-stripes 256 --reps 5 --var RS_AMD_HOST_STAGE=,0 > $O/rs10.log 2>&1 || { tail -5 $O/rs10.log; exit 1; }
grep -E '^\{"(pinned|pageable) ' $O/rs10.log | cut -c1-300
E=$(python3 -c "print(','.join(str(i) for i in range(1, 200, 3)[:55]))")
timeout -k 10 400 python -u tools/e2e_bench.py --k 200 --m 55 --shard-bytes 262144 --stripes 48 --pageable-stripes 48 \
  --erase $E --reps 5 --var RS_AMD_HOST_STAGE=,0 > $O/c4.log 2>&1 || { tail -5 $O/c4.log; exit 1; }
grep -E '^\{"(pinned|pageable) ' $O/c4.log | cut -c1-300

#!/bin/bash
# Round 6: the 2D copy form as the default (unset) against RS_AMD_HOST_COPY2D=0, after the host-batch GPU tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r6c2d2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "host or oneshot or concurrency" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 \
  || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python -u tools/e2e_bench.py --stripes 512 --reps 6 --var RS_AMD_HOST_COPY2D=,0 > $O/rs10.log 2>&1 || { tail -5 $O/rs10.log; exit 1; }
grep -E '^\{"(pinned|pageable) ' $O/rs10.log | cut -c1-300
E=$(python3 -c "print(','.join(str(i) for i in range(1, 200, 3)[:55]))")
timeout -k 10 400 python -u tools/e2e_bench.py --k 200 --m 55 --shard-bytes 262144 --stripes 96 --pageable-stripes 24 \
  --erase $E --reps 6 --var RS_AMD_HOST_COPY2D=,0 > $O/c4.log 2>&1 || { tail -5 $O/c4.log; exit 1; }
grep -E '^\{"(pinned|pageable) ' $O/c4.log | cut -c1-300

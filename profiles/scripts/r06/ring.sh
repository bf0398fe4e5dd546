#!/bin/bash
# Round 6: host ring shape A/B in one process, alternated rep by rep: slots (RS_AMD_HOST_SLOTS) and
# slice size (RS_AMD_HOST_SLICE_MB), c4 and RS(10,4); the host-batch GPU tests first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r6ring; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "host" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 \
  || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
E=$(python3 -c "print(','.join(str(i) for i in range(1, 200, 3)[:55]))")
timeout -k 10 400 python -u tools/e2e_bench.py --k 200 --m 55 --shard-bytes 262144 --stripes 64 --pageable-stripes 16 \
  --erase $E --reps 5 --var RS_AMD_HOST_SLOTS=2,3,4 > $O/c4_slots.log 2>&1 || { tail -5 $O/c4_slots.log; exit 1; }
grep -E '^\{"(pinned|pageable) ' $O/c4_slots.log | cut -c1-300
timeout -k 10 400 python -u tools/e2e_bench.py --k 200 --m 55 --shard-bytes 262144 --stripes 64 --pageable-stripes 16 \
  --erase $E --reps 5 --var RS_AMD_HOST_SLICE_MB=512,256,128,64 > $O/c4_slice.log 2>&1 || { tail -5 $O/c4_slice.log; exit 1; }
grep -E '^\{"(pinned|pageable) ' $O/c4_slice.log | cut -c1-300
timeout -k 10 400 python -u tools/e2e_bench.py --stripes 512 --reps 5 --var RS_AMD_HOST_SLOTS=2,3,4 > $O/rs10_slots.log 2>&1 || { tail -5 $O/rs10_slots.log; exit 1; }
grep -E '^\{"(pinned|pageable) ' $O/rs10_slots.log | cut -c1-300

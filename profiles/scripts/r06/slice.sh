#!/bin/bash
# Round 6: host ring slice size A/B in one process (RS_AMD_HOST_SLICE_MB), alternated rep by rep,
# two orders for c4 and RS(10,4).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r6slice; mkdir -p $O
E=$(python3 -c "print(','.join(str(i) for i in range(1, 200, 3)[:55]))")
for order in 1024,512,256 256,512,1024; do
  timeout -k 10 400 python -u tools/e2e_bench.py --k 200 --m 55 --shard-bytes 262144 --stripes 96 --pageable-stripes 24 \
    --erase $E --reps 5 --var RS_AMD_HOST_SLICE_MB=$order > $O/c4_$order.log 2>&1 || { tail -5 $O/c4_$order.log; exit 1; }
  grep -E '^\{"(pinned|pageable) ' $O/c4_$order.log | cut -c1-300
  timeout -k 10 400 python -u tools/e2e_bench.py --stripes 768 --pageable-stripes 192 --reps 5 --var RS_AMD_HOST_SLICE_MB=$order \
    > $O/rs10_$order.log 2>&1 || { tail -5 $O/rs10_$order.log; exit 1; }
  grep -E '^\{"(pinned|pageable) ' $O/rs10_$order.log | cut -c1-300
done

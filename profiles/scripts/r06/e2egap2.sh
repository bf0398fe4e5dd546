#!/bin/bash
# Round 6: host reconstruct copy shapes A/B in one process, alternated rep by rep (RS_AMD_HOST_GAP:
# -1 one copy per row (round 5), 0 one copy per run of present rows, 1 / 200 runs bridging gaps).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r6gap2; mkdir -p $O
E=$(python3 -c "print(','.join(str(i) for i in range(1, 200, 3)[:55]))")
timeout -k 10 400 python -u tools/e2e_bench.py --k 200 --m 55 --shard-bytes 262144 --stripes 64 --pageable-stripes 16 \
  --erase $E --reps 5 --var RS_AMD_HOST_GAP=-1,0,1,200 > $O/c4.log 2>&1 || { tail -5 $O/c4.log; exit 1; }
grep -E '^\{"(pinned|pageable) ' $O/c4.log | cut -c1-300
timeout -k 10 400 python -u tools/e2e_bench.py --stripes 512 --reps 5 --var RS_AMD_HOST_GAP=-1,0 > $O/rs10.log 2>&1 || { tail -5 $O/rs10.log; exit 1; }
grep -E '^\{"(pinned|pageable) ' $O/rs10.log | cut -c1-300

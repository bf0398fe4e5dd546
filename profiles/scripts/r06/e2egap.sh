#!/bin/bash
# Round 6: host reconstruct copies one run of present rows per copy command (RS_AMD_HOST_GAP =
# missing rows bridged inside a run). c4 (every third data shard lost) and RS(10,4), pinned and
# pageable, per gap setting; the host-batch GPU tests first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r6gap; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "host" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 \
  || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
E=$(python3 -c "print(','.join(str(i) for i in range(1, 200, 3)[:55]))")
for g in 0 1 2 200; do
  RS_AMD_HOST_GAP=$g timeout -k 10 300 python -u tools/e2e_bench.py --k 200 --m 55 --shard-bytes 262144 --stripes 64 \
    --pageable-stripes 16 --erase $E > $O/c4_gap$g.log 2>&1 || { tail -5 $O/c4_gap$g.log; exit 1; }
  echo "gap $g c4: $(grep -E '^\{"(pinned|pageable)' $O/c4_gap$g.log | tr '\n' ' ' | cut -c1-400)"
done
for g in 0 200; do
  RS_AMD_HOST_GAP=$g timeout -k 10 300 python -u tools/e2e_bench.py --stripes 512 > $O/rs10_gap$g.log 2>&1 || { tail -5 $O/rs10_gap$g.log; exit 1; }
  echo "gap $g rs10: $(grep -E '^\{"(pinned|pageable)' $O/rs10_gap$g.log | tr '\n' ' ' | cut -c1-400)"
done

#!/bin/bash
# Round 6: per-stripe pattern rates on the final tree (tools/patterns_bench.py, auto path).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r6pfin; mkdir -p $O
for shp in "256 k=16 m=16 loss=16 max_e=16 sb=1048576" "256 k=40 m=12 loss=12 max_e=12 sb=1048576" \
           "512 k=32 m=8 loss=8 max_e=8 sb=1048576" "256 k=200 m=55 loss=55 max_e=55 sb=262144" \
           "512 k=10 m=4 loss=4 max_e=4 sb=1048576" "512 k=100 m=4 loss=4 max_e=4 sb=1048576"; do
  f=$O/pb_$(echo $shp | tr ' =' '__').log
  timeout -k 10 300 python -u tools/patterns_bench.py $shp > $f 2>&1 || { tail -5 $f; exit 1; }
  echo "$shp: $(grep '"auto"' $f | cut -c1-60 | head -0)$(grep '"auto"' $f | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['ms'], d['frac'], d['launched'][-1][:40], d['verified'], end=' | ')")"
done

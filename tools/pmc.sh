#!/bin/bash
# HBM traffic of the bench kernels from rocprofv3 PMC counters, one counter per
# pass (FETCH_SIZE costs 3 TCC slots, WRITE_SIZE 2: they cannot share a pass).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
ARGS=${PMC_ARGS:---steps 2 --warmup 1 --cpu-seconds 0 --stripes 4096 --no-verify}
for c in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $c"
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$R/gpurun_out/pmc/$c" -o run -- \
      python3 "$R/bench.py" $ARGS > "gpurun_out/pmc/$c.log" 2>&1 || { echo "rc=$?"; tail -20 gpurun_out/pmc/$c.log; exit 1; }
  ls gpurun_out/pmc/$c
done

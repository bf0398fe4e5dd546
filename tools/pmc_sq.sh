#!/bin/bash
# SQ counters for the RS(10,4) kernels (one pass per counter group).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
mkdir -p gpurun_out/sq
rocprofv3 -L > gpurun_out/sq/counters.txt 2>&1 || true
grep -oE '\bSQ_[A-Z_0-9]+|\bTCP_[A-Z_0-9]+|\bTA_[A-Z_0-9]+' gpurun_out/sq/counters.txt | sort -u > gpurun_out/sq/names.txt
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM" "SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $grp --output-format csv -d "$R/gpurun_out/sq/g$i" -o run -- \
    python3 "$R/tools/kernel_sweep.py" --stripes 1024 --nv 4 --rounds 1 --reps 1 > gpurun_out/sq/g$i.log 2>&1 || echo "group $i failed"
done

#!/bin/bash
# SQ / GRBM counters of the wide-code kernels (c4 FFT encode + syndrome map, the
# per-stripe RS(32,8) syndrome network), one rocprofv3 --pmc pass per group (<= 8 SQ).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
mkdir -p gpurun_out/pmcw
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_IFETCH SQ_ACTIVE_INST_SCA" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d "$R/gpurun_out/pmcw/c4_g$i" -o run -- \
    python3 "$R/tools/kernel_sweep.py" --k 200 --m 55 --shard-bytes 262144 --stripes 256 --erase 55:1:3 --nv 4 \
    --rounds 1 --reps 1 --wait > gpurun_out/pmcw/c4_g$i.log 2>&1 || { echo "c4 group $i failed"; exit 1; }
  RS_AMD_JIT_SYNC=1 timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d "$R/gpurun_out/pmcw/p32_g$i" -o run -- \
    python3 "$R/tools/patterns_bench.py" 256 k=32 m=8 sb=1048576 loss=8 max_e=8 > gpurun_out/pmcw/p32_g$i.log 2>&1 || { echo "p32 group $i failed"; exit 1; }
done
echo done

#!/bin/bash
# Round 5 baseline: c4 FFT kernels' decomposition (pattern as data and compiled in), the
# static s_setprio knob, and SQ counters of rs_fft_pdecode (none existed before round 5).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
mkdir -p gpurun_out/r5
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/r5/$name.log" 2>&1
  local rc=$?
  grep -v amdgpu.ids "gpurun_out/r5/$name.log" | grep -v '^round' | cut -c1-330 | tail -n ${TAIL:-8}
  echo "== $name rc=$rc"
  return $rc
}
A="200 55 262144 256 55"
FORM=dyn step dyn_prio 300 python -u tools/fft_decompose.py $A RS_AMD_FFT_SPRIO=0,1,2 || exit $?
FORM=dyn step dyn_decomp 300 python -u tools/fft_decompose.py $A RS_AMD_FFT_DEBUG=0,3,4,8 || exit $?
FORM=pattern step pat_prio 400 python -u tools/fft_decompose.py $A RS_AMD_FFT_SPRIO=0,1 || exit $?
FORM=pattern step pat_decomp 400 python -u tools/fft_decompose.py $A RS_AMD_FFT_DEBUG=3,4 || exit $?
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
           "SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  FORM=pattern ROUNDS=1 REPS=2 step sq_pdec_$i 300 rocprofv3 --pmc $grp --output-format csv -d "$R/gpurun_out/r5/sq_pdec/g$i" -o run -- \
      python3 "$R/tools/fft_decompose.py" $A RS_AMD_FFT_DEBUG=0 || exit $?
done
exit 0

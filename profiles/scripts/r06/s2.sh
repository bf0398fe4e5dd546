#!/bin/bash
# Round 6 session 2: the FFT kernels' unit walk (RS_AMD_FFT_WALK 0 interleaved / 1 blocked; the
# c4 probe's blocked shape moved 0.70 -> 0.75 of HBM) on c4 and other wide codes, interleaved
# A/B; per-stripe pattern rates labelled by the launched kernels; a pattern stream under
# RS_AMD_PDEC_AFTER 2 / 3; low-rate rates and PMC traffic (RS(300,1000) 1 MiB x 16).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
R=$(pwd); export TMPDIR=/tmp
O=gpurun_out/r6s2; mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  grep -v amdgpu.ids "$O/$name.log" | grep -v '^round' | tail -n ${TAIL:-4} | cut -c1-330
  echo "== $name rc=$rc"
  return $rc
}
FORM=pattern ROUNDS=3 TAIL=2 step walk_c4_pattern 300 python -u tools/fft_decompose.py 200 55 262144 512 55 RS_AMD_FFT_WALK=0,1 || exit $?
FORM=dyn ROUNDS=3 TAIL=2 step walk_c4_dyn 300 python -u tools/fft_decompose.py 200 55 262144 512 55 RS_AMD_FFT_WALK=0,1 || exit $?
FORM=dyn ROUNDS=3 TAIL=2 step walk_rs100_20 300 python -u tools/fft_decompose.py 100 20 262144 256 20 RS_AMD_FFT_WALK=0,1 || exit $?
FORM=dyn ROUNDS=3 TAIL=2 step walk_rs32_32 300 python -u tools/fft_decompose.py 32 32 1048576 64 8 RS_AMD_FFT_WALK=0,1 || exit $?
FORM=dyn ROUNDS=3 TAIL=2 step walk_rs64_64_1k 300 python -u tools/fft_decompose.py 64 64 1024 32768 16 RS_AMD_FFT_WALK=0,1 || exit $?
for a in "256 k=200 m=55 sb=262144 loss=55 max_e=55" "256 k=16 m=16 sb=1048576 loss=16 max_e=16" \
         "256 k=40 m=12 sb=1048576 loss=12 max_e=12" "512 k=32 m=8 sb=1048576 loss=8 max_e=8"; do
  n=$(echo $a | tr ' =' '__')
  TAIL=4 step pb_$n 300 python -u tools/patterns_bench.py $a RS_AMD_FFT_WALK=0,1 || exit $?
done
RS_AMD_PDEC_AFTER=3 TAIL=1 step stream_after3 150 python -u tools/pattern_stream.py 35 || exit $?
RS_AMD_PDEC_AFTER=2 TAIL=1 step stream_after2 150 python -u tools/pattern_stream.py 35 || exit $?
TAIL=3 step low_rates 300 python -u tools/kernel_sweep.py --k 300 --m 1000 --shard-bytes 1048576 --stripes 16 \
  --erase 100:0:3 --nv 4 --rounds 3 --reps 3 --wait --var RS_AMD_LOW_BLOCK=1,0 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  cd /tmp
  timeout -k 10 -s KILL 200 rocprofv3 --pmc $c --output-format csv -d "$R/$O/lowpmc/$c" -o run -- \
    python3 "$R/tools/kernel_sweep.py" --k 300 --m 1000 --shard-bytes 1048576 --stripes 16 --erase 100:0:3 --nv 4 \
    --rounds 1 --reps 1 > "$R/$O/lowpmc_$c.log" 2>&1 || { echo "PMC $c FAILED"; tail -5 "$R/$O/lowpmc_$c.log"; exit 1; }
  cd "$R"; echo "== pmc $c ok"
done
exit 0

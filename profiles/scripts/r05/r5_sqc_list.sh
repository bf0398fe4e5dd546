cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r5/sqc; export TMPDIR=/tmp
timeout -k 5 60 rocprofv3 -L > gpurun_out/r5/sqc/counters.txt 2>&1 || true
grep -oE '\bSQC_[A-Z_0-9]+' gpurun_out/sqc_dummy 2>/dev/null; grep -oE '\bSQC_[A-Z_0-9]+' gpurun_out/r5/sqc/counters.txt | sort -u | tr '\n' ' '
echo

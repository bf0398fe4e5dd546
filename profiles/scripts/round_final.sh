# end-of-round evidence: PMC traffic, rocprof kernel stats of the bench, sweeps, default bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/profile_round.sh > gpurun_out/round_profile.log 2>&1 || { tail -30 gpurun_out/round_profile.log; exit 1; }
timeout -k 10 400 python3 bench.py > gpurun_out/round/bench_default.log 2> gpurun_out/round/bench_default.err || { tail -20 gpurun_out/round/bench_default.err; exit 1; }
tail -1 gpurun_out/round/bench_default.log | cut -c1-600
python3 tools/pmc_traffic.py gpurun_out/pmc --stripes 1024 --out gpurun_out/round/traffic.json > gpurun_out/round/traffic.log 2>&1; tail -2 gpurun_out/round/traffic.log

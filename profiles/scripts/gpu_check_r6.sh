# full GPU suite + a short bench after kernel-default changes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r6/suite.log 2>&1 || { tail -40 gpurun_out/r6/suite.log; exit 1; }
tail -1 gpurun_out/r6/suite.log
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --cpu-seconds 0 > gpurun_out/r6/bench.log 2>&1 || { tail -20 gpurun_out/r6/bench.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r6/bench.log').read().strip().splitlines()[-1]);print(d['value'],d['roofline']['frac'],d['encode_GiBps'],d['reconstruct_GiBps'])"

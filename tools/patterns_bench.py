#!/usr/bin/env python3
"""Per-stripe erasure patterns (rs_reconstruct_batch_dev_patterns): RS(10,4) 1 MiB,
4 random erasures per stripe: syndrome network (auto) vs matrix vs FFT path (RS_AMD_PATTERNS).
Each line names the kernels the timed call launched (rs_last_kernels): for codes where the
requested paths coincide (W > 32: matrix and fft both run the generic per-stripe path), the
`launched` field shows it."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-cc_amd"))
import reedsol_amd as R  # noqa: E402

# shape tokens (lower case): k=, m=, sb=, loss= (erasures per stripe), max_e=
shape = {"k": 10, "m": 4, "sb": 1 << 20, "loss": 4, "max_e": 4}
args = [a for a in sys.argv[2:] if not (a.split("=")[0] in shape and shape.update({a.split("=")[0]: int(a.split("=")[1])}) is None)]
k, m, sb, n = shape["k"], shape["m"], shape["sb"], int(sys.argv[1]) if len(sys.argv) > 1 else 2048
loss, max_e = shape["loss"], shape["max_e"]
dev = torch.device("cuda:0")
data = torch.randint(0, 256, (n, k, sb), dtype=torch.uint8, device=dev)
par = torch.empty((n, m, sb), dtype=torch.uint8, device=dev)
R.encode_batch_dev(k, m, data, par)
rng = np.random.default_rng(5)
present = np.ones((n, k + m), np.uint8)
for s in range(n):
    present[s, rng.choice(k + m, size=loss, replace=False)] = 0
dp = torch.from_numpy(present).to(dev)
out = torch.empty((n, max_e, sb), dtype=torch.uint8, device=dev)
status = torch.empty((n,), dtype=torch.int32, device=dev)
# steady state: one untimed call queues the background compiles (encode and syndrome networks),
# net_wait joins them (round 5: without it a fresh box timed the table fallback)
R.reconstruct_batch_dev_patterns(k, m, dp, data, par, out, status)
torch.cuda.synchronize()
R.net_wait()
# extra variants: NAME=v1,v2 arguments after the stripe count (e.g. RS_AMD_JIT=0,1)
variants = [("RS_AMD_PATTERNS", p) for p in ("matrix", "auto", "fft", "matrix", "auto")]
for arg in args:
    name, vals = arg.split("=")
    variants += [(name, v) for v in vals.split(",")] * 2
for var, val in variants:
    os.environ[var] = val
    path = os.environ.get("RS_AMD_PATTERNS", "auto")
    R.reconstruct_batch_dev_patterns(k, m, dp, data, par, out, status)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        R.reconstruct_batch_dev_patterns(k, m, dp, data, par, out, status)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 10
    launched = R.last_kernels()  # what served the call: the label, not the env value
    ok = True
    for s in range(0, n, max(1, n // 64)):
        miss = [i for i in range(k) if not present[s, i]][:max_e]
        ok &= bool(torch.equal(out[s, :len(miss)], data[s, miss]))
    e_mean = float(np.minimum((present[:, :k] == 0).sum(1), max_e).mean())
    alg = n * sb * (k + m - loss + e_mean)  # present shards read + restored written
    print(json.dumps({"requested": path, var: val, "launched": launched, "stripes": n, "ms": round(ms, 3),
                      "alg_TBps": round(alg / ms / 1e9, 3), "frac": round(alg / ms / 8e9, 4), "verified": ok}),
          flush=True)
    if var != "RS_AMD_PATTERNS":
        del os.environ[var]

#!/usr/bin/env python3
"""Single-call latency of the one-shot API (rs_encode / rs_decode via reedsol_amd.encode /
decode, root.zig:14-84) on the reference harness shapes (benchmarks.zig: 1 KiB shards,
Encoder.init + addOriginalShard x k + encode per iteration), against the oracle CPU engine."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-cc_amd"))
import reedsol_amd as R  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
for k, m in ((32, 32), (64, 64), (10, 4)):
    rng = np.random.default_rng(k)
    orig = [bytes(rng.integers(0, 256, 1024, dtype=np.uint8)) for _ in range(k)]
    rec = R.encode(k, m, orig)  # warm-up (plans, kernels, staging)
    t0 = time.perf_counter()
    for _ in range(iters):
        R.encode(k, m, orig)
    enc_us = (time.perf_counter() - t0) / iters * 1e6
    lost = [None] * min(k, m) + orig[min(k, m):]
    assert R.decode(k, m, lost, rec) == orig
    t0 = time.perf_counter()
    for _ in range(iters // 4):
        R.decode(k, m, lost, rec)
    dec_us = (time.perf_counter() - t0) / (iters // 4) * 1e6
    print(json.dumps({"shape": f"RS({k},{m}) 1 KiB", "encode_us_per_call": round(enc_us, 1),
                      "decode_us_per_call (all originals lost)": round(dec_us, 1), "iters": iters}), flush=True)

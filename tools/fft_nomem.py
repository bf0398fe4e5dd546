#!/usr/bin/env python3
"""Measurement aid: the FFT encode kernel's time with its loads and/or stores replaced by
the zero-record buffer resource (RS_AMD_FFT_DEBUG_NOMEM bits 0 / 1: no memory traffic,
wrong bytes) — how much of the kernel's time is memory and how much compute + barriers.
  python tools/fft_nomem.py --k 200 --m 55 --shard-bytes 262144 --stripes 256
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-cc_amd"))
import reedsol_amd as R  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--k", type=int, default=200)
ap.add_argument("--m", type=int, default=55)
ap.add_argument("--shard-bytes", type=int, default=1 << 18)
ap.add_argument("--stripes", type=int, default=256)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--rounds", type=int, default=3)
a = ap.parse_args()
dev = torch.device("cuda:0")
d = torch.randint(0, 256, (a.stripes, a.k, a.shard_bytes), dtype=torch.uint8, device=dev)
p = torch.empty((a.stripes, a.m, a.shard_bytes), dtype=torch.uint8, device=dev)
s = torch.cuda.current_stream()
res = {v: [] for v in ("0", "1", "2", "3")}
for r in range(a.rounds + 1):
    for v in res:
        os.environ["RS_AMD_FFT_DEBUG_NOMEM"] = v
        R.encode_batch_dev(a.k, a.m, d, p, stream=s)  # compiles on first use
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(a.reps):
            R.encode_batch_dev(a.k, a.m, d, p, stream=s)
        e1.record(s)
        torch.cuda.synchronize()
        if r:
            res[v].append(e0.elapsed_time(e1) / a.reps)
names = {"0": "full", "1": "no loads", "2": "no stores", "3": "no loads, no stores"}
for v, t in res.items():
    print(json.dumps({"k": a.k, "m": a.m, "sb": a.shard_bytes, "stripes": a.stripes, "variant": names[v],
                      "kernel": R.encode_kernel_name(a.k, a.m, a.shard_bytes), "ms": round(min(t), 3)}), flush=True)

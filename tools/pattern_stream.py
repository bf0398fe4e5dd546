#!/usr/bin/env python3
"""A repair service's stream of erasure patterns, end to end: for a fixed
wall-clock budget, reconstruct calls of RS(200,55) 256 KiB x STRIPES with 55 losses per call,
the pattern drawn from a pool of POOL random patterns with Zipf(S) popularity, each call timed
(wall, synchronised) and labelled with the kernel that served it (rs_last_kernels). The
background worker's compiles (pattern-compiled kernels from a pattern's RS_AMD_PDEC_AFTER-th
use, at most RS_AMD_PDEC_MAX per code) run meanwhile; a fresh code-object cache per run
(RS_AMD_CACHE_DIR) so no run reuses another's compiles.
  RS_AMD_PDEC_AFTER=3 python tools/pattern_stream.py [seconds] [pool] [stripes] [zipf_s]"""
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-cc_amd"))
os.environ.setdefault("RS_AMD_CACHE_DIR", tempfile.mkdtemp(prefix="rs_stream_cache"))
import reedsol_amd as R  # noqa: E402


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 40.0
    pool = int(sys.argv[2]) if len(sys.argv) > 2 else 48
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    zs = float(sys.argv[4]) if len(sys.argv) > 4 else 1.1
    k, m, sb, e = 200, 55, 256 << 10, 55
    rng = np.random.default_rng(2026)
    pats = []
    for _ in range(pool):
        lost = np.sort(rng.choice(k, size=e, replace=False))
        pats.append((lost, [0 if i in set(lost.tolist()) else 1 for i in range(k)] + [1] * m))
    w = 1.0 / np.arange(1, pool + 1) ** zs
    w /= w.sum()
    dev = torch.device("cuda:0")
    data = torch.randint(0, 256, (n, k, sb), dtype=torch.uint8, device=dev)
    par = torch.empty((n, m, sb), dtype=torch.uint8, device=dev)
    out = torch.empty((n, e, sb), dtype=torch.uint8, device=dev)
    R.encode_batch_dev(k, m, data, par)
    torch.cuda.synchronize()
    calls, t_end = [], time.perf_counter() + secs
    uses = [0] * pool
    bad = 0
    while time.perf_counter() < t_end:
        i = int(rng.choice(pool, p=w))
        lost, present = pats[i]
        t0 = time.perf_counter()
        R.reconstruct_batch_dev(k, m, present, data, par, out)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) * 1e3
        ker = ";".join(R.last_kernels())
        form = "pdecode" if "pdecode" in ker else "decode" if "fft_decode" in ker else "other"
        uses[i] += 1
        calls.append((dt, form, uses[i]))
        if len(calls) % 64 == 1 and not torch.equal(out, data[:, torch.as_tensor(lost, device=dev)]):
            bad += 1
        if len(calls) % 200 == 0:
            print(json.dumps({"t_s": round(secs - (t_end - time.perf_counter()), 1), "calls": len(calls),
                              "pdecode_share": round(sum(c[1] == "pdecode" for c in calls) / len(calls), 3),
                              **R.jit_stats()}), flush=True)
    ms = np.array([c[0] for c in calls])
    forms = {f: int(sum(c[1] == f for c in calls)) for f in ("pdecode", "decode", "other")}
    per_form = {f: round(float(np.median([c[0] for c in calls if c[1] == f])), 3) for f in forms if forms[f]}
    alg = (k + e) * sb * n
    print(json.dumps({
        "workload": f"RS(200,55) 256 KiB x {n}, 55 random losses per call, pool {pool} patterns Zipf({zs})",
        "RS_AMD_PDEC_AFTER": os.environ.get("RS_AMD_PDEC_AFTER", "3 (default)"), "seconds": secs,
        "calls": len(calls), "patterns_seen": int(sum(u > 0 for u in uses)),
        "calls_per_form": forms, "median_ms_per_form": per_form,
        "mean_ms": round(float(ms.mean()), 3), "median_ms": round(float(np.median(ms)), 3),
        "mean_frac": round(alg / (ms.mean() * 1e-3) / 8e12, 4),
        "jit": R.jit_stats(), "spot_checks_bad": bad}), flush=True)


if __name__ == "__main__":
    main()

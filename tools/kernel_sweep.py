#!/usr/bin/env python3
"""A/B sweep of kernel variants in ONE process, interleaved rounds (rule: perf
deltas from interleaved rounds in one process). Variants are selected through
env vars the library reads per call (RS_AMD_NV, RS_AMD_DECODE).

  python tools/kernel_sweep.py --k 10 --m 4 --shard-bytes 1048576 --stripes 1024
"""
import argparse
import itertools
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-cc_amd"))
import reedsol_amd as R  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--shard-bytes", type=int, default=1 << 20)
    ap.add_argument("--stripes", type=int, default=1024)
    ap.add_argument("--erase", type=str, default="0,1,2,3", help="erased indices, or N:first:step")
    ap.add_argument("--rec-erase", type=str, default="", help="lost recovery rows N:first (indices into [0, m))")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--nv", type=str, default="1,2,4")
    ap.add_argument("--decode", type=str, default="", help="comma list of RS_AMD_DECODE values")
    ap.add_argument("--var", action="append", default=[], help="NAME=v1,v2: extra env var to sweep")
    ap.add_argument("--wait", action="store_true", help="after the warmup round, wait for background compiles")
    args = ap.parse_args()
    k, m, sb, n = args.k, args.m, args.shard_bytes, args.stripes
    if ":" in args.erase:
        cnt, first, step = (int(x) for x in args.erase.split(":"))
        erase = list(range(first, first + cnt * step, step))
    else:
        erase = [int(x) for x in args.erase.split(",") if x]
    if any(not 0 <= i < k for i in erase):  # erased data shards only (data[:, erase] below)
        raise SystemExit(f"--erase names shards outside [0, {k}): {erase}")
    e = len(erase)
    present = [0 if i in erase else 1 for i in range(k)] + [1] * m
    if args.rec_erase:
        cnt, first = (int(x) for x in args.rec_erase.split(":"))
        for r in range(first, min(m, first + cnt)):
            present[k + r] = 0
    dev = torch.device("cuda:0")
    data = torch.randint(0, 256, (n, k, sb), dtype=torch.uint8, device=dev)
    parity = torch.empty((n, m, sb), dtype=torch.uint8, device=dev)
    restored = torch.empty((n, max(e, 1), sb), dtype=torch.uint8, device=dev)
    nvs = [x for x in args.nv.split(",") if x]
    decs = [x for x in args.decode.split(",") if x] or [""]
    extra = [(kv.split("=", 1)[0], kv.split("=", 1)[1].split(",")) for kv in args.var]
    variants = [tuple(v[:2]) + (tuple(zip([e[0] for e in extra], v[2:])),)
                for v in itertools.product(nvs, decs, *[e[1] for e in extra])]
    res = {v: {"enc": [], "rec": []} for v in variants}
    s = torch.cuda.current_stream()

    def timed(fn):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(args.reps):
            fn()
        b.record(s)
        torch.cuda.synchronize()
        return a.elapsed_time(b) / args.reps

    ref = None
    for r in range(args.rounds + 1):
        for v in variants:
            for name, val in v[2]:
                os.environ[name] = val
            os.environ["RS_AMD_NV"] = v[0]
            if v[1]:
                os.environ["RS_AMD_DECODE"] = v[1]
            else:
                os.environ.pop("RS_AMD_DECODE", None)
            te = timed(lambda: R.encode_batch_dev(k, m, data, parity, stream=s))
            tr = timed(lambda: R.reconstruct_batch_dev(k, m, present, data, parity, restored, stream=s))
            ok = bool(torch.equal(restored[:, :e], data[:, erase])) if e else True
            if ref is None:
                ref = parity.clone()
            ok = ok and bool(torch.equal(parity, ref))
            if not ok:
                raise SystemExit(f"variant {v} produced wrong bytes")
            if r > 0:  # round 0 = warmup
                res[v]["enc"].append(te)
                res[v]["rec"].append(tr)
        if r == 0 and args.wait:
            R.net_wait()
            for v in variants:  # second pass: the background-compiled kernels are loaded now
                for name, val in v[2]:
                    os.environ[name] = val
                R.encode_batch_dev(k, m, data, parity, stream=s)
                R.reconstruct_batch_dev(k, m, present, data, parity, restored, stream=s)
            R.net_wait()
            torch.cuda.synchronize()
    enc_bytes = (k + m) * sb * n
    rec_bytes = (k + e) * sb * n
    out = []
    for v in variants:
        te, tr = float(np.median(res[v]["enc"])), float(np.median(res[v]["rec"]))
        os.environ["RS_AMD_NV"] = v[0]
        for name, val in v[2]:
            os.environ[name] = val
        if v[1]:
            os.environ["RS_AMD_DECODE"] = v[1]
        else:
            os.environ.pop("RS_AMD_DECODE", None)
        row = {"nv": v[0], "decode": v[1] or "default", **{n: val for n, val in v[2]},
               "enc_kernel": R.encode_kernel_name(k, m, sb), "rec_kernel": R.reconstruct_kernel_name(k, m, sb, present),
               "enc_ms": round(te, 3), "enc_TBps": round(enc_bytes / te / 1e9, 3),
               "rec_ms": round(tr, 3), "rec_TBps": round(rec_bytes / tr / 1e9, 3),
               "enc_min_ms": round(min(res[v]["enc"]), 3), "rec_min_ms": round(min(res[v]["rec"]), 3)}
        out.append(row)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()

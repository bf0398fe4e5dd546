#!/usr/bin/env python3
"""End-to-end (host memory in, host memory out) rate of the codec: the
PCIe-inclusive number DESIGN.md reports beside the device-resident bench.

  python tools/e2e_bench.py --stripes 1024            # RS(10,4) 1 MiB, pinned + pageable
"""
import argparse
import json
import os
import sys
import time

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
    ap.add_argument("--erase", type=str, default="0,1,2,3")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--pageable-stripes", type=int, default=128)
    ap.add_argument("--var", type=str, default="", help="NAME=v1,v2: env values alternated rep by rep in one process")
    a = ap.parse_args()
    vname, vvals = (a.var.split("=", 1)[0], a.var.split("=", 1)[1].split(",")) if a.var else ("", [None])
    k, m, sb = a.k, a.m, a.shard_bytes
    erase = [int(x) for x in a.erase.split(",") if x]
    present = [0 if i in erase else 1 for i in range(k)] + [1] * m
    torch.cuda.init()
    res = {"workload": f"RS({k},{m}) {sb} B shards", "erased": erase}
    for mode, n in (("pinned", a.stripes), ("pageable", a.pageable_stripes)):
        data = torch.randint(0, 256, (n, k, sb), dtype=torch.uint8)
        par = torch.empty((n, m, sb), dtype=torch.uint8)
        out = torch.empty((n, len(erase), sb), dtype=torch.uint8)
        if mode == "pinned":
            data, par, out = data.pin_memory(), par.pin_memory(), out.pin_memory()
        R.encode_batch_host(k, m, data[:1], par[:1])  # plan + warmup
        R.reconstruct_batch_host(k, m, present, data[:1], par[:1], out[:1])
        te, tr = {v: [] for v in vvals}, {v: [] for v in vvals}
        ok = True
        for _ in range(a.reps):
            for v in vvals:
                if v is not None:
                    os.environ[vname] = v
                t0 = time.perf_counter()
                R.encode_batch_host(k, m, data, par)
                te[v].append(time.perf_counter() - t0)
                out.zero_()
                t0 = time.perf_counter()
                R.reconstruct_batch_host(k, m, present, data, par, out)
                tr[v].append(time.perf_counter() - t0)
                ok = ok and bool(torch.equal(out, data[:, erase]))
        gib = k * sb * n / 2**30
        for v in vvals:
            key = mode if v is None else f"{mode} {vname}={v}"
            res[key] = {"stripes": n, "encode_GiBps": round(gib / min(te[v]), 2),
                        "reconstruct_GiBps": round(gib / min(tr[v]), 2),
                        "encode_pcie_GBps": round((k + m) * sb * n / min(te[v]) / 1e9, 2),
                        "reconstruct_pcie_GBps": round((k + len(erase)) * sb * n / min(tr[v]) / 1e9, 2),
                        "verified": ok}
            print(json.dumps({key: res[key]}), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()

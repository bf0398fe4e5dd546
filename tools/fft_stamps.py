#!/usr/bin/env python3
"""Phase timeline of the FFT kernels (measurement build, RS_AMD_FFT_DEBUG bit 6 = 64): every
wave of workgroup 0 stamps s_memtime around each barrier of its third unit. Prints, per wave,
the cycles spent before each barrier (compute since the previous stamp) and waiting in it.
  python tools/fft_stamps.py K M SB STRIPES LOSSES encode|fused|pattern [RS_AMD_X=v ...]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-cc_amd"))
import reedsol_amd as R  # noqa: E402


def main():
    k, m, sb, n, e = (int(x) for x in sys.argv[1:6])
    form = sys.argv[6]
    for kv in sys.argv[7:]:
        a, b = kv.split("=", 1)
        os.environ[a] = b
    dev = torch.device("cuda:0")
    lost = list(range(1, k, 3))[:e]
    present = [0 if i in lost else 1 for i in range(k)] + [1] * m
    data = torch.randint(0, 256, (n, k, sb), dtype=torch.uint8, device=dev)
    par = torch.empty((n, m, sb), dtype=torch.uint8, device=dev)
    out = torch.empty((n, max(e, 1), sb), dtype=torch.uint8, device=dev)
    R.encode_batch_dev(k, m, data, par)  # plain build for the parity
    torch.cuda.synchronize()
    os.environ["RS_AMD_FFT_DEBUG"] = str(int(os.environ.get("RS_AMD_FFT_DEBUG", "0")) | 64)
    if form == "fused":
        os.environ["RS_AMD_FDEC"] = "1"
    if form == "encode":
        par2 = torch.empty_like(par)
        fn = lambda: R.encode_batch_dev(k, m, data, par2)  # noqa: E731
    else:
        if form == "pattern":
            R.reconstruct_warm(k, m, sb, present)
        fn = lambda: R.reconstruct_batch_dev(k, m, present, data, par, out)  # noqa: E731
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    kern = R.last_kernels()
    st = R.debug_fft_stamps().astype(np.int64)
    used = [i for i in range(64) if (st[:, i] != 0).all()]
    t0 = st[:, 62].min()
    rows = []
    for w in range(8):
        rows.append({"wave": w, "total": int(st[w, 63] - st[w, 62]),
                     "stamps": [int(st[w, i] - t0) for i in used]})
    # per barrier b (stamps 2b, 2b+1): arrival spread and the slowest wave's compute since the last release
    phases = []
    prev = st[:, 62]
    for b in range(0, 62, 2):
        if b not in used:
            break
        arr, rel = st[:, b], st[:, b + 1]
        phases.append({"bar": b // 2, "work_max": int((arr - prev).max()), "work_min": int((arr - prev).min()),
                       "wait_max": int((rel - arr).max()), "wait_min": int((rel - arr).min()),
                       "work": [int(x) for x in arr - prev]})
        prev = rel
    tail = int((st[:, 63] - prev).max())
    phases.append({"bar": "end", "work": [int(x) for x in st[:, 63] - prev]})
    print(json.dumps({"code": f"RS({k},{m}) {sb} B x {n}", "form": form, "kernels": kern,
                      "unit_cycles": [r["total"] for r in rows], "after_last_bar_max": tail}))
    for p in phases:
        print(json.dumps(p))


if __name__ == "__main__":
    main()

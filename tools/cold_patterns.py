#!/usr/bin/env python3
"""Cold erasure patterns on RS(200,55) 256 KiB x 256 (verdict r2 item 3): the first calls
of fresh patterns (no net_wait, plan build in the wall time), against the warm path, with
the fused FFT reconstruct (RS_AMD_FDEC=auto) and without it (0). One JSON line per case."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-cc_amd"))
import reedsol_amd as R  # noqa: E402


def main():
    k, m, sb, n = 200, 55, 256 << 10, 256
    dev = torch.device("cuda:0")
    data = torch.randint(0, 256, (n, k, sb), dtype=torch.uint8, device=dev)
    par = torch.empty((n, m, sb), dtype=torch.uint8, device=dev)
    out = torch.empty((n, m, sb), dtype=torch.uint8, device=dev)
    R.encode_batch_dev(k, m, data, par)
    # warm the code's kernels (FFT encode, fused decode, syndrome kernels) on a throwaway pattern
    for mode in ("1", "0"):
        os.environ["RS_AMD_FDEC"] = mode
        lost = list(range(0, 165, 3))
        R.reconstruct_batch_dev(k, m, [0 if i in lost else 1 for i in range(k)] + [1] * m, data, par, out)
    torch.cuda.synchronize()
    first = 2
    for mode in ("auto", "0"):
        os.environ["RS_AMD_FDEC"] = mode
        for e in (55, 20, 8):
            lost = list(range(first, first + 3 * e, 3))
            first += 1
            present = [0 if i in lost else 1 for i in range(k)] + [1] * m
            calls = []
            for _ in range(3):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t0 = time.perf_counter()
                a.record()
                R.reconstruct_batch_dev(k, m, present, data, par, out)
                b.record()
                torch.cuda.synchronize()
                calls.append([round((time.perf_counter() - t0) * 1e3, 2), round(a.elapsed_time(b), 2)])
            ok = bool(torch.equal(out[:, :e], data[:, lost]))
            print(json.dumps({"fdec": mode, "erased": e, "calls_wall_gpu_ms": calls, "verified": ok,
                              "kernel": R.reconstruct_kernel_name(k, m, sb, present)}), flush=True)
    R.net_wait()


if __name__ == "__main__":
    main()

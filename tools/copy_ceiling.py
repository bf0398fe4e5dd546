#!/usr/bin/env python3
"""HBM streaming ceiling on this box: torch device-to-device copy (1 read + 1 write
stream) and a 14-stream pattern like the RS(10,4) kernels (10 reads, 4 writes via
torch ops), for comparison with the network kernels' achieved GB/s."""
import json
import torch

dev = torch.device("cuda:0")
n = 8 << 30
x = torch.empty(n, dtype=torch.uint8, device=dev)
y = torch.empty(n, dtype=torch.uint8, device=dev)
x.fill_(1)
torch.cuda.synchronize()
res = {}
for name, fn, moved in (("copy_8GiB", lambda: y.copy_(x), 2 * n),):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        fn()
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 10
    res[name] = {"ms": round(ms, 3), "GBps": round(moved / ms / 1e6, 1)}
print(json.dumps(res))

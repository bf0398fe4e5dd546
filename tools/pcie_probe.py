import torch, time
dev = torch.device("cuda:0")
for mb in (256, 1024):
    h = torch.empty(mb << 20, dtype=torch.uint8).pin_memory()
    d = torch.empty(mb << 20, dtype=torch.uint8, device=dev)
    d.copy_(h, non_blocking=True); torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(4): d.copy_(h, non_blocking=True)
    torch.cuda.synchronize(); h2d = 4 * (mb << 20) / (time.perf_counter() - t) / 1e9
    t = time.perf_counter()
    for _ in range(4): h.copy_(d, non_blocking=True)
    torch.cuda.synchronize(); d2h = 4 * (mb << 20) / (time.perf_counter() - t) / 1e9
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    h2 = torch.empty(mb << 20, dtype=torch.uint8).pin_memory(); d2 = torch.empty(mb << 20, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(4):
        with torch.cuda.stream(s1): d.copy_(h, non_blocking=True)
        with torch.cuda.stream(s2): h2.copy_(d2, non_blocking=True)
    torch.cuda.synchronize(); both = 8 * (mb << 20) / (time.perf_counter() - t) / 1e9
    print(f"{mb} MiB: H2D {h2d:.1f} GB/s, D2H {d2h:.1f} GB/s, both directions {both:.1f} GB/s", flush=True)

#!/usr/bin/env python3
"""Debug aid: FFT encode kernel vs oracle over several shapes; prints where parity differs."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-cc_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import reedsol_amd as R
import oracle as O
dev = torch.device("cuda:0")
shapes = [tuple(int(x) for x in a.split(",")) for a in sys.argv[1:]]
for k, m in shapes:
    sb, n = 4096, 2
    data = np.random.default_rng(k + m).integers(0, 256, (n, k, sb), dtype=np.uint8)
    d = torch.from_numpy(data).to(dev)
    p = torch.zeros((n, m, sb), dtype=torch.uint8, device=dev)
    R.encode_batch_dev(k, m, d, p, 0)
    torch.cuda.synchronize()
    got = p.cpu().numpy()
    exp = O.encode_batch(k, m, data, threads=8)
    bad = got != exp
    rows = sorted(set(np.nonzero(bad)[1].tolist()))
    cols = np.nonzero(bad)[2]
    print(f"RS({k},{m}) kernel {R.encode_kernel_name(k, m, sb)} bad bytes {bad.sum()} of {bad.size}; rows {rows[:20]}..{len(rows)}; "
          f"col%2048 uniq {len(set((cols % 2048).tolist()))}; stripes {sorted(set(np.nonzero(bad)[0].tolist()))}", flush=True)

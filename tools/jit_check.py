#!/usr/bin/env python3
"""Quick GPU check of the bit-sliced network kernels against the oracle + timing."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-cc_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import reedsol_amd as R  # noqa: E402
import oracle as O  # noqa: E402

os.environ.setdefault("RS_AMD_JIT_VERBOSE", "1")
dev = torch.device("cuda:0")
for (k, m, sb, n, erase) in [(10, 4, 4096, 6, [0, 1, 2, 3]), (10, 4, 8192, 5, [1, 5]), (4, 2, 4096, 4, [0, 3]),
                             (16, 16, 4096, 2, list(range(16))), (5, 5, 4096, 3, [0, 2, 4])]:
    rng = np.random.default_rng(k * 100 + m)
    data = rng.integers(0, 256, (n, k, sb), dtype=np.uint8)
    d = torch.from_numpy(data).to(dev)
    p = torch.zeros((n, m, sb), dtype=torch.uint8, device=dev)
    t0 = time.time()
    R.encode_batch_dev(k, m, d, p)
    torch.cuda.synchronize()
    t1 = time.time()
    exp = O.encode_batch(k, m, data, threads=8)
    ok_enc = bool((p.cpu().numpy() == exp).all())
    present = [0 if i in erase else 1 for i in range(k)] + [1] * m
    out = torch.zeros((n, len(erase), sb), dtype=torch.uint8, device=dev)
    t2 = time.time()
    R.reconstruct_batch_dev(k, m, present, d, p, out)
    torch.cuda.synchronize()
    t3 = time.time()
    ok_rec = bool((out.cpu().numpy() == data[:, erase]).all())
    print(f"RS({k},{m}) sb={sb} enc {R.encode_kernel_name(k, m, sb)} ok={ok_enc} ({(t1-t0)*1e3:.0f} ms first call) "
          f"rec {R.reconstruct_kernel_name(k, m, sb, present)} ok={ok_rec} ({(t3-t2)*1e3:.0f} ms)", flush=True)
    if not (ok_enc and ok_rec):
        bad = np.argwhere(p.cpu().numpy() != exp)
        print("  first enc mismatches:", bad[:5])

#!/usr/bin/env python3
"""Round-2 note: spilled builds of the FFT kernel produced wrong bytes
intermittently (RS(1000,64), prefetch 4). Reproduce: run the encode of a spilled build
(RS_AMD_FFT_PREFETCH=4, RS_AMD_FFT_ALLOW_SPILL=1) `reps` times against the oracle on a
fixed batch, report every mismatching launch (which stripes / shards / bytes), then the
same with the device stack limit raised (more scratch per lane reserved by the runtime)
and with the spill-free build (prefetch 2). One JSON line per configuration.
  RS_AMD_FFT_PREFETCH=4 RS_AMD_FFT_ALLOW_SPILL=1 python tools/spill_repro.py [reps] [stack_bytes]"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-cc_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import reedsol_amd as R  # noqa: E402
import oracle as O  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
stack = int(sys.argv[2]) if len(sys.argv) > 2 else 0
k, m, sb, n = 1000, 64, 4096, 96
dev = torch.device("cuda:0")
if stack:
    hip = C.CDLL("libamdhip64.so")
    st = hip.hipDeviceSetLimit(0, C.c_size_t(stack))  # hipLimitStackSize
    print(json.dumps({"hipDeviceSetLimit(stack)": stack, "status": st}), flush=True)
rng = np.random.default_rng(1000)
data = rng.integers(0, 256, (n, k, sb), dtype=np.uint8)
exp = O.encode_batch(k, m, data, threads=16)
d = torch.from_numpy(data).to(dev)
p = torch.empty((n, m, sb), dtype=torch.uint8, device=dev)
bad_launches = []
for r in range(reps):
    p.fill_(0)
    R.encode_batch_dev(k, m, d, p)
    torch.cuda.synchronize()
    got = p.cpu().numpy()
    diff = got != exp
    if diff.any():
        st_, sh_, by_ = np.nonzero(diff)
        # per bad 1 KiB block (stripe, shard, block): bad bytes, and whether the block
        # reads as the fill value (store missing) or as other bytes (wrong data)
        blocks = {}
        for a, b_, c in zip(st_.tolist(), sh_.tolist(), (by_ // 1024).tolist()):
            blocks[(a, b_, c)] = blocks.get((a, b_, c), 0) + 1
        kinds = {}
        for (a, b_, c), cnt in blocks.items():
            g = got[a, b_, c * 1024:(c + 1) * 1024]
            kind = "zero" if not g.any() else "other"
            if kind == "other":  # the right bytes of another stripe / shard / block?
                for a2 in range(n):
                    for b2 in range(m):
                        for c2 in range(sb // 1024):
                            if (a2, b2, c2) != (a, b_, c) and np.array_equal(g, exp[a2, b2, c2 * 1024:(c2 + 1) * 1024]):
                                kind = "copy_of:%d/%d/%d" % (a2, b2, c2)
                                break
                        if kind != "other":
                            break
                    if kind != "other":
                        break
            offs = np.nonzero(diff[a, b_, c * 1024:(c + 1) * 1024])[0]
            xr = (got[a, b_, c * 1024:(c + 1) * 1024] ^ exp[a, b_, c * 1024:(c + 1) * 1024])[offs]
            kinds.setdefault(kind.split(":")[0], []).append([a, b_, c, cnt] + ([kind] if ":" in kind else []) +
                                                           [offs.tolist()[:64], xr.tolist()[:16]])
        bad_launches.append({"rep": r, "bytes": int(diff.sum()), "stripes": sorted(set(st_.tolist()))[:8],
                             "shards": sorted(set(sh_.tolist()))[:8], "first_byte": int(by_.min()),
                             "blocks_1k": len(blocks), "block_offsets": sorted(set(c for (_, _, c) in blocks)),
                             "kinds": {k: v[:3] for k, v in kinds.items()}})
print(json.dumps({"prefetch": os.environ.get("RS_AMD_FFT_PREFETCH"), "allow_spill": os.environ.get("RS_AMD_FFT_ALLOW_SPILL"),
                  "stack": stack, "kernel": R.encode_kernel_name(k, m, sb), "reps": reps,
                  "bad_launches": len(bad_launches), "detail": bad_launches[:6]}), flush=True)

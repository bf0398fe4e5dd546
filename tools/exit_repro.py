"""Process exit with a pattern's background upgrade (full plan build + pattern-compiled kernel
compile) queued or in flight: the process must exit cleanly (rc 0)."""
import sys
import time

import torch

sys.path.insert(0, "reed-solomon-cc_amd")
import reedsol_amd as R  # noqa: E402

k, m, sb, n = 200, 55, 262144, 64
wait = float(sys.argv[1]) if len(sys.argv) > 1 else 0.0
dev = torch.device("cuda:0")
d = torch.randint(0, 256, (n, k, sb), dtype=torch.uint8, device=dev)
p = torch.empty((n, m, sb), dtype=torch.uint8, device=dev)
R.encode_batch_dev(k, m, d, p)
lost = list(range(2, k, 3))[:m]
present = [0 if i in lost else 1 for i in range(k)] + [1] * m
out = torch.empty((n, m, sb), dtype=torch.uint8, device=dev)
for _ in range(3):
    R.reconstruct_batch_dev(k, m, present, d, p, out)
torch.cuda.synchronize()
print("kernels", R.last_kernels(), "ok", bool(torch.equal(out, d[:, lost])), flush=True)
time.sleep(wait)
print("exiting", flush=True)

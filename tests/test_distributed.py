"""world_size-2 gloo run of the multi-GPU layout (reedsol_amd/sharding.py):
disjoint stripe ranges, per-rank encode, control-plane MAX/AND only. On the CPU
box each rank encodes its range with the oracle; with a GPU (the gpu-marked
variant) both ranks drive librs_amd on cuda:0 (per-process plans, hipRTC
networks and the shared on-disk code-object cache) and rank 0 checks the
gathered parity against the oracle."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from rs_amd import reedsol_amd  # noqa: F401  (puts the package on sys.path)
from reedsol_amd.sharding import stripe_range


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out, use_gpu=False):
    import sys
    import torch
    import torch.distributed as dist

    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "oracle"))
    import oracle as O
    from reedsol_amd.sharding import all_ok, max_over_ranks, stripe_range

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ok_all = True
    t = max_over_ranks(float(rank + 1))
    # (k, m, shard bytes): the headline code, and a wide one (bit-sliced FFT kernel on the GPU)
    for k, m, sb, n in ((10, 4, 4096 if use_gpu else 256, 7), (100, 20, 4096, 5)):
        ok_all &= _encode_range_and_check(O, rank, world, k, m, sb, n, use_gpu)
    if rank == 0:
        out.put((t, ok_all))
    dist.destroy_process_group()


def _encode_range_and_check(O, rank, world, k, m, sb, n, use_gpu):
    import torch
    import torch.distributed as dist
    from reedsol_amd.sharding import all_ok, stripe_range

    rng = np.random.default_rng(123 + k)
    data = rng.integers(0, 256, (n, k, sb), dtype=np.uint8)  # same global batch on every rank
    b, e = stripe_range(n, rank, world)
    if use_gpu:
        from rs_amd import reedsol_amd as R
        dev = torch.device("cuda:0")  # the ranks share one GPU here; one per GPU on a node
        d = torch.from_numpy(np.ascontiguousarray(data[b:e])).to(dev)
        p = torch.zeros((e - b, m, sb), dtype=torch.uint8, device=dev)
        R.encode_batch_dev(k, m, d, p)
        torch.cuda.synchronize()
        par = p.cpu().numpy()
    else:
        par = O.encode_batch(k, m, data[b:e])
    # rank 0 collects the shards only to CHECK the layout (bench never does this)
    sizes = [stripe_range(n, r, world)[1] - stripe_range(n, r, world)[0] for r in range(world)]
    buf = torch.zeros((max(sizes), m, sb), dtype=torch.uint8)
    buf[: e - b] = torch.from_numpy(par)
    gathered = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(gathered, buf)
    full = np.concatenate([g[:s].numpy() for g, s in zip(gathered, sizes)])
    return all_ok(bool((full == O.encode_batch(k, m, data)).all()))


def test_stripe_range_partitions():
    for n in (0, 1, 7, 4096, 32768):
        for world in (1, 2, 3, 8):
            ranges = [stripe_range(n, r, world) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == n
            for (a, b), (c, d) in zip(ranges, ranges[1:]):
                assert b == c
            sizes = [b - a for a, b in ranges]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        stripe_range(10, 2, 2)


def _run_world2(use_gpu):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, use_gpu)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    t, ok = q.get(timeout=10)
    assert t == 2.0 and ok


def test_gloo_world_size_2():
    _run_world2(False)


@pytest.mark.gpu
def test_gloo_world_size_2_on_gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run_world2(True)

"""Multi-GPU layout for the codec: one process per GPU, disjoint stripe ranges.

Stripes are independent codes, so the batch partitions with
no data-path exchange: device d owns stripes [d*N/G, (d+1)*N/G). The only
collectives are control-plane: a barrier around the timed region and a MAX of
the per-rank times (bench.py), which work on gloo (CPU tests) and on
nccl = RCCL (GPU runs) alike.
"""
from __future__ import annotations


def stripe_range(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous, balanced partition of n_total stripes over world ranks."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    base, extra = divmod(n_total, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def max_over_ranks(value: float, device=None) -> float:
    """MAX of a per-rank scalar (timing) over the default process group."""
    import torch
    import torch.distributed as dist

    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_ok(flag: bool, device=None) -> bool:
    """AND of a per-rank verification flag."""
    import torch
    import torch.distributed as dist

    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size() == 1:
        return bool(flag)
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())

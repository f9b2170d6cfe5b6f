"""ofdm_dist — frame sharding and the one end-of-job reduction.

Frames are independent (own pilots, own symbol-0 reference, own sync), so a
batch shards as contiguous frame ranges, remainder to the low ranks, with no
data-path collective. The only collective is a SUM all-reduce of the
{bit_errors, bits, samples, frames} counters plus a MAX of the elapsed time
(RCCL over xGMI on MI355X, gloo in the CPU tests)."""
from __future__ import annotations

import os


def shard(n_units: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [begin, begin+count) of n_units for `rank`; low ranks take the remainder."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, rem = divmod(n_units, world)
    count = base + (1 if rank < rem else 0)
    begin = rank * base + min(rank, rem)
    return begin, count


def env_world() -> tuple[int, int, int]:
    """(world, rank, local_rank) from torch.distributed.run's environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def reduce_counters(counters, dist=None):
    """SUM all-reduce of an int64 tensor [bit_errors, bits, samples, frames] (in place)."""
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(counters)
    return counters


def max_over_ranks(value: float, device, dist=None) -> float:
    import torch
    t = torch.tensor([value], dtype=torch.float64, device=device)
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())

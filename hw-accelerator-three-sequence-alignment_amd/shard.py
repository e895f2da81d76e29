"""Multi-GPU batch sharding: independent triples are split into
contiguous blocks, one block per rank (one process per GPU); the only
collective is the final int32 score gather (RCCL over xGMI on the GPU box,
gloo in the CPU tests). No data-path collective exists: the path shards."""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous block [i0, i1) of triple indices owned by `rank`."""
    i0 = (n_total * rank) // world
    i1 = (n_total * (rank + 1)) // world
    return i0, i1


def gather_scores(local: torch.Tensor, n_total: int, world: int) -> torch.Tensor:
    """All-gather per-rank int32 score blocks into the global order.

    Blocks may differ in length by one; they are padded to the longest block
    for the collective and trimmed afterwards."""
    if world == 1:
        return local
    longest = max(shard_range(n_total, r, world)[1] - shard_range(n_total, r, world)[0]
                  for r in range(world))
    pad = torch.zeros(longest, dtype=local.dtype, device=local.device)
    pad[: local.numel()] = local
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad)
    out = []
    for r in range(world):
        i0, i1 = shard_range(n_total, r, world)
        out.append(parts[r][: i1 - i0])
    return torch.cat(out)


def max_over_ranks(value: float, device) -> float:
    """The slowest rank's time: what the whole job waited for."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())

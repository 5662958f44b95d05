"""Multi-GPU sharding of a QP batch.

QPs are independent, so the batch is cut into contiguous per-rank shards and
solved with no data-path collective.  The only exchange is config 5's argmin
gather: each rank reduces its shard to (fval, local index) on device
(qpb_argmin) and one all_gather of 16 B per rank -- RCCL over xGMI on the GPU,
gloo in the CPU tests -- lets every rank pick the same global winner.
"""
from __future__ import annotations

import numpy as np


def shard_range(rank: int, world: int, per_rank: int) -> tuple[int, int]:
    """Global QP ids [lo, hi) owned by `rank` (weak scaling: fixed per-rank size)."""
    if not (0 <= rank < world) or per_rank < 0:
        raise ValueError("bad shard")
    return rank * per_rank, (rank + 1) * per_rank


def split_even(total: int, world: int, rank: int) -> tuple[int, int]:
    """Global ids [lo, hi) of `rank` when a fixed total is split (strong scaling)."""
    base, extra = divmod(total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def global_winner(gathered, offsets):
    """Pick the global (fval, global index, rank) from per-rank (fval, local
    index) pairs; index -1 marks a rank with no optimal QP.  Lowest fval wins,
    ties go to the lowest global index (the same rule as qpb_argmin)."""
    g = np.asarray(gathered, dtype=np.float64).reshape(-1, 2)
    best = (np.inf, -1, -1)
    for r, (fv, idx) in enumerate(g):
        if idx < 0:
            continue
        gi = int(idx) + int(offsets[r])
        if fv < best[0] or (fv == best[0] and (best[1] < 0 or gi < best[1])):
            best = (float(fv), gi, r)
    return best


def all_gather_winner(best_local, world: int):
    """all_gather of one rank's (fval, index) pair; returns [world, 2].
    best_local: a 2-element float64 tensor on the rank's device (GPU: RCCL
    all_gather_into_tensor; CPU/gloo: list all_gather)."""
    import torch
    import torch.distributed as dist
    if world == 1:
        return best_local.reshape(1, 2)
    if best_local.is_cuda:
        out = torch.empty(2 * world, dtype=best_local.dtype, device=best_local.device)
        dist.all_gather_into_tensor(out, best_local)
        return out.reshape(world, 2)
    parts = [torch.empty_like(best_local) for _ in range(world)]
    dist.all_gather(parts, best_local)
    return torch.stack(parts)

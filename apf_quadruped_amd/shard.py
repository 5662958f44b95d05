"""Multi-GPU sharding of a QP batch.

QPs are independent, so the batch is cut into contiguous per-rank shards and
solved with no data-path collective.  The only exchange is config 5's argmin
gather: each rank reduces its shard to the payload (fval, global index, x*[n])
on device and one all_gather of 16 + 8n B per rank gives every rank the same
global winner and its solution.  On the GPUs that is qpb_argmin_allgather (C ABI:
payload kernel, ncclAllGather over RCCL / xGMI, device-side reduce, all on one
stream; ArgminGather below); the CPU tests run the same logic over gloo
(all_gather_winner + global_winner).
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


def global_winner(gathered, offsets, width: int = 2):
    """Pick the global (fval, global index, rank) from per-rank payloads
    (fval, local index[, x*...]) of `width` doubles; index -1 marks a rank with
    no optimal QP.  Lowest fval wins, ties go to the lowest global index (the
    same rule as qpb_argmin).  The winner's x* is gathered[rank, 2:]."""
    g = np.asarray(gathered, dtype=np.float64).reshape(-1, width)
    best = (np.inf, -1, -1)
    for r, row in enumerate(g):
        fv, idx = row[0], row[1]
        if idx < 0:
            continue
        gi = int(idx) + int(offsets[r])
        if fv < best[0] or (fv == best[0] and (best[1] < 0 or gi < best[1])):
            best = (float(fv), gi, r)
    return best


def all_gather_winner(best_local, world: int):
    """all_gather of one rank's payload (fval, index[, x*...]); returns
    [world, len].  best_local: a float64 tensor on the rank's device (GPU: RCCL
    all_gather_into_tensor; CPU/gloo: list all_gather)."""
    import torch
    import torch.distributed as dist
    w = best_local.numel()
    if world == 1:
        return best_local.reshape(1, w)
    if best_local.is_cuda:
        out = torch.empty(w * world, dtype=best_local.dtype, device=best_local.device)
        dist.all_gather_into_tensor(out, best_local)
        return out.reshape(world, w)
    parts = [torch.empty_like(best_local) for _ in range(world)]
    dist.all_gather(parts, best_local)
    return torch.stack(parts)


def winner_payload(best, x_tiled, n: int, B: int, out=None, stream=None):
    """Device payload {fval, index, x*[n]} of a rank's winner (qpb_winner): one
    small launch on `stream`, no host synchronisation."""
    import ctypes as C
    import torch
    from ._lib import check, lib
    if out is None:
        out = torch.empty(2 + n, dtype=torch.float64, device=best.device)
    if stream is None:
        stream = torch.cuda.current_stream(best.device)
    check(lib().qpb_winner(C.c_void_p(best.data_ptr()), C.c_void_p(x_tiled.data_ptr()), int(n), int(B),
                           C.c_void_p(out.data_ptr()), C.c_void_p(stream.cuda_stream)), "qpb_winner")
    return out


class ArgminGather:
    """The multi-GPU argmin gather through the library's C ABI (RCCL over xGMI).

    Rank 0 creates an RCCL unique id (qpb_comm_get_unique_id); every rank gets
    it through torch.distributed's object broadcast (bootstrap only -- the data
    path never goes through torch) and joins the communicator on its current
    device (qpb_comm_init).  `gather(best, x, n, B, base, out, stream)` is one
    stream-ordered qpb_argmin_allgather: out = {fval, global index, x*[n]} of the
    global winner on every rank."""

    def __init__(self, rank: int, world: int):
        import ctypes as C
        import torch.distributed as dist
        from ._lib import check, lib
        self._C, self._check, self._lib = C, check, lib
        idb = C.create_string_buffer(128)
        err = None
        if rank == 0:
            try:
                check(lib().qpb_comm_get_unique_id(idb), "qpb_comm_get_unique_id")
            except RuntimeError as e:      # still broadcast, so no rank waits forever
                err = str(e)
        obj = [idb.raw if err is None else None, err]
        if world > 1:
            dist.broadcast_object_list(obj, src=0)
        if obj[1] is not None:
            raise RuntimeError(f"rank 0: {obj[1]}")
        idb = C.create_string_buffer(obj[0], 128)
        h = C.c_void_p()
        check(lib().qpb_comm_init(C.byref(h), int(world), idb, int(rank)), "qpb_comm_init")
        self.comm, self.rank, self.world = h, rank, world

    def gather(self, best, x, n: int, B: int, base: int, out, stream):
        C = self._C
        self._check(self._lib().qpb_argmin_allgather(
            C.c_void_p(best.data_ptr()), C.c_void_p(x.data_ptr()), int(n), int(B), int(base), self.comm,
            C.c_void_p(out.data_ptr()), C.c_void_p(stream.cuda_stream)), "qpb_argmin_allgather")
        return out

    def close(self):
        if self.comm is not None and self.comm.value:
            self._lib().qpb_comm_destroy(self.comm)
        self.comm = None

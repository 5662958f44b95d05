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

    def count(self) -> int:
        """Ranks in the communicator as RCCL reports them (ncclCommCount)."""
        C = self._C
        k = C.c_int(0)
        self._check(self._lib().qpb_comm_count(self.comm, C.byref(k)), "qpb_comm_count")
        return int(k.value)

    def gather(self, best, x, n: int, B: int, base: int, out, stream):
        C = self._C
        self._check(self._lib().qpb_argmin_allgather(
            C.c_void_p(best.data_ptr()), C.c_void_p(x.data_ptr()), int(n), int(B), int(base), self.comm,
            C.c_void_p(out.data_ptr()), C.c_void_p(stream.cuda_stream)), "qpb_argmin_allgather")
        return out

    def close(self):
        if getattr(self, "comm", None) is not None and self.comm.value:
            self._lib().qpb_comm_destroy(self.comm)
        self.comm = None


def make_argmin_gather(rank: int, world: int, device):
    """ArgminGather on every rank, or the torch fallback on every rank: the ranks
    agree on the outcome of qpb_comm_init (an all_reduce of a success flag over the
    default process group) so no rank is left waiting in the RCCL gather while
    another has fallen back.  Returns (gather object, info dict for the bench line:
    path, ranks RCCL reports, and the init error if any)."""
    import torch
    import torch.distributed as dist
    ag, err = None, None
    try:
        ag = ArgminGather(rank, world)
    except Exception as e:      # noqa: BLE001 -- reported in the info dict
        err = str(e)
    ok = torch.tensor([0 if ag is None else 1], dtype=torch.int32, device=device)
    if world > 1:
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if int(ok.item()) == 1:
        return ag, {"gather": "qpb_argmin_allgather", "rccl_ranks": ag.count(), "init_error": None}
    if ag is not None:
        ag.close()
    return TorchGather(world), {"gather": "torch_fallback", "rccl_ranks": None,
                                "init_error": err or "qpb_comm_init failed on another rank"}


class TorchGather:
    """Fallback for ArgminGather when the library's RCCL communicator cannot be
    made on every rank: payload (qpb_winner, global index) + torch's
    all_gather_into_tensor (also RCCL) + qpb_argmin_reduce, on the same stream."""

    def __init__(self, world):
        self.world = world
        self.comm = None

    def gather(self, best, x, n, B, base, out, stream):
        import ctypes as C
        import torch
        import torch.distributed as dist
        from ._lib import check, lib
        with torch.cuda.stream(stream):
            pay = winner_payload(best, x, n, B, stream=stream)
            pay[1] = torch.where(pay[1] >= 0, pay[1] + base, pay[1])
            g = torch.empty((2 + n) * self.world, dtype=torch.float64, device=pay.device)
            dist.all_gather_into_tensor(g, pay)
            check(lib().qpb_argmin_reduce(C.c_void_p(g.data_ptr()), self.world, n, C.c_void_p(out.data_ptr()),
                                          C.c_void_p(stream.cuda_stream)), "qpb_argmin_reduce")
        return out

    def close(self):
        pass

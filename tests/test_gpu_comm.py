"""The multi-GPU argmin gather through the C ABI (qpb_comm.hip):
qpb_argmin_reduce on synthetic gathered payloads (ties, ranks without an optimal
QP), and qpb_argmin_allgather end to end on a one-rank RCCL communicator (one GPU
per box: RCCL refuses two ranks on one device).  The gather logic over several
ranks is exercised on CPU by tests/test_multi.py (gloo)."""
import ctypes as C

import numpy as np
import pytest

from apf_quadruped_amd import _lib


def _p(t):
    return C.c_void_p(t.data_ptr())


@pytest.mark.gpu
def test_argmin_reduce_rule():
    import torch
    n = 3
    nan = float("nan")
    rows = [[5.0, 40.0, 1, 2, 3],        # rank 0
            [-2.0, 77.0, 4, 5, 6],       # rank 1: lowest fval ...
            [-2.0, 12.0, 7, 8, 9],       # rank 2: ... tied, lower global index wins
            [np.inf, -1.0, nan, nan, nan]]   # rank 3: no optimal QP
    g = torch.tensor(np.asarray(rows, np.float64).reshape(-1), device="cuda")
    out = torch.zeros(2 + n, dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream()
    _lib.check(_lib.lib().qpb_argmin_reduce(_p(g), 4, n, _p(out), C.c_void_p(s.cuda_stream)), "reduce")
    torch.cuda.synchronize()
    assert out.cpu().numpy().tolist() == [-2.0, 12.0, 7.0, 8.0, 9.0]
    none = torch.tensor([np.inf, -1.0, nan, nan, nan] * 2, dtype=torch.float64, device="cuda")
    _lib.check(_lib.lib().qpb_argmin_reduce(_p(none), 2, n, _p(out), C.c_void_p(s.cuda_stream)), "reduce")
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    assert o[0] == np.inf and o[1] == -1.0 and np.isnan(o[2:]).all()


@pytest.mark.gpu
def test_argmin_allgather_one_rank_communicator():
    import torch
    from apf_quadruped_amd import workloads as W
    from apf_quadruped_amd.batch import Plan, from_tiled
    from apf_quadruped_amd.shard import ArgminGather
    B, base = 1000, 5000
    d = W.contact_force_qp(0xD06B07 + 17, np.arange(B))
    plan = Plan.from_dense(12, 20, 6, d["P"][0], d["A"][0], d["G"][0])
    vals = {k: torch.from_numpy(v).cuda() for k, v in plan.pack(d["P"], d["A"], d["G"], d["c"], d["h"],
                                                                d["b"]).items()}
    out = plan.alloc_outputs(B)
    best = torch.zeros(2, dtype=torch.float64, device="cuda")
    plan.launcher(vals, out, B, best=best)()
    ag = ArgminGather(0, 1)
    try:
        win = torch.zeros(14, dtype=torch.float64, device="cuda")
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        for _ in range(3):                       # repeated, on a side stream
            ag.gather(best, out["x"], 12, B, base, win, s)
        torch.cuda.synchronize()
        w = win.cpu().numpy()
        fv, idx = best.cpu().numpy()
        x = from_tiled(out["x"], B, 12).cpu().numpy()
        assert w[0] == fv and w[1] == base + idx
        np.testing.assert_array_equal(w[2:], x[int(idx)])
    finally:
        ag.close()

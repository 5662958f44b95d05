"""Plan groups (qpb_group_*): one launch for a batch of mixed sparsity patterns
(configs[2]: the four gait phases), through the C ABI.

* every member's outputs are bit-identical to qpb_solve on that plan alone (the
  group kernel runs each member's row-kernel body unchanged);
* against the reference's golden vectors of the four gait patterns
  (tests/golden/mixed_*.npz, made by tests/golden/make_golden.py from
  qpSWIFT itself): |x - x_ref|_inf <= 1e-6 max(1, |x_ref|), same flags;
* the fused argmin over the concatenated batch equals the host argmin of the
  members' fval over optimal QPs (ties -> lowest global index), including
  members of 0 QPs and batches that are not multiples of 4.
CPU-only checks (group creation rules, hiprtc compile for gfx950) are at the end.
"""
import numpy as np
import pytest

from conftest import golden
from test_gpu_parity import _dense

GAITS = ["mixed_stance4", "mixed_trot_blfr", "mixed_trot_brfl", "mixed_crawl_blflfr"]
TOL = 1e-6


def _plans_and_vals(names, sizes=None):
    from apf_quadruped_amd.batch import Plan
    plans, vals, gs = [], [], []
    for k, name in enumerate(names):
        g = golden(name)
        n, m, p, P, A, G = _dense(g)
        B = P.shape[0] if sizes is None else sizes[k]
        idx = np.arange(B) % P.shape[0]
        plan = Plan.from_dense(n, m, p, P[0], A[0], G[0])
        plans.append(plan)
        vals.append(plan.pack(P[idx], A[idx], G[idx], g["c"][idx], g["h"][idx], g["b"][idx]))
        gs.append((g, idx))
    return plans, vals, gs


def _dev(vals):
    import torch
    return [{k: torch.from_numpy(v).cuda() for k, v in vs.items()} for vs in vals]


def _group_solve(plans, dvals, sizes, tol, best=None):
    import torch
    from apf_quadruped_amd.batch import PlanGroup
    grp = PlanGroup(plans)
    outs = [pl.alloc_outputs(max(B, 1), device="cuda") for pl, B in zip(plans, sizes)]
    grp.launcher(dvals, outs, sizes, reltol=tol, abstol=tol, best=best)()
    torch.cuda.synchronize()
    return [pl.unpack(o, B) for pl, o, B in zip(plans, outs, sizes)]


@pytest.mark.gpu
def test_group_bit_identical_to_single_plan_launches():
    sizes = [1000, 37, 1024, 513]
    plans, vals, gs = _plans_and_vals(GAITS, sizes)
    dvals = _dev(vals)
    tol = float(gs[0][0]["tol"])
    rg = _group_solve(plans, dvals, sizes, tol)
    for pl, dv, B, r in zip(plans, dvals, sizes, rg):
        out = pl.solve(**dv, B=B, reltol=tol, abstol=tol)
        r1 = pl.unpack(out, B)
        for k in ("x", "y", "z", "s", "fval", "flag", "iters", "n_rx", "n_mu"):
            np.testing.assert_array_equal(r[k], r1[k], err_msg=k)


@pytest.mark.gpu
def test_group_matches_reference_goldens():
    plans, vals, gs = _plans_and_vals(GAITS)
    sizes = [int(golden(nm)["P"].shape[0]) for nm in GAITS]
    rg = _group_solve(plans, _dev(vals), sizes, float(gs[0][0]["tol"]))
    for name, (g, _), r in zip(GAITS, gs, rg):
        np.testing.assert_array_equal(r["flag"], g["flag"], err_msg=name)
        for k in ("x", "z", "s"):
            scale = np.maximum(1.0, np.abs(g[k]).max(axis=1, keepdims=True))
            err = np.abs(r[k] - g[k]) / scale
            assert err.max() <= TOL, (name, k, err.max())


@pytest.mark.gpu
@pytest.mark.parametrize("sizes", [[1000, 37, 1024, 513], [0, 5, 0, 3], [4096, 0, 0, 0], [1, 1, 1, 1]])
def test_group_fused_argmin(sizes):
    import torch
    plans, vals, gs = _plans_and_vals(GAITS, sizes)
    best = torch.full((2,), -7.0, dtype=torch.float64, device="cuda")
    rg = _group_solve(plans, _dev(vals), sizes, 1e-6, best=best)
    fv = np.concatenate([r["fval"] for r in rg])
    ok = np.concatenate([r["flag"] for r in rg]) == 0
    assert ok.any()
    want = int(np.flatnonzero(ok)[np.argmin(fv[ok])])
    got = best.cpu().numpy()
    assert int(got[1]) == want and got[0] == fv[want]
    # the arrival counter re-arms: a second launch on the same stream gives the same result
    best2 = torch.zeros(2, dtype=torch.float64, device="cuda")
    _group_solve(plans, _dev(vals), sizes, 1e-6, best=best2)
    assert best2.cpu().numpy().tolist() == got.tolist()


@pytest.mark.gpu
def test_group_empty_batch_best_is_none():
    import torch
    plans, vals, _ = _plans_and_vals(GAITS[:2], [0, 0])
    best = torch.zeros(2, dtype=torch.float64, device="cuda")
    _group_solve(plans, _dev(vals), [0, 0], 1e-6, best=best)
    v = best.cpu().numpy()
    assert np.isinf(v[0]) and v[1] == -1


# ---- CPU-only ------------------------------------------------------------

def test_group_rules_and_compile():
    from apf_quadruped_amd import plans as SP
    from apf_quadruped_amd.batch import PlanGroup
    plans, _, _ = _plans_and_vals(GAITS, [1, 1, 1, 1])
    grp = PlanGroup(plans)
    src = grp.source()
    assert src.count("namespace qpb_g0 {") == 1 and src.count("::qpb_row_body(") == 4 and grp.kernel_name().startswith("qpb_rowgroup4_")
    grp.compile()                                          # hiprtc, gfx950, no GPU needed
    with pytest.raises(RuntimeError, match="row-form"):
        PlanGroup([plans[0], SP.standard_plan("mpc_h10")])   # not a row-form plan
    with pytest.raises(RuntimeError, match="1..16"):
        PlanGroup(plans * 5)

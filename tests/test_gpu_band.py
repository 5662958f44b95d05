"""GPU parity of the band kernel (one QP per wavefront, block-tridiagonal LDL' over
the stages of a multi-stage pattern; qpb_band.hip) through the C ABI: the MPC-horizon
QP of configs[3] (120/200/60: 10 stages of 12/20/6) against the reference's golden
vectors and the oracle, and synthetic multi-stage QPs of other block sizes against the
oracle.

Bars: vs the reference's golden vectors 1e-6 * max(1, |ref|) (north-star tolerance);
vs the oracle run with the plan's own permutation (leaves first: the band kernel's
elimination) 1e-9 relative with identical flags and iteration counts -- the same
factor in block form, a different summation order."""
import numpy as np
import pytest

from band_cases import stage_qp
from conftest import golden
from test_gpu_parity import _dense, _solve

TOL = 1e-6


def _close(got, ref, what, tol):
    scale = max(1.0, float(np.max(np.abs(ref)))) if ref.size else 1.0
    err = float(np.max(np.abs(got - ref))) if ref.size else 0.0
    assert err <= tol * scale, (what, err, scale)


@pytest.mark.gpu
def test_band_kernel_vs_reference_golden():
    g = golden("mpc_h10")
    plan, r = _solve(g, perm=None, exact=False, p_upper=True, kernel="band")
    assert plan.kernel_for(g["x"].shape[0]) == "band"
    np.testing.assert_array_equal(r["flag"], g["flag"])
    sel = g["flag"] == 0
    for k in ("x", "y", "z", "s"):
        _close(r[k][sel], g[k][sel], f"mpc_h10.{k}", TOL)


@pytest.mark.gpu
def test_band_kernel_matches_oracle_in_its_order(oracle):
    g = golden("mpc_h10")
    plan, r = _solve(g, perm=None, exact=False, p_upper=True, kernel="band")
    n, m, p = int(g["n"]), int(g["m"]), int(g["p"])
    tol = float(g["tol"])
    for q in range(g["x"].shape[0]):
        o = oracle.solve_dense(n, m, p, g["P"][q], g["A"][q], g["G"][q], g["c"][q], g["h"][q], g["b"][q],
                               perm=plan.perm, ordering=int(g["ordering"]), reltol=tol, abstol=tol,
                               maxit=int(g["maxit"]))
        assert r["flag"][q] == o["flag"] and r["iters"][q] == o["iters"], (q, r["iters"][q], o["iters"])
        for k in ("x", "y", "z", "s"):
            _close(r[k][q], o[k], f"mpc_h10[{q}].{k}", 1e-9)
        assert abs(r["fval"][q] - o["fval"]) <= 1e-9 * max(1.0, abs(o["fval"])), q


def _run(plan, d, B, **kw):
    import torch
    vals = {k: torch.from_numpy(v).cuda() for k, v in plan.pack(d["P"], d["A"] if d["p"] else None, d["G"], d["c"],
                                                                d["h"], d["b"] if d["p"] else None).items()}
    return plan.unpack(plan.solve(**vals, B=B, **kw), B)


@pytest.mark.gpu
@pytest.mark.parametrize("B", [1, 3, 64, 65, 1024])
def test_band_kernel_mpc_batch(B, oracle):
    """configs[3] on the auto-selected kernel: all optimal, KKT residuals small,
    deterministic, a strided sample vs the oracle in the plan's order."""
    from apf_quadruped_amd import plans, workloads as W
    d = W.mpc_qp(plans.SEED + 4, np.arange(B))
    plan = plans.standard_plan("mpc_h10")
    assert plan.kernel_for(B) == "band" and plan.kernel_name(B).startswith("qpb_band_")
    r1 = _run(plan, d, B)
    r2 = _run(plan, d, B)
    for k in ("x", "y", "z", "s", "fval", "iters"):
        np.testing.assert_array_equal(r1[k], r2[k])
    assert (r1["flag"] == 0).all()
    x, y, z, s = r1["x"], r1["y"], r1["z"], r1["s"]
    eq = np.einsum("bij,bj->bi", d["A"], x) - d["b"]
    ineq = np.einsum("bij,bj->bi", d["G"], x) + s - d["h"]
    stat = np.einsum("bij,bj->bi", d["P"], x) + d["c"] + np.einsum("bji,bj->bi", d["A"], y) + \
        np.einsum("bji,bj->bi", d["G"], z)
    assert np.abs(eq).max() < 1e-5 and np.abs(ineq).max() < 1e-5 and np.abs(stat).max() < 1e-5
    assert (s >= 0).all() and (z >= 0).all()
    Pc, Ac, Gc = W.to_colmajor(d["P"]), W.to_colmajor(d["A"]), W.to_colmajor(d["G"])
    for q in sorted({0, B // 2, B - 1} | set(range(0, B, 257))):
        o = oracle.solve_dense(120, 200, 60, Pc[q], Ac[q], Gc[q], d["c"][q], d["h"][q], d["b"][q], perm=plan.perm)
        assert o["flag"] == r1["flag"][q] and o["iters"] == r1["iters"][q]
        for k in ("x", "y", "z", "s"):
            _close(r1[k][q], o[k], f"mpc[{q}].{k}", 1e-9)
        assert abs(r1["fval"][q] - o["fval"]) <= 1e-9 * max(1.0, abs(o["fval"]))


@pytest.mark.gpu
def test_band_kernel_stats_match_tree():
    """The per-QP statistics (residual norms, mu, step lengths) agree with the tree
    kernel's on the same QPs (both follow the same iterates)."""
    from apf_quadruped_amd import plans
    from apf_quadruped_amd.batch import Plan
    B = 64
    d = plans.standard_qp("mpc_h10", np.arange(B))
    out = {}
    for kern in ("band", "tree"):
        plan = Plan.from_dense(d["n"], d["m"], d["p"], d["P"][0], d["A"][0], d["G"][0], kernel=kern)
        out[kern] = _run(plan, d, B)
    np.testing.assert_array_equal(out["band"]["iters"], out["tree"]["iters"])
    for k in ("n_rx", "n_ry", "n_rz", "n_mu", "alpha_p", "alpha_d"):
        a, b = out["band"][k], out["tree"][k]
        assert np.all(np.abs(a - b) <= 1e-6 * np.maximum(1.0, np.abs(b))), k


STAGE_SHAPES = [
    (12, 10, 20, 6),     # the MPC horizon's blocks, random sparsity
    (4, 6, 5, 2),        # small blocks
    (16, 3, 40, 8),      # full DPP rows, z rows across three DPP rows
    (7, 5, 64, 3),       # odd width, every lane a z row
    (9, 4, 11, 0),       # no equality rows (independent stages)
    (10, 8, 3, 10),      # as many equality rows as variables per stage
    (5, 2, 6, 2),        # two stages (the smallest horizon)
]


@pytest.mark.gpu
@pytest.mark.parametrize("shape", STAGE_SHAPES)
@pytest.mark.parametrize("p_upper", [True, False])
def test_band_kernel_stage_shapes_vs_oracle(shape, p_upper, oracle):
    from apf_quadruped_amd import workloads as W
    from apf_quadruped_amd.batch import Plan
    nb, ns, mz, my = shape
    B = 6
    d = stage_qp(nb, ns, mz, my, B=B, seed=sum(shape))
    n, m, p = d["n"], d["m"], d["p"]
    plan = Plan.from_dense(n, m, p, d["P"][0], d["A"][0] if p else None, d["G"][0], p_upper=p_upper, kernel="band")
    r = _run(plan, d, B)
    Pc, Gc = W.to_colmajor(d["P"]), W.to_colmajor(d["G"])
    Ac = W.to_colmajor(d["A"]) if p else None
    for q in range(B):
        o = oracle.solve_dense(n, m, p, Pc[q], Ac[q] if p else None, Gc[q], d["c"][q], d["h"][q],
                               d["b"][q] if p else None, perm=plan.perm)
        assert r["flag"][q] == o["flag"] and r["iters"][q] == o["iters"], (shape, q, r["iters"][q], o["iters"])
        for k in ("x", "z", "s") + (("y",) if p else ()):
            _close(r[k][q], o[k], f"{shape}[{q}].{k}", 1e-7)


@pytest.mark.gpu
def test_band_kernel_regularised_pivot_vs_oracle(oracle):
    """A variable with no cost and no constraint row gives a zero pivot: the fast
    factor pass sees |D| <= 1e-14 and the factor is redone with the reference's
    regularisation (ldl.c:273-274), as the oracle does."""
    from apf_quadruped_amd import workloads as W
    from apf_quadruped_amd.batch import Plan
    B = 4
    d = stage_qp(6, 4, 8, 2, B=B, seed=11)
    dead = 8                                           # stage 1, variable 2
    for key in ("P", "G", "A"):
        d[key][:, :, dead] = 0.0
    d["P"][:, dead, :] = 0.0
    d["c"][:, dead] = 0.0
    for r in range(d["m"]):                            # keep every G row non-empty
        if not d["G"][0, r].any():
            st = r // 8
            d["G"][:, r, 6 * st] = 1.0
    d["h"] = np.einsum("bij,bj->bi", d["G"], np.zeros((B, d["n"]))) + 1.0
    d["b"] = np.zeros((B, d["p"]))
    n, m, p = d["n"], d["m"], d["p"]
    plan = Plan.from_dense(n, m, p, d["P"][0], d["A"][0], d["G"][0], kernel="band")
    r = _run(plan, d, B)
    Pc, Ac, Gc = W.to_colmajor(d["P"]), W.to_colmajor(d["A"]), W.to_colmajor(d["G"])
    for q in range(B):
        o = oracle.solve_dense(n, m, p, Pc[q], Ac[q], Gc[q], d["c"][q], d["h"][q], d["b"][q], perm=plan.perm)
        assert r["flag"][q] == o["flag"] and r["iters"][q] == o["iters"], (q, r["iters"][q], o["iters"])
        for k in ("x", "z", "s"):
            _close(r[k][q], o[k], f"reg[{q}].{k}", 1e-7)


@pytest.mark.gpu
@pytest.mark.parametrize("tol,maxit,sigma_d", [(1e-2, 100, 0.0), (1e-6, 3, 0.0), (1e-6, 100, 0.05)])
def test_band_kernel_mpc_options_vs_oracle(tol, maxit, sigma_d, oracle):
    """The IPM's options on the band kernel: loose tolerance, maxit truncation (QP_MAXIT,
    the third iterate), and sigma_d > 0 (the pure-centering branch, qpSWIFT.c:572-579)
    -- against the oracle given the same CSC data and the plan's permutation."""
    from apf_quadruped_amd import plans
    from apf_quadruped_amd.batch import Plan, _gather_values
    B = 8
    d = plans.standard_qp("mpc_h10", np.arange(B))
    n, m, p = d["n"], d["m"], d["p"]
    plan = Plan.from_dense(n, m, p, d["P"][0], d["A"][0], d["G"][0], p_upper=False, kernel="band")
    assert plan.kernel_for(B) == "band"
    r = _run(plan, d, B, reltol=tol, abstol=tol, maxit=maxit, sigma_d=sigma_d)
    (Pjc, Pir), (Ajc, Air), (Gjc, Gir) = plan.patterns.P, plan.patterns.A, plan.patterns.G
    Pv, Av, Gv = (_gather_values(d[k], jc, ir) for k, (jc, ir) in (("P", (Pjc, Pir)), ("A", (Ajc, Air)),
                                                                  ("G", (Gjc, Gir))))
    # loosely converged / truncated iterates (an ill-conditioned KKT after 3 iterations)
    # amplify the summation-order rounding of the block form: 1e-7, still 10x inside the
    # north-star tolerance
    bar = 1e-9 if (tol < 1e-3 and maxit == 100) else 1e-7
    for q in range(B):
        o = oracle.solve_csc(n, m, p, Pjc, Pir, Pv[q], Ajc, Air, Av[q], Gjc, Gir, Gv[q], d["c"][q], d["h"][q],
                             d["b"][q], sigma_d=sigma_d, perm=plan.perm, reltol=tol, abstol=tol, maxit=maxit)
        assert r["flag"][q] == o["flag"] and r["iters"][q] == o["iters"], (q, r["flag"][q], o["flag"], r["iters"][q],
                                                                            o["iters"])
        for k in ("x", "y", "z", "s"):
            _close(r[k][q], o[k], f"opts[{q}].{k}", bar)


@pytest.mark.gpu
@pytest.mark.parametrize("horizon", [3, 16])
def test_band_kernel_mpc_horizons_vs_oracle(horizon, oracle):
    """MPC horizons other than configs[3]'s ten stages: a short one (three stages, a
    single stage-parallel round) and a long one (16 stages, 69 KB of LDS per QP: two QPs
    per CU, more than 64 KB per workgroup)."""
    from apf_quadruped_amd import plans, workloads as W
    from apf_quadruped_amd.batch import Plan
    B = 5
    d = W.mpc_qp(plans.SEED + 40 + horizon, np.arange(B), horizon=horizon)
    n, m, p = d["n"], d["m"], d["p"]
    plan = Plan.from_dense(n, m, p, d["P"][0], d["A"][0], d["G"][0], kernel="band")
    r = _run(plan, d, B)
    Pc, Ac, Gc = W.to_colmajor(d["P"]), W.to_colmajor(d["A"]), W.to_colmajor(d["G"])
    for q in range(B):
        o = oracle.solve_dense(n, m, p, Pc[q], Ac[q], Gc[q], d["c"][q], d["h"][q], d["b"][q], perm=plan.perm)
        assert r["flag"][q] == o["flag"] == 0 and r["iters"][q] == o["iters"], (horizon, q, r["iters"][q], o["iters"])
        for k in ("x", "y", "z", "s"):
            _close(r[k][q], o[k], f"h{horizon}[{q}].{k}", 1e-9)



@pytest.mark.gpu
@pytest.mark.parametrize("cut", [0, 2, 4])
def test_band_kernel_warm_solve_continues_the_cold_one(cut, oracle):
    """Warm solves of multi-stage plans run on the band kernel's QPB_WARM variant (round 6;
    the tree kernel before).  The drop-in's sequence on one QP object: QP_SETUP
    (kkt_initialize: a cold launch with maxit 0), a first QP_SOLVE stopped after `cut`
    passes, a second QP_SOLVE continuing from the object's x, y, z, s, IterationCount,
    Flag and sigma (qpSWIFT.c:502-601) -- the same passes as one uninterrupted cold solve:
    identical flags and iteration counts, iterates within 1e-12 (the two variants are
    separate compilations of the same source); the tree kernel's warm variant continuing
    from the same state agrees to 1e-9."""
    import torch
    from apf_quadruped_amd import plans, workloads as W
    from apf_quadruped_amd.batch import Plan
    B = 65
    d = W.mpc_qp(plans.SEED + 4, np.arange(B))
    plan = plans.standard_plan("mpc_h10")
    assert plan.kernel_for(B) == "band"
    vals = {k: torch.from_numpy(v).cuda() for k, v in plan.pack(d["P"], d["A"], d["G"], d["c"], d["h"], d["b"]).items()}
    full = plan.unpack(plan.solve(**vals, B=B), B)
    out = plan.solve(**vals, B=B, maxit=0)                     # QP_SETUP's initial point
    sig = torch.full((B,), 100.0, dtype=torch.float64, device="cuda")
    if cut:
        plan.solve_warm(**vals, B=B, maxit=cut, out=out, sigma=sig)
        torch.cuda.synchronize()
        first = plan.unpack(out, B)
        assert (first["iters"] == cut).all() and (first["flag"] == 2).all()
    tree = Plan(120, 200, 60, *plan.patterns.P, *plan.patterns.A, *plan.patterns.G, perm=plan.perm,
                p_upper=plan.p_upper, kernel="tree")
    tout = {k: v.clone() for k, v in out.items()}
    tsig = sig.clone()
    plan.solve_warm(**vals, B=B, maxit=100, out=out, sigma=sig)
    tree.solve_warm(**vals, B=B, maxit=100, out=tout, sigma=tsig)
    torch.cuda.synchronize()
    w, t = plan.unpack(out, B), tree.unpack(tout, B)
    np.testing.assert_array_equal(w["flag"], full["flag"])
    np.testing.assert_array_equal(w["iters"], full["iters"])
    np.testing.assert_array_equal(t["iters"], w["iters"])
    for k in ("x", "y", "z", "s"):
        _close(w[k], full[k], f"warm vs cold .{k}", 1e-12)
        for q in range(0, B, 8):
            _close(t[k][q], w[k][q], f"tree vs band warm [{q}].{k}", 1e-9)
    # and against the oracle in the plan's order (the cold path's bar)
    Pc, Ac, Gc = W.to_colmajor(d["P"]), W.to_colmajor(d["A"]), W.to_colmajor(d["G"])
    for q in (0, B - 1):
        o = oracle.solve_dense(120, 200, 60, Pc[q], Ac[q], Gc[q], d["c"][q], d["h"][q], d["b"][q], perm=plan.perm)
        assert o["iters"] == w["iters"][q] and o["flag"] == w["flag"][q]
        for k in ("x", "y", "z", "s"):
            _close(w[k][q], o[k], f"mpc warm[{q}].{k}", 1e-9)

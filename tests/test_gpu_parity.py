"""GPU parity: the generated HIP kernels against the reference's golden vectors
and the oracle, through the C ABI (qpb_solve).

* exact plans (QPB_EXACT) given the reference's own AMD permutation must be
  BIT-IDENTICAL to reference qpSWIFT (x, y, z, s, flag, iterations, fval);
* fast plans (FMA, reciprocal pivots) and plans with our own ordering must agree
  with the reference within the north-star tolerance: |x - x_ref|_inf <= 1e-6
  ("primal/dual within 1e-6 of reference qpSWIFT");
* large batches are checked through size-independent properties (KKT residuals,
  tile independence, determinism) and a strided sample against the oracle.
"""
import numpy as np
import pytest

from conftest import golden

TOL = 1e-6
DENSE_CASES = ["c1_tol1e-6", "c1_tol1e-2", "c1_rowmajor", "c1_noeq", "edge_zero_g_row",
               "mixed_stance4", "mixed_trot_blfr", "mixed_trot_brfl", "mixed_crawl_blflfr",
               "edge_infeasible"] + \
              [f"c1_maxit{k}" for k in range(7)]
# primal-infeasible QPs cut at 8 iterations: the iterates diverge, so only the exact
# kernel (same operations, same bits) is held to them; the fast kernels are checked
# on flag / iteration count (test_infeasible_runs_to_maxit)
EXACT_ONLY_CASES = ["edge_infeasible_maxit8"]


def _dense(g):
    """Golden dense inputs -> row-major [B, r, c] arrays."""
    n, m, p = int(g["n"]), int(g["m"]), int(g["p"])
    B = g["P"].shape[0]
    if int(g["ordering"]) == 20:
        P = g["P"].reshape(B, n, n); G = g["G"].reshape(B, m, n)
        A = g["A"].reshape(B, p, n) if p else None
    else:
        P = g["P"].reshape(B, n, n).transpose(0, 2, 1); G = g["G"].reshape(B, n, m).transpose(0, 2, 1)
        A = g["A"].reshape(B, n, p).transpose(0, 2, 1) if p else None
    return n, m, p, P, A, G


def _solve(g, perm, exact, p_upper=False, kernel="lane"):
    from apf_quadruped_amd.batch import Plan
    n, m, p, P, A, G = _dense(g)
    B = P.shape[0]
    plan = Plan.from_dense(n, m, p, P[0], A[0] if p else None, G[0], perm=perm, p_upper=p_upper, exact=exact,
                           kernel=kernel)
    vals = plan.pack(P, A, G, g["c"], g["h"], g["b"] if p else None)
    tol = float(g["tol"])
    out = plan.solve(**vals, B=B, reltol=tol, abstol=tol, maxit=int(g["maxit"]))
    return plan, plan.unpack(out, B)


@pytest.mark.gpu
@pytest.mark.parametrize("name", DENSE_CASES + EXACT_ONLY_CASES)
def test_exact_kernel_bit_identical_to_reference(name):
    g = golden(name)
    _, r = _solve(g, perm=g["perm"][0], exact=True, p_upper=False)
    for k in ("x", "z", "s") + (("y",) if int(g["p"]) else ()):
        np.testing.assert_array_equal(r[k], g[k], err_msg=f"{name}.{k}")
    np.testing.assert_array_equal(r["flag"], g["flag"])
    np.testing.assert_array_equal(r["iters"], g["iters"])
    if int(g["maxit"]) > 0:
        np.testing.assert_array_equal(r["fval"], g["fval"])
        np.testing.assert_array_equal(r["n_rx"], g["n_rx"])
        np.testing.assert_array_equal(r["n_mu"], g["n_mu"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", DENSE_CASES)
@pytest.mark.parametrize("exact,own_order,kernel", [(False, False, "lane"), (False, True, "lane"),
                                                    (True, True, "lane"), (False, True, "wave"),
                                                    (False, False, "wave"), (False, True, "wave1"),
                                                    (False, False, "wave1")])
def test_kernel_within_tolerance_of_reference(name, exact, own_order, kernel):
    """Fast kernel and/or own ordering vs the reference: |.|_inf <= 1e-6 * max(1, |ref|).
    The wave kernel always eliminates in its own order [z | y | x].

    With another KKT ordering the dynamic regularisation (ldl.c:319-320) lands on
    other pivots; where A has a row-rank defect (2-foot trot: rank 5) the dual y
    is then only unique modulo null(A^T), so y is compared through A^T y there.
    Truncated iterates (maxit < 100) are compared only under the reference order."""
    g = golden(name)
    truncated = int(g["maxit"]) < 100
    if own_order and (name == "edge_zero_g_row" or truncated):
        pytest.skip("depends on the reference's own KKT order")
    if kernel.startswith("wave") and name == "edge_zero_g_row":
        pytest.skip("the wave kernel needs every G row non-empty")
    _, r = _solve(g, perm=None if own_order else g["perm"][0], exact=exact, p_upper=True, kernel=kernel)
    n, m, p, P, A, G = _dense(g)
    sel = slice(None) if truncated else (g["flag"] == 0)
    if not truncated:
        np.testing.assert_array_equal(r["flag"], g["flag"])

    def close(got, ref, what, tol=TOL):
        scale = max(1.0, float(np.max(np.abs(ref)))) if ref.size else 1.0
        err = float(np.max(np.abs(got - ref))) if ref.size else 0.0
        assert err <= tol * scale, (name, what, err)

    tol = 10 * TOL if truncated else TOL
    for k in ("x", "z", "s"):
        close(r[k][sel], g[k][sel], k, tol)
    if p:
        rank = np.linalg.matrix_rank(A[0])
        if rank == p or not own_order:
            close(r["y"][sel], g["y"][sel], "y", tol)
        else:
            close(np.einsum("bji,bj->bi", A[sel], r["y"][sel]), np.einsum("bji,bj->bi", A[sel], g["y"][sel]),
                  "A^T y", tol)


@pytest.mark.gpu
def test_exact_kernel_matches_oracle_with_own_ordering(oracle):
    """Own min-degree ordering: GPU exact == oracle (same ordering) bit for bit."""
    g = golden("c1_tol1e-6")
    plan, r = _solve(g, perm=None, exact=True)
    n, m, p, P, A, G = _dense(g)
    for q in range(0, P.shape[0], 5):
        o = oracle.solve_dense(n, m, p, g["P"][q], g["A"][q], g["G"][q], g["c"][q], g["h"][q], g["b"][q],
                               perm=plan.perm)
        for k in ("x", "y", "z", "s"):
            np.testing.assert_array_equal(r[k][q], o[k])
        assert r["iters"][q] == o["iters"] and r["fval"][q] == o["fval"]


@pytest.mark.gpu
@pytest.mark.parametrize("name,ref_perm", [("c30_tol1e-6", False), ("c30_tol1e-6", True), ("c30_tol1e-2", True),
                                           ("c30_trot_tol1e-6", False), ("c30_trot_tol1e-6", True),
                                           ("c30_trot_tol1e-2", True), ("c30_crawl_tol1e-6", False),
                                           ("c30_crawl_tol1e-6", True), ("c30_crawl_tol1e-2", True)])
def test_wave_kernel_controller_shape_vs_reference(name, ref_perm):
    """Controller-shape QPs (stance 30/68/18, trot 30/70/12, crawl 30/69/15; N = 116: two z rows per lane, dense block
    of 48-51 rows over several 16-lane rows) on the wave kernel vs the reference
    golden vectors.  Given the reference's permutation the wave kernel factors
    with the reference's pivots (and regularisations), so even the loosely
    converged tol-1e-2 solutions agree to 1e-6."""
    g = golden(name)
    _, r = _solve(g, perm=g["perm"][0] if ref_perm else None, exact=False, p_upper=True, kernel="wave")
    np.testing.assert_array_equal(r["flag"], g["flag"])
    for k in ("x", "y", "z", "s"):
        scale = max(1.0, float(np.abs(g[k]).max()))
        err = float(np.abs(r[k] - g[k]).max())
        assert err <= TOL * scale, (name, k, err, scale)


def _oracle_perm(plan):
    return plan.perm if plan.kernel == "wave" else plan.perm


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["c1_tol1e-6", "c1_tol1e-2", "c1_noeq", "mixed_stance4", "mixed_trot_blfr",
                                  "mixed_trot_brfl", "mixed_crawl_blflfr", "c1_maxit3", "c30_tol1e-6", "c30_tol1e-2",
                                  "c30_trot_tol1e-6", "c30_trot_tol1e-2", "c30_crawl_tol1e-6", "c30_crawl_tol1e-2"])
@pytest.mark.parametrize("kernel", ["wave", "wave1"])
def test_wave_kernel_matches_oracle_in_its_order(name, kernel, oracle):
    """Wave kernel (row form where the pattern fits, and one QP per wavefront) vs
    the oracle run with the kernel's elimination order: same factorisation, so
    agreement is at rounding level (1e-9 relative)."""
    g = golden(name)
    plan, r = _solve(g, perm=None, exact=False, p_upper=True, kernel=kernel)
    n, m, p = int(g["n"]), int(g["m"]), int(g["p"])
    tol = float(g["tol"])
    for q in range(0, g["x"].shape[0], 3):
        o = oracle.solve_dense(n, m, p, g["P"][q], g["A"][q] if p else None, g["G"][q], g["c"][q], g["h"][q],
                               g["b"][q] if p else None, perm=plan.perm, ordering=int(g["ordering"]),
                               reltol=tol, abstol=tol, maxit=int(g["maxit"]))
        assert r["flag"][q] == o["flag"] and r["iters"][q] == o["iters"], (name, q)
        got, ref = {k: r[k][q] for k in ("x", "z", "s")}, {k: o[k] for k in ("x", "z", "s")}
        if p:
            # y is unique only modulo null(A^T) when A is rank deficient (2-foot trot)
            Aq = _dense(g)[4][q]
            if np.linalg.matrix_rank(Aq) < p:
                got["Aty"], ref["Aty"] = Aq.T @ r["y"][q], Aq.T @ o["y"]
            else:
                got["y"], ref["y"] = r["y"][q], o["y"]
        for k in got:
            scale = max(1.0, float(np.abs(ref[k]).max()))
            assert np.abs(got[k] - ref[k]).max() <= 1e-9 * scale, (name, q, k)


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", ["lane", "wave", "wave1", "tree"])
@pytest.mark.parametrize("B", [1, 2, 3, 5, 63, 65, 1000])
def test_ragged_batches(B, kernel, oracle):
    from apf_quadruped_amd import workloads as W
    from apf_quadruped_amd.batch import Plan
    d = W.contact_force_qp(0xD06B07 + 11, np.arange(B))
    plan = Plan.from_dense(12, 20, 6, d["P"][0], d["A"][0], d["G"][0], kernel=kernel)
    out = plan.solve(**plan.pack(d["P"], d["A"], d["G"], d["c"], d["h"], d["b"]), B=B)
    r = plan.unpack(out, B)
    Pc, Ac, Gc = W.to_colmajor(d["P"]), W.to_colmajor(d["A"]), W.to_colmajor(d["G"])
    for q in sorted({0, B // 2, B - 1}):
        o = oracle.solve_dense(12, 20, 6, Pc[q], Ac[q], Gc[q], d["c"][q], d["h"][q], d["b"][q],
                               perm=_oracle_perm(plan))
        assert np.max(np.abs(o["x"] - r["x"][q])) <= TOL * max(1, np.max(np.abs(o["x"])))


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", ["lane", "wave", "wave1"])
def test_large_batch_properties(kernel, oracle):
    """B = 65536 (config 5's global batch on one GPU): all optimal, KKT residuals
    small, deterministic, each QP independent of its neighbours."""
    import torch
    from apf_quadruped_amd import workloads as W
    from apf_quadruped_amd.batch import Plan
    B = 65536
    d = W.contact_force_qp(0xD06B07 + 5, np.arange(B))
    plan = Plan.from_dense(12, 20, 6, d["P"][0], d["A"][0], d["G"][0], kernel=kernel)
    vals = plan.pack(d["P"], d["A"], d["G"], d["c"], d["h"], d["b"])
    vals = {k: torch.from_numpy(v).cuda() for k, v in vals.items()}
    r1 = plan.unpack(plan.solve(**vals, B=B), B)
    r2 = plan.unpack(plan.solve(**vals, B=B), B)
    for k in ("x", "y", "z", "s", "fval", "iters"):
        np.testing.assert_array_equal(r1[k], r2[k])         # deterministic
    assert (r1["flag"] == 0).all()
    x, y, z, s = r1["x"], r1["y"], r1["z"], r1["s"]
    eq = np.einsum("bij,bj->bi", d["A"], x) - d["b"]
    ineq = np.einsum("bij,bj->bi", d["G"], x) + s - d["h"]
    stat = np.einsum("bij,bj->bi", d["P"], x) + d["c"] + np.einsum("bji,bj->bi", d["A"], y) + \
        np.einsum("bji,bj->bi", d["G"], z)
    assert np.abs(eq).max() < 1e-5 and np.abs(ineq).max() < 1e-5 and np.abs(stat).max() < 1e-5
    assert (s >= 0).all() and (z >= 0).all() and (s * z).sum(1).max() / 20 < 1e-5
    # shuffled batch: same per-QP answers (tile independence)
    perm = np.random.default_rng(1).permutation(B)
    sh = {k: d[k][perm] for k in ("P", "A", "G", "c", "h", "b")}
    r3 = plan.unpack(plan.solve(**plan.pack(sh["P"], sh["A"], sh["G"], sh["c"], sh["h"], sh["b"]), B=B), B)
    np.testing.assert_array_equal(r3["x"], r1["x"][perm])
    Pc, Ac, Gc = W.to_colmajor(d["P"]), W.to_colmajor(d["A"]), W.to_colmajor(d["G"])
    for q in range(0, B, 4099):
        o = oracle.solve_dense(12, 20, 6, Pc[q], Ac[q], Gc[q], d["c"][q], d["h"][q], d["b"][q],
                               perm=_oracle_perm(plan))
        assert np.max(np.abs(o["x"] - r1["x"][q])) <= TOL * max(1, np.max(np.abs(o["x"])))


@pytest.mark.gpu
def test_row_two_wave_kernel_bit_identical(monkeypatch):
    """Large batches launch the row kernel allocated for two waves per SIMD
    (qpb_plan_kernel_name names it); same source and arithmetic as the one-wave
    kernel, so its results are bit-identical to it."""
    import torch
    from apf_quadruped_amd import workloads as W
    from apf_quadruped_amd.batch import Plan
    B = 8192 + 37
    d = W.contact_force_qp(0xD06B07 + 7, np.arange(B))
    plans = {}
    for occ in ("4096", "-1"):
        monkeypatch.setenv("QPB_ROW_OCC_BATCH", occ)
        plans[occ] = Plan.from_dense(12, 20, 6, d["P"][0], d["A"][0], d["G"][0], kernel="wave")
    assert plans["4096"].kernel_name(B) != plans["-1"].kernel_name(B)
    assert plans["4096"].kernel_name(1024) == plans["-1"].kernel_name(B)
    vals = {k: torch.from_numpy(v).cuda() for k, v in plans["-1"].pack(d["P"], d["A"], d["G"], d["c"], d["h"], d["b"]).items()}
    r2 = plans["4096"].unpack(plans["4096"].solve(**vals, B=B), B)
    r1 = plans["-1"].unpack(plans["-1"].solve(**vals, B=B), B)
    for k in ("x", "y", "z", "s", "fval", "iters", "flag"):
        np.testing.assert_array_equal(r1[k], r2[k])
    assert (r1["flag"] == 0).all()


@pytest.mark.gpu
def test_argmin_device_reduction():
    import torch
    from apf_quadruped_amd.batch import argmin
    fv = torch.tensor([3.0, -1.0, -1.0, -5.0, 2.0], dtype=torch.float64, device="cuda")
    fl = torch.tensor([0, 0, 0, 2, 0], dtype=torch.int32, device="cuda")
    r = argmin(fv, fl).cpu().numpy()
    assert r[0] == -1.0 and r[1] == 1.0            # flag 2 excluded, tie -> lowest index
    big = torch.randn(100003, dtype=torch.float64, device="cuda")
    flg = torch.zeros(100003, dtype=torch.int32, device="cuda")
    r = argmin(big, flg).cpu().numpy()
    assert r[1] == float(torch.argmin(big).item())


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", ["lane", "wave", "wave1", "tree"])
def test_solve_best_fused_argmin(kernel):
    """qpb_solve_best == qpb_solve + qpb_argmin, repeatedly, for ragged batch sizes
    (1 and 1024 take the single-block argmin, 3000 too; 100003 the two-stage one)."""
    import torch
    from apf_quadruped_amd import workloads as W
    from apf_quadruped_amd.batch import Plan, argmin
    for B in (1, 100, 1024, 3000):
        d = W.contact_force_qp(0xD06B07 + 13, np.arange(B))
        plan = Plan.from_dense(12, 20, 6, d["P"][0], d["A"][0], d["G"][0], kernel=kernel)
        vals = {k: torch.from_numpy(v).cuda() for k, v in plan.pack(d["P"], d["A"], d["G"], d["c"], d["h"],
                                                                    d["b"]).items()}
        out = plan.alloc_outputs(B)
        best = torch.zeros(4, dtype=torch.float64, device="cuda")
        go = plan.launcher(vals, out, B, best=best)
        for _ in range(3):
            best[:2] = -7.0
            go()
            torch.cuda.synchronize()
            ref = argmin(out["fval"], out["flag"]).cpu().numpy()
            got = best.cpu().numpy()
            assert got[0] == ref[0] and got[1] == ref[1], (kernel, B, got, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("B", [1, 5, 257, 1024])
def test_controller_shape_batch_auto_dispatch(B, oracle):
    """Controller stance QPs (30/68/18) as the bench runs them: auto dispatch (the
    wide row kernel, four QPs per wavefront, at every batch size),
    ragged and full batches; a strided sample vs the oracle run with the plan's
    order: same flags and iteration counts, x / z / s within 1e-9 relative;
    deterministic across launches."""
    import torch
    from apf_quadruped_amd import plans, workloads as W
    from apf_quadruped_amd.batch import Plan
    d = W.controller_qp(plans.SEED + 30, np.arange(B))
    plan = Plan.from_dense(30, 68, 18, d["P"][0], d["A"][0], d["G"][0])
    assert plan.kernel_for(B) == "wave"
    vals = {k: torch.from_numpy(v).cuda() for k, v in plan.pack(d["P"], d["A"], d["G"], d["c"], d["h"],
                                                                d["b"]).items()}
    r1 = plan.unpack(plan.solve(**vals, B=B), B)
    r2 = plan.unpack(plan.solve(**vals, B=B), B)
    for k in ("x", "z", "s", "iters"):
        np.testing.assert_array_equal(r1[k], r2[k])
    Pc, Ac, Gc = W.to_colmajor(d["P"]), W.to_colmajor(d["A"]), W.to_colmajor(d["G"])
    for q in sorted(set(range(0, B, max(1, B // 12))) | {B - 1}):
        o = oracle.solve_dense(30, 68, 18, Pc[q], Ac[q], Gc[q], d["c"][q], d["h"][q], d["b"][q], perm=plan.perm)
        assert r1["flag"][q] == o["flag"] and r1["iters"][q] == o["iters"], q
        for k in ("x", "z", "s"):
            assert np.abs(r1[k][q] - o[k]).max() <= 1e-9 * max(1.0, np.abs(o[k]).max()), (q, k)


@pytest.mark.gpu
@pytest.mark.parametrize("B", [1, 1000, 4096])
def test_winner_payload(B):
    """qpb_winner: the multi-GPU gather's payload {fval, index, x*[n]} built on the
    device after qpb_solve_best equals the host argmin and that QP's x; an index
    of -1 yields NaN for x*."""
    import torch
    from apf_quadruped_amd import workloads as W
    from apf_quadruped_amd.batch import Plan
    from apf_quadruped_amd.shard import winner_payload
    d = W.contact_force_qp(0xD06B07 + 21, np.arange(B))
    plan = Plan.from_dense(12, 20, 6, d["P"][0], d["A"][0], d["G"][0])
    vals = {k: torch.from_numpy(v).cuda() for k, v in plan.pack(d["P"], d["A"], d["G"], d["c"], d["h"],
                                                                d["b"]).items()}
    out = plan.alloc_outputs(B, device="cuda")
    best = torch.zeros(2, dtype=torch.float64, device="cuda")
    plan.launcher(vals, out, B, best=best)()
    pay = winner_payload(best, out["x"], 12, B)
    torch.cuda.synchronize()
    r = plan.unpack(out, B)
    ok = r["flag"] == 0
    want = int(np.flatnonzero(ok)[np.argmin(r["fval"][ok])])
    p = pay.cpu().numpy()
    assert int(p[1]) == want and p[0] == r["fval"][want]
    np.testing.assert_array_equal(p[2:], r["x"][want])
    none = torch.tensor([np.inf, -1.0], dtype=torch.float64, device="cuda")
    p2 = winner_payload(none, out["x"], 12, B).cpu().numpy()
    assert p2[1] == -1 and np.isnan(p2[2:]).all()


@pytest.mark.gpu
def test_wave_two_rows_per_lane_factor_bit_identical(monkeypatch):
    """The 17-32-row dense blocks (leaves-first controller QPs: 30 rows) are
    factored with two rows per lane (QPB_W_DUP, DPP broadcasts); it performs the
    one-row-per-lane factor's operations in the same order, so every output is
    bit-identical to the QPB_W_DUP=0 build."""
    import torch
    from apf_quadruped_amd import workloads as W
    from apf_quadruped_amd.batch import Plan
    B = 256
    d = W.controller_qp(0xD06B07 + 33, np.arange(B))
    res = {}
    for opt in ("", "QPB_W_DUP=0"):
        monkeypatch.setenv("QPB_WAVE_OPTS", opt)
        plan = Plan.from_dense(30, 68, 18, d["P"][0], d["A"][0], d["G"][0], kernel="wave1")
        assert "#define QPB_ND 30" in plan.wave_source()
        vals = {k: torch.from_numpy(v).cuda() for k, v in plan.pack(d["P"], d["A"], d["G"], d["c"], d["h"], d["b"]).items()}
        res[opt] = plan.unpack(plan.solve(**vals, B=B), B)
    for k in ("x", "y", "z", "s", "fval", "iters", "flag"):
        np.testing.assert_array_equal(res[""][k], res["QPB_W_DUP=0"][k])
    assert (res[""]["flag"] == 0).all()


@pytest.mark.gpu
@pytest.mark.parametrize("order", ["amd", "own"])
def test_wave_structure_knobs_match_plain_build(monkeypatch, order):
    """Round 4's wave-kernel changes -- the LDL' skipping structurally zero H(j,k)
    (QPB_W_LSKIP), the branch-free H0 (QPB_W_H0BF), the unmasked descending -L transpose
    (QPB_W_TRUNM) and the backward solve's zero slot (QPB_W_LTZS) -- against the build
    with all four off, on controller QPs in the drop-in's AMD order (51 dense rows) and
    leaves first (30): the same flags and iteration counts, iterates within 1e-9
    (the skipped terms are exact zeros; H0BF rounds the 1e7 A'A terms differently)."""
    import torch
    from apf_quadruped_amd import workloads as W
    from apf_quadruped_amd.batch import Plan
    B = 256
    d = W.controller_qp(0xD06B07 + 34, np.arange(B))
    plain = "QPB_W_LSKIP=0 QPB_W_H0BF=0 QPB_W_TRUNM=0 QPB_W_LTZS=0"
    res = {}
    for opt in ("", plain):
        monkeypatch.setenv("QPB_WAVE_OPTS", opt)
        plan = Plan.from_dense(30, 68, 18, d["P"][0], d["A"][0], d["G"][0], kernel="wave1", order=order)
        vals = {k: torch.from_numpy(v).cuda() for k, v in plan.pack(d["P"], d["A"], d["G"], d["c"], d["h"], d["b"]).items()}
        res[opt] = plan.unpack(plan.solve(**vals, B=B), B)
    np.testing.assert_array_equal(res[""]["flag"], res[plain]["flag"])
    np.testing.assert_array_equal(res[""]["iters"], res[plain]["iters"])
    for k in ("x", "y", "z", "s"):
        a, b = res[""][k], res[plain][k]
        assert np.abs(a - b).max() <= 1e-9 * max(1.0, np.abs(b).max()), (order, k)
    assert (res[""]["flag"] == 0).all()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["edge_infeasible", "edge_infeasible_maxit8"])
@pytest.mark.parametrize("own_order,kernel", [(False, "lane"), (True, "lane"), (False, "wave"), (True, "wave"),
                                              (True, "wave1"), (False, "tree"), (True, "tree")])
def test_infeasible_runs_to_maxit(name, own_order, kernel):
    """Primal-infeasible contact-force QPs (a 3 kN lateral force against ~100 N of
    friction): qpSWIFT stops at maxit with QP_MAXIT (golden flags / iterations);
    every fast kernel, in either KKT order, must report the same flag and iteration
    count and keep its iterates finite."""
    g = golden(name)
    _, r = _solve(g, perm=None if own_order else g["perm"][0], exact=False, p_upper=True, kernel=kernel)
    np.testing.assert_array_equal(r["flag"], g["flag"])
    np.testing.assert_array_equal(r["iters"], g["iters"])
    for k in ("x", "y", "z", "s"):
        assert np.isfinite(r[k]).all(), (name, kernel, k)



@pytest.mark.gpu
def test_row_kernel_zero_pivot_refactor_matches_oracle(oracle, monkeypatch):
    """The one-wave row kernel checks the pivot regularisation once per factor
    (QPB_R_LAZYREG) and redoes the factor with the regularised reciprocals
    (ldl.c:318-319) only when some pivot is <= 1e-14.  Force that path: variable 0 of
    the contact QPs decoupled (its P row / column, G and A columns and c entry zeroed),
    so its pivot is exactly 0 in every factor; the kernel vs the oracle in the plan's
    order, flags and iterations equal, x / y / z / s within 1e-9, and the two-wave
    kernel (which regularises every pivot inline) bit-identical."""
    from apf_quadruped_amd import workloads as W
    from apf_quadruped_amd.batch import Plan
    B = 200
    d = {k: np.array(v, copy=True) if isinstance(v, np.ndarray) else v
         for k, v in W.contact_force_qp(0xD06B07 + 23, np.arange(B)).items()}
    d["P"][:, 0, :] = 0.0
    d["P"][:, :, 0] = 0.0
    d["G"][:, :, 0] = 0.0
    d["A"][:, :, 0] = 0.0
    d["c"][:, 0] = 0.0
    plan = Plan.from_dense(12, 20, 6, d["P"][0], d["A"][0], d["G"][0], kernel="wave")
    assert plan.kernel_name(B).startswith("qpb_row")
    r = plan.unpack(plan.solve(**plan.pack(d["P"], d["A"], d["G"], d["c"], d["h"], d["b"]), B=B), B)
    Pc, Ac, Gc = W.to_colmajor(d["P"]), W.to_colmajor(d["A"]), W.to_colmajor(d["G"])
    for q in (0, 1, B // 2, B - 1):
        o = oracle.solve_dense(12, 20, 6, Pc[q], Ac[q], Gc[q], d["c"][q], d["h"][q], d["b"][q], perm=plan.perm)
        assert r["flag"][q] == o["flag"] and r["iters"][q] == o["iters"], q
        for k in ("x", "y", "z", "s"):
            scale = max(1.0, float(np.abs(o[k]).max()))
            assert np.abs(r[k][q] - o[k]).max() <= 1e-9 * scale, (q, k)
        assert r["x"][q][0] == 0.0
    monkeypatch.setenv("QPB_ROW_OCC_BATCH", "100")       # B = 200 on the two-wave kernel
    plan2 = Plan.from_dense(12, 20, 6, d["P"][0], d["A"][0], d["G"][0], kernel="wave")
    assert plan2.kernel_name(B) != plan.kernel_name(B)
    r2 = plan2.unpack(plan2.solve(**plan2.pack(d["P"], d["A"], d["G"], d["c"], d["h"], d["b"]), B=B), B)
    for k in ("x", "y", "z", "s", "fval", "iters", "flag"):
        np.testing.assert_array_equal(r[k], r2[k])

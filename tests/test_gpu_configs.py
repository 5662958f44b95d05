"""One GPU parity test per BASELINE.json config, collected FIRST (tests/conftest.py
moves this module to the front), so a driver run of `pytest -m gpu` verifies every
config before anything else.  Everything goes through the C ABI; the checkers are
the reference's golden vectors (tests/golden/, made from qpSWIFT itself by
tests/golden/make_golden.py) and the oracle (oracle/qpswift_oracle.c, bit-exact to
the reference on every golden, tests/test_oracle.py).

Bars: vs the reference |v - v_ref|_inf <= 1e-6 max(1, |v_ref|_inf) (north-star
tolerance), vs the oracle run with the kernel's own elimination order 1e-9 relative
with identical flags and iteration counts (same factorisation, FMA rounding only).

  configs[0]  single tick through the drop-in: QP_SETUP_dense(..., Permut = NULL,
              COLUMN_MAJOR_ORDERING) -> reltol/abstol override -> QP_SOLVE
              (main.cpp:1649-1656), C1 and the controller's C30 shapes
  configs[1]  1 024 C1 QPs on the headline row kernel with the fused argmin
              (qpb_solve_best, exactly the bench's step)
  configs[2]  4 x 1 024 QPs over the four gait patterns as ONE group launch
  configs[3]  MPC horizon (120/200/60, N = 380), 1 024 QPs, the 192-thread tree form
  configs[4]  65 536 QPs: 8 shards of 8 192 solved on one GPU, each reduced on the
              device, the 8 payloads reduced as the RCCL gather delivers them, and
              the whole qpb_argmin_allgather on a one-rank communicator
"""
import numpy as np
import pytest

from conftest import golden
from test_gpu_parity import _dense

TOL = 1e-6


def _rel(got, ref):
    ref = np.asarray(ref)
    return float(np.max(np.abs(np.asarray(got) - ref))) / max(1.0, float(np.max(np.abs(ref)))) if ref.size else 0.0


def _dense_args(g, q):
    n, m, p = int(g["n"]), int(g["m"]), int(g["p"])
    return (n, m, p, g["P"][q], g["A"][q] if p else None, g["G"][q], g["c"][q], g["h"][q], g["b"][q] if p else None)


def _fval(d, x):
    return 0.5 * np.einsum("bi,bij,bj->b", x, d["P"], x) + np.einsum("bi,bi->b", d["c"], x)


def _oracle_batch(oracle, d, perm, tol=1e-6, threads=8):
    from apf_quadruped_amd import workloads as W
    n, m, p = int(d["n"]), int(d["m"]), int(d["p"])
    return oracle.solve_dense_batch(n, m, p, W.to_colmajor(d["P"]), W.to_colmajor(d["A"]), W.to_colmajor(d["G"]),
                                    d["c"], d["h"], d["b"], perm=perm, reltol=tol, abstol=tol, threads=threads)


# ------------------------------------------------------------------ configs[0]


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["c1_tol1e-6", "c1_tol1e-2", "c30_tol1e-2", "c30_trot_tol1e-2",
                                  "c30_crawl_tol1e-2"])
def test_config0_dropin_single_tick(name):
    """configs[0]: one controller tick through the drop-in, the call the controller
    makes (Permut = NULL -> the AMD restatement, fast kernels), vs the reference's
    golden vectors: same flag and iteration count, x/y/z/s within 1e-6."""
    from apf_quadruped_amd import dropin
    g = golden(name)
    tol, maxit = float(g["tol"]), int(g["maxit"])
    for q in range(0, g["x"].shape[0], 2):
        r = dropin.solve_dense(*_dense_args(g, q), ordering=int(g["ordering"]), reltol=tol, abstol=tol, maxit=maxit)
        assert r["flag"] == int(g["flag"][q]), (name, q, r["error"])
        assert r["iters"] == int(g["iters"][q]), (name, q)
        assert r["amd_result"] == 0
        for k in ("x", "z", "s") + (("y",) if int(g["p"]) else ()):
            assert _rel(r[k], g[k][q]) <= TOL, (name, q, k, _rel(r[k], g[k][q]))


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["c1_tol1e-6", "c1_tol1e-2", "mixed_crawl_blflfr"])
def test_config0_dropin_exact_bit_identical(name, monkeypatch):
    """configs[0] with QPSWIFT_HIP_EXACT=1: bit-identical to the reference."""
    from apf_quadruped_amd import dropin
    monkeypatch.setenv("QPSWIFT_HIP_EXACT", "1")
    g = golden(name)
    tol, maxit = float(g["tol"]), int(g["maxit"])
    for q in range(0, g["x"].shape[0], 5):
        r = dropin.solve_dense(*_dense_args(g, q), ordering=int(g["ordering"]), reltol=tol, abstol=tol, maxit=maxit)
        assert r["flag"] == int(g["flag"][q]) and r["iters"] == int(g["iters"][q]), (name, q)
        for k in ("x", "y", "z", "s"):
            np.testing.assert_array_equal(r[k], g[k][q], err_msg=f"{name}[{q}].{k}")
        assert r["fval"] == float(g["fval"][q])


# ------------------------------------------------------------------ configs[1]


@pytest.mark.gpu
def test_config1_headline_batch_row_kernel(oracle):
    """configs[1]: the bench's step -- 1 024 C1 QPs (bench.make_shard, resident on
    the device) through qpb_solve_best on the row kernel -- every QP vs the oracle in
    the plan's order, the fused argmin vs the oracle's argmin, and the reference's
    C1 golden vectors through the same plan."""
    import torch
    from apf_quadruped_amd import plans, workloads as W
    from apf_quadruped_amd.batch import Plan
    B = 1024
    plan = plans.standard_plan("c1")
    assert plan.kernel_name(B).startswith("qpb_row_"), plan.kernel_name(B)
    d = W.contact_force_qp(plans.SEED + 1, np.arange(B))
    vals = {k: torch.from_numpy(v).cuda() for k, v in plan.pack(d["P"], d["A"], d["G"], d["c"], d["h"],
                                                                d["b"]).items()}
    out = plan.alloc_outputs(B)
    best = torch.zeros(2, dtype=torch.float64, device="cuda")
    go = plan.launcher(vals, out, B, best=best)
    go()
    torch.cuda.synchronize()
    r = plan.unpack(out, B)
    x_o, fl_o, it_o = _oracle_batch(oracle, d, plan.perm)
    np.testing.assert_array_equal(r["flag"], fl_o)
    np.testing.assert_array_equal(r["iters"], it_o)
    err = np.abs(r["x"] - x_o).max(1) / np.maximum(1.0, np.abs(x_o).max(1))
    assert err.max() <= 1e-9, err.max()
    # fused argmin: the GPU's winner is the oracle's winner (or ties it to rounding)
    fv_o = _fval(d, x_o)
    ok = fl_o == 0
    i_o = int(np.flatnonzero(ok)[np.argmin(fv_o[ok])])
    bv, bi = best.cpu().numpy()
    assert bv == r["fval"][int(bi)] and r["flag"][int(bi)] == 0
    assert int(bi) == i_o or abs(fv_o[int(bi)] - fv_o[i_o]) <= 1e-9 * max(1.0, abs(fv_o[i_o])), (bi, i_o)
    # repeated launches: same answer (the arrival counter re-arms)
    best2 = best.clone()
    go()
    torch.cuda.synchronize()
    assert best.cpu().numpy().tolist() == best2.cpu().numpy().tolist()
    # the reference's C1 goldens (tol 1e-6 and 1e-2) on the same plan
    for name in ("c1_tol1e-6", "c1_tol1e-2"):
        g = golden(name)
        tol = float(g["tol"])
        _, _, _, Pg, Ag, Gg = _dense(g)
        Bg = Pg.shape[0]
        gp = Plan.from_dense(12, 20, 6, Pg[0], Ag[0], Gg[0])
        assert gp.kernel_name(Bg).startswith("qpb_row_")
        rg = gp.unpack(gp.solve(**gp.pack(Pg, Ag, Gg, g["c"], g["h"], g["b"]), B=Bg, reltol=tol, abstol=tol), Bg)
        np.testing.assert_array_equal(rg["flag"], g["flag"])
        for k in ("x", "y", "z", "s"):
            assert _rel(rg[k], g[k]) <= TOL, (name, k, _rel(rg[k], g[k]))


# ------------------------------------------------------------------ configs[2]


@pytest.mark.gpu
def test_config2_four_gait_patterns_group_launch(oracle):
    """configs[2]: 4 096 QPs over the four gait contact patterns (stance4, trot
    BL+FR, trot BR+FL, crawl BL+FL+FR), bucketed into one plan each and solved as
    ONE group launch with the argmin over all 4 096 -- every QP vs the oracle in its
    plan's order, the group argmin vs the host argmin of the group's outputs."""
    import torch
    from apf_quadruped_amd import plans, workloads as W
    from apf_quadruped_amd.batch import Plan, PlanGroup
    per = 1024
    ps, dvals, outs, ds = [], [], [], []
    for k, name in enumerate(("stance4", "trot_blfr", "trot_brfl", "crawl_blflfr")):
        d = W.contact_force_qp(plans.SEED + 3, np.arange(k * per, (k + 1) * per), stance=W.STANCE_SETS[name],
                               feasible_wrench=True)
        pl = Plan.from_dense(12, d["m"], 6, d["P"][0], d["A"][0], d["G"][0])
        ps.append(pl)
        ds.append(d)
        dvals.append({kk: torch.from_numpy(v).cuda() for kk, v in pl.pack(d["P"], d["A"], d["G"], d["c"], d["h"],
                                                                        d["b"]).items()})
        outs.append(pl.alloc_outputs(per))
    grp = PlanGroup(ps)
    best = torch.zeros(2, dtype=torch.float64, device="cuda")
    grp.launcher(dvals, outs, [per] * 4, best=best)()
    torch.cuda.synchronize()
    fvs, fls = [], []
    for pl, d, o in zip(ps, ds, outs):
        r = pl.unpack(o, per)
        x_o, fl_o, it_o = _oracle_batch(oracle, d, pl.perm)
        np.testing.assert_array_equal(r["flag"], fl_o)
        np.testing.assert_array_equal(r["iters"], it_o)
        opt = fl_o == 0
        err = np.abs(r["x"][opt] - x_o[opt]).max(1) / np.maximum(1.0, np.abs(x_o[opt]).max(1))
        assert err.max() <= 1e-9, (d["m"], err.max())
        fvs.append(r["fval"])
        fls.append(r["flag"])
    fv, ok = np.concatenate(fvs), np.concatenate(fls) == 0
    want = int(np.flatnonzero(ok)[np.argmin(fv[ok])])
    got = best.cpu().numpy()
    assert int(got[1]) == want and got[0] == fv[want]


# ------------------------------------------------------------------ configs[3]


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", ["auto", "tree"])
def test_config3_mpc_horizon(kernel, oracle):
    """configs[3]: 1 024 MPC-horizon QPs (N = 10 stages, 120/200/60, KKT N = 380) on
    the band kernel (auto dispatch: the bench's launch) and on the tree kernel's
    192-thread form -- all optimal, KKT residuals < 1e-5, deterministic, a strided
    sample vs the oracle in the plan's order (1e-9 relative, identical iteration
    counts)."""
    import torch
    from apf_quadruped_amd import plans, workloads as W
    from apf_quadruped_amd.batch import Plan
    B = 1024
    d = W.mpc_qp(plans.SEED + 4, np.arange(B))
    plan = Plan.from_dense(d["n"], d["m"], d["p"], d["P"][0], d["A"][0], d["G"][0], kernel=kernel)
    if kernel == "auto":
        assert plan.kernel_for(B) == "band" and plan.kernel_name(B).startswith("qpb_band_"), plan.kernel_name(B)
    else:
        assert plan.kernel_for(B) == "tree" and "_w192_" in plan.kernel_name(B), plan.kernel_name(B)
    vals = {k: torch.from_numpy(v).cuda() for k, v in plan.pack(d["P"], d["A"], d["G"], d["c"], d["h"],
                                                                d["b"]).items()}
    r1 = plan.unpack(plan.solve(**vals, B=B), B)
    r2 = plan.unpack(plan.solve(**vals, B=B), B)
    for k in ("x", "y", "z", "s", "fval", "iters"):
        np.testing.assert_array_equal(r1[k], r2[k])
    assert (r1["flag"] == 0).all()
    x, y, z, s = r1["x"], r1["y"], r1["z"], r1["s"]
    eq = np.einsum("bij,bj->bi", d["A"], x) - d["b"]
    ineq = np.einsum("bij,bj->bi", d["G"], x) + s - d["h"]
    stat = np.einsum("bij,bj->bi", d["P"], x) + d["c"] + np.einsum("bji,bj->bi", d["A"], y) + \
        np.einsum("bji,bj->bi", d["G"], z)
    assert np.abs(eq).max() < 1e-5 and np.abs(ineq).max() < 1e-5 and np.abs(stat).max() < 1e-5
    Pc, Ac, Gc = W.to_colmajor(d["P"]), W.to_colmajor(d["A"]), W.to_colmajor(d["G"])
    for q in sorted(set(range(0, B, 97)) | {B - 1}):
        o = oracle.solve_dense(120, 200, 60, Pc[q], Ac[q], Gc[q], d["c"][q], d["h"][q], d["b"][q], perm=plan.perm)
        assert o["flag"] == r1["flag"][q] and o["iters"] == r1["iters"][q], q
        for k in ("x", "y", "z", "s"):
            assert _rel(r1[k][q], o[k]) <= 1e-9, (q, k, _rel(r1[k][q], o[k]))


# ------------------------------------------------------------------ configs[4]


@pytest.mark.gpu
def test_config4_sharded_argmin_gather(oracle):
    """configs[4]: 65 536 APF-sampled C1 QPs as 8 shards of 8 192 (the ranks of an
    8-GPU run, here one after another on one GPU): each shard qpb_solve_best on its
    own ids, its payload {fval, global index, x*} built on the device (qpb_winner),
    the 8 payloads reduced by qpb_argmin_reduce exactly as qpb_argmin_allgather
    reduces what ncclAllGather delivers -- equal to the argmin over all 65 536 and to
    the oracle's -- and the whole qpb_argmin_allgather path on a one-rank RCCL
    communicator."""
    import ctypes as C
    import torch
    from apf_quadruped_amd import _lib, plans, workloads as W
    from apf_quadruped_amd.batch import from_tiled
    from apf_quadruped_amd.shard import ArgminGather, shard_range, winner_payload
    world, per = 8, 8192
    plan = plans.standard_plan("c1")
    d = W.contact_force_qp(plans.SEED + 5, np.arange(world * per))
    pays, xs, fvs, fls = [], [], [], []
    last = None
    for r in range(world):
        lo, hi = shard_range(r, world, per)
        sub = {k: d[k][lo:hi] for k in ("P", "A", "G", "c", "h", "b")}
        vals = {k: torch.from_numpy(v).cuda() for k, v in plan.pack(sub["P"], sub["A"], sub["G"], sub["c"], sub["h"],
                                                                    sub["b"]).items()}
        out = plan.alloc_outputs(per)
        best = torch.zeros(2, dtype=torch.float64, device="cuda")
        plan.launcher(vals, out, per, best=best)()
        pay = winner_payload(best, out["x"], 12, per)
        pay[1] = torch.where(pay[1] >= 0, pay[1] + lo, pay[1])
        pays.append(pay)
        rr = plan.unpack(out, per)
        xs.append(rr["x"]); fvs.append(rr["fval"]); fls.append(rr["flag"])
        last = (best, out, lo)
    g = torch.cat(pays)
    win = torch.zeros(14, dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream()
    _lib.check(_lib.lib().qpb_argmin_reduce(C.c_void_p(g.data_ptr()), world, 12, C.c_void_p(win.data_ptr()),
                                            C.c_void_p(s.cuda_stream)), "qpb_argmin_reduce")
    torch.cuda.synchronize()
    w = win.cpu().numpy()
    X, FV, OK = np.concatenate(xs), np.concatenate(fvs), np.concatenate(fls) == 0
    assert OK.all()
    want = int(np.argmin(FV))
    assert int(w[1]) == want and w[0] == FV[want]
    np.testing.assert_array_equal(w[2:], X[want])
    # vs the oracle over all 65 536 (plan's order): every x within the north-star
    # 1e-6, all but a handful at rounding level (1e-9: measured 1 of 65 536 at 1.2e-8,
    # an ill-conditioned QP where FMA rounding is amplified), and the winner is the
    # oracle's (or ties it to rounding)
    x_o, fl_o, it_o = _oracle_batch(oracle, d, plan.perm, threads=16)
    assert (fl_o == 0).all()
    err = np.abs(X - x_o).max(1) / np.maximum(1.0, np.abs(x_o).max(1))
    assert err.max() <= TOL, err.max()
    assert (err > 1e-9).sum() <= 8, np.sort(err)[-10:]
    fv_o = _fval(d, x_o)
    i_o = int(np.argmin(fv_o))
    assert want == i_o or abs(fv_o[want] - fv_o[i_o]) <= 1e-9 * max(1.0, abs(fv_o[i_o]))
    # the C-ABI gather itself (payload kernel + ncclAllGather + device reduce) on a
    # one-rank communicator: the last shard's winner with its global index
    best, out, lo = last
    ag = ArgminGather(0, 1)
    try:
        assert ag.count() == 1
        one = torch.zeros(14, dtype=torch.float64, device="cuda")
        ag.gather(best, out["x"], 12, per, lo, one, torch.cuda.current_stream())
        torch.cuda.synchronize()
        o1 = one.cpu().numpy()
        bv, bi = best.cpu().numpy()
        assert o1[0] == bv and int(o1[1]) == lo + int(bi)
        np.testing.assert_array_equal(o1[2:], from_tiled(out["x"], per, 12).cpu().numpy()[int(bi)])
    finally:
        ag.close()

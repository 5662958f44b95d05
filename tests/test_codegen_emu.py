"""Code-generation tests on the CPU through tests/kernel_emu.py (a lane-by-lane
host execution of the generated HIP kernel; test tool only).

* exact kernels, given the reference's AMD permutation, reproduce the
  reference's golden vectors BIT FOR BIT (so the generated code is the
  reference's arithmetic, independently of the GPU);
* every fast-kernel placement variant agrees with the oracle to 1e-9.
"""
import os

import numpy as np
import pytest

from conftest import golden
from kernel_emu import emulate

from apf_quadruped_amd.batch import Plan, from_tiled

CASES = ["c1_tol1e-6", "c1_tol1e-2", "c1_noeq", "c1_maxit3", "mixed_trot_blfr", "mixed_crawl_blflfr",
         "edge_zero_g_row"]


def _dense(g):
    n, m, p = int(g["n"]), int(g["m"]), int(g["p"])
    B = g["P"].shape[0]
    P = g["P"].reshape(B, n, n).transpose(0, 2, 1)
    G = g["G"].reshape(B, n, m).transpose(0, 2, 1)
    A = g["A"].reshape(B, n, p).transpose(0, 2, 1) if p else None
    return n, m, p, P, A, G


@pytest.mark.parametrize("name", CASES)
def test_emulated_exact_kernel_bit_identical_to_reference(name):
    g = golden(name)
    n, m, p, P, A, G = _dense(g)
    B = min(P.shape[0], 24)
    plan = Plan.from_dense(n, m, p, P[0], A[0] if p else None, G[0], perm=g["perm"][0], p_upper=False, exact=True)
    vals = plan.pack(P[:B], A[:B] if p else None, G[:B], g["c"][:B], g["h"][:B], g["b"][:B] if p else None)
    tol = float(g["tol"])
    out = emulate(plan, vals, B, reltol=tol, abstol=tol, maxit=int(g["maxit"]))
    np.testing.assert_array_equal(from_tiled(out["x"], B, n), g["x"][:B])
    np.testing.assert_array_equal(from_tiled(out["z"], B, m), g["z"][:B])
    np.testing.assert_array_equal(from_tiled(out["s"], B, m), g["s"][:B])
    if p:
        np.testing.assert_array_equal(from_tiled(out["y"], B, p), g["y"][:B])
    np.testing.assert_array_equal(out["iters"], g["iters"][:B])
    np.testing.assert_array_equal(out["flag"], g["flag"][:B])


@pytest.mark.parametrize("variant", ["128:3", "128:2", "256:1", "256:0"])
def test_emulated_fast_variants_match_oracle(variant, oracle, monkeypatch):
    from apf_quadruped_amd import workloads as W
    wg, lds = variant.split(":")
    monkeypatch.setenv("QPB_WG", wg)
    monkeypatch.setenv("QPB_LDS", lds)
    B = 20
    d = W.contact_force_qp(0xD06B07 + 21, np.arange(B))
    plan = Plan.from_dense(12, 20, 6, d["P"][0], d["A"][0], d["G"][0])
    out = emulate(plan, plan.pack(d["P"], d["A"], d["G"], d["c"], d["h"], d["b"]), B)
    x = from_tiled(out["x"], B, 12)
    Pc, Ac, Gc = W.to_colmajor(d["P"]), W.to_colmajor(d["A"]), W.to_colmajor(d["G"])
    for q in range(B):
        r = oracle.solve_dense(12, 20, 6, Pc[q], Ac[q], Gc[q], d["c"][q], d["h"][q], d["b"][q], perm=plan.perm)
        assert np.max(np.abs(r["x"] - x[q])) < 1e-9 * max(1.0, np.max(np.abs(r["x"])))
        assert out["iters"][q] == r["iters"]


@pytest.mark.parametrize("name", ["resolve_c1", "resolve_c1_maxit", "resolve_csc_sigma0.05"])
def test_emulated_exact_kernel_resolve_sequence(name):
    """Warm solves (qpb_solve_warm): kkt_initialize alone (a cold maxit = 0 launch,
    what QP_SETUP leaves in the QP, qpSWIFT.c:447), then one warm launch per
    QP_SOLVE of the reference's sequence, each continuing from the previous
    launch's x, y, z, s, iterations, flag and sigma (qpSWIFT.c:502-601) --
    bit-identical to the reference's state after every call."""
    from apf_quadruped_amd.batch import to_tiled
    g = golden(name)
    n, m, p = int(g["n"]), int(g["m"]), int(g["p"])
    B = min(g["st_x"].shape[0], 8)
    if "Pjc" in g:
        plan = Plan(n, m, p, g["Pjc"], g["Pir"], g["Ajc"], g["Air"], g["Gjc"], g["Gir"], perm=g["perm"][0],
                    p_upper=False, exact=True)
        vals = dict(P=to_tiled(g["Ppr"][:B]), A=to_tiled(g["Apr"][:B]), G=to_tiled(g["Gpr"][:B]),
                    c=to_tiled(g["c"][:B]), h=to_tiled(g["h"][:B]), b=to_tiled(g["b"][:B]))
        sigma_d = float(g["sigma_d"])
    else:
        _, _, _, P, A, G = _dense(g)
        plan = Plan.from_dense(n, m, p, P[0], A[0], G[0], perm=g["perm"][0], p_upper=False, exact=True)
        vals = plan.pack(P[:B], A[:B], G[:B], g["c"][:B], g["h"][:B], g["b"][:B])
        sigma_d = 0.0

    def check(out, k):
        for key, nv in (("x", n), ("y", p), ("z", m), ("s", m)):
            np.testing.assert_array_equal(from_tiled(out[key], B, nv), g["st_" + key][:B, k], err_msg=f"{k}.{key}")

    out = emulate(plan, vals, B, maxit=0, sigma_d=sigma_d)          # QP_SETUP's initial point
    check(out, 0)
    out["flag"][:] = 3                                               # QP_FATAL after setup
    out["iters"][:] = 0
    out["sigma"] = np.full(B, 100.0)                                 # SIGMA (GlobalOptions.h:49)
    for k, (tol, maxit) in enumerate(g["calls"], start=1):
        emulate(plan, vals, B, reltol=tol, abstol=tol, maxit=int(maxit), sigma_d=sigma_d, warm=out)
        check(out, k)
        np.testing.assert_array_equal(out["flag"], g["st_flag"][:B, k])
        np.testing.assert_array_equal(out["iters"], g["st_iters"][:B, k])
        np.testing.assert_array_equal(out["sigma"], g["st_sigma"][:B, k])
        if maxit > 0:
            np.testing.assert_array_equal(out["fval"], g["st_fval"][:B, k])

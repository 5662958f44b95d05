"""CPU-side tests: the C ABI loads and exports what include/*.h declares, plans
match the reference's symbolic analysis, the tiled layout round-trips, and the
generated kernels compile for gfx950 (hiprtc; no GPU needed)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from conftest import ROOT, golden

from apf_quadruped_amd import _lib
from apf_quadruped_amd.batch import Plan, from_tiled, to_tiled


def declared_symbols(header):
    txt = open(os.path.join(ROOT, "include", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    txt = re.sub(r"^\s*#.*$", "", txt, flags=re.M)   # macros are not symbols
    return sorted(set(re.findall(r"\b(qpb_[a-z_]+|QP_[A-Z_a-z]+)\s*\(", txt)))


@pytest.mark.parametrize("header", ["qpswift_hip.h", "qpSWIFT.h"])
def test_library_exports_every_declared_symbol(header):
    L = C.CDLL(_lib.LIB_PATH)
    syms = declared_symbols(header)
    assert syms, header
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing


def _c1_plan(perm=None, exact=False, name="c1_tol1e-6"):
    g = golden(name)
    n, m, p = int(g["n"]), int(g["m"]), int(g["p"])
    P0 = g["P"][0].reshape(n, n).T
    A0 = g["A"][0].reshape(n, p).T if p else None
    G0 = g["G"][0].reshape(n, m).T
    return g, Plan.from_dense(n, m, p, P0, A0, G0, perm=perm, exact=exact)


@pytest.mark.parametrize("name", ["c1_tol1e-6", "c1_noeq", "mixed_trot_blfr", "mixed_crawl_blflfr",
                                  "edge_zero_g_row", "mpc_h10"])
def test_symbolic_matches_reference(name):
    """With the reference's own AMD permutation, nnz(L) equals the reference's Lp[N]."""
    g = golden(name)
    _, plan = _c1_plan(perm=g["perm"][0], name=name)
    assert plan.info.lnz == int(g["lnz"][0])
    assert np.array_equal(plan.perm, g["perm"][0])


def test_own_ordering_is_a_permutation_and_sparse():
    _, plan = _c1_plan(perm=None)
    assert sorted(plan.perm.tolist()) == list(range(38))
    assert plan.info.ordering == 3       # small QP: leaves first (z, y, then x in natural order)
    assert plan.perm.tolist() == list(range(18, 38)) + list(range(12, 18)) + list(range(12))
    assert plan.info.lnz <= 138          # no worse than the reference AMD order


def test_own_ordering_of_larger_plans():
    """Multi-stage patterns (the MPC horizon) are ordered leaves first -- the band
    kernel's elimination; other plans beyond the wave kernel's range by minimum degree."""
    from apf_quadruped_amd import plans
    plan = plans.standard_plan("mpc_h10")
    assert plan.info.ordering == 3
    assert plan.perm.tolist() == list(range(180, 380)) + list(range(120, 180)) + list(range(120))
    rng = np.random.default_rng(5)
    n, m = 80, 100
    P = rng.standard_normal((n, n)) * (rng.random((n, n)) < 0.1)
    P = P @ P.T + np.eye(n)
    G = rng.standard_normal((m, n)) * (rng.random((m, n)) < 0.1)
    G[np.arange(m), rng.integers(0, n, m)] = 1.0
    plan = Plan.from_dense(n, m, 0, P, None, G)
    assert plan.info.ordering == 1 and sorted(plan.perm.tolist()) == list(range(n + m))
    assert plan.kernel_for(1024) == "tree"


def test_plan_rejects_bad_input():
    with pytest.raises(RuntimeError):
        Plan(12, 20, 6, np.zeros(13), np.zeros(0), None, None, np.zeros(13), np.zeros(0),
             perm=np.zeros(38, np.int64))          # perm is not a permutation
    with pytest.raises(RuntimeError):
        Plan(0, 20, 0, np.zeros(1), np.zeros(0), None, None, np.zeros(1), np.zeros(0))


def test_tiled_roundtrip():
    rng = np.random.default_rng(0)
    for B in (1, 63, 64, 65, 200):
        V = rng.standard_normal((B, 7))
        t = to_tiled(V)
        assert t.size == ((B + 63) // 64) * 64 * 7
        np.testing.assert_array_equal(from_tiled(t, B, 7), V)
        # value j of QP q at [(q//64)*nv*64 + j*64 + q%64]
        q, j = B - 1, 3
        assert t[(q // 64) * 7 * 64 + j * 64 + q % 64] == V[q, j]


@pytest.mark.parametrize("exact", [False, True])
def test_kernel_compiles_for_gfx950(exact, tmp_path, monkeypatch):
    _, plan = _c1_plan(exact=exact)
    src = plan.source()
    assert "__global__" in src and ("[exact]" in src) == exact
    plan.compile()                     # hiprtc --offload-arch=gfx950 (or cache hit)


@pytest.mark.parametrize("name,kernel,qpw", [("c1", "wave", 4), ("c1", "wave1", 1), ("c1", "auto", 4),
                                             ("c1", "auto1", 1), ("stance4", "wave", 4),
                                             ("crawl_blflfr", "wave", 4), ("trot_blfr", "wave", 4),
                                             ("trot_brfl", "auto", 4), ("trot_blfr", "wave1", 1)])
def test_wave_kernel_form(name, kernel, qpw):
    """The wave kernel takes its row form (four QPs per wavefront) exactly for
    patterns whose z / y rows are all leaves with the x block in natural order
    and n, p <= 16, m <= 32; "wave1" / "auto1" keep one QP per wavefront."""
    from apf_quadruped_amd import plans
    d = plans.standard_qp(name)
    plan = Plan.from_dense(d["n"], d["m"], d["p"], d["P"][0], d["A"][0], d["G"][0], kernel=kernel)
    assert plan.info.wave_ok == 1 and plan.info.wave_qpw == qpw
    src = plan.wave_source()
    assert ("[row-cooperative" in src) == (qpw == 4)
    plan.compile()                     # hiprtc for gfx950 (or cache hit), no GPU needed


def test_controller_shape_row_forms():
    """30/68/18: leaves first it takes the wide row form (four QPs per wavefront,
    qpb_rowx.hip); in the reference's AMD order (51 dense rows) and with
    QPB_KERNEL_NOROW one QP per wavefront."""
    from apf_quadruped_amd import plans, workloads as W
    d = W.controller_qp(plans.SEED + 30, [0])
    plan = Plan.from_dense(d["n"], d["m"], d["p"], d["P"][0], d["A"][0], d["G"][0], kernel="wave")
    assert plan.info.wave_ok == 1 and plan.info.wave_qpw == 4
    for kw in (dict(kernel="wave1"), dict(order="amd")):
        plan = Plan.from_dense(d["n"], d["m"], d["p"], d["P"][0], d["A"][0], d["G"][0], **kw)
        assert plan.info.wave_ok == 1 and plan.info.wave_qpw == 1, kw


@pytest.mark.parametrize("name,mask,ok", [("c1", 0b1111, True), ("trot_blfr", 0b1010, True),
                                          ("trot_brfl", 0b0101, True), ("crawl_blflfr", 0b1110, True),
                                          ("trot_blfr", 0b1111, False), ("mpc_h10", 0b1111, False)])
def test_assemble_contact_checks_the_plan_pattern(name, mask, ok):
    """qpb_assemble_contact accepts exactly the plans whose P/A/G patterns are those
    of a contact-force QP with the given stance (checked on the host, no GPU)."""
    from apf_quadruped_amd import _lib, plans
    p = plans.standard_plan(name)
    rc = _lib.lib().qpb_assemble_contact(p._h, 0, None, None, mask, 0.5, *([None] * 7))
    assert (rc == 0) == ok, _lib.lib().qpb_last_error()

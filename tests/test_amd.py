"""AMD ordering restatement (csrc/qpb_amd.cpp) vs the reference's amd_l_order.

qpSWIFT orders the KKT with SuiteSparse AMD whenever Permut = NULL
(src/qpSWIFT/qpSWIFT.c:424-440), which is how dogbot_controller calls it
(src/client/main.cpp:1649, 2005, 3232).  A permutation is integer work: the bar
is bit-for-bit equality.

* every golden vector stores the permutation the reference computed for its QP
  (tests/golden/make_golden.py): the plan built with order="amd", the C ABI
  qpb_amd_order and the drop-in's QP_SETUP_dense(..., Permut = NULL) must all
  reproduce it (CPU, no GPU needed);
* where oracle/_ref (the reference compiled from its own sources) is present,
  random patterns -- symmetric and not, jumbled columns with duplicates, dense
  rows, and sizes that make AMD compact its workspace -- are ordered by both.
"""
import ctypes as C
import glob
import os

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, golden

from apf_quadruped_amd import _lib, dropin
from apf_quadruped_amd.batch import Plan

REF_SO = os.path.join(ROOT, "oracle", "_ref", "libqpswift_ref.so")
LP = C.POINTER(C.c_long)
DENSE = sorted(os.path.basename(f)[:-4] for f in glob.glob(os.path.join(GOLDEN, "*.npz"))
               if "csc_" not in os.path.basename(f))


def amd(n, jc, ir):
    jc = np.ascontiguousarray(jc, np.int64)
    ir = np.ascontiguousarray(ir if len(ir) else [0], np.int64)
    perm = np.full(n, -1, np.int64)
    rc = _lib.lib().qpb_amd_order(n, jc.ctypes.data_as(LP), ir.ctypes.data_as(LP), perm.ctypes.data_as(LP))
    return rc, perm


def _dense_plan(g, q):
    n, m, p = int(g["n"]), int(g["m"]), int(g["p"])
    A = g["A"][q].reshape(n, p).T if p else None            # goldens hold column-major dense inputs
    if int(g["ordering"]) == 20:
        P, G = g["P"][q].reshape(n, n), g["G"][q].reshape(m, n)
        A = g["A"][q].reshape(p, n) if p else None
    else:
        P, G = g["P"][q].reshape(n, n).T, g["G"][q].reshape(n, m).T
    return Plan.from_dense(n, m, p, P, A, G, p_upper=False, order="amd")


@pytest.mark.parametrize("name", DENSE)
def test_plan_amd_order_equals_reference_perm(name):
    g = golden(name)
    seen = set()
    for q in range(g["perm"].shape[0]):
        plan = _dense_plan(g, q)
        assert plan.info.ordering == 2
        assert np.array_equal(plan.perm, g["perm"][q]), (name, q)
        seen.add(tuple(g["perm"][q]))
    assert seen


@pytest.mark.parametrize("name", ["csc_sigma0", "csc_sigma0.05"])
def test_plan_amd_order_equals_reference_perm_csc(name):
    g = golden(name)
    plan = Plan(12, 20, 6, g["Pjc"], g["Pir"], g["Ajc"], g["Air"], g["Gjc"], g["Gir"], p_upper=False, order="amd")
    for q in range(g["perm"].shape[0]):
        assert np.array_equal(plan.perm, g["perm"][q])


@pytest.mark.parametrize("name", ["c1_tol1e-6", "c30_tol1e-2", "c30_trot_tol1e-2", "c30_crawl_tol1e-2", "mpc_h10"])
def test_dropin_setup_with_null_permut_uses_reference_perm(name):
    """QP_SETUP_dense(..., Permut = NULL): the KKT ordering the drop-in factors
    with is the reference's (kkt->P), AMD_RESULT = AMD_OK."""
    g = golden(name)
    n, m, p = int(g["n"]), int(g["m"]), int(g["p"])
    qp, keep = dropin.setup_dense(n, m, p, g["P"][0], g["A"][0] if p else None, g["G"][0], g["c"][0],
                                  g["h"][0], g["b"][0] if p else None, ordering=int(g["ordering"]))
    q = qp.contents
    N = n + m + p
    perm = np.ctypeslib.as_array(q.kkt.contents.P, (N,)).copy()
    assert q.stats.contents.AMD_RESULT == 0
    assert np.array_equal(perm, g["perm"][0])
    _lib.lib().QP_CLEANUP_dense(qp)


def test_amd_small_cases():
    # empty matrix / no off-diagonal entries: identity, isolated rows first
    assert amd(0, [0], [])[0] == 0
    rc, perm = amd(3, [0, 1, 2, 3], [0, 1, 2])
    assert rc == 0 and perm.tolist() == [0, 1, 2]
    # a path 0-1-2: an end first
    rc, perm = amd(3, [0, 1, 3, 4], [1, 0, 2, 1])
    assert rc == 0 and sorted(perm.tolist()) == [0, 1, 2]
    # unsorted column: still ordered, status "jumbled"
    rc, perm = amd(3, [0, 2, 3, 4], [2, 1, 0, 0])
    assert rc == 1 and sorted(perm.tolist()) == [0, 1, 2]
    # invalid: row index out of range
    assert amd(2, [0, 1, 2], [0, 5])[0] == -1


def _random_pattern(rng, n):
    kind = rng.integers(0, 4)
    if kind == 0:
        M = rng.random((n, n)) < rng.uniform(0.0, 0.5)
    else:
        M = rng.random((n, n)) < rng.uniform(1.0, 6.0) / n
        if kind == 2:
            M[np.arange(n - 1), np.arange(1, n)] = True
    if rng.random() < 0.7:
        M = M | M.T
    if rng.random() < 0.3:
        M[:, rng.integers(0, n, rng.integers(1, 4))] = True
    jc, ir = [0], []
    for j in range(n):
        rows = list(np.nonzero(M[:, j])[0])
        if rows and rng.random() < 0.05:
            rng.shuffle(rows)
            rows = rows + rows[:1]
        ir += rows
        jc.append(len(ir))
    return np.asarray(jc, np.int64), np.asarray(ir, np.int64)


@pytest.mark.skipif(not os.path.exists(REF_SO), reason="oracle/_ref not built (needs /root/reference)")
def test_amd_matches_reference_amd_l_order_on_random_patterns():
    R = C.CDLL(REF_SO)
    rng = np.random.default_rng(20260)
    ncmpa = ndense = 0
    for trial in range(1500):
        n = int(rng.integers(1, 400))
        jc, ir = _random_pattern(rng, n)
        rc, perm = amd(n, jc, ir)
        ref = np.zeros(n, np.int64)
        ctl, info = (C.c_double * 5)(), (C.c_double * 20)()
        R.amd_l_defaults(ctl)
        irr = np.ascontiguousarray(ir if len(ir) else [0], np.int64)
        rrc = R.amd_l_order(C.c_long(n), jc.ctypes.data_as(LP), irr.ctypes.data_as(LP), ref.ctypes.data_as(LP),
                            ctl, info)
        assert rc == rrc and np.array_equal(perm, ref), (trial, n)
        ncmpa += info[8] > 0      # AMD_NCMPA: workspace compactions
        ndense += info[6] > 0     # AMD_NDENSE
    assert ncmpa > 100 and ndense > 50

"""The oracle (oracle/qpswift_oracle.c) against the reference's own golden vectors.

The fixtures were produced by the reference qpSWIFT compiled from its sources
(tests/golden/make_golden.py); the restatement must reproduce them bit for bit
when given the reference's AMD permutation.
"""
import glob
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden

# resolve_*: QP_SOLVE sequences on one QP object (tests/test_dropin.py,
# tests/test_codegen_emu.py); the oracle solves one call per QP
DENSE = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "*.npz"))
               if not os.path.basename(p).startswith(("csc_", "resolve_")))
SPARSE = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "csc_*.npz")))


@pytest.mark.parametrize("name", DENSE)
def test_oracle_dense_bit_exact(oracle, name):
    g = golden(name)
    n, m, p = int(g["n"]), int(g["m"]), int(g["p"])
    B = g["P"].shape[0]
    for q in range(B):
        r = oracle.solve_dense(n, m, p, g["P"][q], g["A"][q] if p else None, g["G"][q], g["c"][q],
                               g["h"][q], g["b"][q] if p else None, perm=g["perm"][q],
                               ordering=int(g["ordering"]), reltol=float(g["tol"]),
                               abstol=float(g["tol"]), maxit=int(g["maxit"]))
        for k in ("x", "y", "z", "s"):
            np.testing.assert_array_equal(r[k], g[k][q], err_msg=f"{name}[{q}].{k}")
        assert r["flag"] == g["flag"][q] and r["iters"] == g["iters"][q]
        if int(g["maxit"]) > 0:
            assert r["fval"] == g["fval"][q] or (np.isnan(r["fval"]) and np.isnan(g["fval"][q]))
            assert r["n_rx"] == g["n_rx"][q] and r["n_rz"] == g["n_rz"][q] and r["n_mu"] == g["n_mu"][q]
        assert r["lnz"] == g["lnz"][q]


@pytest.mark.parametrize("name", SPARSE)
def test_oracle_csc_bit_exact(oracle, name):
    g = golden(name)
    for q in range(g["Ppr"].shape[0]):
        r = oracle.solve_csc(12, 20, 6, g["Pjc"], g["Pir"], g["Ppr"][q], g["Ajc"], g["Air"], g["Apr"][q],
                             g["Gjc"], g["Gir"], g["Gpr"][q], g["c"][q], g["h"][q], g["b"][q],
                             sigma_d=float(g["sigma_d"]), perm=g["perm"][q])
        for k in ("x", "y", "z", "s"):
            np.testing.assert_array_equal(r[k], g[k][q])
        assert r["flag"] == g["flag"][q] and r["iters"] == g["iters"][q] and r["fval"] == g["fval"][q]


def test_regularisation_fires_on_c1(oracle):
    """5 of 38 pivots are regularised on the 12/20/6 KKT with AMD order."""
    g = golden("c1_tol1e-6")
    r = oracle.solve_dense(12, 20, 6, g["P"][0], g["A"][0], g["G"][0], g["c"][0], g["h"][0], g["b"][0],
                           perm=g["perm"][0])
    assert r["n_regularised"] == 5 and r["lnz"] == 138

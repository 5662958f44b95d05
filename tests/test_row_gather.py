"""Host-side check of the row kernel's gathered sparse products (qpb_row.hip
QPB_R_GATHER; tables from qpb_wave.cpp row_gather_tables): for every standard
row-form plan, the per-lane term lists -- LDS slot + staged-matrix coefficient --
reproduce G'z + A'y (x rows), G x (z rows), A x (y rows) and the G'diag(w)G update
(qpb_xtpos) exactly as the dense products, on random values.  Reference ops:
Auxilary.c:745-786 (residual products), :802-860 (SpMV), ldl.c:253-326 (the
x block's Schur update).  No GPU."""
import re

import numpy as np
import pytest

from apf_quadruped_amd import plans


def _tables(src):
    def arr(name):
        m = re.search(r"qpb_%s\[(\d+)\]\[(\d+)\] = \{(.*?)\};\n" % name, src, re.S)
        rows, cols = int(m.group(1)), int(m.group(2))
        vals = [int(v) for v in re.findall(r"-?\d+", m.group(3))]
        return np.array(vals).reshape(rows, cols)
    lens = {k: int(re.search(r"#define QPB_%s_LEN (\d+)" % k, src).group(1)) for k in ("XT", "ZX0", "ZX1", "AX", "XG")}
    t = {k: (arr("slot_" + k), arr("src_" + k)) for k in ("XT", "ZX0", "ZX1", "AX")}
    return lens, t, arr("xtpos")


@pytest.mark.parametrize("name", plans.STANDARD)
def test_row_gather_tables_reproduce_products(name):
    pl = plans.standard_plan(name)
    src = pl.wave_source()
    if "row-cooperative" not in src:
        pytest.skip("not a row-form plan")
    d = plans.standard_qp(name)
    n, m, p = d["n"], d["m"], d["p"]
    rng = np.random.default_rng(5)
    G = np.where(d["G"][0] != 0, rng.standard_normal((m, n)), 0.0)
    A = np.where(d["A"][0] != 0, rng.standard_normal((p, n)), 0.0)
    # the staged dense matrices as the kernel lays them out (column-major, Ls)
    Ls = np.zeros(n * n + max(p, 1) * n + m * n)
    Ls[n * n:n * n + p * n] = A.T.reshape(-1)
    Ls[n * n + max(p, 1) * n:] = G.T.reshape(-1)
    lens, t, xtpos = _tables(src)
    x, z, y, w = rng.standard_normal(n), rng.standard_normal(m), rng.standard_normal(p), rng.random(m)
    V = np.zeros(66)
    V[:m] = z
    V[32:32 + p] = y
    V[48:48 + n] = x

    def gathered(key, lane):
        slot, srcs = t[key]
        L = lens[key]
        return sum((-Ls[srcs[lane, k]] if srcs[lane, k] >= 0 else 0.0) * V[slot[lane, k]] for k in range(L))

    # x rows: -(G'z + A'y)
    for c in range(n):
        assert gathered("XT", c) == pytest.approx(-(G[:, c] @ z + A[:, c] @ y), abs=1e-12)
    # z rows: -G x (rows c and 16 + c), y rows: -A x
    for c in range(16):
        if c < m:
            assert gathered("ZX0", c) == pytest.approx(-(G[c] @ x), abs=1e-12)
        if 16 + c < m:
            assert gathered("ZX1", c) == pytest.approx(-(G[16 + c] @ x), abs=1e-12)
        if c < p:
            assert gathered("AX", c) == pytest.approx(-(A[c] @ x), abs=1e-12)
    # padding lanes read the zero slot with a zero coefficient
    for key in ("XT", "ZX0", "ZX1", "AX"):
        slot, srcs = t[key]
        assert np.all((srcs >= 0) | (slot == 64))
    # G'diag(w)G through the x lanes' gathered sources: lane j's term for row r
    V[:m] = w
    slot, srcs = t["XT"]
    H = np.zeros((n, n))
    for r in range(m):
        for j in range(n):
            if G[r, j] != 0 or d["G"][0][r, j] != 0:
                k = xtpos[r, j]
                assert 0 <= k < lens["XG"] and slot[j, k] == r
                gw = -Ls[srcs[j, k]] * V[slot[j, k]]              # -G(r, j) w_r in lane j
                H[:, j] += gw * -G[r, :]                            # x -G(r, c) in lane c
    assert np.allclose(H, G.T @ np.diag(w) @ G, atol=1e-12)

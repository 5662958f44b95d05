"""Synthetic QPs for the wide row kernel's tests (qpb_rowx.hip): n <= 32 variables
with sparse G (every row non-empty), dense-ish A and a sparse symmetric P -- shapes
beyond the row kernel's n, p <= 16, m <= 32.  Feasible by construction
(h = G x0 + slack, b = A x0)."""
import numpy as np


def dense_qp(n, m, p, B=4, seed=0, g_density=0.3, a_density=0.6, p_density=0.3, zero_var=None, p_offdiag_from=0,
             linear_var=None):
    """zero_var: a variable decoupled from everything (its P row / column, G and A
    columns, c entry zero) -- its pivot is exactly 0 in every factor.
    p_offdiag_from: P's off-diagonal entries only among variables >= it (the
    controller's skyline P: its coupled block sits in variables 18-29).
    linear_var: a variable with only a linear cost (its P row / column structurally
    empty, so P(v, v) is absent from P's pattern), boxed by G rows 0 and 1 (+-e_v)."""
    rng = np.random.default_rng(seed)
    others = np.array([j for j in range(n) if j != zero_var])
    # one sparsity pattern per plan (every QP of the batch shares it), values per QP
    gpat = rng.random((m, n)) < g_density
    gpat[np.arange(m), others[rng.integers(0, len(others), m)]] = True    # no empty G row
    apat = rng.random((p, n)) < a_density
    apat[np.arange(p), others[np.arange(p) % len(others)]] = True
    ppat = rng.random((n, n)) < p_density
    ppat = ppat | ppat.T
    ppat[:p_offdiag_from, :] = ppat[:, :p_offdiag_from] = False
    ppat = ppat | np.eye(n, dtype=bool)
    if zero_var is not None:
        gpat[:, zero_var] = apat[:, zero_var] = ppat[zero_var, :] = ppat[:, zero_var] = False
    if linear_var is not None:
        ppat[linear_var, :] = ppat[:, linear_var] = False
        gpat[:2, :] = False
        gpat[:2, linear_var] = True
    M = rng.standard_normal((B, n, n)) * 0.4
    P = (np.einsum("bij,bkj->bik", M, M) + (1.0 + 0.1 * n) * np.eye(n)[None]) * ppat[None]
    G = rng.standard_normal((B, m, n)) * gpat[None]
    if linear_var is not None:
        G[:, 0, linear_var], G[:, 1, linear_var] = 1.0, -1.0
    A = (rng.standard_normal((B, p, n)) + 2.0 * np.eye(p, n)[None]) * apat[None]
    x0 = rng.standard_normal((B, n)) * 0.3
    c = rng.standard_normal((B, n))
    if zero_var is not None:
        c[:, zero_var] = 0.0
    h = np.einsum("bij,bj->bi", G, x0) + rng.random((B, m)) + 0.1
    b = np.einsum("bij,bj->bi", A, x0)
    return dict(n=n, m=m, p=p, P=P, A=A, G=G, c=c, h=h, b=b)

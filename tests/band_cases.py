"""Synthetic multi-stage QPs for the band kernel's tests (qpb_band.hip): NS stages of
NB variables, MZ inequality rows on each stage, MY equality rows coupling each stage
to the previous one -- the structure of an MPC horizon (workloads.mpc_qp) with other
block sizes and sparsity.  Feasible by construction (h = G x0 + slack, b = A x0)."""
import numpy as np


def stage_qp(nb, ns, mz, my, B=4, seed=0, g_density=0.4, a_density=0.7):
    rng = np.random.default_rng(seed)
    n, m, p = nb * ns, mz * ns, my * ns
    # one sparsity pattern per plan (every QP of the batch shares it), values per QP
    gpat = rng.random((ns, mz, nb)) < g_density
    gpat[:, np.arange(mz), rng.integers(0, nb, mz)] = True          # no empty G row
    arpat = rng.random((ns, my, nb)) < a_density
    alpat = rng.random((ns, my, nb)) < a_density * 0.5
    ppat = rng.random((ns, nb, nb)) < 0.5
    ppat = ppat | ppat.transpose(0, 2, 1) | np.eye(nb, dtype=bool)[None]
    P = np.zeros((B, n, n)); G = np.zeros((B, m, n)); A = np.zeros((B, p, n))
    for k in range(ns):
        xs = slice(nb * k, nb * k + nb)
        M = rng.standard_normal((B, nb, nb)) * 0.5
        Pk = np.einsum("bij,bkj->bik", M, M) * ppat[k] + (1.0 + nb * 0.1) * np.eye(nb)[None]
        P[:, xs, xs] = Pk
        G[:, mz * k:mz * k + mz, xs] = rng.standard_normal((B, mz, nb)) * gpat[k]
        if my:
            A[:, my * k:my * k + my, xs] = (rng.standard_normal((B, my, nb)) + 2.0 * np.eye(my, nb)[None]) * \
                (arpat[k] | np.eye(my, nb, dtype=bool))
            if k > 0:
                A[:, my * k:my * k + my, nb * (k - 1):nb * k] = rng.standard_normal((B, my, nb)) * alpat[k]
    x0 = rng.standard_normal((B, n)) * 0.3
    c = rng.standard_normal((B, n))
    h = np.einsum("bij,bj->bi", G, x0) + rng.random((B, m)) + 0.1
    b = np.einsum("bij,bj->bi", A, x0)
    return dict(n=n, m=m, p=p, P=P, A=A, G=G, c=c, h=h, b=b)

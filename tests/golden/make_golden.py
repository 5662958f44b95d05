"""Generate the golden vectors in tests/golden/ from the reference qpSWIFT itself.

Run in the build container (needs oracle/_ref/libqpswift_ref.so, which
`make -C oracle ref` compiles from /root/reference's own C sources):

    python tests/golden/make_golden.py          # every case
    python tests/golden/make_golden.py c30      # only the controller-shape cases
    python tests/golden/make_golden.py c30_swing  # only the swing-phase controller shapes

Every case calls the reference exactly as dogbot_controller does
(QP_SETUP_dense -> options override -> QP_SOLVE, main.cpp:1649-1656) and records
inputs, the reference's own AMD permutation, and outputs x, y, z, s, flag,
iteration count, fval and the final residual norms.  Files are plain .npz
(numbers only; load with allow_pickle=False).
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from apf_quadruped_amd import workloads as W  # noqa: E402
from oracle_py import Reference  # noqa: E402

SEED_BASE = 0xD06B07


def dense_case(ref, d, qp_ids, tol, maxit=None, ordering=30, perm=None, drop_eq=False):
    n, m, p = d["n"], d["m"], d["p"]
    if drop_eq:
        p = 0
    B = len(qp_ids)
    P, A, G = W.to_colmajor(d["P"]), W.to_colmajor(d["A"]), W.to_colmajor(d["G"])
    if ordering == 20:  # row-major inputs
        P = d["P"].reshape(B, -1); A = d["A"].reshape(B, -1); G = d["G"].reshape(B, -1)
    out = {k: [] for k in ("x", "y", "z", "s", "flag", "iters", "fval", "n_rx", "n_ry", "n_rz",
                           "n_mu", "perm", "lnz")}
    for q in range(B):
        r = ref.solve_dense(n, m, p, P[q], None if drop_eq else A[q], G[q], d["c"][q], d["h"][q],
                            None if drop_eq else d["b"][q], perm=perm, ordering=ordering,
                            reltol=tol, abstol=tol, maxit=maxit)
        for k in out:
            out[k].append(r[k])
    res = {k: np.asarray(v) for k, v in out.items()}
    res.update(dict(n=n, m=m, p=p, tol=tol, maxit=100 if maxit is None else maxit, ordering=ordering,
                    qp_ids=np.asarray(qp_ids), P=P, A=A if not drop_eq else np.zeros((B, 0)), G=G,
                    c=d["c"], h=d["h"], b=d["b"] if not drop_eq else np.zeros((B, 0))))
    return res


def save(name, **arrs):
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **arrs)
    print(f"{name}: {os.path.getsize(path) / 1024:.1f} KiB")


def c30_cases(ref):
    """Controller-shape stance QP 30/68/18 (main.cpp:1471-1647),
    at the default tolerance and at the controller's 1e-2 (main.cpp:1651-1652)."""
    ids = np.arange(8)
    d = W.controller_qp(SEED_BASE + 30, ids)
    save("c30_tol1e-6", seed=SEED_BASE + 30, **dense_case(ref, d, ids, 1e-6))
    save("c30_tol1e-2", seed=SEED_BASE + 30, **dense_case(ref, d, ids, 1e-2))


def c30_swing_cases(ref):
    """Controller-shape swing-phase QPs: trot 30/70/12 (main.cpp:1730-2005) and
    crawl 30/69/15 (main.cpp:2919-3232), at 1e-6 and at the controller's 1e-2."""
    ids = np.arange(8)
    for phase in ("trot", "crawl"):
        d = W.controller_qp(SEED_BASE + 31, ids, phase=phase)
        save(f"c30_{phase}_tol1e-6", seed=SEED_BASE + 31, **dense_case(ref, d, ids, 1e-6))
        save(f"c30_{phase}_tol1e-2", seed=SEED_BASE + 31, **dense_case(ref, d, ids, 1e-2))


def main(only=None):
    ref = Reference()
    if only == "c30":
        c30_cases(ref)
        return
    if only == "c30_swing":
        c30_swing_cases(ref)
        return
    if only == "edge_infeasible":
        infeasible_case(ref)
        return
    # C1: 12-var / 20-ineq / 6-eq contact-force QP (configs 1, 2, 5).
    ids = np.arange(64)
    d = W.contact_force_qp(SEED_BASE + 1, ids)
    save("c1_tol1e-6", seed=SEED_BASE + 1, **dense_case(ref, d, ids, 1e-6))
    save("c1_tol1e-2", seed=SEED_BASE + 1, **dense_case(ref, d, ids, 1e-2))
    # k-truncated iterates via options->maxit = k (flag QP_MAXIT).
    ids8 = np.arange(8)
    d8 = W.contact_force_qp(SEED_BASE + 1, ids8)
    for k in range(0, 7):
        save(f"c1_maxit{k}", seed=SEED_BASE + 1, **dense_case(ref, d8, ids8, 1e-6, maxit=k))
    # Row-major input ordering (ROW_MAJOR_ORDERING = 20).
    save("c1_rowmajor", seed=SEED_BASE + 1, **dense_case(ref, d8, ids8, 1e-6, ordering=20))
    # No equality constraints (p = 0 path, qpSWIFT.c:306-312, :527-533).
    save("c1_noeq", seed=SEED_BASE + 1, **dense_case(ref, d8, ids8, 1e-6, drop_eq=True))
    # Config 3: four gait contact patterns (mixed KKT sparsity).
    for i, (name, stance) in enumerate(W.STANCE_SETS.items()):
        ids16 = np.arange(16)
        dm = W.contact_force_qp(SEED_BASE + 3, ids16, stance=stance, feasible_wrench=True)
        save(f"mixed_{name}", seed=SEED_BASE + 3, stance=np.asarray(stance),
             **dense_case(ref, dm, ids16, 1e-6))
    # Config 4: MPC horizon QP (N = 10 stages; 120 vars, 200 ineq, 60 eq).
    ids4 = np.arange(4)
    dmpc = W.mpc_qp(SEED_BASE + 4, ids4)
    save("mpc_h10", seed=SEED_BASE + 4, horizon=10, **dense_case(ref, dmpc, ids4, 1e-6))
    # Edge: an all-zero G row (no -I diagonal is inserted, Auxilary.c:126-131).
    dz = W.contact_force_qp(SEED_BASE + 6, ids8)
    dz["G"] = np.concatenate([dz["G"], np.zeros((8, 1, 12))], 1)
    dz["h"] = np.concatenate([dz["h"], np.ones((8, 1))], 1)
    dz["m"] = 21
    save("edge_zero_g_row", seed=SEED_BASE + 6, **dense_case(ref, dz, ids8, 1e-6))
    # Sparse QP_SETUP with sigma_d > 0: the pure-centering branch (qpSWIFT.c:572-579).
    sparse_cases(ref)
    c30_cases(ref)
    c30_swing_cases(ref)
    infeasible_case(ref)


def infeasible_case(ref):
    """Edge: primal-infeasible contact-force QPs -- a lateral force of 3 kN against
    a friction cone that allows ~100 N -- which qpSWIFT runs to maxit = 100
    (QP_MAXIT) with diverging iterates; plus a maxit-truncated copy (tol 1e-6)."""
    ids8 = np.arange(8)
    r, Wr = W.contact_inputs(SEED_BASE + 7, ids8)
    Wr = Wr.copy()
    Wr[:, 0] += 3000.0
    d = W.contact_qp_from_terms(r, Wr)
    save("edge_infeasible", seed=SEED_BASE + 7, **dense_case(ref, d, ids8, 1e-6))
    save("edge_infeasible_maxit8", seed=SEED_BASE + 7, **dense_case(ref, d, ids8, 1e-6, maxit=8))


def to_csc(M):
    """Dense [r, c] -> CSC (jc, ir, pr) dropping exact zeros (column order)."""
    r, c = M.shape
    jc, ir, pr = [0], [], []
    for j in range(c):
        for i in range(r):
            if M[i, j] != 0.0:
                ir.append(i); pr.append(M[i, j])
        jc.append(len(ir))
    return np.asarray(jc, np.int64), np.asarray(ir, np.int64), np.asarray(pr, np.float64)


def sparse_cases(ref):
    ids = np.arange(8)
    d = W.contact_force_qp(SEED_BASE + 7, ids)
    for sigma_d in (0.0, 0.05):
        rows = []
        for q in range(8):
            Pjc, Pir, Ppr = to_csc(d["P"][q]); Ajc, Air, Apr = to_csc(d["A"][q]); Gjc, Gir, Gpr = to_csc(d["G"][q])
            r = ref.solve_csc(12, 20, 6, Pjc, Pir, Ppr, Ajc, Air, Apr, Gjc, Gir, Gpr,
                              d["c"][q], d["h"][q], d["b"][q], sigma_d=sigma_d)
            rows.append((Pjc, Pir, Ppr, Ajc, Air, Apr, Gjc, Gir, Gpr, r))
        out = dict(n=12, m=20, p=6, sigma_d=sigma_d, tol=1e-6, maxit=100,
                   Pjc=rows[0][0], Pir=rows[0][1], Ajc=rows[0][3], Air=rows[0][4], Gjc=rows[0][6], Gir=rows[0][7],
                   Ppr=np.stack([r[2] for r in rows]), Apr=np.stack([r[5] for r in rows]),
                   Gpr=np.stack([r[8] for r in rows]), c=d["c"], h=d["h"], b=d["b"])
        for k in ("x", "y", "z", "s", "flag", "iters", "fval", "perm"):
            out[k] = np.asarray([r[9][k] for r in rows])
        save(f"csc_sigma{sigma_d:g}", seed=SEED_BASE + 7, **out)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else None)

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
    if only == "resolve":
        resolve_cases(ref)
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
    resolve_cases(ref)


def _state(lib, qp, n, m):
    """The QP object's state as a caller sees it: x, y, z, s, stats, options->sigma."""
    q = qp.contents
    st, o = q.stats.contents, q.options.contents
    return dict(x=np.ctypeslib.as_array(q.x, (n,)).copy(),
                y=np.ctypeslib.as_array(q.y, (q.p,)).copy() if q.p else np.zeros(0),
                z=np.ctypeslib.as_array(q.z, (m,)).copy(), s=np.ctypeslib.as_array(q.s, (m,)).copy(),
                flag=int(st.Flag), iters=int(st.IterationCount), fval=float(st.fval), sigma=float(o.sigma),
                n_rx=st.n_rx, n_ry=st.n_ry, n_rz=st.n_rz, n_mu=st.n_mu)


def resolve_sequence(ref, setup, n, m, calls, dense=True):
    """One QP object: setup, then QP_SOLVE once per (reltol = abstol, maxit) in
    `calls`, the options changed in between -- qpSWIFT's QP_SOLVE continues from
    the object's iterate, IterationCount and options->sigma (qpSWIFT.c:502-596).
    Returns the state after setup and after every call."""
    L = ref.lib
    qp = setup()
    states = [_state(L, qp, n, m)]
    for tol, maxit in calls:
        o = qp.contents.options.contents
        o.reltol = tol
        o.abstol = tol
        o.maxit = maxit
        rc = int(L.QP_SOLVE(qp))
        stt = _state(L, qp, n, m)
        assert rc == stt["flag"]
        states.append(stt)
    N = n + m + qp.contents.p
    perm = np.ctypeslib.as_array(qp.contents.kkt.contents.P, (N,)).copy()
    (L.QP_CLEANUP_dense if dense else L.QP_CLEANUP)(qp)
    return states, perm


def resolve_cases(ref):
    """QP_SOLVE called repeatedly on one QP object (qpSWIFT.c:502-596 never
    re-initialises; QP_SETUP leaves kkt_initialize's point in x, s, z, :447):
    state after setup and after each call of a sequence of (tol, maxit) calls --
    the controller's tol 1e-2 solve then tightened to 1e-6, the same tol again (no
    iteration), maxit-truncated calls whose IterationCount passes maxit (the
    :598-601 QP_MAXIT rule), and sigma_d = 0.05 (QP_SETUP, options->sigma carried)."""
    from apf_quadruped_amd.qpswift_abi import dptr, lptr

    def dense_seq(name, d, ids, calls, seed):
        n, m, p = d["n"], d["m"], d["p"]
        P, A, G = W.to_colmajor(d["P"]), W.to_colmajor(d["A"]), W.to_colmajor(d["G"])
        per = []
        for q in range(len(ids)):
            keep = [np.ascontiguousarray(a, dtype=np.float64) for a in (P[q], A[q], G[q], d["c"][q], d["h"][q],
                                                                        d["b"][q])]
            setup = lambda k=keep: ref.lib.QP_SETUP_dense(n, m, p, *[dptr(a) for a in k], lptr(None), 30)
            per.append(resolve_sequence(ref, setup, n, m, calls))
        out = dict(n=n, m=m, p=p, ordering=30, calls=np.asarray(calls, dtype=np.float64), qp_ids=np.asarray(ids),
                   P=P, A=A, G=G, c=d["c"], h=d["h"], b=d["b"], perm=np.asarray([pp for _, pp in per]))
        for k in per[0][0][0]:
            out["st_" + k] = np.asarray([[stt[k] for stt in sts] for sts, _ in per])
        save(name, seed=seed, **out)

    ids = np.arange(16)
    d = W.contact_force_qp(SEED_BASE + 1, ids)
    dense_seq("resolve_c1", d, ids, [(1e-2, 100), (1e-6, 100), (1e-6, 100)], SEED_BASE + 1)
    dense_seq("resolve_c1_maxit", {k: (v[:8] if hasattr(v, "shape") else v) for k, v in d.items()}, ids[:8],
              [(1e-6, 0), (1e-6, 2), (1e-6, 2), (1e-6, 3), (1e-6, 100)], SEED_BASE + 1)
    ids4 = np.arange(4)
    dc = W.controller_qp(SEED_BASE + 30, ids4)
    dense_seq("resolve_c30", dc, ids4, [(1e-2, 100), (1e-6, 100)], SEED_BASE + 30)
    # QP_SETUP (CSC) with sigma_d = 0.05: the options->sigma carried between calls
    # decides the sigma > sigma_d branch (qpSWIFT.c:540) of the next call
    ids8 = np.arange(8)
    d7 = W.contact_force_qp(SEED_BASE + 7, ids8)
    per, rows = [], []
    for q in range(8):
        Pjc, Pir, Ppr = to_csc(d7["P"][q]); Ajc, Air, Apr = to_csc(d7["A"][q]); Gjc, Gir, Gpr = to_csc(d7["G"][q])
        keep = [Pjc, Pir, Ppr, Ajc, Air, Apr, Gjc, Gir, Gpr] + \
            [np.ascontiguousarray(d7[k][q], dtype=np.float64) for k in ("c", "h", "b")]
        setup = lambda k=keep: ref.lib.QP_SETUP(12, 20, 6, lptr(k[0]), lptr(k[1]), dptr(k[2]), lptr(k[3]),
                                                lptr(k[4]), dptr(k[5]), lptr(k[6]), lptr(k[7]), dptr(k[8]),
                                                dptr(k[9]), dptr(k[10]), dptr(k[11]), 0.05, lptr(None))
        per.append(resolve_sequence(ref, setup, 12, 20, [(1e-2, 100), (1e-6, 100), (1e-8, 100)], dense=False))
        rows.append(keep)
    out = dict(n=12, m=20, p=6, sigma_d=0.05, calls=np.asarray([(1e-2, 100), (1e-6, 100), (1e-8, 100)]),
               Pjc=rows[0][0], Pir=rows[0][1], Ajc=rows[0][3], Air=rows[0][4], Gjc=rows[0][6], Gir=rows[0][7],
               Ppr=np.stack([r[2] for r in rows]), Apr=np.stack([r[5] for r in rows]),
               Gpr=np.stack([r[8] for r in rows]), c=d7["c"], h=d7["h"], b=d7["b"],
               perm=np.asarray([pp for _, pp in per]))
    for k in per[0][0][0]:
        out["st_" + k] = np.asarray([[stt[k] for stt in sts] for sts, _ in per])
    save("resolve_csc_sigma0.05", seed=SEED_BASE + 7, **out)


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

"""Python face of the qpSWIFT drop-in (include/qpSWIFT.h, csrc/qpswift_dropin.cpp).

Same call sequence as the controller (dogbot_controller/src/client/main.cpp:
1649-1663): QP_SETUP_dense -> options override -> QP_SOLVE -> read x/y/z/s and
stats -> QP_CLEANUP_dense.  The solve runs on the GPU through libqpswift_hip.so;
there is no host solver behind it.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .qpswift_abi import COLUMN_MAJOR_ORDERING, dptr, lptr


def _f64(a):
    return None if a is None else np.ascontiguousarray(a, dtype=np.float64).ravel()


def _i64(a):
    return None if a is None else np.ascontiguousarray(a, dtype=np.int64).ravel()


def _finish(L, qp, n, m, reltol, abstol, maxit, cleanup, dense):
    if not qp:
        raise MemoryError("QP_SETUP returned NULL")
    o = qp.contents.options.contents
    if reltol is not None:
        o.reltol = reltol
    if abstol is not None:
        o.abstol = abstol
    if maxit is not None:
        o.maxit = maxit
    flag = int(L.QP_SOLVE(qp))
    q = qp.contents
    st = q.stats.contents
    N = n + m + q.p
    k = q.kkt.contents
    out = dict(
        x=np.ctypeslib.as_array(q.x, (n,)).copy(),
        y=np.ctypeslib.as_array(q.y, (q.p,)).copy() if q.p else np.zeros(0),
        z=np.ctypeslib.as_array(q.z, (m,)).copy(),
        s=np.ctypeslib.as_array(q.s, (m,)).copy(),
        flag=flag, iters=int(st.IterationCount), fval=float(st.fval),
        n_rx=st.n_rx, n_ry=st.n_ry, n_rz=st.n_rz, n_mu=st.n_mu,
        alpha_p=st.alpha_p, alpha_d=st.alpha_d, amd_result=int(st.AMD_RESULT),
        tsetup=st.tsetup, tsolve=st.tsolve,
        error=L.qpb_last_error().decode(errors="replace") if flag == 3 else "")
    if k.P:
        out["perm"] = np.ctypeslib.as_array(k.P, (N,)).copy()
        out["lnz"] = int(k.Lp[N]) if k.Lp else -1
    if cleanup:
        (L.QP_CLEANUP_dense if dense else L.QP_CLEANUP)(qp)
    return out


def solve_dense(n, m, p, P, A, G, c, h, b, perm=None, ordering=COLUMN_MAJOR_ORDERING,
                reltol=None, abstol=None, maxit=None, cleanup=True):
    """One QP_SETUP_dense -> QP_SOLVE round trip.  P, A, G are the dense buffers
    in `ordering` (ROW_MAJOR_ORDERING 20 / COLUMN_MAJOR_ORDERING 30)."""
    L = _lib.lib()
    P, A, G, c, h, b = (_f64(a) for a in (P, A, G, c, h, b))
    perm = _i64(perm)
    qp = L.QP_SETUP_dense(n, m, p, dptr(P), dptr(A), dptr(G), dptr(c), dptr(h), dptr(b), lptr(perm), ordering)
    return _finish(L, qp, n, m, reltol, abstol, maxit, cleanup, True)


def solve_csc(n, m, p, Pjc, Pir, Ppr, Ajc, Air, Apr, Gjc, Gir, Gpr, c, h, b, sigma_d=0.0, perm=None,
              reltol=None, abstol=None, maxit=None, cleanup=True):
    """One QP_SETUP (CSC, P with both triangles) -> QP_SOLVE round trip."""
    L = _lib.lib()
    Pjc, Pir, Ajc, Air, Gjc, Gir, perm = (_i64(a) for a in (Pjc, Pir, Ajc, Air, Gjc, Gir, perm))
    Ppr, Apr, Gpr, c, h, b = (_f64(a) for a in (Ppr, Apr, Gpr, c, h, b))
    qp = L.QP_SETUP(n, m, p, lptr(Pjc), lptr(Pir), dptr(Ppr), lptr(Ajc), lptr(Air), dptr(Apr),
                    lptr(Gjc), lptr(Gir), dptr(Gpr), dptr(c), dptr(h), dptr(b), sigma_d, lptr(perm))
    return _finish(L, qp, n, m, reltol, abstol, maxit, cleanup, False)


def setup_dense(n, m, p, P, A, G, c, h, b, perm=None, ordering=COLUMN_MAJOR_ORDERING):
    """QP_SETUP_dense only (no GPU work); returns (QP pointer, keep-alive arrays)."""
    L = _lib.lib()
    keep = [_f64(a) for a in (P, A, G, c, h, b)] + [_i64(perm)]
    P, A, G, c, h, b, perm = keep
    qp = L.QP_SETUP_dense(n, m, p, dptr(P), dptr(A), dptr(G), dptr(c), dptr(h), dptr(b), lptr(perm), ordering)
    return qp, keep


def state(qp, n, m):
    """The QP object's state as the caller sees it: x, y, z, s, stats and
    options->sigma (what a further QP_SOLVE continues from, qpSWIFT.c:502-596)."""
    L = _lib.lib()
    q = qp.contents
    st, o = q.stats.contents, q.options.contents
    return dict(x=np.ctypeslib.as_array(q.x, (n,)).copy(),
                y=np.ctypeslib.as_array(q.y, (q.p,)).copy() if q.p else np.zeros(0),
                z=np.ctypeslib.as_array(q.z, (m,)).copy(), s=np.ctypeslib.as_array(q.s, (m,)).copy(),
                flag=int(st.Flag), iters=int(st.IterationCount), fval=float(st.fval), sigma=float(o.sigma),
                n_rx=st.n_rx, n_ry=st.n_ry, n_rz=st.n_rz, n_mu=st.n_mu,
                error=L.qpb_last_error().decode(errors="replace") if st.Flag == 3 else "")


def solve_again(qp, n, m, reltol=None, abstol=None, maxit=None):
    """Options override -> QP_SOLVE on an existing QP object -> its state."""
    o = qp.contents.options.contents
    if reltol is not None:
        o.reltol = reltol
    if abstol is not None:
        o.abstol = abstol
    if maxit is not None:
        o.maxit = maxit
    rc = int(_lib.lib().QP_SOLVE(qp))
    out = state(qp, n, m)
    out["rc"] = rc
    return out


def setup_csc(n, m, p, Pjc, Pir, Ppr, Ajc, Air, Apr, Gjc, Gir, Gpr, c, h, b, sigma_d=0.0, perm=None):
    """QP_SETUP only; returns (QP pointer, keep-alive arrays: CSC and c, h, b are
    borrowed by the QP, qpSWIFT.c:60-234)."""
    L = _lib.lib()
    keep = [_i64(a) for a in (Pjc, Pir, Ajc, Air, Gjc, Gir, perm)] + [_f64(a) for a in (Ppr, Apr, Gpr, c, h, b)]
    Pjc, Pir, Ajc, Air, Gjc, Gir, perm, Ppr, Apr, Gpr, c, h, b = keep
    qp = L.QP_SETUP(n, m, p, lptr(Pjc), lptr(Pir), dptr(Ppr), lptr(Ajc), lptr(Air), dptr(Apr),
                    lptr(Gjc), lptr(Gir), dptr(Gpr), dptr(c), dptr(h), dptr(b), sigma_d, lptr(perm))
    return qp, keep

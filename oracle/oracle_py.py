"""Python bindings for the oracle (TEST INFRASTRUCTURE ONLY).

* `Oracle`    -- ctypes binding of liboracle.so, this repo's from-scratch C
                 restatement of qpSWIFT (oracle/qpswift_oracle.c).
* `Reference` -- ctypes binding of oracle/_ref/libqpswift_ref.so, the reference
                 qpSWIFT compiled from /root/reference's own C sources by
                 oracle/Makefile (`make ref`).  Used to make golden vectors and as
                 the CPU baseline in bench.py; never part of the product.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from apf_quadruped_amd.qpswift_abi import (  # noqa: E402
    COLUMN_MAJOR_ORDERING, bind_qpswift, dptr, lptr)

ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libqpswift_ref.so")


def build(ref: bool = True) -> None:
    """Compile the oracle (and, when /root/reference is present, oracle/_ref)."""
    targets = ["oracle"]
    if ref and os.path.isdir("/root/reference/dogbot_controller/src/qpSWIFT"):
        targets.append("ref")
    subprocess.run(["make", "-s", "-C", HERE, "-j8", *targets], check=True)


class OracleResult(C.Structure):
    _fields_ = [("flag", C.c_long), ("iters", C.c_long), ("fval", C.c_double),
                ("n_rx", C.c_double), ("n_ry", C.c_double), ("n_rz", C.c_double),
                ("n_mu", C.c_double), ("alpha_p", C.c_double), ("alpha_d", C.c_double),
                ("n_regularised", C.c_long), ("lnz", C.c_long)]


def _f64(a):
    return None if a is None else np.ascontiguousarray(a, dtype=np.float64)


def _i64(a):
    return None if a is None else np.ascontiguousarray(a, dtype=np.int64)


class Oracle:
    def __init__(self, path: str = ORACLE_SO):
        if not os.path.exists(path):
            build(ref=False)
        lib = C.CDLL(path)
        dp, lp = C.POINTER(C.c_double), C.POINTER(C.c_long)
        lib.oracle_solve_dense.restype = C.c_int
        lib.oracle_solve_dense.argtypes = [C.c_long] * 3 + [dp] * 6 + [lp, C.c_int, C.c_double,
                                                                        C.c_double, C.c_long] + [dp] * 4 + [C.POINTER(OracleResult)]
        lib.oracle_solve_csc.restype = C.c_int
        lib.oracle_solve_csc.argtypes = [C.c_long] * 3 + [lp, lp, dp] * 3 + [dp] * 3 + [C.c_double, lp, C.c_double, C.c_double, C.c_long] + [dp] * 4 + [C.POINTER(OracleResult)]
        lib.oracle_solve_dense_batch.restype = C.c_int
        lib.oracle_solve_dense_batch.argtypes = [C.c_long] * 4 + [dp] * 6 + [lp, C.c_double, C.c_double, C.c_long, dp, lp, lp, C.c_int]
        self.lib = lib

    def solve_dense(self, n, m, p, P, A, G, c, h, b, perm=None, ordering=COLUMN_MAJOR_ORDERING,
                    reltol=1e-6, abstol=1e-6, maxit=100):
        """P, A, G flattened in the given ordering.  Returns a dict."""
        P, A, G, c, h, b = map(_f64, (P, A, G, c, h, b))
        perm = _i64(perm)
        x, y, z, s = np.zeros(n), np.zeros(max(p, 1)), np.zeros(m), np.zeros(m)
        r = OracleResult()
        self.lib.oracle_solve_dense(n, m, p, dptr(P), dptr(A), dptr(G), dptr(c), dptr(h), dptr(b),
                                    lptr(perm), ordering, reltol, abstol, maxit,
                                    dptr(x), dptr(y), dptr(z), dptr(s), C.byref(r))
        return dict(x=x, y=y[:p], z=z, s=s, flag=r.flag, iters=r.iters, fval=r.fval,
                    n_rx=r.n_rx, n_ry=r.n_ry, n_rz=r.n_rz, n_mu=r.n_mu,
                    alpha_p=r.alpha_p, alpha_d=r.alpha_d, n_regularised=r.n_regularised, lnz=r.lnz)

    def solve_csc(self, n, m, p, Pjc, Pir, Ppr, Ajc, Air, Apr, Gjc, Gir, Gpr, c, h, b,
                  sigma_d=0.0, perm=None, reltol=1e-6, abstol=1e-6, maxit=100):
        Pjc, Pir, Ajc, Air, Gjc, Gir, perm = map(_i64, (Pjc, Pir, Ajc, Air, Gjc, Gir, perm))
        Ppr, Apr, Gpr, c, h, b = map(_f64, (Ppr, Apr, Gpr, c, h, b))
        x, y, z, s = np.zeros(n), np.zeros(max(p, 1)), np.zeros(m), np.zeros(m)
        r = OracleResult()
        self.lib.oracle_solve_csc(n, m, p, lptr(Pjc), lptr(Pir), dptr(Ppr), lptr(Ajc), lptr(Air), dptr(Apr),
                                  lptr(Gjc), lptr(Gir), dptr(Gpr), dptr(c), dptr(h), dptr(b), sigma_d,
                                  lptr(perm), reltol, abstol, maxit, dptr(x), dptr(y), dptr(z), dptr(s), C.byref(r))
        return dict(x=x, y=y[:p], z=z, s=s, flag=r.flag, iters=r.iters, fval=r.fval,
                    n_rx=r.n_rx, n_ry=r.n_ry, n_rz=r.n_rz, n_mu=r.n_mu,
                    alpha_p=r.alpha_p, alpha_d=r.alpha_d, n_regularised=r.n_regularised, lnz=r.lnz)

    def solve_dense_batch(self, n, m, p, P, A, G, c, h, b, perm=None, reltol=1e-6, abstol=1e-6,
                          maxit=100, threads=1):
        """Column-major batched inputs P [B, n*n] ...; returns x [B, n], flags, iters."""
        P, A, G, c, h, b = map(_f64, (P, A, G, c, h, b))
        B = P.shape[0]
        x = np.zeros((B, n)); flags = np.zeros(B, np.int64); iters = np.zeros(B, np.int64)
        self.lib.oracle_solve_dense_batch(B, n, m, p, dptr(P), dptr(A), dptr(G), dptr(c), dptr(h), dptr(b),
                                          lptr(_i64(perm)), reltol, abstol, maxit, dptr(x), lptr(flags),
                                          lptr(iters), threads)
        return x, flags, iters


class Reference:
    """The reference qpSWIFT itself (oracle/_ref), driven through its C API."""

    def __init__(self, path: str = REF_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle ref` where /root/reference exists")
        self.lib = bind_qpswift(C.CDLL(path))

    def solve_dense(self, n, m, p, P, A, G, c, h, b, perm=None, ordering=COLUMN_MAJOR_ORDERING,
                    reltol=None, abstol=None, maxit=None, cleanup=True):
        """One QP_SETUP_dense -> [option override] -> QP_SOLVE, as main.cpp:1649-1656 does."""
        keep = [_f64(a) for a in (P, A, G, c, h, b)]
        P, A, G, c, h, b = keep
        perm = _i64(perm)
        qp = self.lib.QP_SETUP_dense(n, m, p, dptr(P), dptr(A), dptr(G), dptr(c), dptr(h), dptr(b),
                                     lptr(perm), ordering)
        return self._solve(qp, n, m, p, reltol, abstol, maxit, cleanup, dense=True)

    def solve_csc(self, n, m, p, Pjc, Pir, Ppr, Ajc, Air, Apr, Gjc, Gir, Gpr, c, h, b,
                  sigma_d=0.0, perm=None, reltol=None, abstol=None, maxit=None, cleanup=True):
        arrs = [_i64(a) for a in (Pjc, Pir, Ajc, Air, Gjc, Gir)] + [_f64(a) for a in (Ppr, Apr, Gpr, c, h, b)]
        Pjc, Pir, Ajc, Air, Gjc, Gir, Ppr, Apr, Gpr, c, h, b = arrs
        perm = _i64(perm)
        qp = self.lib.QP_SETUP(n, m, p, lptr(Pjc), lptr(Pir), dptr(Ppr), lptr(Ajc), lptr(Air), dptr(Apr),
                               lptr(Gjc), lptr(Gir), dptr(Gpr), dptr(c), dptr(h), dptr(b), sigma_d, lptr(perm))
        return self._solve(qp, n, m, p, reltol, abstol, maxit, cleanup, dense=False)

    def _solve(self, qp, n, m, p, reltol, abstol, maxit, cleanup, dense):
        o = qp.contents.options.contents
        if reltol is not None:
            o.reltol = reltol
        if abstol is not None:
            o.abstol = abstol
        if maxit is not None:
            o.maxit = maxit
        flag = self.lib.QP_SOLVE(qp)
        q = qp.contents
        st = q.stats.contents
        N = n + m + q.p
        out = dict(
            x=np.ctypeslib.as_array(q.x, (n,)).copy(),
            y=np.ctypeslib.as_array(q.y, (q.p,)).copy() if q.p else np.zeros(0),
            z=np.ctypeslib.as_array(q.z, (m,)).copy(),
            s=np.ctypeslib.as_array(q.s, (m,)).copy(),
            flag=int(flag), iters=int(st.IterationCount), fval=float(st.fval),
            n_rx=st.n_rx, n_ry=st.n_ry, n_rz=st.n_rz, n_mu=st.n_mu,
            alpha_p=st.alpha_p, alpha_d=st.alpha_d, amd_result=int(st.AMD_RESULT),
            perm=np.ctypeslib.as_array(q.kkt.contents.P, (N,)).copy(),
            lnz=int(q.kkt.contents.Lp[N]))
        if cleanup:
            (self.lib.QP_CLEANUP_dense if dense else self.lib.QP_CLEANUP)(qp)
        return out

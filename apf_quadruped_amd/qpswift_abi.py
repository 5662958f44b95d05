"""ctypes mirror of the qpSWIFT C ABI (struct layouts and entry points).

The layouts follow dogbot_controller/include/qpSWIFT/Auxilary.h:18-151 field for
field (qp_int = long, qp_real = double, GlobalOptions.h:36-43), which is also the
layout exported by this repository's drop-in library (include/qpSWIFT.h).  The
same mirror therefore binds either library: `bind_qpswift(cdll)` declares the
QP_SETUP / QP_SETUP_dense / QP_SOLVE / QP_CLEANUP / QP_CLEANUP_dense prototypes
(qpSWIFT.h:14-26) on any CDLL that exports them.
"""
from __future__ import annotations

import ctypes as C

c_long_p = C.POINTER(C.c_long)
c_double_p = C.POINTER(C.c_double)

# GlobalOptions.h:54-60
QP_OPTIMAL, QP_KKTFAIL, QP_MAXIT, QP_FATAL = 0, 1, 2, 3
ROW_MAJOR_ORDERING, COLUMN_MAJOR_ORDERING = 20, 30


class smat(C.Structure):          # Auxilary.h:18-26
    _fields_ = [("jc", c_long_p), ("ir", c_long_p), ("pr", c_double_p),
                ("n", C.c_long), ("m", C.c_long), ("nnz", C.c_long)]


class kkt(C.Structure):           # Auxilary.h:31-50
    _fields_ = [("kktmatrix", C.POINTER(smat)), ("b", c_double_p),
                ("Parent", c_long_p), ("Flag", c_long_p), ("Lnz", c_long_p),
                ("Li", c_long_p), ("Lp", c_long_p), ("Lti", c_long_p), ("Ltp", c_long_p),
                ("Pattern", c_long_p), ("UPattern", c_long_p), ("Y", c_double_p),
                ("Lx", c_double_p), ("D", c_double_p), ("P", c_long_p), ("Pinv", c_long_p)]


class stats(C.Structure):         # Auxilary.h:55-84
    _fields_ = [("tsetup", C.c_double), ("tsolve", C.c_double), ("kkt_time", C.c_double),
                ("ldl_numeric", C.c_double), ("IterationCount", C.c_long),
                ("n_rx", C.c_double), ("n_ry", C.c_double), ("n_rz", C.c_double),
                ("n_mu", C.c_double), ("alpha_p", C.c_double), ("alpha_d", C.c_double),
                ("fval", C.c_double), ("Flag", C.c_long), ("AMD_RESULT", C.c_long),
                ("resolve_kkt", C.c_long)]


class settings(C.Structure):      # Auxilary.h:89-100
    _fields_ = [("maxit", C.c_long), ("reltol", C.c_double), ("abstol", C.c_double),
                ("sigma", C.c_double), ("verbose", C.c_long)]


class QP(C.Structure):            # Auxilary.h:106-151
    _fields_ = [("n", C.c_long), ("m", C.c_long), ("p", C.c_long),
                ("sigma_d", C.c_double), ("mu", C.c_double), ("rho", C.c_double),
                ("x", c_double_p), ("y", c_double_p), ("z", c_double_p), ("s", c_double_p),
                ("rx", c_double_p), ("ry", c_double_p), ("rz", c_double_p),
                ("delta", c_double_p), ("delta_x", c_double_p), ("delta_y", c_double_p),
                ("delta_z", c_double_p), ("delta_s", c_double_p), ("ds", c_double_p),
                ("lambda", c_double_p), ("temp", c_double_p),
                ("P", C.POINTER(smat)), ("c", c_double_p), ("G", C.POINTER(smat)),
                ("h", c_double_p), ("A", C.POINTER(smat)), ("b", c_double_p),
                ("At", C.POINTER(smat)), ("Gt", C.POINTER(smat)), ("kkt", C.POINTER(kkt)),
                ("options", C.POINTER(settings)), ("stats", C.POINTER(stats))]


QP_p = C.POINTER(QP)


def bind_qpswift(lib: C.CDLL) -> C.CDLL:
    """Declare the five qpSWIFT.h entry points on `lib`."""
    lib.QP_SETUP.restype = QP_p
    lib.QP_SETUP.argtypes = [C.c_long, C.c_long, C.c_long,
                             c_long_p, c_long_p, c_double_p,
                             c_long_p, c_long_p, c_double_p,
                             c_long_p, c_long_p, c_double_p,
                             c_double_p, c_double_p, c_double_p, C.c_double, c_long_p]
    lib.QP_SETUP_dense.restype = QP_p
    lib.QP_SETUP_dense.argtypes = [C.c_long, C.c_long, C.c_long,
                                   c_double_p, c_double_p, c_double_p,
                                   c_double_p, c_double_p, c_double_p, c_long_p, C.c_int]
    lib.QP_SOLVE.restype = C.c_long
    lib.QP_SOLVE.argtypes = [QP_p]
    lib.QP_CLEANUP.restype = None
    lib.QP_CLEANUP.argtypes = [QP_p]
    lib.QP_CLEANUP_dense.restype = None
    lib.QP_CLEANUP_dense.argtypes = [QP_p]
    return lib


def dptr(a):
    """double* of a C-contiguous float64 numpy array (None -> NULL)."""
    if a is None:
        return None
    return a.ctypes.data_as(c_double_p)


def lptr(a):
    """long* of a C-contiguous int64 numpy array (None -> NULL)."""
    if a is None:
        return None
    return a.ctypes.data_as(c_long_p)

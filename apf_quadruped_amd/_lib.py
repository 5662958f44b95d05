"""Loader for the native library (libqpswift_hip.so, built in-tree).

The product path has no CPU fallback: if the HIP library is missing or fails to
load, every entry point raises.  Build it with `python -c "import
__graft_entry__ as g; g.build()"` (or `make -C apf_quadruped_amd`).
"""
from __future__ import annotations

import ctypes as C
import os

from .qpswift_abi import bind_qpswift

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libqpswift_hip.so")


class QpbSettings(C.Structure):
    _fields_ = [("maxit", C.c_long), ("reltol", C.c_double), ("abstol", C.c_double),
                ("sigma_d", C.c_double)]


class QpbIo(C.Structure):
    """qpb_io: one member's batch of a plan group (device pointers)."""
    _fields_ = [("B", C.c_long)] + [(k, C.c_void_p) for k in ("P", "A", "G", "c", "h", "b", "x", "y", "z", "s",
                                                              "flag", "iters", "fval", "stats")]


class QpbApfState(C.Structure):
    """qpb_apf_state (include/qpswift_hip.h): one tick's state for qpb_apf_wrench."""
    _fields_ = [("ee", (C.c_double * 2) * 4), ("com", C.c_double * 6), ("com_vel", C.c_double * 6),
                ("acc_des", C.c_double * 6), ("des_orient", C.c_double * 2), ("rob_foot", C.c_double * 4),
                ("versor", (C.c_double * 2) * 4), ("lat_versor", C.c_double * 2), ("R_wb", C.c_double * 9),
                ("Mcom", C.c_double * 36), ("mass", C.c_double), ("rep_field", C.c_int), ("min_exit", C.c_int),
                ("fake_crawl", C.c_int)]


class QpbPlanInfo(C.Structure):
    _fields_ = [("n", C.c_long), ("m", C.c_long), ("p", C.c_long), ("N", C.c_long),
                ("nnzP", C.c_long), ("nnzA", C.c_long), ("nnzG", C.c_long),
                ("nnzK", C.c_long), ("lnz", C.c_long),
                ("fac_updates", C.c_long), ("fac_divs", C.c_long),
                ("ordering", C.c_int), ("exact", C.c_int), ("hash", C.c_uint64),
                ("wave_ok", C.c_int), ("wave_max_batch", C.c_long), ("wave_qpw", C.c_int),
                ("tree_ok", C.c_int), ("large_kernel", C.c_int)]


_lib = None


class NativeLibraryMissing(RuntimeError):
    pass


def lib() -> C.CDLL:
    """The loaded native library; raises NativeLibraryMissing if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeLibraryMissing(
            f"{LIB_PATH} not built -- the HIP path is the only path (no CPU fallback); "
            "run __graft_entry__.build() first")
    L = C.CDLL(LIB_PATH)
    lp, dp, vp = C.POINTER(C.c_long), C.POINTER(C.c_double), C.c_void_p
    L.qpb_last_error.restype = C.c_char_p
    L.qpb_version.restype = C.c_char_p
    L.qpb_compiler.restype = C.c_char_p
    L.qpb_audit_dpp.argtypes = [vp, C.c_long, C.c_char_p, C.c_long]
    L.qpb_join_fixup.argtypes = [C.c_char_p, C.c_long, C.c_char_p, C.c_long]
    L.qpb_join_fixup.restype = C.c_long
    L.qpb_default_settings.argtypes = [C.POINTER(QpbSettings)]
    L.qpb_plan_create.restype = C.c_int
    L.qpb_plan_create.argtypes = [C.POINTER(vp), C.c_long, C.c_long, C.c_long, C.c_int,
                                  lp, lp, lp, lp, lp, lp, lp]
    L.qpb_plan_destroy.argtypes = [vp]
    L.qpb_plan_destroy.restype = None
    L.qpb_plan_get_info.argtypes = [vp, C.POINTER(QpbPlanInfo)]
    L.qpb_plan_get_perm.argtypes = [vp, lp]
    L.qpb_comm_get_unique_id.argtypes = [vp]
    L.qpb_comm_init.argtypes = [C.POINTER(vp), C.c_int, vp, C.c_int]
    L.qpb_comm_destroy.argtypes = [vp]
    L.qpb_comm_count.argtypes = [vp, C.POINTER(C.c_int)]
    L.qpb_comm_destroy.restype = None
    L.qpb_argmin_allgather.argtypes = [vp, vp, C.c_long, C.c_long, C.c_long, vp, vp, vp]
    L.qpb_argmin_reduce.argtypes = [vp, C.c_long, C.c_long, vp, vp]
    L.qpb_assemble_controller.argtypes = [vp, C.c_long, vp, C.c_int, vp, C.c_double] + [vp] * 8
    L.qpb_apf_wrench.argtypes = [C.c_long, C.POINTER(QpbApfState), vp, vp, vp, vp]
    L.qpb_apf_update.argtypes = [C.POINTER(QpbApfState), dp, C.c_double, dp]
    L.qpb_amd_order.restype = C.c_int
    L.qpb_amd_order.argtypes = [C.c_long, lp, lp, lp]
    L.qpb_plan_source.restype = C.c_long
    L.qpb_plan_source.argtypes = [vp, C.c_char_p, C.c_long]
    L.qpb_plan_wave_source.restype = C.c_long
    L.qpb_plan_wave_source.argtypes = [vp, C.c_char_p, C.c_long]
    L.qpb_plan_kernel_name.restype = C.c_long
    L.qpb_plan_kernel_name.argtypes = [vp, C.c_long, C.c_char_p, C.c_long]
    L.qpb_plan_tree_source.restype = C.c_long
    L.qpb_plan_tree_source.argtypes = [vp, C.c_char_p, C.c_long]
    L.qpb_plan_tree_tables.restype = C.c_long
    L.qpb_plan_tree_tables.argtypes = [vp, C.c_void_p, C.c_long]
    L.qpb_plan_compile.argtypes = [vp]
    L.qpb_plan_compile_warm.argtypes = [vp, C.c_long]
    L.qpb_plan_compile_serve.argtypes = [vp]
    L.qpb_dropin_serve_stats.argtypes = [C.POINTER(C.c_long)]
    L.qpb_serve_config.argtypes = [C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.qpb_serve_config.restype = C.c_int
    L.qpb_solve.restype = C.c_int
    L.qpb_solve.argtypes = [vp, C.c_long] + [vp] * 6 + [C.POINTER(QpbSettings)] + [vp] * 7 + [vp, vp]
    L.qpb_solve_warm.restype = C.c_int
    L.qpb_solve_warm.argtypes = [vp, C.c_long] + [vp] * 6 + [C.POINTER(QpbSettings)] + [vp] * 7 + [vp, vp, vp]
    L.qpb_solve_best.restype = C.c_int
    L.qpb_solve_best.argtypes = [vp, C.c_long] + [vp] * 6 + [C.POINTER(QpbSettings)] + [vp] * 7 + [vp, vp, vp]
    L.qpb_assemble_contact.restype = C.c_int
    L.qpb_assemble_contact.argtypes = [vp, C.c_long, vp, vp, C.c_int, C.c_double] + [vp] * 7
    L.qpb_group_create.restype = C.c_int
    L.qpb_group_create.argtypes = [C.POINTER(vp), C.POINTER(vp), C.c_int]
    L.qpb_group_destroy.argtypes = [vp]
    L.qpb_group_destroy.restype = None
    L.qpb_group_source.restype = C.c_long
    L.qpb_group_source.argtypes = [vp, C.c_char_p, C.c_long]
    L.qpb_group_compile.argtypes = [vp]
    L.qpb_group_solve.restype = C.c_int
    L.qpb_group_solve.argtypes = [vp, C.POINTER(QpbIo), C.POINTER(QpbSettings), vp, vp]
    L.qpb_winner.restype = C.c_int
    L.qpb_winner.argtypes = [vp, vp, C.c_long, C.c_long, vp, vp]
    L.qpb_argmin.restype = C.c_int
    L.qpb_argmin.argtypes = [C.c_long, vp, vp, vp, vp]
    if hasattr(L, "QP_SETUP"):
        bind_qpswift(L)
    _lib = L
    return L


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().qpb_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed ({rc}): {msg}")

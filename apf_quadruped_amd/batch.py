"""Batched qpSWIFT solve on MI355X: Python host side of include/qpswift_hip.h.

    plan = Plan.from_dense(n, m, p, P0, A0, G0)        # pattern of one QP
    vals = plan.pack(P, A, G, c, h, b)                  # [B, ...] dense -> SoA
    out  = plan.solve(**vals, reltol=1e-6)              # one HIP launch, B QPs

A Plan is the pattern half of QP_SETUP (dogbot_controller/src/qpSWIFT/
qpSWIFT.c:60-234): KKT assembly, ordering, symbolic factorisation, and the
generated gfx950 kernel.  `solve` is the value half (kkt_initialize) plus
QP_SOLVE (qpSWIFT.c:473-644) for every QP of the batch.  Torch is used only to
own device memory and streams; the arithmetic is the generated HIP kernel.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import QpbApfState, QpbIo, QpbPlanInfo, QpbSettings, check
check_ = check

QPB_P_FULL, QPB_P_UPPER, QPB_EXACT = 0x0, 0x1, 0x10
# KKT ordering when no permutation is given: "own" (leaves first for small QPs,
# else minimum degree), "amd" (the reference's AMD: what qpSWIFT computes for
# Permut = NULL, qpSWIFT.c:424-440), "mindeg", "leaves"
ORDER_FLAGS = {"own": 0x0, "amd": 0x20, "mindeg": 0x40, "leaves": 0x80}
QPB_KERNEL_LANE, QPB_KERNEL_WAVE, QPB_KERNEL_NOROW, QPB_KERNEL_TREE, QPB_KERNEL_BAND = 0x100, 0x200, 0x400, 0x800, 0x1000
# "wave" = the wave kernel in the form the plan picks (row form: four QPs per
# wavefront, where it fits); "wave1" = one QP per wavefront regardless
KERNEL_FLAGS = {"auto": 0, "lane": QPB_KERNEL_LANE, "wave": QPB_KERNEL_WAVE,
                "wave1": QPB_KERNEL_WAVE | QPB_KERNEL_NOROW, "auto1": QPB_KERNEL_NOROW,
                "tree": QPB_KERNEL_TREE, "band": QPB_KERNEL_BAND}
QP_OPTIMAL, QP_KKTFAIL, QP_MAXIT, QP_FATAL = 0, 1, 2, 3


def dense_pattern(M: np.ndarray, upper: bool = False):
    """CSC (jc, ir) of the non-zeros of dense M (exact zeros dropped, as
    densetosparse does, Auxilary.c:1154-1206); upper=True keeps rows <= col."""
    M = np.asarray(M)
    rows, cols = M.shape
    nz = M != 0.0
    if upper:
        nz = nz & (np.arange(rows)[:, None] <= np.arange(cols)[None, :])
    jc = np.zeros(cols + 1, np.int64)
    jc[1:] = np.cumsum(nz.sum(0))
    ir = np.nonzero(nz.T)[1].astype(np.int64)       # column-major scan, rows ascending
    return jc, ir


TILE = 64


def ntiles(B: int) -> int:
    return (int(B) + TILE - 1) // TILE


def to_tiled(V: np.ndarray) -> np.ndarray:
    """[B, nv] per-QP rows -> flat tiled-SoA array (include/qpswift_hip.h):
    value j of QP q at [(q//64)*nv*64 + j*64 + q%64]; the last tile is zero-padded."""
    V = np.asarray(V, dtype=np.float64)
    if V.ndim == 1:
        V = V[:, None]
    B, nv = V.shape
    T = ntiles(B)
    buf = np.zeros((T * TILE, nv))
    buf[:B] = V
    return np.ascontiguousarray(buf.reshape(T, TILE, nv).transpose(0, 2, 1)).reshape(-1)


def from_tiled(flat, B: int, nv: int):
    """Inverse of to_tiled (numpy or torch): flat tiled array -> [B, nv]."""
    T = ntiles(B)
    t = flat[:T * nv * TILE].reshape(T, nv, TILE)     # buffers may hold spare tiles
    if hasattr(t, "permute"):
        return t.permute(0, 2, 1).reshape(T * TILE, nv)[:B]
    return t.transpose(0, 2, 1).reshape(T * TILE, nv)[:B]


def _gather_values(M: np.ndarray, jc, ir) -> np.ndarray:
    """[B, r, c] dense -> [B, nnz] values in CSC order."""
    cols = np.repeat(np.arange(len(jc) - 1), np.diff(jc))
    return np.ascontiguousarray(M[:, ir, cols])


@dataclass
class Patterns:
    P: tuple
    A: tuple
    G: tuple


class Plan:
    """One sparsity pattern (+ KKT ordering) and its generated gfx950 kernel."""

    def __init__(self, n, m, p, Pjc, Pir, Ajc, Air, Gjc, Gir, perm=None, p_upper=True, exact=False, kernel="auto",
                 order="own"):
        L = _lib.lib()
        self.n, self.m, self.p = int(n), int(m), int(p)
        self.p_upper, self.exact = bool(p_upper), bool(exact)
        arr = lambda a: None if a is None else np.ascontiguousarray(a, dtype=np.int64)
        self._keep = [arr(a) for a in (Pjc, Pir, Ajc, Air, Gjc, Gir, perm)]
        Pjc, Pir, Ajc, Air, Gjc, Gir, perm = self._keep
        self.patterns = Patterns((Pjc, Pir), (Ajc, Air), (Gjc, Gir))
        lp = lambda a: None if a is None else a.ctypes.data_as(C.POINTER(C.c_long))
        h = C.c_void_p()
        flags = ((QPB_P_UPPER if p_upper else QPB_P_FULL) | (QPB_EXACT if exact else 0) | KERNEL_FLAGS[kernel]
                 | ORDER_FLAGS[order])
        self.kernel, self.order = kernel, order
        check(L.qpb_plan_create(C.byref(h), self.n, self.m, self.p, flags, lp(Pjc), lp(Pir),
                                lp(Ajc) if self.p else None, lp(Air) if self.p else None,
                                lp(Gjc), lp(Gir), lp(perm)), "qpb_plan_create")
        self._h = h
        self.info = QpbPlanInfo()
        check(L.qpb_plan_get_info(h, C.byref(self.info)), "qpb_plan_get_info")
        self.N = self.info.N
        self.perm = np.zeros(self.N, np.int64)
        check(L.qpb_plan_get_perm(h, self.perm.ctypes.data_as(C.POINTER(C.c_long))), "qpb_plan_get_perm")

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                _lib.lib().qpb_plan_destroy(h)
            except Exception:       # interpreter shutdown: the library may be gone
                pass
            self._h = None

    @classmethod
    def from_dense(cls, n, m, p, P, A, G, perm=None, p_upper=True, exact=False, kernel="auto", order="own"):
        """Plan for the non-zero pattern of one dense QP (P [n,n], A [p,n], G [m,n]).
        kernel: "auto" (wave kernel for small batches when eligible), "lane", "wave"
        (its row form -- four QPs per wavefront -- where the pattern fits a 16-lane
        row), "wave1" / "auto1" (as "wave" / "auto" but one QP per wavefront),
        "tree" (one QP per workgroup, level-scheduled sparse LDL'; any pattern).
        order: KKT ordering without `perm` (ORDER_FLAGS; "amd" = the reference's)."""
        Pjc, Pir = dense_pattern(P, upper=p_upper)
        Ajc, Air = dense_pattern(A) if p else (None, None)
        Gjc, Gir = dense_pattern(G)
        return cls(n, m, p, Pjc, Pir, Ajc, Air, Gjc, Gir, perm=perm, p_upper=p_upper, exact=exact, kernel=kernel,
                   order=order)

    # -- inspection ---------------------------------------------------------
    def source(self) -> str:
        L = _lib.lib()
        size = L.qpb_plan_source(self._h, None, 0)
        buf = C.create_string_buffer(size + 1)
        L.qpb_plan_source(self._h, buf, size + 1)
        return buf.value.decode()

    def kernel_for(self, B: int) -> str:
        """Which kernel qpb_solve runs for a batch of B ("wave", "lane" or "tree";
        the wave kernel's form is info.wave_qpw: 4 QPs per wavefront = row form)."""
        i = self.info
        if i.wave_ok and (i.wave_max_batch < 0 or B <= i.wave_max_batch):
            return "wave"
        return {1: "lane", 2: "wave", 3: "tree", 4: "band"}[i.large_kernel]

    def oracle_perm(self, B: int) -> np.ndarray:
        """The KKT permutation the kernels factor with (both kernels follow the
        plan's permutation; the oracle run with it is their arithmetic reference)."""
        return self.perm

    def wave_source(self) -> str:
        L = _lib.lib()
        size = L.qpb_plan_wave_source(self._h, None, 0)
        check(0 if size >= 0 else int(size), "qpb_plan_wave_source")
        buf = C.create_string_buffer(size + 1)
        L.qpb_plan_wave_source(self._h, buf, size + 1)
        return buf.value.decode()

    def tree_source(self) -> str:
        L = _lib.lib()
        size = L.qpb_plan_tree_source(self._h, None, 0)
        check(0 if size >= 0 else int(size), "qpb_plan_tree_source")
        buf = C.create_string_buffer(size + 1)
        L.qpb_plan_tree_source(self._h, buf, size + 1)
        return buf.value.decode()

    def tree_tables(self) -> bytes:
        """The tree kernel's plan tables (the device buffer it reads)."""
        L = _lib.lib()
        size = L.qpb_plan_tree_tables(self._h, None, 0)
        check(0 if size >= 0 else int(size), "qpb_plan_tree_tables")
        buf = C.create_string_buffer(max(size, 1))
        L.qpb_plan_tree_tables(self._h, buf, size)
        return buf.raw[:size]

    def compile(self, warm: bool = False, B: int = 1, serve: bool = False) -> bool:
        """Compile (or fetch from the code-object cache) the plan's kernels; warm:
        the warm-solve variant qpb_solve_warm launches for a batch of B; serve: the
        persistent forms of the one-QP kernel the drop-in's device solves use
        (False when that kernel has none)."""
        if serve:
            rc = _lib.lib().qpb_plan_compile_serve(self._h)
            check(min(rc, 0), "qpb_plan_compile_serve")
            return rc == 0
        if warm:
            check(_lib.lib().qpb_plan_compile_warm(self._h, int(B)), "qpb_plan_compile_warm")
        else:
            check(_lib.lib().qpb_plan_compile(self._h), "qpb_plan_compile")

    @property
    def nnz(self):
        return self.info.nnzP, self.info.nnzA, self.info.nnzG

    def bytes_per_qp(self) -> int:
        """Algorithmic HBM bytes per QP: inputs read once + outputs
        written once + flag/iteration words."""
        i = self.info
        ins = i.nnzP + i.nnzA + i.nnzG + i.n + i.m + i.p
        outs = i.n + i.p + 2 * i.m
        return 8 * (ins + outs) + 8

    # -- data ---------------------------------------------------------------
    def pack(self, P, A, G, c, h, b):
        """Dense numpy batches [B, ...] -> flat tiled-SoA numpy arrays for this
        plan (values at the plan's pattern positions, CSC order)."""
        (Pjc, Pir), (Ajc, Air), (Gjc, Gir) = self.patterns.P, self.patterns.A, self.patterns.G
        out = dict(P=to_tiled(_gather_values(np.asarray(P), Pjc, Pir)),
                   G=to_tiled(_gather_values(np.asarray(G), Gjc, Gir)),
                   c=to_tiled(np.asarray(c)), h=to_tiled(np.asarray(h)))
        if self.p:
            out["A"] = to_tiled(_gather_values(np.asarray(A), Ajc, Air))
            out["b"] = to_tiled(np.asarray(b))
        return out

    def alloc_outputs(self, B, device="cuda"):
        import torch
        T = ntiles(B) * TILE
        f = dict(dtype=torch.float64, device=device)
        return dict(x=torch.empty(self.n * T, **f), y=torch.empty(max(self.p, 1) * T, **f),
                    z=torch.empty(self.m * T, **f), s=torch.empty(self.m * T, **f),
                    flag=torch.empty(B, dtype=torch.int32, device=device),
                    iters=torch.empty(B, dtype=torch.int32, device=device),
                    fval=torch.empty(B, **f), stats=torch.empty(6 * T, **f))

    def assemble_contact(self, feet, wrench, stance=0xF, mu=0.5, B=None, out=None, stream=None):
        """On-device assembly of contact-force QPs (qpb_assemble_contact): feet
        [tiled nv=12] and wrench [tiled nv=6] float64 device tensors -> dict of the
        plan's tiled inputs P, A, G, c, h, b (device tensors, reused from `out`)."""
        import torch
        if B is None:
            B = wrench.numel() // 6
        B = int(B)
        T = ntiles(B) * TILE
        dev = wrench.device
        if out is None:
            f = dict(dtype=torch.float64, device=dev)
            out = dict(P=torch.empty(self.info.nnzP * T, **f), A=torch.empty(self.info.nnzA * T, **f),
                       G=torch.empty(self.info.nnzG * T, **f), c=torch.empty(self.n * T, **f),
                       h=torch.empty(self.m * T, **f), b=torch.empty(self.p * T, **f))
        if stream is None:
            stream = torch.cuda.current_stream(dev)
        ptr = lambda a: C.c_void_p(a.data_ptr())
        check(_lib.lib().qpb_assemble_contact(self._h, B, ptr(feet), ptr(wrench), int(stance), float(mu),
                                              ptr(out["P"]), ptr(out["A"]), ptr(out["G"]), ptr(out["c"]),
                                              ptr(out["h"]), ptr(out["b"]), C.c_void_p(stream.cuda_stream)),
              "qpb_assemble_contact")
        return out

    def assemble_controller(self, terms, B=None, shared=False, wdes=None, mu=0.5, out=None, check=None,
                            stream=None):
        """On-device assembly of the controller's stance QP 30/68/18
        (qpb_assemble_controller): terms = float64 device tensor of robot terms
        (tiled, nv = workloads.ROBOT_NV; or one shared copy with shared=True),
        wdes = optional tiled [nv = 6] per-QP desired wrench (e.g. from apf_wrench),
        check = optional int32 device tensor [B] (1: the QP has the plan's pattern).
        Returns the dict of the plan's tiled inputs P, A, G, c, h, b."""
        import torch
        if B is None:
            B = wdes.numel() // 6 if (shared and wdes is not None) else terms.numel() // 480
        B = int(B)
        T = ntiles(B) * TILE
        dev = terms.device
        if out is None:
            f = dict(dtype=torch.float64, device=dev)
            out = dict(P=torch.empty(self.info.nnzP * T, **f), A=torch.empty(self.info.nnzA * T, **f),
                       G=torch.empty(self.info.nnzG * T, **f), c=torch.empty(self.n * T, **f),
                       h=torch.empty(self.m * T, **f), b=torch.empty(self.p * T, **f))
        if stream is None:
            stream = torch.cuda.current_stream(dev)
        ptr = lambda a: None if a is None else C.c_void_p(a.data_ptr())
        check_(_lib.lib().qpb_assemble_controller(self._h, B, ptr(terms), int(bool(shared)), ptr(wdes), float(mu),
                                                  ptr(out["P"]), ptr(out["A"]), ptr(out["G"]), ptr(out["c"]),
                                                  ptr(out["h"]), ptr(out["b"]), ptr(check),
                                                  C.c_void_p(stream.cuda_stream)), "qpb_assemble_controller")
        return out

    def unpack(self, out, B):
        """Device tiled outputs -> dict of host numpy arrays [B, n] etc."""
        r = dict(x=from_tiled(out["x"], B, self.n).cpu().numpy(),
                 z=from_tiled(out["z"], B, self.m).cpu().numpy(),
                 s=from_tiled(out["s"], B, self.m).cpu().numpy(),
                 flag=out["flag"][:B].cpu().numpy(), iters=out["iters"][:B].cpu().numpy(),
                 fval=out["fval"][:B].cpu().numpy())
        r["y"] = from_tiled(out["y"], B, self.p).cpu().numpy() if self.p else np.zeros((B, 0))
        if out.get("stats") is not None:
            st = from_tiled(out["stats"], B, 6).cpu().numpy()
            for k, name in enumerate(("n_rx", "n_ry", "n_rz", "n_mu", "alpha_p", "alpha_d")):
                r[name] = st[:, k]
        return r

    def solve(self, P, G, c, h, A=None, b=None, B=None, reltol=1e-6, abstol=1e-6, maxit=100,
              sigma_d=0.0, out=None, stream=None):
        """Solve B QPs.  Inputs are flat tiled-SoA float64 arrays (torch device
        tensors, or numpy arrays which are uploaded).  Asynchronous on `stream`
        (torch stream or None = current stream)."""
        import torch
        dev = torch.device("cuda", torch.cuda.current_device())

        def t(a):
            if a is None:
                return None
            if isinstance(a, np.ndarray):
                a = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).to(dev)
            if not (a.dtype == torch.float64 and a.is_cuda and a.is_contiguous()):
                raise TypeError("inputs must be contiguous float64 device tensors")
            return a

        P, G, c, h, A, b = map(t, (P, G, c, h, A, b))
        if B is None:
            B = c.numel() // self.n
        B = int(B)
        T = ntiles(B) * TILE
        for name, a, nv in (("P", P, self.info.nnzP), ("G", G, self.info.nnzG), ("c", c, self.n),
                            ("h", h, self.m), ("A", A, self.info.nnzA), ("b", b, self.p)):
            if a is not None and nv and a.numel() < nv * T:
                raise ValueError(f"{name}: need {nv * T} values for B={B}, got {a.numel()}")
        if out is None:
            out = self.alloc_outputs(B, device=dev)
        st = QpbSettings(int(maxit), float(reltol), float(abstol), float(sigma_d))
        if stream is None:
            stream = torch.cuda.current_stream(dev)
        ptr = lambda a: None if a is None else C.c_void_p(a.data_ptr())
        check(_lib.lib().qpb_solve(self._h, B, ptr(P), ptr(A) if self.p else None, ptr(G), ptr(c), ptr(h),
                                   ptr(b) if self.p else None, C.byref(st), ptr(out["x"]),
                                   ptr(out["y"]) if self.p else None, ptr(out["z"]), ptr(out["s"]),
                                   ptr(out["flag"]), ptr(out["iters"]), ptr(out["fval"]),
                                   ptr(out.get("stats")), C.c_void_p(stream.cuda_stream)), "qpb_solve")
        return out


    def solve_warm(self, P, G, c, h, A=None, b=None, B=None, reltol=1e-6, abstol=1e-6, maxit=100,
                   sigma_d=0.0, out=None, sigma=None, stream=None):
        """Warm solve (qpb_solve_warm): continue every QP from out's x, y, z, s,
        iters and flag and from sigma (float64 device tensor [B], in/out), as a
        second QP_SOLVE on the same QP object does (qpSWIFT.c:502-596).  Inputs as
        solve(); `out` must hold the previous state."""
        import torch
        dev = torch.device("cuda", torch.cuda.current_device())

        def t(a):
            if a is None:
                return None
            if isinstance(a, np.ndarray):
                a = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).to(dev)
            return a

        P, G, c, h, A, b = map(t, (P, G, c, h, A, b))
        if B is None:
            B = c.numel() // self.n
        if out is None or sigma is None:
            raise ValueError("solve_warm needs the previous outputs and sigma")
        st = QpbSettings(int(maxit), float(reltol), float(abstol), float(sigma_d))
        if stream is None:
            stream = torch.cuda.current_stream(dev)
        ptr = lambda a: None if a is None else C.c_void_p(a.data_ptr())
        check(_lib.lib().qpb_solve_warm(self._h, int(B), ptr(P), ptr(A) if self.p else None, ptr(G), ptr(c), ptr(h),
                                        ptr(b) if self.p else None, C.byref(st), ptr(out["x"]),
                                        ptr(out["y"]) if self.p else None, ptr(out["z"]), ptr(out["s"]),
                                        ptr(out["flag"]), ptr(out["iters"]), ptr(out["fval"]),
                                        ptr(out.get("stats")), ptr(sigma), C.c_void_p(stream.cuda_stream)),
              "qpb_solve_warm")
        return out

    def launcher(self, vals, out, B, reltol=1e-6, abstol=1e-6, maxit=100, sigma_d=0.0, stream=None, best=None):
        """A zero-argument callable that launches qpb_solve on fixed device buffers
        with every C argument pre-built: one ctypes call per launch, so a Python
        loop of launches stays GPU-bound even for small batches.  With `best` (a
        float64 device tensor of >= 2) it calls qpb_solve_best: the batch's
        argmin {fval, index} lands in best[0:2]."""
        import torch
        if stream is None:
            stream = torch.cuda.current_stream()
        ptr = lambda a: None if a is None else C.c_void_p(a.data_ptr())
        st = QpbSettings(int(maxit), float(reltol), float(abstol), float(sigma_d))
        args = (self._h, int(B), ptr(vals["P"]), ptr(vals.get("A")) if self.p else None, ptr(vals["G"]),
                ptr(vals["c"]), ptr(vals["h"]), ptr(vals.get("b")) if self.p else None, C.byref(st),
                ptr(out["x"]), ptr(out["y"]) if self.p else None, ptr(out["z"]), ptr(out["s"]),
                ptr(out["flag"]), ptr(out["iters"]), ptr(out["fval"]), ptr(out.get("stats")))
        if best is not None:
            if best.numel() < 2 or best.dtype != torch.float64:
                raise ValueError("best must be a float64 device tensor of >= 2 elements")
            args = args + (ptr(best), C.c_void_p(stream.cuda_stream))
            fn = _lib.lib().qpb_solve_best
        else:
            args = args + (C.c_void_p(stream.cuda_stream),)
            fn = _lib.lib().qpb_solve
        keep = (vals, out, st, best)

        def go():
            rc = fn(*args)
            if rc:
                check(rc, "qpb_solve")
        go.keep = keep
        return go

    def kernel_name(self, B: int) -> str:
        """Name of the kernel qpb_solve launches for a batch of B."""
        L = _lib.lib()
        buf = C.create_string_buffer(128)
        check(0 if L.qpb_plan_kernel_name(self._h, int(B), buf, 128) >= 0 else -1, "qpb_plan_kernel_name")
        return buf.value.decode()


class PlanGroup:
    """Several row-form plans (e.g. one per gait phase) solved as ONE launch
    (qpb_group_solve, include/qpswift_hip.h): member i's QPs run the exact code
    of Plan.solve on plans[i], and with `best` the argmin over the concatenated
    batch (plans[0]'s QPs first) is reduced inside the same launch."""

    def __init__(self, plans):
        L = _lib.lib()
        self.plans = list(plans)
        hs = (C.c_void_p * len(self.plans))(*[p._h.value for p in self.plans])
        h = C.c_void_p()
        check(L.qpb_group_create(C.byref(h), hs, len(self.plans)), "qpb_group_create")
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                _lib.lib().qpb_group_destroy(h)
            except Exception:
                pass
            self._h = None

    def source(self) -> str:
        L = _lib.lib()
        size = L.qpb_group_source(self._h, None, 0)
        buf = C.create_string_buffer(size + 1)
        L.qpb_group_source(self._h, buf, size + 1)
        return buf.value.decode()

    def kernel_name(self) -> str:
        return self.source().split("\n", 1)[0].split()[-1]

    def compile(self) -> None:
        check(_lib.lib().qpb_group_compile(self._h), "qpb_group_compile")

    def launcher(self, vals, outs, Bs, reltol=1e-6, abstol=1e-6, maxit=100, sigma_d=0.0, stream=None, best=None):
        """Zero-argument callable launching qpb_group_solve on fixed device buffers:
        vals[i] / outs[i] as Plan.launcher's, Bs[i] QPs of member i."""
        import torch
        if not (len(vals) == len(outs) == len(Bs) == len(self.plans)):
            raise ValueError("one vals / outs / B per member plan")
        if stream is None:
            stream = torch.cuda.current_stream()
        ptr = lambda a: None if a is None else a.data_ptr()
        io = (QpbIo * len(self.plans))()
        for i, (pl, v, o, B) in enumerate(zip(self.plans, vals, outs, Bs)):
            io[i] = QpbIo(int(B), ptr(v["P"]), ptr(v.get("A")) if pl.p else None, ptr(v["G"]), ptr(v["c"]),
                          ptr(v["h"]), ptr(v.get("b")) if pl.p else None, ptr(o["x"]),
                          ptr(o["y"]) if pl.p else None, ptr(o["z"]), ptr(o["s"]), ptr(o["flag"]),
                          ptr(o["iters"]), ptr(o["fval"]), ptr(o.get("stats")))
        st = QpbSettings(int(maxit), float(reltol), float(abstol), float(sigma_d))
        if best is not None and (best.numel() < 2 or best.dtype != torch.float64):
            raise ValueError("best must be a float64 device tensor of >= 2 elements")
        args = (self._h, io, C.byref(st), None if best is None else C.c_void_p(best.data_ptr()),
                C.c_void_p(stream.cuda_stream))
        fn = _lib.lib().qpb_group_solve
        keep = (vals, outs, st, best, io)

        def go():
            rc = fn(*args)
            if rc:
                check(rc, "qpb_group_solve")
        go.keep = keep
        return go


def argmin_launcher(fval, flag, out, stream=None):
    """Pre-built qpb_argmin launch (see Plan.launcher)."""
    import torch
    if stream is None:
        stream = torch.cuda.current_stream(fval.device)
    fn = _lib.lib().qpb_argmin
    args = (int(fval.numel()), C.c_void_p(fval.data_ptr()), C.c_void_p(flag.data_ptr()),
            C.c_void_p(out.data_ptr()), C.c_void_p(stream.cuda_stream))

    def go():
        rc = fn(*args)
        if rc:
            check(rc, "qpb_argmin")
    go.keep = (fval, flag, out)
    return go


def argmin(fval, flag, out=None, stream=None):
    """Device-side (fval, index) of the lowest-fval optimal QP (qpb_argmin)."""
    import torch
    if out is None:
        out = torch.empty(2, dtype=torch.float64, device=fval.device)
    if stream is None:
        stream = torch.cuda.current_stream(fval.device)
    check(_lib.lib().qpb_argmin(fval.numel(), C.c_void_p(fval.data_ptr()), C.c_void_p(flag.data_ptr()),
                                C.c_void_p(out.data_ptr()), C.c_void_p(stream.cuda_stream)), "qpb_argmin")
    return out


def bucket_by_pattern(P, A, G):
    """Group dense QPs by their exact-zero pattern (config 3, mixed sparsity).
    Returns {key: index array}, key = (P mask, A mask, G mask) bytes."""
    B = P.shape[0]
    keys = {}
    mP = (np.asarray(P) != 0).reshape(B, -1)
    mA = (np.asarray(A) != 0).reshape(B, -1)
    mG = (np.asarray(G) != 0).reshape(B, -1)
    allm = np.concatenate([mP, mA, mG], 1)
    packed = np.packbits(allm, axis=1)
    uniq, inv = np.unique(packed, axis=0, return_inverse=True)
    for u in range(len(uniq)):
        keys[u] = np.nonzero(inv.reshape(-1) == u)[0]
    return keys


def apf_state(**kw) -> QpbApfState:
    """qpb_apf_state from keyword arrays (ee [4,2], com [6], com_vel [6], acc_des [6],
    des_orient [2], rob_foot [4], versor [4,2], lat_versor [2], R_wb [3,3], Mcom [6,6],
    mass, rep_field, min_exit, fake_crawl)."""
    st = QpbApfState()
    for name, _ in QpbApfState._fields_:
        if name not in kw:
            continue
        v = kw[name]
        if name in ("mass",):
            st.mass = float(v)
        elif name in ("rep_field", "min_exit", "fake_crawl"):
            setattr(st, name, int(bool(v)))
        else:
            flat = np.asarray(v, np.float64).reshape(-1)
            arr = getattr(st, name)
            if name in ("ee", "versor"):
                for i in range(4):
                    for j in range(2):
                        arr[i][j] = flat[2 * i + j]
            else:
                for i, x in enumerate(flat):
                    arr[i] = x
    return st


def apf_update(state: QpbApfState, h_prev, period_st: float) -> float:
    """qpb_apf_update: one gait step's robustness smoothing and fake_crawl
    (main.cpp:1273-1321), in place; returns robf_to_mean."""
    h = np.ascontiguousarray(h_prev, dtype=np.float64).reshape(4)
    mean = C.c_double(0.0)
    check(_lib.lib().qpb_apf_update(C.byref(state), h.ctypes.data_as(C.POINTER(C.c_double)), float(period_st),
                                    C.byref(mean)), "qpb_apf_update")
    return float(mean.value)


def apf_wrench(state: QpbApfState, targets, K=None, wrench=None, com_des=None, stream=None):
    """qpb_apf_wrench: APF-sampled targets (tiled nv = 2 float64 device tensor) ->
    desired CoM wrench (tiled nv = 6) [and CoMPosDes] per candidate."""
    import torch
    K = int(targets.numel() // 2 if K is None else K)
    T = ntiles(K) * TILE
    if wrench is None:
        wrench = torch.empty(6 * T, dtype=torch.float64, device=targets.device)
    if stream is None:
        stream = torch.cuda.current_stream(targets.device)
    p = lambda a: None if a is None else C.c_void_p(a.data_ptr())
    check(_lib.lib().qpb_apf_wrench(K, C.byref(state), p(targets), p(wrench), p(com_des),
                                    C.c_void_p(stream.cuda_stream)), "qpb_apf_wrench")
    return wrench

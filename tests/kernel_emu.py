"""CPU emulation of a generated IPM kernel -- TEST TOOL ONLY (never the product).

The generated kernels have no cross-lane communication (each lane owns one QP
and a private LDS column), so executing the kernel body once per lane on the
host is an exact emulation of its arithmetic.  The HIP source is compiled with
g++ after a handful of textual shims (builtins, thread ids, the opaque-offset
asm statements).  Exact-mode kernels must then be bit-identical to the oracle;
this lets the CPU suite validate code generation without a GPU.
"""
from __future__ import annotations

import ctypes as C
import hashlib
import os
import re
import subprocess
import tempfile

import numpy as np

PRELUDE = r"""
#include <cmath>
#include <cstring>
struct qpb_dim3 { unsigned x, y, z; };
static qpb_dim3 threadIdx, blockIdx;
#define __global__
#define __device__
#define __forceinline__ inline
#define __launch_bounds__(a, b)
#define __shared__ static
static inline double qpb_emu_rcp(double v) { return 1.0 / v; }
#define __builtin_amdgcn_rcp(v) qpb_emu_rcp(v)
#define __builtin_amdgcn_readfirstlane(v) (v)
#define __builtin_amdgcn_s_memrealtime() 0UL
"""

DRIVER = r"""
extern "C" void qpb_emu_run(qpb_args a, int wg, long B) {
  for (long q = 0; q < B; q++) {
    blockIdx.x = (unsigned)(q / wg); threadIdx.x = (unsigned)(q % wg);
    KERNEL(a);
  }
}
"""


class QpbArgs(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("P", "A", "G", "c", "h", "b", "x", "y", "z", "s", "flag", "iters",
                                          "fval", "stats")] + \
               [("B", C.c_long), ("tol", C.c_double), ("abstol", C.c_double), ("sigma_d", C.c_double),
                ("maxit", C.c_long)] + [(n, C.c_void_p) for n in ("tab", "best", "part", "ctr", "sig")] + \
               [("warm", C.c_long), ("trace", C.c_void_p)]


def build_emulator(src: str, exact: bool, cache_dir=None):
    kname = re.search(r"void __launch_bounds__\([^)]*\) (\w+)\(qpb_args a\)", src).group(1)
    wg = int(re.search(r"__launch_bounds__\((\d+),", src).group(1))
    body = re.sub(r'asm volatile\(""\s*:\s*"\+v"\((\w+)\)\);', r"(void)\1;", src)
    body = body.replace('extern "C" ', "")
    code = PRELUDE + body + DRIVER.replace("KERNEL", kname)
    h = hashlib.sha1((code + str(exact)).encode()).hexdigest()[:16]
    d = cache_dir or os.path.join(tempfile.gettempdir(), "qpb_emu")
    os.makedirs(d, exist_ok=True)
    so = os.path.join(d, f"emu_{h}.so")
    if not os.path.exists(so):
        cpp = os.path.join(d, f"emu_{h}.cpp")
        open(cpp, "w").write(code)
        flags = ["-O1", "-ffp-contract=off"] if exact else ["-O1", "-ffp-contract=fast"]
        subprocess.run(["g++", "-std=c++17", "-shared", "-fPIC", "-w", *flags, "-o", so, cpp], check=True)
    lib = C.CDLL(so)
    lib.qpb_emu_run.argtypes = [QpbArgs, C.c_int, C.c_long]
    lib.qpb_emu_run.restype = None
    return lib, wg


def emulate(plan, vals, B, reltol=1e-6, abstol=1e-6, maxit=100, sigma_d=0.0, warm=None):
    """Run plan's generated kernel on the CPU for B QPs (tiled numpy inputs).
    warm = the `out` dict of a previous call plus "sigma" ([B]): a warm solve
    (qpb_solve_warm) continuing from it, updated in place and returned."""
    from apf_quadruped_amd.batch import TILE, ntiles
    # the warm variant is the same source with QPB_WARM = 1 (qpb_solve_warm)
    lib, wg = build_emulator(("#define QPB_WARM 1\n" if warm is not None else "") + plan.source(), plan.exact)
    T = ntiles(B) * TILE
    keep = {k: np.ascontiguousarray(v, dtype=np.float64) for k, v in vals.items()}
    out = warm if warm is not None else \
        dict(x=np.zeros(plan.n * T), y=np.zeros(max(plan.p, 1) * T), z=np.zeros(plan.m * T),
             s=np.zeros(plan.m * T), flag=np.zeros(B, np.int32), iters=np.zeros(B, np.int32),
             fval=np.zeros(B), stats=np.zeros(6 * T))
    a = QpbArgs()
    for k in ("P", "A", "G", "c", "h", "b"):
        setattr(a, k, keep[k].ctypes.data if k in keep else None)
    for k in ("x", "y", "z", "s", "flag", "iters", "fval", "stats"):
        setattr(a, k, out[k].ctypes.data)
    if warm is not None:
        a.sig = warm["sigma"].ctypes.data
        a.warm = 1
    a.B, a.tol, a.abstol, a.sigma_d, a.maxit = B, reltol / np.sqrt(3.0), abstol, sigma_d, maxit
    lib.qpb_emu_run(a, wg, B)
    return out

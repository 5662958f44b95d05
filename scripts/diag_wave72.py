"""Diagnose the leaves-first wave-kernel NaN under the pinned
ROCm 7.2 clang: one child process per compile variant (a process keeps one code
object per kernel name), each solving trot / stance / crawl controller QPs in
leaves-first order on the wave kernel and comparing with the oracle run in the
same order.

    python scripts/diag_wave72.py                 # all variants
    python scripts/diag_wave72.py child <variant> # one variant (internal)
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VARIANTS = {
    "base": {},
    "O1": {"QPB_CLANG_FLAGS": "-O1"},
    "O2": {"QPB_CLANG_FLAGS": "-O2"},
    "mfma_pad": {"QPB_CLANG_FLAGS": "-mllvm -amdgpu-mfma-padding-ratio=100"},
    "mfma_vgpr": {"QPB_CLANG_FLAGS": "-mllvm -amdgpu-mfma-vgpr-form=1"},
    "no_dppcomb": {"QPB_CLANG_FLAGS": "-mllvm -amdgpu-dpp-combine=0"},
    "mfma_off": {"QPB_WAVE_OPTS": "QPB_W_MFMA=0"},
    "ldsb_off": {"QPB_WAVE_OPTS": "QPB_W_LDSB=0"},
    "ltlds_off": {"QPB_WAVE_OPTS": "QPB_W_LTLDS=0"},
}


def child(variant):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import torch  # noqa: F401  (device memory for Plan.solve)
    from apf_quadruped_amd import workloads as W, plans, _lib
    from apf_quadruped_amd.batch import Plan
    from oracle_py import Oracle
    o = Oracle()
    res = {"variant": variant, "compiler": _lib.lib().qpb_compiler().decode().split("\n")[0]}
    B = 64
    for phase, seed in (("trot", plans.SEED + 31), ("stance", plans.SEED + 30), ("crawl", plans.SEED + 31)):
        d = (W.controller_qp(seed, np.arange(B)) if phase == "stance"
             else W.controller_qp(seed, np.arange(B), phase=phase))
        n, m, p = 30, d["m"], d["p"]
        pl = Plan.from_dense(n, m, p, d["P"][0], d["A"][0], d["G"][0], kernel="wave1", order="leaves")
        out = pl.unpack(pl.solve(**pl.pack(d["P"], d["A"], d["G"], d["c"], d["h"], d["b"]), B=B), B)
        worst, nbad = 0.0, 0
        for q in range(0, B, 8):
            ref = o.solve_dense(n, m, p, W.to_colmajor(d["P"])[q], W.to_colmajor(d["A"])[q],
                                W.to_colmajor(d["G"])[q], d["c"][q], d["h"][q], d["b"][q], perm=pl.perm)
            dx = float(np.abs(out["x"][q] - ref["x"]).max())
            worst = max(worst, dx if np.isfinite(dx) else np.inf)
            nbad += int(out["flag"][q] != ref["flag"] or not np.isfinite(dx) or dx > 1e-6)
        res[phase] = {"max_dx": worst, "bad": nbad, "nan": int(np.isnan(out["x"]).any()),
                      "kernel": pl.kernel_name(B)}
    print(json.dumps(res), flush=True)


def main():
    names = sys.argv[1:] or list(VARIANTS)
    for v in names:
        env = dict(os.environ, **VARIANTS[v])
        r = subprocess.run([sys.executable, __file__, "child", v], env=env, capture_output=True, text=True,
                           timeout=300)
        line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else f'{{"variant": "{v}", "rc": {r.returncode}}}'
        print(line, flush=True)
        if r.returncode != 0:
            print(r.stderr[-2000:], flush=True)
            if r.returncode < 0 or r.returncode in (124, 134, 137, 139):
                break


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "child":
        child(sys.argv[2])
    else:
        main()

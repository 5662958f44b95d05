"""Diagnose the leaves-first wave-kernel NaN (DESIGN_HISTORY §7 item 4) under the pinned
ROCm 7.2 clang: one child process per compile variant (a process keeps one code
object per kernel name), each solving trot / stance / crawl controller QPs in
leaves-first order on the wave kernel and comparing with the oracle run in the
same order.

    python scripts/diag_wave72.py                 # all variants
    python scripts/diag_wave72.py child <variant> # one variant (internal)
    python scripts/diag_wave72.py bisect LO HI     # -mllvm -opt-bisect-limit search (trot only)
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
    # round 2, after the opt-bisect found amdgpu-pre-ra-optimizations as the first bad pass
    "no_prera": {"QPB_CLANG_FLAGS": "-mllvm -amdgpu-enable-pre-ra-optimizations=0"},
    "ldsb_sync": {"QPB_WAVE_OPTS": "QPB_W_LDSB_SYNC=1"},
    "no_postra_sched": {"QPB_CLANG_FLAGS": "-mllvm -disable-post-ra"},
    "no_dce_in_ra": {"QPB_CLANG_FLAGS": "-mllvm -amdgpu-dce-in-ra=0"},
    "sgpr_ra_fast": {"QPB_CLANG_FLAGS": "-mllvm -sgpr-regalloc=fast"},
    "no_prealloc_spill": {"QPB_CLANG_FLAGS": "-mllvm -amdgpu-prealloc-sgpr-spill-vgprs=0"},
    # the row kernel's parked fault (illegal address with all three knobs on)
    "row_knobs": {"QPB_WAVE_OPTS": "QPB_R_ZF128=1 QPB_R_AADPP=1 QPB_R_LATEFAC=1", "QPB_DIAG_PHASES": "c1row"},
    # round 3: the workaround off, with / without the DPP wait-state padding (qpb_hazard.cpp)
    "prera_on": {},
    "prera_on_unpadded": {"QPB_NO_ASM_FIXUP": "1"},
    "prera_on_opq0": {"QPB_WAVE_OPTS": "QPB_W_OPQ=0"},
    "prera_on_opq0_h0re0": {"QPB_WAVE_OPTS": "QPB_W_OPQ=0 QPB_W_H0RE=0"},
    "prera_off_opq0": {"QPB_PRERA_OFF": "1", "QPB_WAVE_OPTS": "QPB_W_OPQ=0"},
    "prera_on_dup0": {"QPB_WAVE_OPTS": "QPB_W_DUP=0"},
    "prera_on_dup0_opq0": {"QPB_WAVE_OPTS": "QPB_W_DUP=0 QPB_W_OPQ=0"},
    "prera_off_dup0_opq0": {"QPB_PRERA_OFF": "1", "QPB_WAVE_OPTS": "QPB_W_DUP=0 QPB_W_OPQ=0"},
    "padded": {"QPB_PRERA_OFF": "1"},
    "unpadded": {"QPB_PRERA_OFF": "1", "QPB_NO_ASM_FIXUP": "1"},
    "maxit0": {"QPB_DIAG_MAXIT": "0"},
    "maxit1": {"QPB_DIAG_MAXIT": "1"},
    "maxit2": {"QPB_DIAG_MAXIT": "2"},
}


def child(variant, phases=("trot", "stance", "crawl")):
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
    if os.environ.get("QPB_DIAG_PHASES"):
        phases = tuple(os.environ["QPB_DIAG_PHASES"].split(","))
    for phase, seed in (("trot", plans.SEED + 31), ("stance", plans.SEED + 30), ("crawl", plans.SEED + 31),
                        ("c1row", plans.SEED + 1)):
        if phase not in phases:
            continue
        if phase == "c1row":                 # C1 contact-force QPs on the row kernel, B = 1024
            B = 1024
            d = W.contact_force_qp(seed, np.arange(B))
            n, m, p = 12, 20, 6
            pl = Plan.from_dense(n, m, p, d["P"][0], d["A"][0], d["G"][0], kernel="wave")
        else:
            d = (W.controller_qp(seed, np.arange(B)) if phase == "stance"
                 else W.controller_qp(seed, np.arange(B), phase=phase))
            n, m, p = 30, d["m"], d["p"]
            pl = Plan.from_dense(n, m, p, d["P"][0], d["A"][0], d["G"][0], kernel="wave1", order="leaves")
        maxit = int(os.environ.get("QPB_DIAG_MAXIT", "100"))
        out = pl.unpack(pl.solve(**pl.pack(d["P"], d["A"], d["G"], d["c"], d["h"], d["b"]), B=B, maxit=maxit), B)
        worst, nbad = 0.0, 0
        for q in range(0, B, B // 8):
            ref = o.solve_dense(n, m, p, W.to_colmajor(d["P"])[q], W.to_colmajor(d["A"])[q],
                                W.to_colmajor(d["G"])[q], d["c"][q], d["h"][q], d["b"][q], perm=pl.perm, maxit=maxit)
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


def bisect(lo, hi):
    """lo: a limit known good, hi: known bad.  Each probe runs in a child under
    its own timeout; a compile failure shifts the probe by a few passes."""
    def probe(n):
        for shift in (0, 7, 19, 41):
            env = dict(os.environ, QPB_CLANG_FLAGS=f"-mllvm -opt-bisect-limit={n + shift}")
            try:
                r = subprocess.run([sys.executable, __file__, "childtrot", f"lim{n + shift}"], env=env,
                                   capture_output=True, text=True, timeout=90)
            except subprocess.TimeoutExpired:
                print(f"probe {n + shift}: TIMEOUT -- stopping", flush=True)
                sys.exit(3)
            if r.returncode == 0 and r.stdout.strip():
                res = json.loads(r.stdout.strip().splitlines()[-1])["trot"]
                good = res["bad"] == 0
                print(f"probe {n + shift}: {'good' if good else 'BAD'} max_dx {res['max_dx']:.3e}", flush=True)
                return n + shift, good
            if r.returncode < 0 or r.returncode in (124, 134, 137, 139) or "ECOMPILE" not in r.stderr + r.stdout \
                    and "clang" not in r.stderr:
                print(f"probe {n + shift}: rc {r.returncode} -- stopping\n{r.stderr[-1500:]}", flush=True)
                sys.exit(4)
            print(f"probe {n + shift}: compile failed, shifting", flush=True)
        sys.exit(5)
    while hi - lo > 1:
        mid = (lo + hi) // 2
        n, good = probe(mid)
        if good:
            lo = n
        else:
            hi = min(hi, n)
        print(f"range [{lo}, {hi}]", flush=True)
    print(f"FIRST BAD PASS: {hi}", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "child":
        child(sys.argv[2])
    elif len(sys.argv) > 2 and sys.argv[1] == "childtrot":
        child(sys.argv[2], phases=("trot",))
    elif len(sys.argv) > 3 and sys.argv[1] == "bisect":
        bisect(int(sys.argv[2]), int(sys.argv[3]))
    else:
        main()

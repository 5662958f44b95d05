"""Could the drop-in solve on the device in the leaves-first order instead of the AMD
order the reference uses (Permut = NULL)?  The leaves-first wave kernel is ~1.7x faster
per iteration on the 30-variable controller QPs (profiles/r04_wave_abl.jsonl), but the
order decides which y pivots are regularised (ldl.c:273-274), so the iterates differ by
more than rounding.  CPU only: the oracle (the reference's algorithm) in the leaves-first
order against the reference's AMD-ordered goldens -- flag / iteration mismatches and the
largest relative x/y/z/s difference (per vector).  Output: profiles/r04_order_equiv.jsonl.

    python scripts/order_equiv.py > profiles/r04_order_equiv.jsonl
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from oracle_py import Oracle  # noqa: E402
from apf_quadruped_amd.batch import Plan  # noqa: E402

NAMES = ["c1_tol1e-6", "c1_tol1e-2", "c30_tol1e-6", "c30_tol1e-2", "c30_trot_tol1e-6", "c30_trot_tol1e-2",
         "c30_crawl_tol1e-6", "c30_crawl_tol1e-2", "mixed_stance4", "mixed_crawl_blflfr", "mixed_trot_brfl",
         "mixed_trot_blfr"]


def main():
    o = Oracle()
    F = lambda M, r, c: np.asarray(M).reshape(r, c, order="F")
    for name in NAMES:
        g = np.load(os.path.join(ROOT, "tests/golden", name + ".npz"))
        n, m, p = int(g["n"]), int(g["m"]), int(g["p"])
        tol, maxit = float(g["tol"]), int(g["maxit"])
        mism, worst, per = 0, 0.0, {}
        for q in range(g["x"].shape[0]):
            A = F(g["A"][q], p, n) if p else np.zeros((0, n))
            pl = Plan.from_dense(n, m, p, F(g["P"][q], n, n), A, F(g["G"][q], m, n), kernel="wave", order="own")
            r = o.solve_dense(n, m, p, g["P"][q], g["A"][q] if p else None, g["G"][q], g["c"][q], g["h"][q], g["b"][q],
                              perm=pl.perm, ordering=int(g["ordering"]), reltol=tol, abstol=tol, maxit=maxit)
            mism += int(r["iters"] != int(g["iters"][q]) or r["flag"] != int(g["flag"][q]))
            for k in ("x", "z", "s") + (("y",) if p else ()):
                d = float(np.max(np.abs(r[k] - g[k][q])) / max(1.0, np.max(np.abs(g[k][q]))))
                per[k] = max(per.get(k, 0.0), d)
                worst = max(worst, d)
        print(json.dumps({"golden": name, "n": n, "m": m, "p": p, "qps": int(g["x"].shape[0]), "tol": tol,
                          "iter_or_flag_mismatches": mism, "max_rel_diff": worst, "per_vector": per, "within_1e-6": worst <= 1e-6}))


if __name__ == "__main__":
    main()

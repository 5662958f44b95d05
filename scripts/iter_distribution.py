"""Iteration-count distribution of the synthetic C1 QPs (the oracle run in the
reference's arithmetic, tol 1e-6) and what it means for a wave that holds four
QPs (the row kernel): the wave runs to the slowest of its four.  Analysis only
(the oracle is the checker, never the product).

    python scripts/iter_distribution.py [B] > profiles/r02_iter_distribution.json
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    from apf_quadruped_amd import plans
    from oracle_py import Oracle
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    q = plans.standard_qp("c1", np.arange(B))
    cm = lambda M: np.ascontiguousarray(np.swapaxes(M, 1, 2)).reshape(M.shape[0], -1)
    _, flags, it = Oracle().solve_dense_batch(q["n"], q["m"], q["p"], cm(q["P"]), cm(q["A"]), cm(q["G"]),
                                              q["c"], q["h"], q["b"], threads=os.cpu_count() or 1)
    res = {"qps": B, "tol": 1e-6, "optimal_frac": float((flags == 0).mean()),
           "histogram": {int(k): int(v) for k, v in enumerate(np.bincount(it)) if v},
           "mean_iters": float(it.mean())}
    for per_wave in (4, 64):
        w = it[: B // per_wave * per_wave].reshape(-1, per_wave).max(1)
        res[f"mean_max_of_{per_wave}"] = float(w.mean())
        res[f"lockstep_overhead_{per_wave}"] = float(w.mean() / it.mean())
    for b in (1024,):
        res[f"max_over_batch_{b}"] = [int(it[s:s + b].max()) for s in range(0, min(B, 8 * b), b)]
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

"""Compile (no GPU) the wide row kernels of the rowx tests and benches into the in-tree
kcache, so GPU runs find them: python scripts/rowx_precompile.py [--all]"""
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
import sys, numpy as np, os
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'tests'))
from rowx_cases import dense_qp
from apf_quadruped_amd import plans, workloads as W
from apf_quadruped_amd.batch import Plan
def P(d, **kw):
    return Plan.from_dense(d["n"], d["m"], d["p"], d["P"][0], d["A"][0] if d["p"] else None, d["G"][0], p_upper=False, **kw)
for ph in ("stance","trot","crawl"):
    d = W.controller_qp(plans.SEED + 30, np.arange(1), phase=ph)
    P(d).compile()
    Plan.from_dense(30, d["m"], d["p"], d["P"][0], d["A"][0], d["G"][0]).compile()
    Plan.from_dense(30, d["m"], d["p"], d["P"][0], d["A"][0], d["G"][0], order="own").compile()
if "--all" in sys.argv:
    for (n,m,p) in [(20, 40, 10), (32, 48, 16), (17, 33, 0), (12, 40, 6), (16, 20, 20), (30, 24, 30)]:
        P(dense_qp(n, m, p, B=1, seed=n * 1000 + m * 10 + p)).compile()
    P(dense_qp(24, 40, 8, B=1, seed=5, zero_var=3)).compile()
print("ok")
if "--all" in sys.argv:
    # round 6: upper-triangle P past 16 variables (tests/test_gpu_rowx.py, tests/test_gpu_limits.py)
    from test_gpu_limits import random_qps
    for (n, m, p) in [(17, 20, 6), (32, 48, 16)]:
        d = random_qps(n, m, p, 1, seed=1000 * n + m + p)
        Plan.from_dense(n, m, p, d["P"][0], d["A"][0], d["G"][0], kernel="wave").compile()
    for (n, m, p), off, lin in [((24, 40, 8), 16, None), ((20, 40, 10), 16, None), ((30, 68, 18), 16, None),
                                ((17, 20, 6), 0, None), ((24, 40, 8), 0, None), ((17, 40, 5), 0, 16)]:
        d = dense_qp(n, m, p, B=1, seed=7 * n + m, p_offdiag_from=off, linear_var=lin)
        Plan.from_dense(n, m, p, d["P"][0], d["A"][0], d["G"][0], p_upper=True, kernel="wave").compile()
    print("ok (upper P)")

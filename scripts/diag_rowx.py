"""Diagnostic: the wide row kernel on one synthetic shape, repeated, vs the oracle (the
QPs whose flags / iterations differ).  python scripts/diag_rowx.py n m p [compile]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    if not (len(sys.argv) > 4 and sys.argv[4] == "compile"):
        import torch  # noqa: F401  (before the library: HIP initialised by torch first)
    from rowx_cases import dense_qp
    from apf_quadruped_amd.batch import Plan, _gather_values
    n, m, p = (int(v) for v in sys.argv[1:4])
    B = 70
    d = dense_qp(n, m, p, B=B, seed=n * 1000 + m * 10 + p)
    plan = Plan.from_dense(n, m, p, d["P"][0], d["A"][0] if p else None, d["G"][0], p_upper=False)
    if len(sys.argv) > 4 and sys.argv[4] == "compile":
        plan.compile()
        print(plan.kernel_name(B))
        return
    import torch
    from oracle_py import Oracle
    o = Oracle()
    vals = {k: torch.from_numpy(v).cuda() for k, v in plan.pack(d["P"], d["A"] if p else None, d["G"], d["c"], d["h"],
                                                                d["b"] if p else None).items()}
    (Pjc, Pir), (Gjc, Gir) = plan.patterns.P, plan.patterns.G
    Pv, Gv = _gather_values(d["P"], Pjc, Pir), _gather_values(d["G"], Gjc, Gir)
    Ajc, Air = plan.patterns.A if p else (None, None)
    Av = _gather_values(d["A"], Ajc, Air) if p else None
    ref = [o.solve_csc(n, m, p, Pjc, Pir, Pv[q], Ajc, Air, Av[q] if p else None, Gjc, Gir, Gv[q], d["c"][q], d["h"][q],
                       d["b"][q] if p else None, perm=plan.perm) for q in range(B)]
    for rep in range(3):
        r = plan.unpack(plan.solve(**vals, B=B), B)
        diff = [q for q in range(B) if ref[q]["flag"] != r["flag"][q] or ref[q]["iters"] != r["iters"][q]]
        print(os.environ.get("QPB_WAVE_OPTS", ""), (n, m, p), rep, plan.kernel_name(B), "differ:", diff, flush=True)


if __name__ == "__main__":
    main()

"""Diagnostic: the setup factor's pivots D of the wide row kernel (QPB_X_DBG=1) against a
numpy LDL' of H = P + 1e7 A'A + G'G in natural order.  python scripts/diag_rowx_d.py n m p [compile]"""
import os
import sys

import numpy as np

DBG = int(os.environ.get("DBG", "1"))
os.environ["QPB_WAVE_OPTS"] = (os.environ.get("QPB_WAVE_OPTS", "") + f" QPB_X_DBG={DBG}").strip()
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def ldl_d(H):
    H = H.copy()
    n = len(H)
    D = np.zeros(n)
    for k in range(n):
        D[k] = H[k, k]
        for i in range(k + 1, n):
            l = H[i, k] / D[k]
            H[i, k + 1:] -= l * H[k, k + 1:]
    return D


def main():
    comp = len(sys.argv) > 4 and sys.argv[4] == "compile"
    if not comp:
        import torch  # noqa: F401
    from rowx_cases import dense_qp
    from apf_quadruped_amd.batch import Plan
    n, m, p = (int(v) for v in sys.argv[1:4])
    B = 8
    d = dense_qp(n, m, p, B=B, seed=n * 1000 + m * 10 + p)
    plan = Plan.from_dense(n, m, p, d["P"][0], d["A"][0] if p else None, d["G"][0], p_upper=False)
    if comp:
        plan.compile()
        print(plan.kernel_name(B))
        return
    import torch
    vals = {k: torch.from_numpy(v).cuda() for k, v in plan.pack(d["P"], d["A"] if p else None, d["G"], d["c"], d["h"],
                                                                d["b"] if p else None).items()}
    if DBG == 0:                    # residual statistics after maxit passes (stats output)
        for mi in (3, 4, 5, 6):
            r = plan.unpack(plan.solve(**vals, B=B, maxit=mi), B)
            for q in range(3):
                print(os.environ["QPB_WAVE_OPTS"], "maxit", mi, q, int(r["flag"][q]), int(r["iters"][q]),
                      " ".join(f"{r[k][q]:.6e}" for k in ("n_rx", "n_ry", "n_rz", "n_mu", "alpha_p", "alpha_d")),
                      flush=True)
        return
    r = plan.unpack(plan.solve(**vals, B=B), B)
    for q in range(B):
        H = d["P"][q] + 1e7 * d["A"][q].T @ d["A"][q] + d["G"][q].T @ d["G"][q]
        if DBG >= 3:                # the iterate after DBG - 2 passes: printed, compared across builds
            print(os.environ["QPB_WAVE_OPTS"], q, int(r["flag"][q]), " ".join(f"{v:.17g}" for v in r["x"][q][:4]))
            continue
        if DBG == 1:
            D = ldl_d(H)
        else:                       # x0 of kkt_initialize: H x = -c + G'h + 1e7 A'b
            D = np.linalg.solve(H, -d["c"][q] + d["G"][q].T @ d["h"][q] + (1e7 * d["A"][q].T @ d["b"][q] if p else 0))
        rel = np.abs(r["x"][q] - D) / np.abs(D).max()
        print(os.environ["QPB_WAVE_OPTS"], q, int(r["flag"][q]), "max rel", float(rel.max()), "at", int(rel.argmax()),
              flush=True)


if __name__ == "__main__":
    main()

"""One random dense QP batch through Plan.from_dense and the oracle (the case of
tests/test_gpu_limits.py), with the P storage selectable -- to isolate a failing
plan outside pytest: python scripts/diag_rowx_case.py n m p [full|upper] [B]."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from test_gpu_limits import random_qps, _colmajor  # noqa: E402


def main():
    n, m, p = (int(v) for v in sys.argv[1:4])
    upper = (sys.argv[4] if len(sys.argv) > 4 else "upper") == "upper"
    B = int(sys.argv[5]) if len(sys.argv) > 5 else 5
    torch.zeros(1, device="cuda")
    from apf_quadruped_amd.batch import Plan
    from oracle_py import Oracle
    d = random_qps(n, m, p, B, seed=1000 * n + m + p)
    plan = Plan.from_dense(n, m, p, d["P"][0], d["A"][0], d["G"][0], p_upper=upper)
    print("kernel", plan.kernel_name(B), "upper", upper, flush=True)
    vals = plan.pack(d["P"], d["A"], d["G"], d["c"], d["h"], d["b"])
    r = plan.unpack(plan.solve(**vals, B=B, reltol=1e-6, abstol=1e-6), B)
    torch.cuda.synchronize()
    o_ = Oracle()
    Pc, Ac, Gc = _colmajor(d["P"]), _colmajor(d["A"]), _colmajor(d["G"])
    worst = 0.0
    for q in range(B):
        o = o_.solve_dense(n, m, p, Pc[q], Ac[q], Gc[q], d["c"][q], d["h"][q], d["b"][q], perm=plan.perm,
                           reltol=1e-6, abstol=1e-6)
        assert r["flag"][q] == o["flag"] and r["iters"][q] == o["iters"], (q, r["flag"][q], o["flag"])
        for k in ("x", "y", "z", "s"):
            worst = max(worst, float(np.abs(r[k][q] - o[k]).max()) / max(1.0, float(np.abs(o[k]).max())))
    print("ok worst rel", worst, flush=True)


if __name__ == "__main__":
    main()

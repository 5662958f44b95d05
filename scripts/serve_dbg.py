"""Drop-in trot golden, QP by QP: iterations and max |x - golden| with the
persistent solver, in file order and QP 1 alone first (debug of a mismatch)."""
import os, sys, json
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from apf_quadruped_amd import dropin
g = np.load(os.path.join(ROOT, "tests/golden/mixed_trot_brfl.npz"))
n, m, p = int(g["n"]), int(g["m"]), int(g["p"])
tol, maxit = float(g["tol"]), int(g["maxit"])
order = [int(v) for v in sys.argv[1].split(",")] if len(sys.argv) > 1 else list(range(g["x"].shape[0]))
for q in order:
    # QP_SETUP (its initial point is the cold wave's answer), then QP_SOLVE (the warm wave)
    qp, keep = dropin.setup_dense(n, m, p, g["P"][q], g["A"][q], g["G"][q], g["c"][q], g["h"][q], g["b"][q],
                                  ordering=int(g["ordering"]))
    s0 = dropin.state(qp, n, m)
    r = dropin.solve_again(qp, n, m, reltol=tol, abstol=tol, maxit=maxit)
    dropin._lib.lib().QP_CLEANUP_dense(qp)
    dx = float(np.abs(r["x"] - g["x"][q]).max())
    print(json.dumps({"q": q, "ok": bool(dx < 1e-6 and r["iters"] == int(g["iters"][q])), "flag": r["flag"], "iters": r["iters"], "g_iters": int(g["iters"][q]),
                      "dx": dx, "dz": float(np.abs(r["z"] - g["z"][q]).max()),
                      "init": [float(np.abs(s0[k]).sum()) for k in ("x", "y", "z", "s")] + [s0["sigma"]]}))
import ctypes as C
from apf_quadruped_amd import _lib
st = (C.c_long * 4)()
_lib.lib().qpb_dropin_serve_stats(st)
print(json.dumps({"serve_requests": int(st[0]), "serve_launches": int(st[1])}))

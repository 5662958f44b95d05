"""QP_SETUP only (the cold persistent wave's kkt_initialize), QP by QP over the trot
drop-in golden, no QP_SOLVE in between: each QP's initial point as |.|-sums (compare
across modes; the one-request-per-wave mode is the reference)."""
import os, sys, json
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from apf_quadruped_amd import dropin
g = np.load(os.path.join(ROOT, "tests/golden/mixed_trot_brfl.npz"))
n, m, p = int(g["n"]), int(g["m"]), int(g["p"])
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 1
for rep in range(reps):
    for q in range(g["x"].shape[0]):
        qp, keep = dropin.setup_dense(n, m, p, g["P"][q], g["A"][q], g["G"][q], g["c"][q], g["h"][q], g["b"][q],
                                      ordering=int(g["ordering"]))
        s0 = dropin.state(qp, n, m)
        dropin._lib.lib().QP_CLEANUP_dense(qp)
        print(json.dumps({"rep": rep, "q": q, "init": [float(np.abs(s0[k]).sum()) for k in ("x", "y", "z", "s")]}))

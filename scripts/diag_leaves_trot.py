"""Leaves-first trot QP: optimal share per launch for B in (64, 256, 1024), first a
fresh output each launch, then five launches into one reused output."""
import sys
import numpy as np
sys.path.insert(0, "/root/repo")
import torch  # noqa: E402
from apf_quadruped_amd import workloads as W, plans  # noqa: E402
from apf_quadruped_amd.batch import Plan  # noqa: E402
for B in (64, 256, 1024):
    d = W.controller_qp(plans.SEED + 31, np.arange(B), phase="trot")
    n, m, pp = 30, d["m"], d["p"]
    lf = np.array(list(range(n + pp, n + pp + m)) + list(range(n, n + pp)) + list(range(n)))
    p = Plan.from_dense(30, m, pp, d["P"][0], d["A"][0], d["G"][0], kernel="wave", perm=lf)
    vals = {k: torch.from_numpy(v).cuda() for k, v in p.pack(d["P"], d["A"], d["G"], d["c"], d["h"], d["b"]).items()}
    fresh = [float((p.unpack(p.solve(**vals, B=B), B)["flag"] == 0).mean()) for _ in range(3)]
    out = p.alloc_outputs(B, device="cuda")
    reuse = []
    for _ in range(5):
        p.solve(**vals, B=B, out=out)
        r = p.unpack(out, B)
        reuse.append((float((r["flag"] == 0).mean()), int(np.isnan(r["x"]).any(1).sum())))
    print("B", B, "fresh", fresh, "reuse(opt, nan rows)", reuse, flush=True)

"""Kernel-only latency of small batches (HIP events around back-to-back
qpb_solve launches on resident inputs): what the drop-in's per-call time is made
of, without the host copies.

    python scripts/lat_bench.py c30:amd:1 c30:own:1 c1:own:1 ...   (name:order:B[:tol[:kernel[:maxit]]]; tol 0 + maxit = a fixed iteration count)"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
from tree_bench import qp  # noqa: E402


def main():
    import torch
    from apf_quadruped_amd.batch import Plan
    for case in sys.argv[1:]:
        f = case.split(":")
        name, order, B = f[0], f[1] or "own", int(f[2])
        tol = float(f[3]) if len(f) > 3 and f[3] else 1e-2
        kernel = f[4] if len(f) > 4 and f[4] else "auto"
        maxit = int(f[5]) if len(f) > 5 else 100
        d = qp(name, np.arange(B))
        plan = Plan.from_dense(d["n"], d["m"], d["p"], d["P"][0], d["A"][0], d["G"][0], order=order,
                               kernel=kernel)
        vals = {k: torch.from_numpy(v).cuda() for k, v in plan.pack(d["P"], d["A"], d["G"], d["c"], d["h"], d["b"]).items()}
        out = plan.alloc_outputs(B)
        go = plan.launcher(vals, out, B, reltol=tol, abstol=tol, maxit=maxit)
        for _ in range(3):
            go()
        torch.cuda.synchronize()
        n = 50
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            go()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / n
        it = out["iters"][:B].float().mean().item()
        print(json.dumps({"case": case, "opts": os.environ.get("QPB_WAVE_OPTS", ""), "kernel": plan.kernel_name(B),
                          "us_per_launch": us, "mean_iters": it, "us_per_iter": us / max(it, 1)}), flush=True)


if __name__ == "__main__":
    main()

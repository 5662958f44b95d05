"""Warm-solve timing (qpb_solve_warm) of the MPC horizon plan: the band kernel's QPB_WARM
variant (round 6) against the tree kernel's, each continuing from QP_SETUP's initial
point (a cold maxit-0 launch) for a full solve.  HIP events around each warm launch
alone (the state is restored between launches, outside the events).

    python scripts/warm_bench.py [B ...]        (default 1 1024)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main():
    import torch
    from apf_quadruped_amd import plans, workloads as W
    from apf_quadruped_amd.batch import Plan
    band = plans.standard_plan("mpc_h10")
    tree = Plan(120, 200, 60, *band.patterns.P, *band.patterns.A, *band.patterns.G, perm=band.perm,
                p_upper=band.p_upper, kernel="tree")
    for B in [int(a) for a in sys.argv[1:]] or [1, 1024]:
        d = W.mpc_qp(plans.SEED + 4, np.arange(B))
        vals = {k: torch.from_numpy(v).cuda() for k, v in band.pack(d["P"], d["A"], d["G"], d["c"], d["h"], d["b"]).items()}
        init = band.solve(**vals, B=B, maxit=0)
        torch.cuda.synchronize()
        for name, plan in (("band", band), ("tree", tree)):
            out = {k: v.clone() for k, v in init.items()}
            sig = torch.full((B,), 100.0, dtype=torch.float64, device="cuda")
            ms = []
            for rep in range(6):
                for k in out:
                    out[k].copy_(init[k])
                sig.fill_(100.0)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                plan.solve_warm(**vals, B=B, maxit=100, out=out, sigma=sig)
                e1.record()
                torch.cuda.synchronize()
                if rep:
                    ms.append(e0.elapsed_time(e1))
            r = plan.unpack(out, B)
            print(json.dumps(dict(kernel=name, B=B, warm_ms=float(np.median(ms)), qps=B / np.median(ms) * 1e3,
                                  optimal=float((r["flag"] == 0).mean()), mean_iters=float(r["iters"].mean()))),
                  flush=True)


if __name__ == "__main__":
    main()

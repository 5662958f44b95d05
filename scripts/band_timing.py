"""Per-phase cycles of the band kernel (QPB_B_TIMING=1 build: s_memtime deltas per
phase into the stats slots) on the MPC-horizon QP, per IPM iteration.

    QPB_WAVE_OPTS="QPB_B_TIMING=1" python scripts/band_timing.py [B ...]
    QPB_WAVE_OPTS="QPB_B_TIMING=2" ...: factor / solve parts instead of phases"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PHASES = ("w+residuals+setup", "factor", "predictor", "corrector", "steps+update", "staging")
PARTS = ("factor stage-parallel", "factor sequential", "solve rhs", "forward recursion", "S^-1 chains + backward recursion",
         "solve directions")


def main():
    import torch
    from apf_quadruped_amd import plans
    from apf_quadruped_amd.batch import Plan, from_tiled
    opts = os.environ.get("QPB_WAVE_OPTS", "")
    mode2 = "QPB_B_TIMING=2" in opts
    assert mode2 or "QPB_B_TIMING=1" in opts
    for B in [int(v) for v in sys.argv[1:]] or [1, 1024]:
        d = plans.standard_qp("mpc_h10", np.arange(B))
        plan = Plan.from_dense(d["n"], d["m"], d["p"], d["P"][0], d["A"][0], d["G"][0], kernel="band")
        vals = {k: torch.from_numpy(v).cuda() for k, v in plan.pack(d["P"], d["A"], d["G"], d["c"], d["h"],
                                                                    d["b"]).items()}
        out = plan.solve(**vals, B=B)
        out = plan.solve(**vals, B=B)
        torch.cuda.synchronize()
        st = from_tiled(out["stats"], B, 6).cpu().numpy()
        it = out["iters"][:B].cpu().numpy().astype(float)
        per_it = st / (it[:, None] + 1)          # + the setup pass
        if mode2:
            rec = {"B": B, "kernel": plan.kernel_name(B), "mean_iters": float(it.mean()),
                   "cycles_per_pass": {p: float(per_it[:, k].mean()) for k, p in enumerate(PARTS)}}
        else:
            rec = {"B": B, "kernel": plan.kernel_name(B), "mean_iters": float(it.mean()),
                   "cycles_per_pass": {p: float(per_it[:, k].mean()) for k, p in enumerate(PHASES[:5])},
                   "staging_cycles": float(st[:, 5].mean()),
                   "total_cycles_qp0": float(st[0].sum())}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()

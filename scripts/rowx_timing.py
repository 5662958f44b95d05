"""Per-phase cycle counts of the wide row kernel (knob QPB_X_TIMING=3, in-kernel
s_memtime stamps) on the controller's stance QP (30/68/18): H0 + setup solve,
residuals + reductions, factor, predictor (solve + step length + rho), corrector
(solve + step + update) + tail, input staging; per QP, summed over its wave's
iterations, and per pass.  One JSON line per batch size.

    python scripts/rowx_timing.py [--parts] [B ...]   (QPB_WAVE_OPTS adds further knobs)

--parts (QPB_X_TIMING=2): G'WG, pivots, -L parking, the solves' right-hand sides,
triangular chains, dz / dy instead (the solve parts summed over predictor and corrector)."""
import json
import os
import sys

PARTS = "--parts" in sys.argv
if PARTS:
    sys.argv.remove("--parts")
os.environ["QPB_WAVE_OPTS"] = (os.environ.get("QPB_WAVE_OPTS", "") + (" QPB_X_TIMING=2" if PARTS
                                                                        else " QPB_X_TIMING=3")).strip()
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from apf_quadruped_amd import plans, workloads as W  # noqa: E402
from apf_quadruped_amd.batch import Plan, from_tiled  # noqa: E402

NAMES = (("gwg", "pivots", "park", "rhs", "chains", "dzdy") if PARTS
         else ("h0_setup", "resid", "factor", "pred", "corr_tail", "staging"))


def main():
    import torch
    d0 = W.controller_qp(plans.SEED + 30, np.arange(1))
    plan = Plan.from_dense(30, 68, 18, d0["P"][0], d0["A"][0], d0["G"][0], order="own")
    if len(sys.argv) > 1 and sys.argv[1] == "compile":
        plan.compile()
        print(plan.kernel_name(1024))
        return
    for B in [int(a) for a in sys.argv[1:]] or [1, 1024]:
        d = W.controller_qp(plans.SEED + 30, np.arange(B))
        vals = {k: torch.from_numpy(v).cuda() for k, v in plan.pack(d["P"], d["A"], d["G"], d["c"], d["h"],
                                                                    d["b"]).items()}
        out = plan.alloc_outputs(B, device="cuda")
        for _ in range(3):
            plan.solve(**vals, B=B, out=out)
        torch.cuda.synchronize()
        st = from_tiled(out["stats"], B, 6).cpu().numpy()
        it = out["iters"].cpu().numpy()
        Bp = (B + 3) // 4 * 4
        wit = np.pad(it, (0, Bp - B), mode="edge").reshape(-1, 4).max(1).repeat(4)[:B]
        k = int(np.argmax(st.sum(1)))
        rec = {"B": B, "kernel": plan.kernel_name(B), "mean_iters": float(it.mean()), "max_wave_iters": int(wit.max())}
        rec.update({f"{n}_cyc_per_pass": float((st[:, i] / np.maximum(wit + 1, 1)).mean()) for i, n in enumerate(NAMES)})
        rec["slowest"] = {n: float(st[k, i]) for i, n in enumerate(NAMES)}
        rec["slowest_iters"] = int(wit[k])
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()

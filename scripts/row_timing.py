"""Per-phase cycle counts of the row kernel (knob QPB_R_TIMING=3, in-kernel
s_memtime stamps): H0 + setup solve, residuals + reductions, factor, predictor (solve + step
length + rho), corrector (solve + step + update) + tail, input staging; per QP, summed over its wave's iterations.  One JSON line per batch size."""
import json
import os
import sys

os.environ["QPB_WAVE_OPTS"] = (os.environ.get("QPB_WAVE_OPTS", "") + " QPB_R_TIMING=3").strip()
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from apf_quadruped_amd import plans  # noqa: E402
from apf_quadruped_amd.batch import from_tiled  # noqa: E402
from bench import make_shard  # noqa: E402

NAMES = ("h0_setup", "resid", "factor", "pred", "corr_tail", "staging")
for B in [int(a) for a in sys.argv[1:]] or [1024]:
    plan = plans.standard_plan("c1")
    host = make_shard(plan, plans.SEED + 1, 0, B)
    vals = {k: torch.from_numpy(v).cuda() for k, v in host.items()}
    out = plan.alloc_outputs(B, device="cuda")
    for _ in range(3):
        plan.solve(**vals, B=B, out=out)
    torch.cuda.synchronize()
    st = from_tiled(out["stats"], B, 6).cpu().numpy()
    it = out["iters"].cpu().numpy()
    # every row of a wave runs the wave's iteration count: the wave max
    wit = it.reshape(-1, 4).max(1).repeat(4)[:B] if B % 4 == 0 else it
    k = int(np.argmax(st.sum(1)))
    rec = {"B": B, "kernel": plan.kernel_name(B), "mean_iters": float(it.mean()), "max_wave_iters": int(wit.max())}
    rec.update({f"{n}_cyc_mean": float(st[:, i].mean()) for i, n in enumerate(NAMES)})
    rec.update({f"{n}_cyc_per_it": float((st[:, i] / np.maximum(wit + 1, 1)).mean()) for i, n in enumerate(NAMES)})
    rec["slowest"] = {n: float(st[k, i]) for i, n in enumerate(NAMES)}
    rec["slowest_iters"] = int(wit[k])
    print(json.dumps(rec), flush=True)

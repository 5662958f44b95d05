"""Phase stamps of the wave kernel (knob QPB_W_TIMING=1: s_memtime of QP 0 of each
tile into stats) for one QP of a standard shape; prints the cycle deltas between
consecutive stamps of iteration 1 (loop top 8+8i, after residuals / exit test 9,
after the L transpose 10, predictor 11, step 12, corrector 13, update 14) and the
prologue (0 start, 1 after staging + H0, 2..6 setup pass)."""
import json
import os
import sys

os.environ["QPB_WAVE_OPTS"] = (os.environ.get("QPB_WAVE_OPTS", "") + " QPB_W_TIMING=1").strip()
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from tree_bench import qp  # noqa: E402
from apf_quadruped_amd.batch import Plan  # noqa: E402

for spec in sys.argv[1:] or ["c30"]:
    name, _, order = spec.partition(":")      # "c30:amd" -> the AMD-ordered plan
    d = qp(name, np.arange(1))
    plan = Plan.from_dense(d["n"], d["m"], d["p"], d["P"][0], d["A"][0], d["G"][0], kernel="wave1",
                           order=order or "own")
    vals = {k: torch.from_numpy(v).cuda() for k, v in plan.pack(d["P"], d["A"], d["G"], d["c"], d["h"], d["b"]).items()}
    out = plan.alloc_outputs(1)
    out["stats"] = torch.zeros(384, dtype=torch.float64, device="cuda")
    for _ in range(2):
        plan.solve(**vals, B=1, out=out)
    torch.cuda.synchronize()
    st = out["stats"].cpu().numpy()
    it = int(out["iters"][0].item())
    stamps = {i: st[i] for i in range(384) if st[i] != 0}
    keys = sorted(stamps)
    deltas = {f"{a}->{b}": stamps[b] - stamps[a] for a, b in zip(keys, keys[1:])}
    print(json.dumps({"shape": spec, "opts": os.environ["QPB_WAVE_OPTS"], "iters": it, "kernel": plan.kernel_name(1),
                      "total": stamps[keys[-1]] - stamps[keys[0]], "deltas": deltas}), flush=True)

"""In-step cycle breakdown of the tree kernel (QPB_TREE_OPTS=QPB_T_TIMING=2): per
program step, cycles waiting for the step's descriptors, summing its terms,
writing its results and at the barrier (wave 0 of one QP)."""
import os, sys, json
import numpy as np
os.environ["QPB_TREE_OPTS"] = os.environ.get("QPB_TREE_OPTS", "") + " QPB_T_TIMING=2"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import torch
from tree_bench import qp
from apf_quadruped_amd.batch import Plan
for case in (sys.argv[1:] or ["mpc_h10:1", "c1:1"]):
    name, B = case.split(":"); B = int(B)
    d = qp(name, np.arange(B))
    plan = Plan.from_dense(d["n"], d["m"], d["p"], d["P"][0], d["A"][0], d["G"][0], kernel="tree")
    vals = {k: torch.from_numpy(v).cuda() for k, v in plan.pack(d["P"], d["A"], d["G"], d["c"], d["h"], d["b"]).items()}
    out = plan.alloc_outputs(B)
    go = plan.launcher(vals, out, B)
    go(); torch.cuda.synchronize()
    r = plan.unpack(out, B)
    n = r["alpha_p"][0]
    seg = [r[k][0] / n for k in ("n_rx", "n_ry", "n_rz", "n_mu")]
    pv = float(r["alpha_d"][0])
    npanel = int(pv // 1e9)
    pcyc = pv - 1e9 * npanel
    print(json.dumps(dict(case=case, steps=float(n), desc_wait=seg[0], terms=seg[1], epilogue=seg[2], barrier=seg[3],
                          per_step=sum(seg), panel_steps=npanel, cycles_per_panel_step=pcyc / max(npanel, 1),
                          panel_share=pcyc / (sum(seg) * n))), flush=True)

"""Per-phase cycle counts of the tree kernel (QPB_TREE_OPTS=QPB_T_TIMING=1):
factor / solve / residual-product cycles and the total, per QP (s_memtime)."""
import os, sys, json
import numpy as np
os.environ["QPB_TREE_OPTS"] = os.environ.get("QPB_TREE_OPTS", "") + " QPB_T_TIMING=1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import torch
from tree_bench import qp
from apf_quadruped_amd.batch import Plan
for case in (sys.argv[1:] or ["mpc_h10:1", "mpc_h10:1024", "c30:1", "c1:1"]):
    name, B = case.split(":"); B = int(B)
    d = qp(name, np.arange(B))
    plan = Plan.from_dense(d["n"], d["m"], d["p"], d["P"][0], d["A"][0], d["G"][0], kernel="tree")
    vals = {k: torch.from_numpy(v).cuda() for k, v in plan.pack(d["P"], d["A"], d["G"], d["c"], d["h"], d["b"]).items()}
    out = plan.alloc_outputs(B)
    go = plan.launcher(vals, out, B)
    go(); torch.cuda.synchronize(); go(); torch.cuda.synchronize()
    r = plan.unpack(out, B)
    it = r["iters"].astype(float)
    res = dict(case=case, iters=float(it.mean()), fac_cyc=float(r["n_rx"].mean()), sol_cyc=float(r["n_ry"].mean()),
               mv_cyc=float(r["n_rz"].mean()), total_cyc=float(r["n_mu"].mean()), fac_steps=float(r["alpha_p"][0]),
               solve_steps=float(r["alpha_d"][0]))
    nf = it + 1  # factorisations per solve (setup + one per iteration)
    res["cyc_per_fac_step"] = res["fac_cyc"] / (nf * res["fac_steps"]).mean()
    res["cyc_per_solve_step"] = res["sol_cyc"] / ((2 * it + 1) * res["solve_steps"]).mean()
    print(json.dumps(res), flush=True)

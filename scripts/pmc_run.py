"""Small fixed workload for rocprofv3 PMC passes: solve B QPs of one shape (C1 by default) `reps` times
with the kernel variant selected by QPB_WG / QPB_LDS (or --exact)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=262144)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--exact", action="store_true")
    ap.add_argument("--kernel", default="auto", choices=["auto", "lane", "wave", "tree", "band"])
    ap.add_argument("--shape", default="c1", help="plans.standard_qp name (c1, mpc_h10, ...)")
    a = ap.parse_args()
    import torch
    from apf_quadruped_amd import plans
    from apf_quadruped_amd.batch import Plan
    import bench
    torch.cuda.set_device(0)
    d0 = plans.standard_qp(a.shape)
    plan = Plan.from_dense(d0["n"], d0["m"], d0["p"], d0["P"][0], d0["A"][0], d0["G"][0], exact=a.exact,
                           kernel=a.kernel)
    vals = {k: torch.from_numpy(v).cuda() for k, v in bench.make_shard(
        plan, plans.SEED + 1, 0, a.batch, chunk=4096,
        gen=None if a.shape == "c1" else (lambda ids: plans.standard_qp(a.shape, ids))).items()}
    out = plan.solve(**vals, B=a.batch)
    for _ in range(a.reps):
        plan.solve(**vals, B=a.batch, out=out)
    torch.cuda.synchronize()
    print("iters", float(out["iters"].float().mean()))


if __name__ == "__main__":
    main()

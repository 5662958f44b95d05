"""A/B: controller QPs (stance / trot / crawl) with the default plan ordering vs
leaves-first (z, y, x), B=1024, wave kernel; prints us/launch, optimal share and
max |x - x_oracle| on QP 0."""
import sys
import numpy as np
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/oracle")
import torch  # noqa: E402
from apf_quadruped_amd import workloads as W, plans  # noqa: E402
from apf_quadruped_amd.batch import Plan  # noqa: E402
from oracle_py import Oracle  # noqa: E402
o = Oracle()
B = 1024
for phase in ("stance", "trot", "crawl"):
    d = W.controller_qp(plans.SEED + 31, np.arange(B), phase=phase)
    n, m, pp = 30, d["m"], d["p"]
    lf = np.array(list(range(n + pp, n + pp + m)) + list(range(n, n + pp)) + list(range(n)))
    for name, perm in (("default", None), ("leaves", lf)):
        p = Plan.from_dense(30, m, pp, d["P"][0], d["A"][0], d["G"][0], kernel="wave", perm=perm)
        vals = {k: torch.from_numpy(v).cuda() for k, v in p.pack(d["P"], d["A"], d["G"], d["c"], d["h"], d["b"]).items()}
        out = p.alloc_outputs(B, device="cuda")
        for _ in range(3):
            p.solve(**vals, B=B, out=out)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            p.solve(**vals, B=B, out=out)
        e1.record(); torch.cuda.synchronize()
        r = p.unpack(out, B)
        ref = o.solve_dense(30, m, pp, W.to_colmajor(d["P"])[0], W.to_colmajor(d["A"])[0], W.to_colmajor(d["G"])[0],
                            d["c"][0], d["h"][0], d["b"][0])
        print(phase, name, p.kernel_name(B), "us %.1f" % (e0.elapsed_time(e1) / 20 * 1e3),
              "optimal", float((r["flag"] == 0).mean()), "dx0 %.2e" % np.abs(r["x"][0] - ref["x"]).max(), flush=True)

"""A/B kernel variants in one process on one GPU (cdna guide rule 24).

    python scripts/sweep.py [--batch B] [--reps R] VARIANT...
VARIANT = "wg:lds" (fast lane kernel), "exact" (lane) or "wave" (wave-cooperative).  Prints one JSON line per variant.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--maxit", type=int, default=100)
    ap.add_argument("--shape", default="c1", choices=["c1", "c30"])
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    import torch
    from apf_quadruped_amd import plans, workloads as W
    from apf_quadruped_amd.batch import Plan
    import bench
    torch.cuda.set_device(0)
    seed = plans.SEED + 1
    if a.shape == "c1":
        gen = lambda ids: W.contact_force_qp(seed, ids)
        n, m, p = 12, 20, 6
    else:
        gen = lambda ids: W.controller_qp(seed, ids)
        n, m, p = 30, 68, 18
    d0 = gen(np.arange(1))
    base = Plan.from_dense(n, m, p, d0["P"][0], d0["A"][0], d0["G"][0], kernel="wave" if a.shape == "c30" else "auto")
    host = bench.make_shard(base, seed, 0, a.batch, gen=gen)
    vals = {k: torch.from_numpy(v).cuda() for k, v in host.items()}
    plans_ = {}
    for v in a.variants:
        if v == "exact":
            os.environ.pop("QPB_WG", None); os.environ.pop("QPB_LDS", None)
            plans_[v] = Plan.from_dense(n, m, p, d0["P"][0], d0["A"][0], d0["G"][0], exact=True)
        elif v.startswith("wave"):
            # "wave[1]" or "wave[1]:KNOB=V,KNOB=V" (QPB_W_* knobs of qpb_wave.hip, QPB_R_*
            # of qpb_row.hip); "wave" takes the row form where it fits, "wave1" never
            kind = v.split(":", 1)[0]
            opts = v.split(":", 1)[1].replace(",", " ") if ":" in v else ""
            os.environ["QPB_WAVE_OPTS"] = " ".join(f"QPB_W_{o} QPB_R_{o}" for o in opts.split())
            plans_[v] = Plan.from_dense(n, m, p, d0["P"][0], d0["A"][0], d0["G"][0], kernel=kind)
            plans_[v].compile()
            os.environ.pop("QPB_WAVE_OPTS", None)
        else:
            parts = v.split(":")
            os.environ["QPB_WG"], os.environ["QPB_LDS"] = parts[0], parts[1]
            os.environ["QPB_PARKZ"] = parts[2] if len(parts) > 2 else "1"
            plans_[v] = Plan.from_dense(n, m, p, d0["P"][0], d0["A"][0], d0["G"][0], kernel="lane")
        t0 = time.time(); plans_[v].compile(); ct = time.time() - t0
        print(f"compiled {v} in {ct:.1f}s", file=sys.stderr)
    for k in ("QPB_WG", "QPB_LDS", "QPB_PARKZ"):
        os.environ.pop(k, None)
    from oracle_py import Oracle
    o = Oracle()
    ids = np.arange(0, a.batch, a.batch // 16)
    dd = gen(ids)
    Pc, Ac, Gc = W.to_colmajor(dd["P"]), W.to_colmajor(dd["A"]), W.to_colmajor(dd["G"])
    times = {v: [] for v in a.variants}
    outs = {}
    for r in range(a.rounds):
        for v in a.variants:
            pl = plans_[v]
            out = pl.solve(**vals, B=a.batch, maxit=a.maxit)
            torch.cuda.synchronize()
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(); pl.solve(**vals, B=a.batch, out=out, maxit=a.maxit); e1.record(); torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1))
            outs[v] = out
    for v in a.variants:
        pl = plans_[v]
        if "TIMING=2" in v:      # per QP: start / end realtime (100 MHz) and cycles, iterations, XCC
            st = outs[v]["stats"].cpu().numpy().reshape(-1, 6, 64)[: (a.batch + 63) // 64]
            f = lambda k: st[:, k, :].reshape(-1)[: a.batch]
            rt0, rt1, cy0, cy1, itn, hw = (f(k) for k in range(6))
            dur_us = (rt1 - rt0) / 100.0
            cyc = cy1 - cy0
            xcc = (hw // 4294967296).astype(int)
            span = (rt1.max() - rt0.min()) / 100.0
            summ = dict(variant=v, span_us=span, start_spread_us=(rt0.max() - rt0.min()) / 100.0,
                        dur_us_median=float(np.median(dur_us)), dur_us_max=float(dur_us.max()),
                        clock_ghz=float(np.median(cyc / np.maximum(dur_us, 1e-3)) / 1e3),
                        cycles_per_iter=float(np.median(cyc / np.maximum(itn + 1, 1))),
                        iters_hist={int(k): int((itn == k).sum()) for k in np.unique(itn)},
                        dur_by_iters={int(k): float(np.median(dur_us[itn == k])) for k in np.unique(itn)},
                        end_by_xcc={int(k): float((rt1[xcc == k].max() - rt0.min()) / 100.0) for k in np.unique(xcc)},
                        start_by_xcc={int(k): float((rt0[xcc == k].min() - rt0.min()) / 100.0) for k in np.unique(xcc)})
            print(json.dumps(summ))
            continue
        if "TIMING=1" in v:      # phase timestamps of QP 0 of tile 0 (s_memtime cycles)
            t = outs[v]["stats"][:384].cpu().numpy()
            base = t[0]
            ph = {"stage": t[1] - t[0], "init_factor": t[6] - t[1], "init_solve": t[3] - t[6],
                  "init_sz": t[4] - t[3]}
            its = []
            for it in range(int(outs[v]["iters"][0].item())):
                r = t[8 + 8 * it: 16 + 8 * it]
                its.append(dict(resid_ldl=r[1] - r[0], transpose=r[2] - r[1], pred_solve=r[3] - r[2], pred_step=r[4] - r[3],
                                corr_solve=r[5] - r[4], corr_step=r[6] - r[5],
                                update=(t[16 + 8 * it] if t[16 + 8 * it] > 0 else t[370]) - r[6]))
            ph["out"] = t[371] - t[370]
            if t[305] > 0:
                ss = t[300:306]
                ph["solve_inner"] = dict(publish=ss[1] - ss[0], leaf_fwd=ss[2] - ss[1], dense=ss[3] - ss[2],
                                         publish_dx=ss[4] - ss[3], leaf_back=ss[5] - ss[4])
            ph["total"] = t[371] - base
            print(json.dumps(dict(variant=v, phases=ph, iterations=its)))
            continue
        res = pl.unpack(outs[v], a.batch)
        err = 0.0
        for k, q in enumerate(ids):
            perm = pl.perm
            ref = o.solve_dense(n, m, p, Pc[k], Ac[k], Gc[k], dd["c"][k], dd["h"][k], dd["b"][k], perm=perm,
                                maxit=a.maxit)
            err = max(err, float(np.max(np.abs(ref["x"] - res["x"][q]))))
        ms = float(np.median(times[v]))
        print(json.dumps(dict(variant=v, kernel=pl.info.hash, ms_median=ms, ms_min=float(np.min(times[v])),
                              qps=a.batch / ms * 1e3, gbs=pl.bytes_per_qp() * a.batch / ms / 1e6,
                              mean_iters=float(res["iters"].mean()), optimal=float((res["flag"] == 0).mean()),
                              max_err_vs_oracle=err)))


if __name__ == "__main__":
    main()

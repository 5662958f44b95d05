"""Reproducer (parked, DESIGN_HISTORY.md §7): the wave kernel on the trot controller QP
(30/70/12) with a leaves-first KKT order (z rows, y rows, then x -- pass it as the
plan's permutation) goes NaN at IPM iteration 1 when QPB_W_MFMA, QPB_W_LDSB and
QPB_W_LTLDS are all on; turning any one off (QPB_WAVE_OPTS) gives the oracle's
answer to 1e-12.  Stance and crawl QPs with the same order are correct.

    QPB_WAVE_OPTS="QPB_W_MFMA=0" python scripts/repro_leaves_first_trot.py
"""
import os, sys, numpy as np
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/oracle")
import torch
from apf_quadruped_amd import workloads as W, plans
from apf_quadruped_amd.batch import Plan
from oracle_py import Oracle
o = Oracle()
d = W.controller_qp(plans.SEED + 31, np.arange(4), phase="trot")
n, m, pp = 30, d["m"], d["p"]
leaves_first = np.array(list(range(n + pp, n + pp + m)) + list(range(n, n + pp)) + list(range(n)))
p = Plan.from_dense(30, d["m"], d["p"], d["P"][0], d["A"][0], d["G"][0], kernel="wave", perm=leaves_first)
for maxit in (1, 100):
    r = p.unpack(p.solve(**p.pack(d["P"], d["A"], d["G"], d["c"], d["h"], d["b"]), B=4, maxit=maxit), 4)
    ref = o.solve_dense(30, d["m"], d["p"], W.to_colmajor(d["P"])[0], W.to_colmajor(d["A"])[0], W.to_colmajor(d["G"])[0],
                        d["c"][0], d["h"][0], d["b"][0], perm=p.perm, maxit=maxit)
    print(os.environ.get("QPB_WAVE_OPTS"), maxit, "flag", r["flag"][0], ref["flag"], "dx %.3e" % np.abs(r["x"][0] - ref["x"]).max(),
          "dz %.3e" % np.abs(r["z"][0] - ref["z"]).max(), flush=True)

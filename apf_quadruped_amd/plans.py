"""Standard plans: the sparsity patterns of the benchmark / test workloads.

Patterns are taken from one synthetic QP of each workload (value-dependent,
exact zeros dropped as QP_SETUP_dense does) and ordered by our own
minimum-degree ordering (no dependence on the reference at run time)."""
from __future__ import annotations

import functools

import numpy as np

from . import workloads as W
from .batch import Plan

SEED = 0xD06B07
STANDARD = ("c1", "stance4", "trot_blfr", "trot_brfl", "crawl_blflfr")


def standard_qp(name: str, ids=(0,)):
    ids = np.asarray(ids)
    if name == "c1":
        return W.contact_force_qp(SEED + 1, ids)
    if name in W.STANCE_SETS:
        return W.contact_force_qp(SEED + 3, ids, stance=W.STANCE_SETS[name], feasible_wrench=True)
    if name == "mpc_h10":
        return W.mpc_qp(SEED + 4, ids)
    raise KeyError(name)


@functools.lru_cache(maxsize=None)
def standard_plan(name: str, exact: bool = False) -> Plan:
    d = standard_qp(name)
    return Plan.from_dense(d["n"], d["m"], d["p"], d["P"][0], d["A"][0], d["G"][0], exact=exact)

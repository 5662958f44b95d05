"""Host-side checks of the band kernel's plan logic (no GPU): which patterns are
multi-stage (band_shape, csrc/qpb_plan.cpp), the dispatch that sends them to the band
kernel (qpb::pick_kernel), its conditions (leaves-first permutation, cold solves),
and that its generated source compiles for gfx950 and passes the DPP audit."""
import glob
import os

import numpy as np
import pytest

from band_cases import stage_qp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _plan(d, **kw):
    from apf_quadruped_amd.batch import Plan
    return Plan.from_dense(d["n"], d["m"], d["p"], d["P"][0], d["A"][0] if d["p"] else None, d["G"][0], **kw)


def test_mpc_horizon_dispatches_to_band_kernel():
    from apf_quadruped_amd import plans
    plan = plans.standard_plan("mpc_h10")
    assert plan.kernel_for(1) == "band" and plan.kernel_for(1 << 20) == "band"
    assert plan.kernel_name(1024).startswith("qpb_band_")


@pytest.mark.parametrize("shape", [(12, 10, 20, 6), (4, 6, 5, 2), (16, 3, 40, 8), (7, 5, 64, 3), (9, 4, 11, 0),
                                   (10, 8, 3, 10)])
def test_stage_shapes_are_detected(shape):
    d = stage_qp(*shape, B=1, seed=sum(shape))
    assert _plan(d).info.ordering == 3, shape                       # leaves first
    assert _plan(d, kernel="band").kernel_for(64) == "band", shape   # eligible


def test_band_needs_the_leaves_first_order_and_a_stage_pattern():
    from apf_quadruped_amd import plans
    d = plans.standard_qp("mpc_h10")
    # the reference's AMD order: a different elimination -> the tree kernel
    plan = _plan(d, order="amd")
    assert plan.kernel_for(1024) == "tree"
    with pytest.raises(RuntimeError):
        _plan(d, order="amd", kernel="band")
    # a coupling outside the stage blocks (P entry between stages 0 and 5)
    P = d["P"].copy()
    P[:, 0, 60] = P[:, 60, 0] = 0.5
    with pytest.raises(RuntimeError):
        _plan(dict(d, P=P), kernel="band")
    assert _plan(dict(d, P=P)).kernel_for(1024) == "tree"
    # y rows of stage k touching stage k - 2
    A = d["A"].copy()
    A[:, 30, 0] = 1.0
    assert _plan(dict(d, A=A)).kernel_for(1024) == "tree"


def test_band_kernel_compiles_and_audits_clean():
    from apf_quadruped_amd import plans
    plan = plans.standard_plan("mpc_h10")
    plan.compile()
    kn = plan.kernel_name(1024)
    objs = glob.glob(os.path.join(ROOT, "apf_quadruped_amd", "kcache", kn + ".*.hsaco"))
    assert objs, kn
    audit = open(objs[0] + ".audit").read()
    assert audit.split("audit:")[-1].strip().startswith("clean"), audit


def test_python_flags_match_the_header():
    """batch.py's mirrors of the plan flags (orderings, kernels) equal the #defines of
    include/qpswift_hip.h -- QPB_KERNEL_BAND included."""
    import re
    from apf_quadruped_amd import batch
    text = open(os.path.join(ROOT, "include", "qpswift_hip.h")).read()
    defs = {k: int(v, 0) for k, v in re.findall(r"#define (QPB_\w+)\s+(0x[0-9a-fA-F]+)", text)}
    assert defs["QPB_KERNEL_BAND"] == batch.QPB_KERNEL_BAND == batch.KERNEL_FLAGS["band"]
    assert defs["QPB_KERNEL_TREE"] == batch.QPB_KERNEL_TREE == batch.KERNEL_FLAGS["tree"]
    assert defs["QPB_KERNEL_LANE"] == batch.KERNEL_FLAGS["lane"] and defs["QPB_KERNEL_WAVE"] == batch.KERNEL_FLAGS["wave"]
    assert batch.KERNEL_FLAGS["wave1"] == defs["QPB_KERNEL_WAVE"] | defs["QPB_KERNEL_NOROW"]
    for name, key in (("amd", "QPB_ORDER_AMD"), ("mindeg", "QPB_ORDER_MINDEG"), ("leaves", "QPB_ORDER_LEAVES")):
        assert batch.ORDER_FLAGS[name] == defs[key], name
    # no two plan flags share a bit
    flags = [v for k, v in defs.items() if k.startswith(("QPB_KERNEL_", "QPB_ORDER_")) or k in ("QPB_P_UPPER", "QPB_EXACT")]
    assert all(bin(f).count("1") == 1 for f in flags) and len(set(flags)) == len(flags)

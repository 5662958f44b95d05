"""The code-object cache files a kernel under the name the plan was made with (a hash
of its source).  A source generated under other knobs defines another kernel: the
runtime refuses to file it under the plan's name (round 6: a ZF128 test that unset
QPB_WAVE_OPTS before the first solve left such an object in the cache, and every later
load of that name failed with 'named symbol not found').  CPU only (cross-compile)."""
import numpy as np
import pytest


def test_source_generated_under_other_knobs_is_refused(monkeypatch):
    from apf_quadruped_amd import plans, workloads as W
    from apf_quadruped_amd.batch import Plan
    d = W.contact_force_qp(plans.SEED + 1, np.arange(1))
    # explicit defaults: the same kernel code, a different source text, hence a new name
    monkeypatch.setenv("QPB_WAVE_OPTS", "QPB_R_SELSLICE=1 QPB_R_ZF128=0 QPB_R_TIMING=0")
    monkeypatch.setenv("QPB_NO_DISK_CACHE", "1")
    plan = Plan.from_dense(12, 20, 6, d["P"][0], d["A"][0], d["G"][0])
    kn = plan.kernel_name(1024)
    monkeypatch.delenv("QPB_WAVE_OPTS")
    with pytest.raises(RuntimeError, match="defines another kernel"):
        plan.compile()
    monkeypatch.setenv("QPB_WAVE_OPTS", "QPB_R_SELSLICE=1 QPB_R_ZF128=0 QPB_R_TIMING=0")
    plan.compile()                   # under the plan's own knobs it builds
    assert plan.kernel_name(1024) == kn

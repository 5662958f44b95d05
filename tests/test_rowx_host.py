"""Host-side checks of the wide row kernel's plan logic (no GPU): which plans take it
(qpb::rowx_eligible, csrc/qpb_wave.cpp) -- the controller's 30-variable QPs in
leaves-first order, not in the reference's AMD order, not where the row kernel fits,
not where four QPs' dense copies exceed the LDS -- its LDS layout, and that its
generated source compiles for gfx950 and passes the DPP audit."""
import glob
import os

import numpy as np
import pytest

from rowx_cases import dense_qp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _plan(d, **kw):
    from apf_quadruped_amd.batch import Plan
    return Plan.from_dense(d["n"], d["m"], d["p"], d["P"][0], d["A"][0] if d["p"] else None, d["G"][0], **kw)


@pytest.mark.parametrize("phase", ["stance", "trot", "crawl"])
def test_controller_shapes_take_the_wide_row_kernel(phase):
    from apf_quadruped_amd import plans, workloads as W
    d = W.controller_qp(plans.SEED + 30, np.arange(2), phase=phase)
    plan = _plan(d)
    assert plan.info.wave_qpw == 4
    for B in (1, 1024, 1 << 20):
        assert plan.kernel_for(B) == "wave" and plan.kernel_name(B).startswith("qpb_rowx_"), (phase, B)
    # the one-QP-per-wavefront form on request, and the reference's AMD order keeps it
    assert _plan(d, kernel="wave1").kernel_name(64).startswith("qpb_wave_")
    assert _plan(d, order="amd").kernel_name(64).startswith("qpb_wave_")


def test_row_kernel_keeps_the_small_plans():
    from apf_quadruped_amd import plans
    assert plans.standard_plan("c1").kernel_name(1024).startswith("qpb_row_")


@pytest.mark.parametrize("shape,ok", [((20, 40, 10), True), ((32, 48, 16), True), ((12, 40, 6), True),
                                      ((16, 20, 20), True), ((33, 10, 2), False), ((32, 64, 16), False),
                                      ((24, 130, 4), False)])
def test_eligibility_by_shape(shape, ok):
    d = dense_qp(*shape, B=1, seed=sum(shape))
    name = _plan(d, p_upper=False).kernel_name(64)
    assert name.startswith("qpb_rowx_") == ok, (shape, name)


@pytest.mark.parametrize("shape,ok", [((20, 40, 10), True), ((17, 20, 6), True), ((16, 33, 6), True),
                                      ((12, 40, 6), True)])
def test_upper_p_eligibility(shape, ok):
    """An upper-triangle P takes the wide row form at any n <= 32 (round 5 kept plans past
    16 variables whose off-diagonal entries reach rows < 16 on the wave form after an
    aperture violation; its cause -- a register-allocator copy ahead of an EXEC restore --
    is repaired in every kernel since round 6)."""
    d = dense_qp(*shape, B=1, seed=sum(shape))
    name = _plan(d, p_upper=True).kernel_name(64)
    assert name.startswith("qpb_rowx_") == ok, (shape, name)


def test_layout_fits_four_controller_qps_per_cu():
    """Dense column-major G (leading dimension 2 mod 4: conflict-free column reads), A,
    P, the packed H0 and the row-padded -L of four QPs in the 160 KB of a CU."""
    from apf_quadruped_amd import plans, workloads as W
    d = W.controller_qp(plans.SEED + 30, np.arange(1))
    src = _plan(d).wave_source()
    defs = dict(line.split()[1:3] for line in src.splitlines() if line.startswith("#define ") and len(line.split()) >= 3)
    assert int(defs["LDG"]) == 70 and int(defs["LDA"]) == 18 and int(defs["LDP"]) == 30
    assert int(defs["LDG"]) % 4 == 2 and int(defs["LDP"]) % 4 == 2
    assert 4 * int(defs["LDS_QP"]) * 8 <= 160 * 1024
    assert int(defs["OFF_H0"]) + 30 * 31 // 2 <= int(defs["OFF_L"])
    assert int(defs["OFF_L"]) + 17 * 16 + 33 * 14 <= int(defs["O_DUMP"])
    assert int(defs["LDS_QP"]) % 32 == 17


def test_wide_row_kernel_compiles_and_audits_clean():
    from apf_quadruped_amd import plans, workloads as W
    d = W.controller_qp(plans.SEED + 30, np.arange(1))
    plan = _plan(d)
    plan.compile()
    kn = plan.kernel_name(1024)
    objs = glob.glob(os.path.join(ROOT, "apf_quadruped_amd", "kcache", kn + ".*.hsaco"))
    assert objs, kn
    audit = open(objs[0] + ".audit").read()
    assert audit.split("audit:")[-1].strip().startswith("clean"), audit

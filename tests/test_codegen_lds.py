"""Code-generation guard for round 6's finding: the register allocator serialised LDS
loads (one `s_waitcnt lgkmcnt(0)` per lone load, ~120 cycles each on a wave's chain) in
the row kernel's prologue, the wide row kernel's H0 staging, the wave kernel's residual
/ solve products and the band kernel's per-row passes.  The kernels of the bench's
workloads are compiled (CPU cross-compile; the in-tree cache makes this fast) and their
disassembly is counted with scripts/lds_roundtrips.py.  Bounds: what the shipped sources
give, with a little slack; the round-5 forms had 29 (row), 45 (wide row), 99 (AMD-ordered
C30 wave) and 21 (band).  CPU only."""
import glob
import os
import sys

import numpy as np
import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "scripts"))
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def _object(plan, B):
    plan.compile()
    name = plan.kernel_name(B)
    objs = sorted(glob.glob(os.path.join(ROOT, "apf_quadruped_amd", "kcache", name + ".*.hsaco")),
                  key=os.path.getmtime)
    assert objs, name
    return objs[-1]


def _plans():
    from apf_quadruped_amd import plans, workloads as W
    from apf_quadruped_amd.batch import Plan
    d = W.controller_qp(plans.SEED + 30, np.arange(1))
    return {
        "row (configs[1] C1)": (plans.standard_plan("c1"), 1024, 2),
        "wide row (stance 30/68/18)": (Plan.from_dense(30, 68, 18, d["P"][0], d["A"][0], d["G"][0]), 1024, 5),
        "wave (stance, AMD order)": (Plan.from_dense(30, 68, 18, d["P"][0], d["A"][0], d["G"][0], order="amd",
                                                     kernel="wave"), 8192, 65),
        "band (configs[3] MPC)": (plans.standard_plan("mpc_h10"), 1024, 25),
    }


@pytest.mark.skipif(not os.path.exists(OBJDUMP), reason="llvm-objdump not present")
@pytest.mark.parametrize("which", ["row (configs[1] C1)", "wide row (stance 30/68/18)", "wave (stance, AMD order)",
                                   "band (configs[3] MPC)"])
def test_shipped_kernels_batch_their_lds_loads(which):
    import lds_roundtrips
    plan, B, bound = _plans()[which]
    ins = lds_roundtrips.disasm(_object(plan, B))
    n = len(lds_roundtrips.lone_sites(ins))
    assert n <= bound, f"{which}: {n} lone LDS round trips (bound {bound})"


def test_counter_sees_a_lone_round_trip():
    # synthetic instruction stream: one batched pair, then a lone load
    ins = [(0, "ds_read_b64", "v[0:1], v2"), (4, "ds_read_b64", "v[2:3], v2 offset:8"),
           (8, "s_waitcnt", "lgkmcnt(0)"), (12, "ds_read_b64", "v[4:5], v2 offset:16"),
           (16, "v_add_f64", "v[6:7], v[0:1], v[2:3]"), (20, "s_waitcnt", "lgkmcnt(0)")]
    import lds_roundtrips
    assert [w for w, _ in lds_roundtrips.lone_sites(ins)] == [5]

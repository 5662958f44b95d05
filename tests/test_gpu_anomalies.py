"""The parked device anomalies of earlier rounds, run once each after their cause was
found.

The row kernel's illegal-address abort with `QPB_R_ZF128=1` (16-byte staging zero-fill;
rounds 1 and 4) came from the same compiler defect as the wide row kernel's aperture
violation: the register allocator copied q and tile into a4:a7 under the `c < NX`
region's EXEC, ahead of its restore, and the z / s stores of lanes 12-15 formed their
addresses from stale AGPRs (the round-4 object, rebuilt offline, holds exactly that
join).  Every kernel now passes `join_fixup` and the audit, so the variant is built
with the knob and run once on the headline workload (1 024 C1 QPs), against the oracle
in the plan's order (1e-9 relative, identical flags and iteration counts) and against
the shipped kernel."""
import numpy as np
import pytest


@pytest.mark.gpu
def test_row_kernel_zf128_variant_runs_clean(oracle, monkeypatch):
    import torch
    from apf_quadruped_amd import plans, workloads as W
    from apf_quadruped_amd.batch import Plan
    B = 1024
    d = W.contact_force_qp(plans.SEED + 1, np.arange(B))
    base = Plan.from_dense(12, 20, 6, d["P"][0], d["A"][0], d["G"][0])
    monkeypatch.setenv("QPB_WAVE_OPTS", "QPB_R_ZF128=1")
    plan = Plan.from_dense(12, 20, 6, d["P"][0], d["A"][0], d["G"][0])
    kn = plan.kernel_name(B)
    plan.compile(B=B)               # the variant is generated from the options in force: compile it now
    monkeypatch.delenv("QPB_WAVE_OPTS")
    assert kn.startswith("qpb_row_") and kn != base.kernel_name(B), (kn, base.kernel_name(B))
    vals = plan.pack(d["P"], d["A"], d["G"], d["c"], d["h"], d["b"])
    r = plan.unpack(plan.solve(**vals, B=B), B)
    torch.cuda.synchronize()
    r0 = base.unpack(base.solve(**vals, B=B), B)
    assert (r["flag"] == 0).all()
    np.testing.assert_array_equal(r["iters"], r0["iters"])
    np.testing.assert_array_equal(r["x"], r0["x"])          # the zero-fill changes no arithmetic
    cm = lambda M: np.ascontiguousarray(M.transpose(0, 2, 1)).reshape(M.shape[0], -1)
    Pc, Ac, Gc = cm(d["P"]), cm(d["A"]), cm(d["G"])
    for q in range(0, B, 97):
        o = oracle.solve_dense(12, 20, 6, Pc[q], Ac[q], Gc[q], d["c"][q], d["h"][q], d["b"][q], perm=plan.perm)
        assert r["flag"][q] == o["flag"] and r["iters"][q] == o["iters"], q
        for k in ("x", "z", "s"):
            err = np.max(np.abs(r[k][q] - o[k])) / max(1.0, np.max(np.abs(o[k])))
            assert err < 1e-9, (q, k, err)

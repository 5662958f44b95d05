"""On-device assembly of the controller's own 30-variable stance QP and the
APF-sampled candidates: qpb_assemble_controller restates
main.cpp:1471-1647 from the robot terms, qpb_apf_wrench main.cpp:1263-1422 +
1484-1571 (numpy checkers: workloads.controller_qp_from_terms, tests/apf_ref.py).

CPU: the synthetic controller QP is exactly controller_qp_from_terms of its robot
terms (so the golden vectors' inputs are reproduced bit for bit), and the ctypes
mirror of qpb_apf_state has the C layout.
GPU: assembled inputs equal the numpy restatement to rounding, every QP has the
plan's pattern (check = 1), a perturbed off-pattern term is caught (check = 0),
the assembled QPs solve to the oracle's answer, and the APF pipeline (targets ->
wrench -> shared-terms assembly -> solve + argmin) matches the numpy chain."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, golden

from apf_quadruped_amd import workloads as W
from apf_quadruped_amd._lib import QpbApfState


@pytest.mark.parametrize("name", ["c30_tol1e-6", "c30_tol1e-2"])
def test_controller_qp_is_the_restatement_of_its_terms(name):
    g = golden(name)
    t = W.controller_terms(int(g["seed"]), g["qp_ids"])
    d = W.controller_qp_from_terms(t)
    for k in ("P", "A", "G"):
        assert np.array_equal(W.to_colmajor(d[k]), g[k]), k
    for k in ("c", "h", "b"):
        assert np.array_equal(d[k], g[k]), k
    assert W.pack_terms(t).shape == (len(g["qp_ids"]), W.ROBOT_NV) and W.ROBOT_NV == 480


def test_apf_state_layout(tmp_path):
    src = tmp_path / "probe.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "qpswift_hip.h"\n'
                   'int main(void){printf("%zu %zu %zu %zu\\n", sizeof(qpb_apf_state), offsetof(qpb_apf_state, R_wb),'
                   ' offsetof(qpb_apf_state, mass), offsetof(qpb_apf_state, fake_crawl));return 0;}\n')
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(v) for v in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    assert got == [C.sizeof(QpbApfState), QpbApfState.R_wb.offset, QpbApfState.mass.offset,
                   QpbApfState.fake_crawl.offset]


def _plan(order="amd"):
    from apf_quadruped_amd.batch import Plan
    d = W.controller_qp(0xD06B07 + 30, np.arange(1))
    return Plan.from_dense(30, 68, 18, d["P"][0], d["A"][0], d["G"][0], order=order)


def _dense_from_tiled(plan, out, B):
    """Tiled CSC values -> dense [B, r, c] with the plan's patterns (P upper mirrored)."""
    from apf_quadruped_amd.batch import from_tiled
    res = {}
    for k, (jc, ir), shape in (("P", plan.patterns.P, (30, 30)), ("A", plan.patterns.A, (18, 30)),
                               ("G", plan.patterns.G, (68, 30))):
        v = from_tiled(out[k], B, len(ir)).cpu().numpy()
        M = np.zeros((B,) + shape)
        cols = np.repeat(np.arange(len(jc) - 1), np.diff(jc))
        M[:, ir, cols] = v
        if k == "P":
            M = M + np.transpose(M, (0, 2, 1)) - M * np.eye(30)[None]
        res[k] = M
    for k, nv in (("c", 30), ("h", 68), ("b", 18)):
        res[k] = from_tiled(out[k], B, nv).cpu().numpy()
    return res


@pytest.mark.gpu
def test_assemble_controller_matches_restatement_and_solves(oracle):
    import torch
    from apf_quadruped_amd.batch import to_tiled
    B = 200
    t = W.controller_terms(0xD06B07 + 41, np.arange(B))
    ref = W.controller_qp_from_terms(t)
    plan = _plan()
    terms = torch.from_numpy(to_tiled(W.pack_terms(t))).cuda()
    chk = torch.zeros(B, dtype=torch.int32, device="cuda")
    vals = plan.assemble_controller(terms, B=B, check=chk)
    torch.cuda.synchronize()
    assert (chk.cpu().numpy() == 1).all()
    got = _dense_from_tiled(plan, vals, B)
    for k in ("P", "A", "G", "c", "h", "b"):
        scale = max(1.0, float(np.abs(ref[k]).max()))
        assert np.abs(got[k] - ref[k]).max() <= 1e-14 * scale, k
    r = plan.unpack(plan.solve(**vals, B=B, reltol=1e-2, abstol=1e-2), B)
    for q in range(0, B, 23):
        o = oracle.solve_dense(30, 68, 18, W.to_colmajor(ref["P"])[q], W.to_colmajor(ref["A"])[q],
                               W.to_colmajor(ref["G"])[q], ref["c"][q], ref["h"][q], ref["b"][q], perm=plan.perm,
                               reltol=1e-2, abstol=1e-2)
        assert r["flag"][q] == o["flag"] and r["iters"][q] == o["iters"]
        assert np.abs(r["x"][q] - o["x"]).max() <= 1e-8 * max(1.0, np.abs(o["x"]).max()), q


@pytest.mark.gpu
def test_assemble_controller_flags_off_pattern_terms():
    import torch
    from apf_quadruped_amd.batch import Plan, to_tiled
    t = W.controller_terms(0xD06B07 + 42, np.arange(64))
    t["Jst"][:, 0, 9] = 0.0            # foot BR row x, a joint of another leg: an exact zero ...
    d = W.controller_qp_from_terms(t)
    plan = Plan.from_dense(30, 68, 18, d["P"][0], d["A"][0], d["G"][0], order="amd")
    t["Jst"][5, 0, 9] = 1e-3           # ... which QP 5 violates
    terms = torch.from_numpy(to_tiled(W.pack_terms(t))).cuda()
    chk = torch.zeros(64, dtype=torch.int32, device="cuda")
    plan.assemble_controller(terms, B=64, check=chk)
    c = chk.cpu().numpy()
    assert c[5] == 0 and (np.delete(c, 5) == 1).all()


@pytest.mark.gpu
def test_apf_candidates_end_to_end(oracle):
    """One tick, K APF candidate targets: wrench per candidate on the device,
    shared robot terms, assembled stance QPs, one solve + argmin."""
    import sys
    import torch
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import apf_ref
    from apf_quadruped_amd.batch import apf_state, apf_wrench, from_tiled, to_tiled
    K = 300
    for flags in ((True, False, False), (False, True, False), (True, True, True)):
        s = apf_ref.sample_state(rep_field=flags[0], min_exit=flags[1], fake_crawl=flags[2])
        rng = np.random.default_rng(3)
        targets = s["com"][None, :2] + rng.uniform(-0.6, 0.6, (K, 2))
        wd = apf_wrench(apf_state(**s), torch.from_numpy(to_tiled(targets)).cuda())
        w_ref, _ = apf_ref.apf_wrench(s, targets)
        w = from_tiled(wd, K, 6).cpu().numpy()
        assert np.abs(w - w_ref).max() <= 1e-12 * np.abs(w_ref).max()
    # shared robot terms of one tick + the candidates' wrenches
    t = W.controller_terms(0xD06B07 + 43, np.arange(1))
    plan = _plan()
    terms = torch.from_numpy(W.pack_terms(t)[0].copy()).cuda()
    vals = plan.assemble_controller(terms, B=K, shared=True, wdes=wd)
    best = torch.zeros(2, dtype=torch.float64, device="cuda")
    out = plan.alloc_outputs(K)
    plan.launcher(vals, out, K, reltol=1e-2, abstol=1e-2, best=best)()
    r = plan.unpack(out, K)
    tt = {k: np.repeat(v, K, 0) for k, v in t.items()}
    tt["wdes"] = w
    ref = W.controller_qp_from_terms(tt)
    fv = []
    for q in range(K):
        o = oracle.solve_dense(30, 68, 18, W.to_colmajor(ref["P"])[q], W.to_colmajor(ref["A"])[q],
                               W.to_colmajor(ref["G"])[q], ref["c"][q], ref["h"][q], ref["b"][q], perm=plan.perm,
                               reltol=1e-2, abstol=1e-2)
        fv.append(o["fval"] if o["flag"] == 0 else np.inf)
        if q % 37 == 0:
            assert np.abs(r["x"][q] - o["x"]).max() <= 1e-8 * max(1.0, np.abs(o["x"]).max())
    b = best.cpu().numpy()
    fv = np.asarray(fv)
    # the winner is the oracle's (up to rounding-level near-ties between candidates)
    assert abs(fv[int(b[1])] - fv.min()) <= 1e-9 * max(1.0, abs(fv.min()))
    assert abs(b[0] - fv.min()) <= 1e-9 * max(1.0, abs(fv.min()))


@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5])
def test_apf_update_matches_restatement(seed):
    """qpb_apf_update (host C, no GPU): the step's robustness smoothing and the
    fake_crawl decision (main.cpp:1273-1276, 1307-1321) equal the restatement in
    tests/apf_ref.py bit for bit, over successive steps of one robot; both sides of
    the 0.34 threshold occur."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import apf_ref
    from apf_quadruped_amd.batch import apf_state, apf_update
    rng = np.random.default_rng(seed)
    s = apf_ref.sample_state(seed)
    st = apf_state(**s)
    seen = set()
    for step in range(40):
        h = rng.uniform(0.0, 0.3, 4)
        period = rng.uniform(0.2, 0.6)
        m_ref = apf_ref.apf_update(s, h, period)
        m = apf_update(st, h, period)
        assert m == m_ref
        assert list(st.rob_foot) == list(s["rob_foot"])
        assert bool(st.fake_crawl) == s["fake_crawl"]
        seen.add(s["fake_crawl"])
    assert seen == {True, False}

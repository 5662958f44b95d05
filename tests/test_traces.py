"""Recorded Gazebo traces as a QP-input source (traces.py).

CPU: the committed data file (apf_quadruped_amd/data/gazebo_traces.npz, made by
scripts/extract_gazebo_traces.py from the reference's DogBotV4/log state logs)
holds physically consistent states (total mass 21.261 kg as the URDF, CoM height,
foot geometry, gait stance sets); the parser reads a minimal log of the same
format; the host QP builder from robot terms equals the synthetic generator's.
GPU: every stance set's QPs assembled on the device (qpb_assemble_contact) and
solved as ONE group launch agree with the oracle run with the plan's
permutation: same flags (infeasible 2-foot stances end at QP_MAXIT in both),
|x - x_oracle| <= 1e-6 max(1, |x|) for the optimal ones.
"""
import base64
import zlib

import numpy as np
import pytest


def _inputs():
    from apf_quadruped_amd import traces
    return [(run, traces.contact_inputs_from_trace(run)) for run in traces.load()]


def test_trace_data_is_physical():
    from apf_quadruped_amd import traces, workloads as W
    runs = traces.load()
    assert len(runs) == 5 and sum(len(r["t"]) for r in runs) > 6000
    assert abs(runs[0]["mass"].sum() - W.ROBOT_MASS) < 1e-9
    masks = set()
    for run, (r, Wr, st, t) in _inputs():
        assert np.all(np.diff(t) > 0)
        h = -r[st == 15][:, :, 2].mean() if (st == 15).any() else 0.35
        assert 0.2 < h < 0.45                                    # CoM height over the feet
        assert np.all(np.abs(np.abs(r[..., 1]) - W.Y_NOM) < 0.2)   # longitudinal foot offsets (swing feet reach)
        assert 150 < np.median(Wr[:, 2]) < 260                    # ~ m g = 208.6 N
        masks |= set(st.tolist())
    assert {15, 7, 11, 13, 14}.issubset(masks)                    # stance + the four crawl phases


def test_parse_minimal_log(tmp_path):
    from apf_quadruped_amd import traces
    ins = "".join(f"<link name='{n}'>\n<pose frame=''>0 0 0 0 -0 0</pose>\n<inertial>\n"
                  f"<pose frame=''>0 0 -0.1 0 -0 0</pose>\n<mass>1.5</mass></inertial></link>\n" for n in traces.LINKS)
    ins += ("<collision name='back_left_lowerleg_fixed_joint_lump__back_left_foot_collision_5'>\n"
            "<pose frame=''>0 -0.035 -0.3 0 -0 0</pose></collision>\n")

    def state(t, z):
        links = "".join(f"<link name='{n}'><pose>0.1 0.2 {z:.5f} 0.00000 0.01000 0.00000 </pose>"
                        f"<velocity>0.0 0.0 0.0 0.0 0.0 0.0123 </velocity></link>" for n in traces.LINKS)
        return (f"<sdf version='1.6'><state world_name='default'><sim_time>{t} 500000000</sim_time>"
                f"<model name='dogbot'><pose>0 0 0 0 0 0 </pose>{links}</model></state></sdf>")
    chunk1 = "<sdf><state world_name='default'><insertions><model name='dogbot'>" + ins + "</model></insertions></state></sdf>"
    body = state(1, 0.4) + state(2, 0.41) + state(0, 0.39)
    log = ("<?xml version='1.0'?>\n<gazebo_log>\n<header></header>\n"
           f"<chunk encoding='txt'><![CDATA[{chunk1}]]></chunk>\n"
           f"<chunk encoding='zlib'><![CDATA[{base64.b64encode(zlib.compress(body.encode())).decode()}]]></chunk>\n"
           "</gazebo_log>\n")
    p = tmp_path / "state.log"
    p.write_text(log)
    d = traces.parse_state_log(str(p))
    np.testing.assert_allclose(d["t"], [0.5, 1.5, 2.5])          # sorted by sim time
    assert d["pose"].shape == (3, len(traces.LINKS), 6)
    assert d["pose"][0, 0, 2] == 39000 and d["pose"][2, 0, 2] == 41000 and d["pose"][1, 3, 4] == 1000
    assert d["twist_base"][0, 5] == 123
    np.testing.assert_allclose(d["mass"], 1.5)
    np.testing.assert_allclose(d["com"][:, 2], -0.1)
    np.testing.assert_allclose(d["foot"], [0, -0.035, -0.3])


def test_qp_from_terms_matches_generator():
    from apf_quadruped_amd import workloads as W
    ids = np.arange(16)
    for stance in ((0, 1, 2, 3), (1, 3), (1, 2, 3)):
        d = W.contact_force_qp(7, ids, stance=stance)
        r, Wr = W.contact_inputs(7, ids)
        e = W.contact_qp_from_terms(r, Wr, stance)
        for k in ("P", "c", "A", "b", "G", "h"):
            np.testing.assert_array_equal(e[k], d[k], err_msg=k)


@pytest.mark.gpu
def test_trace_qps_group_vs_oracle(oracle):
    import torch
    from apf_quadruped_amd import traces, workloads as W
    from apf_quadruped_amd.batch import PlanGroup, to_tiled
    batches = traces.stance_batches()
    plans = traces.stance_plans(batches)
    masks, vals, outs, Bs, qps = [], [], [], [], []
    for (mask, r, Wr), plan in zip(batches, plans):
        B = len(r)
        feet = torch.from_numpy(to_tiled(r.reshape(B, 12))).cuda()
        wrench = torch.from_numpy(to_tiled(Wr)).cuda()
        vals.append(plan.assemble_contact(feet, wrench, stance=mask, mu=W.MU, B=B))
        outs.append(plan.alloc_outputs(B, device="cuda"))
        masks.append(mask); Bs.append(B)
        qps.append(W.contact_qp_from_terms(r, Wr, traces.stance_tuple(mask)))
    grp = PlanGroup(plans)
    best = torch.zeros(2, dtype=torch.float64, device="cuda")
    grp.launcher(vals, outs, Bs, best=best)()
    torch.cuda.synchronize()
    n_opt = 0
    for plan, o, B, q, mask in zip(plans, outs, Bs, qps, masks):
        res = plan.unpack(o, B)
        Pc, Ac, Gc = W.to_colmajor(q["P"]), W.to_colmajor(q["A"]), W.to_colmajor(q["G"])
        for i in range(0, B, max(1, B // 25)):
            ref = oracle.solve_dense(12, q["m"], 6, Pc[i], Ac[i], Gc[i], q["c"][i], q["h"][i], q["b"][i],
                                     perm=plan.oracle_perm(B))
            assert res["flag"][i] == ref["flag"], (mask, i)
            if ref["flag"] == 0:
                n_opt += 1
                err = np.abs(res["x"][i] - ref["x"]).max() / max(1.0, np.abs(ref["x"]).max())
                assert err <= 1e-6, (mask, i, err)
                assert res["iters"][i] == ref["iters"]
    assert n_opt > 100
    fv = np.concatenate([plan.unpack(o, B)["fval"] for plan, o, B in zip(plans, outs, Bs)])
    ok = np.concatenate([plan.unpack(o, B)["flag"] for plan, o, B in zip(plans, outs, Bs)]) == 0
    assert int(best[1].item()) == int(np.flatnonzero(ok)[np.argmin(fv[ok])])

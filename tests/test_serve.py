"""The drop-in's persistent solver (include/qpSWIFT.h "Device solves", csrc/
qpb_runtime.hip qpb::serve_ex): QP_SETUP's initial point and QP_SOLVE go to a
resident wave that polls a mailbox in mapped host memory instead of a launch +
stream synchronisation per call.

GPU tests: the controller's call sequence (QP_SETUP_dense -> QP_SOLVE ->
QP_CLEANUP_dense, main.cpp:1649-1663) through the served path agrees with the
reference's golden vectors as the launched path does (1e-6 of scale, equal
flags), the server is really what answered (qpb_dropin_serve_stats), it is
relaunched after leaving idle, and alternating patterns (a new kernel each call)
stop and relaunch it without mixing results up.
CPU test: the library exports the serve entry points.
"""
import ctypes as C
import os
import time

import numpy as np
import pytest

from conftest import golden

from apf_quadruped_amd import _lib, dropin


def _args(g, q):
    n, m, p = int(g["n"]), int(g["m"]), int(g["p"])
    return (n, m, p, g["P"][q], g["A"][q] if p else None, g["G"][q], g["c"][q], g["h"][q],
            g["b"][q] if p else None)


def _stats():
    out = (C.c_long * 4)()
    assert _lib.lib().qpb_dropin_serve_stats(out) == 0
    return int(out[0]), int(out[1])


def _check(r, g, q, name):
    assert r["flag"] == int(g["flag"][q]), (name, q, r["error"])
    # the iteration count too: a solve that starts from another QP's state (a stale
    # read of the slab by the resident wave) still converges, in a different count
    assert r["iters"] == int(g["iters"][q]), (name, q, r["iters"])
    for k in ("x", "z", "s") + (("y",) if int(g["p"]) else ()):
        scale = max(1.0, float(np.abs(g[k][q]).max()))
        assert np.abs(r[k] - g[k][q]).max() <= 1e-6 * scale, (name, q, k)


def _solve(g, q, null_perm=False):
    tol, maxit = float(g["tol"]), int(g["maxit"])
    return dropin.solve_dense(*_args(g, q), perm=None if null_perm else g["perm"][q],
                              ordering=int(g["ordering"]), reltol=tol, abstol=tol, maxit=maxit)


def test_serve_symbols_exported():
    L = _lib.lib()
    for s in ("qpb_dropin_serve_stats", "qpb_plan_compile_serve"):
        assert hasattr(L, s), s


@pytest.mark.gpu
@pytest.mark.skipif(os.environ.get("QPSWIFT_HIP_SERVE") == "0", reason="persistent solver switched off")
@pytest.mark.parametrize("name", ["c1_tol1e-6", "c1_tol1e-2", "c30_tol1e-2", "c30_trot_tol1e-2", "mixed_trot_brfl"])
def test_served_solves_match_reference(name):
    """Many QP objects of one pattern: every setup + solve answered by the two
    persistent solvers (cold, warm), results and iteration counts as the golden.
    (mixed_trot_brfl, 16 QPs of one pattern, is the case that showed the resident
    wave reading the previous request's slab lines when its acquire's L1 invalidate
    had not completed: iteration counts 6 instead of 5 from the third QP on.)"""
    g = golden(name)
    req0, lau0 = _stats()
    nq = g["x"].shape[0]
    for q in range(nq):
        _check(_solve(g, q), g, q, name)
    req, lau = _stats()
    assert req - req0 == 2 * nq            # QP_SETUP's initial point + QP_SOLVE, per QP
    # one request per launch, each next wave launched behind the answering one
    assert lau - lau0 <= 2 * nq + 2, (lau - lau0, nq)


@pytest.mark.gpu
@pytest.mark.skipif(os.environ.get("QPSWIFT_HIP_SERVE") == "0", reason="persistent solver switched off")
def test_served_solver_relaunches_after_idle_exit():
    """The resident wave leaves after QPSWIFT_HIP_SERVE_IDLE_MS (20 ms) without a
    call; the next call finds it gone, launches it again and gets the right answer."""
    g = golden("c1_tol1e-6")
    _check(_solve(g, 0), g, 0, "first")
    _, lau0 = _stats()
    time.sleep(0.2)
    _check(_solve(g, 1), g, 1, "after idle")
    _, lau = _stats()
    assert lau - lau0 >= 2                  # cold and warm solvers both came back


@pytest.mark.gpu
@pytest.mark.skipif(os.environ.get("QPSWIFT_HIP_SERVE") == "0", reason="persistent solver switched off")
def test_served_alternating_patterns():
    """Stance / trot / C1 patterns in turn (as a gait change does): each call has
    another kernel and other arguments, so the solver is stopped and relaunched
    every time -- and every result is the golden one (Permut = NULL as well)."""
    gs = [golden(n) for n in ("c30_tol1e-2", "c30_trot_tol1e-2", "c1_tol1e-2")]
    for rnd in range(3):
        for g, name in zip(gs, ("c30", "trot", "c1")):
            q = rnd % g["x"].shape[0]
            _check(_solve(g, q), g, q, name)
            r = _solve(g, q, null_perm=True)
            assert r["flag"] == int(g["flag"][q]), (name, r["error"])


@pytest.mark.gpu
@pytest.mark.skipif(os.environ.get("QPSWIFT_HIP_SERVE") == "0", reason="persistent solver switched off")
def test_served_solvers_per_thread():
    """Two solving threads at once (C1 and C30 stance): each thread's workspace has
    its own resident solvers, mailboxes and slab, so concurrent ticks neither block
    nor mix up each other's results."""
    import threading
    gs = {"c1": golden("c1_tol1e-2"), "c30": golden("c30_tol1e-2")}
    errors = []

    def worker(name):
        try:
            g = gs[name]
            for rnd in range(6):
                q = rnd % g["x"].shape[0]
                _check(_solve(g, q), g, q, name)
        except Exception as e:            # surfaced below: pytest sees only the main thread
            errors.append(f"{name}: {e!r}")

    ts = [threading.Thread(target=worker, args=(n,)) for n in gs]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in ts), "a solving thread hung"
    assert not errors, errors


_LAUNCH_PATH = r"""
import sys, json
import numpy as np
sys.path.insert(0, sys.argv[1])
sys.path.insert(0, sys.argv[1] + "/tests")
from conftest import golden
from apf_quadruped_amd import dropin
out = {}
for name in sys.argv[3].split(","):
    g = golden(name)
    n, m, p = int(g["n"]), int(g["m"]), int(g["p"])
    tol, maxit = float(g["tol"]), int(g["maxit"])
    for q in range(g["x"].shape[0]):
        r = dropin.solve_dense(n, m, p, g["P"][q], g["A"][q] if p else None, g["G"][q], g["c"][q], g["h"][q],
                               g["b"][q] if p else None, ordering=int(g["ordering"]), reltol=tol, abstol=tol,
                               maxit=maxit)
        out[f"{name}/{q}"] = {"flag": r["flag"], "iters": r["iters"], "x": r["x"].tolist(), "z": r["z"].tolist()}
json.dump(out, open(sys.argv[2], "w"))
"""


@pytest.mark.gpu
@pytest.mark.skipif(os.environ.get("QPSWIFT_HIP_SERVE") == "0", reason="persistent solver switched off")
def test_served_matches_launch_path(tmp_path):
    """The controller's call (Permut = NULL) on every QP of four goldens, through the
    persistent solver here and through launch + synchronise in a child process
    (QPSWIFT_HIP_SERVE=0): the same flags and iteration counts and x, z within 1e-12
    of scale -- a request that saw anything of an earlier one would differ."""
    import json
    import subprocess
    import sys
    names = ["c1_tol1e-2", "mixed_trot_brfl", "c30_tol1e-2", "c30_trot_tol1e-2"]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, QPSWIFT_HIP_SERVE="0")
    res = tmp_path / "launch.json"
    subprocess.run([sys.executable, "-c", _LAUNCH_PATH, root, str(res), ",".join(names)], env=env, check=True,
                   timeout=180)
    ref = json.load(open(res))
    for name in names:
        g = golden(name)
        tol, maxit = float(g["tol"]), int(g["maxit"])
        for q in range(g["x"].shape[0]):
            r = dropin.solve_dense(*_args(g, q), ordering=int(g["ordering"]), reltol=tol, abstol=tol, maxit=maxit)
            e = ref[f"{name}/{q}"]
            assert (r["flag"], r["iters"]) == (e["flag"], e["iters"]), (name, q)
            for k in ("x", "z"):
                v = np.asarray(e[k])
                assert np.abs(r[k] - v).max() <= 1e-12 * max(1.0, float(np.abs(v).max())), (name, q, k)


@pytest.mark.gpu
@pytest.mark.skipif(os.environ.get("QPSWIFT_HIP_SERVE") == "0", reason="persistent solver switched off")
def test_tick_then_batched_solve_then_device_sync_is_fast():
    """One thread ticks the drop-in (which leaves the next call's wave queued, polling
    for up to QPSWIFT_HIP_SERVE_IDLE_MS = 20 ms), then runs a batched solve and a
    device-wide synchronisation (torch.cuda.synchronize = hipDeviceSynchronize): the
    batched entry point retires the queued wave, so the whole sequence stays well
    inside the controller's 2.5 ms tick (main.cpp:1107) -- and the next drop-in tick
    relaunches and is still right.  qpb_dropin_quiesce does the same explicitly."""
    import torch
    from apf_quadruped_amd import plans, workloads as W
    g = golden("c1_tol1e-2")
    plan = plans.standard_plan("c1")
    plan.compile()
    B = 1024
    d = W.contact_force_qp(plans.SEED + 1, np.arange(B))
    vals = {k: torch.from_numpy(v).cuda() for k, v in plan.pack(d["P"], d["A"], d["G"], d["c"], d["h"], d["b"]).items()}
    out = plan.alloc_outputs(B, device="cuda")
    best = torch.zeros(2, dtype=torch.float64, device="cuda")
    solve = plan.launcher(vals, out, B, reltol=1e-6, abstol=1e-6, best=best)
    solve()
    torch.cuda.synchronize()
    # one untimed round of the whole sequence first: the first retire of a queued wave in
    # a process pays one-time costs (a 7.7 ms first round was seen once on the box)
    _check(_solve(g, 0), g, 0, "tick")
    solve()
    torch.cuda.synchronize()
    times = []
    for rnd in range(6):
        q = rnd % g["x"].shape[0]
        _check(_solve(g, q), g, q, "tick")
        t0 = time.perf_counter()
        if rnd % 2:
            assert _lib.lib().qpb_dropin_quiesce() == 0
            torch.cuda.synchronize()
        else:
            solve()
            torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
        assert (out["flag"][:B] == 0).all()
    assert max(times) < 2.5e-3, times


def _serve_config(env):
    """qpb_serve_config in a fresh process (the settings are read once per process)."""
    import json
    import subprocess
    import sys
    code = ("import ctypes as C, json\n"
            "from apf_quadruped_amd import _lib\n"
            "L = _lib.lib()\n"
            "i, l = C.c_double(), C.c_double()\n"
            "assert L.qpb_serve_config(C.byref(i), C.byref(l)) == 0\n"
            "print(json.dumps([i.value, l.value]))\n")
    e = {k: v for k, v in os.environ.items() if k not in ("QPSWIFT_HIP_SERVE_LIFE_MS", "QPB_SERVE_DIAG")}
    e.update(env)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], env=e, cwd=root, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1]), r.stderr


def test_multi_request_wave_refused_without_diag_guard():
    """The multi-request persistent wave has an open defect (DESIGN_HISTORY §7.5): a lifetime
    (QPSWIFT_HIP_SERVE_LIFE_MS > 0) alone is refused -- one request per wave, with a
    message -- and only QPB_SERVE_DIAG=1 turns the diagnostics mode on.  No GPU needed."""
    (idle, life), _ = _serve_config({})
    assert life == 0.0 and abs(idle - 20.0) < 1e-9
    (idle, life), err = _serve_config({"QPSWIFT_HIP_SERVE_LIFE_MS": "5"})
    assert life == 0.0 and "ignored" in err
    (idle, life), _ = _serve_config({"QPSWIFT_HIP_SERVE_LIFE_MS": "5", "QPB_SERVE_DIAG": "1"})
    assert abs(life - 5.0) < 1e-9

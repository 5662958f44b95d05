"""The drop-in boundary exercised by a compiled C caller (tests/c_caller/
controller_tick.c): it includes include/qpSWIFT.h, links libqpswift_hip.so the
way INTEGRATION.md's CMake relink does, and replays main.cpp:1649-1663 --
QP_SETUP_dense(..., NULL, COLUMN_MAJOR_ORDERING), tol override, QP_SOLVE, read x,
QP_CLEANUP_dense -- one tick per golden QP.

CPU: the program builds and links, and without a GPU QP_SOLVE returns QP_FATAL.
GPU: x of every tick is within 1e-6 of the reference's golden vector (the drop-in
orders the KKT with the AMD restatement, i.e. the reference's permutation)."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, golden

LIBDIR = os.path.join(ROOT, "apf_quadruped_amd")
SRC = os.path.join(ROOT, "tests", "c_caller", "controller_tick.c")


@pytest.fixture(scope="module")
def tick_exe(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("c_caller") / "controller_tick")
    subprocess.run(["gcc", "-O2", "-Wall", "-Werror", "-std=c99", "-I", os.path.join(ROOT, "include"), SRC,
                    "-o", exe, "-L", LIBDIR, "-lqpswift_hip", f"-Wl,-rpath,{LIBDIR}"], check=True)
    return exe


def _write_inputs(path, g, ticks):
    n, m, p = int(g["n"]), int(g["m"]), int(g["p"])
    with open(path, "wb") as f:
        np.asarray([n, m, p, len(ticks)], np.int64).tofile(f)
        np.asarray([float(g["tol"])], np.float64).tofile(f)
        for q in ticks:
            for k in ("P", "A", "G", "c", "h", "b"):
                np.ascontiguousarray(g[k][q], np.float64).tofile(f)


def _run(exe, tmp_path, name, ticks=None):
    g = golden(name)
    ticks = range(g["x"].shape[0]) if ticks is None else ticks
    inp = tmp_path / f"{name}.bin"
    _write_inputs(inp, g, ticks)
    r = subprocess.run([exe, str(inp)], check=True, capture_output=True, text=True, timeout=300)
    rows = []
    for line in r.stdout.splitlines():
        t = line.split()
        rows.append(dict(tick=int(t[1]), exit=int(t[3]), iters=int(t[5]), amd=int(t[7]),
                         x=np.asarray([float(v) for v in t[9:]])))
    return g, list(ticks), rows


def _no_gpu():
    try:
        import torch
        return not torch.cuda.is_available()
    except Exception:
        return True


@pytest.mark.skipif(not _no_gpu(), reason="checks the no-GPU failure mode")
def test_c_caller_links_and_fails_loudly_without_gpu(tick_exe, tmp_path):
    g, ticks, rows = _run(tick_exe, tmp_path, "c1_tol1e-2", ticks=[0, 1])
    assert [r["tick"] for r in rows] == [0, 1]
    assert all(r["exit"] == 3 and r["amd"] == 0 for r in rows)     # QP_FATAL, AMD_OK


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["c1_tol1e-2", "c30_tol1e-2", "c30_trot_tol1e-2", "c30_crawl_tol1e-2"])
def test_c_caller_controller_ticks_match_reference(tick_exe, tmp_path, name):
    g, ticks, rows = _run(tick_exe, tmp_path, name)
    assert len(rows) == len(ticks)
    for q, r in zip(ticks, rows):
        assert r["exit"] == int(g["flag"][q]) and r["iters"] == int(g["iters"][q]) and r["amd"] == 0
        scale = max(1.0, float(np.abs(g["x"][q]).max()))
        assert np.abs(r["x"] - g["x"][q]).max() <= 1e-6 * scale, (name, q)

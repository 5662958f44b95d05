"""CPU checks of the tree kernel's generated programs (tests/tree_emu.py): the
KKT assembly + level-scheduled LDL' + solves reproduce a dense solve of the KKT
system, and the residual / objective products reproduce the dense products, for
the C1, gait-pattern, controller-shape and MPC-horizon plans (no GPU needed)."""
import numpy as np
import pytest

from tree_emu import TreeEmu


def _qp(name):
    from apf_quadruped_amd import plans, workloads as W
    if name == "c30":
        return W.controller_qp(plans.SEED + 30, np.arange(1))
    return plans.standard_qp(name)


def _plan(d, perm=None):
    from apf_quadruped_amd.batch import Plan
    return Plan.from_dense(d["n"], d["m"], d["p"], d["P"][0], d["A"][0] if d["p"] else None, d["G"][0],
                           perm=perm, kernel="tree")


def _pag(plan, d):
    v = plan.pack(d["P"][:1], d["A"][:1] if d["p"] else None, d["G"][:1], d["c"][:1], d["h"][:1],
                  d["b"][:1] if d["p"] else None)
    from apf_quadruped_amd.batch import from_tiled
    parts = [from_tiled(v["P"], 1, plan.info.nnzP)[0]]
    if d["p"]:
        parts.append(from_tiled(v["A"], 1, plan.info.nnzA)[0])
    parts.append(from_tiled(v["G"], 1, plan.info.nnzG)[0])
    return np.concatenate(parts + [np.zeros(1)])


def _kkt(d, zdiag):
    n, m, p = d["n"], d["m"], d["p"]
    N = n + m + p
    K = np.zeros((N, N))
    K[:n, :n] = d["P"][0]
    if p:
        K[n:n + p, :n] = d["A"][0]
        K[:n, n:n + p] = d["A"][0].T
    K[n + p:, :n] = d["G"][0]
    K[:n, n + p:] = d["G"][0].T
    K[n + p:, n + p:] = np.diag(zdiag)
    return K


@pytest.mark.parametrize("name", ["c1", "stance4", "trot_blfr", "crawl_blflfr", "c30", "mpc_h10"])
def test_tree_programs_solve_the_kkt(name):
    d = _qp(name)
    plan = _plan(d)
    emu = TreeEmu(plan)
    pag = _pag(plan, d)
    n, m, p, N = d["n"], d["m"], d["p"], d["n"] + d["m"] + d["p"]
    rng = np.random.default_rng(7)
    xt = rng.standard_normal(N)
    # setup solve: the -I block (kkt_initialize)
    LD, rD = emu.assemble(pag, loop=False)
    emu.factor(LD, rD)
    K = _kkt(d, -np.ones(m))
    rhs = K @ xt                    # consistent rhs (2-foot trot: A has a rank defect)
    sol = emu.solve(LD, rD, rhs)
    # zero pivots of the y block are regularised to -1e-7 (ldl.c:319-320): the
    # factor is of a 1e-7-perturbed K, so compare the residual, not the solution
    res = np.abs(K @ sol - rhs).max() / max(1.0, np.abs(rhs).max())
    assert res < 1e-5, res
    # loop solve: z diagonal -s/z
    s, z = rng.uniform(0.1, 2.0, m), rng.uniform(0.1, 2.0, m)
    LD, rD = emu.assemble(pag, loop=True, s=s, z=z)
    emu.factor(LD, rD)
    K = _kkt(d, -s / z)
    rhs = K @ xt
    sol = emu.solve(LD, rD, rhs)
    res = np.abs(K @ sol - rhs).max() / max(1.0, np.abs(rhs).max())
    assert res < 1e-5, res


@pytest.mark.parametrize("name", ["c1", "c30", "mpc_h10"])
def test_tree_residual_products(name):
    d = _qp(name)
    plan = _plan(d)
    emu = TreeEmu(plan)
    pag = _pag(plan, d)
    n, m, p, N = d["n"], d["m"], d["p"], d["n"] + d["m"] + d["p"]
    v = np.random.default_rng(3).standard_normal(N)
    K = _kkt(d, np.zeros(m))
    np.testing.assert_allclose(emu.products(pag, v), K @ v, rtol=1e-12, atol=1e-12)
    Px = emu.products(pag, v, prog="obj")[:n]
    np.testing.assert_allclose(Px, d["P"][0] @ v[:n], rtol=1e-12, atol=1e-12)


def test_tree_kernel_compiles_for_gfx950():
    """hiprtc compiles the MPC-horizon tree kernel (N = 380) without a GPU."""
    d = _qp("mpc_h10")
    plan = _plan(d)
    plan.compile()
    assert plan.kernel_for(1024) == "tree"
    assert plan.kernel_name(1024).startswith("qpb_tree_")

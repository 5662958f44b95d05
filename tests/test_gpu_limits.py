"""GPU parity at the size limits of each kernel form, on random dense QPs.

The dispatch rules (include/qpswift_hip.h, qpb_plan_info): the row form of the
wave kernel holds n, p <= 16, m <= 32 (four QPs per wavefront); the wide row form
n, p <= 32, m <= 128 in leaves-first order while four QPs' dense copies fit the LDS
(four QPs per wavefront, two x rows per lane; round 6 lifted round 5's exclusion of
upper-triangle P past 16 variables once its fault was root-caused);
the one-QP-per-wavefront form holds
n, p <= 64, m <= 256 with every G row non-empty; beyond that a plan runs the lane or
tree kernel.  Each case sits on or just past one of those edges and is checked
against the oracle run with the plan's own KKT permutation (same factorisation, so
rounding-level agreement: 1e-9 relative, the bar of test_gpu_parity.py) with
identical flags and iteration counts, on a ragged batch of 5 QPs.

The QPs: P = M M' + n I (dense SPD), A dense with full row rank, G dense, and
h = G x0 + slack, b = A x0 for a random x0 (feasible, strictly inside)."""
import numpy as np
import pytest

# (n, m, p, expected kernel form: "row" | "rowx" | "wave" | "other")
LIMIT_CASES = [
    (16, 32, 16, "row"),     # the row form at its limit
    (12, 20, 0, "row"),      # no equality rows (round 6: the row kernel's select-form A slices at NY = 0)
    (16, 32, 0, "row"),
    (16, 33, 6, "rowx"),     # one inequality too many for a 16-lane row: the wide row form
    (17, 20, 6, "rowx"),     # one variable too many: the wide row form (dense upper-triangle P; the
                             # round-5 aperture-violation case)
    (32, 48, 16, "rowx"),    # the wide row form's variable limit (dense upper-triangle P)
    (12, 128, 6, "rowx"),    # ... and at its inequality limit
    (12, 129, 6, "wave"),    # one inequality past it
    (32, 64, 16, "wave"),    # four QPs' dense copies past the LDS of a CU
    (48, 96, 24, "wave"),
    (64, 128, 8, "wave"),    # the one-QP-per-wavefront form at its variable limit
    (65, 40, 10, "other"),   # past it: lane or tree kernel
    (12, 256, 6, "wave"),    # four z rows per lane: the inequality limit
    (12, 257, 6, "other"),   # one inequality past it
    (40, 64, 40, "wave"),    # as many equalities as variables
]


def random_qps(n, m, p, B, seed):
    rng = np.random.default_rng(seed)
    M = rng.standard_normal((B, n, n)) / np.sqrt(n)
    P = M @ M.transpose(0, 2, 1) + np.eye(n)
    A = rng.standard_normal((B, p, n))
    G = rng.standard_normal((B, m, n))
    x0 = rng.standard_normal((B, n))
    h = np.einsum("bmn,bn->bm", G, x0) + rng.uniform(0.5, 1.5, (B, m))
    b = np.einsum("bpn,bn->bp", A, x0)
    c = rng.standard_normal((B, n))
    return dict(n=n, m=m, p=p, P=P, A=A, G=G, c=c, h=h, b=b)


def _colmajor(M):
    return np.ascontiguousarray(M.transpose(0, 2, 1)).reshape(M.shape[0], -1)


@pytest.mark.gpu
@pytest.mark.parametrize("n,m,p,form", LIMIT_CASES)
def test_kernel_limits_match_oracle(n, m, p, form, oracle):
    from apf_quadruped_amd.batch import Plan
    B = 5
    d = random_qps(n, m, p, B, seed=1000 * n + m + p)
    plan = Plan.from_dense(n, m, p, d["P"][0], d["A"][0], d["G"][0])
    info = plan.info
    kn = plan.kernel_name(B)
    got_form = ("rowx" if kn.startswith("qpb_rowx_") else "row" if info.wave_qpw == 4 else "wave") \
        if info.wave_ok else "other"
    assert got_form == form, (n, m, p, got_form)
    vals = plan.pack(d["P"], d["A"], d["G"], d["c"], d["h"], d["b"])
    r = plan.unpack(plan.solve(**vals, B=B, reltol=1e-6, abstol=1e-6), B)
    Pc, Ac, Gc = _colmajor(d["P"]), _colmajor(d["A"]), _colmajor(d["G"])
    for q in range(B):
        o = oracle.solve_dense(n, m, p, Pc[q], Ac[q], Gc[q], d["c"][q], d["h"][q], d["b"][q], perm=plan.perm,
                               reltol=1e-6, abstol=1e-6)
        assert o["flag"] == 0, (n, m, p, q)
        assert r["flag"][q] == o["flag"] and r["iters"][q] == o["iters"], (n, m, p, q, r["iters"][q], o["iters"])
        for k in ("x", "y", "z", "s"):
            if np.size(o[k]) == 0:          # y with p = 0
                continue
            scale = max(1.0, float(np.abs(o[k]).max()))
            err = float(np.abs(r[k][q] - o[k]).max())
            assert err <= 1e-9 * scale, (n, m, p, q, k, err)

"""Synthetic QP workloads of the controller's own shape.

Every generator is a pure function of (seed, qp_id): uniforms come from a
counter-based splitmix64 hash of (seed, qp_id, draw), so any shard of a batch can
be regenerated independently on any rank.

Contact-force QP ("C1", 12 vars / 20 ineq / 6 eq) -- the contact-force
sub-problem of the stance QP built in dogbot_controller/src/client/main.cpp:
  * foot order BR, BL, FL, FR (Jacobian stacking, main.cpp:825-837)
  * nominal foot offsets x=0.186571, y=0.289186 (main.cpp:433-443)
  * P = 50 Jc Jc^T + I           (main.cpp:1476-1480, force block)
  * c = -50 Jc W                 (main.cpp:1573)
  * A = Jc^T, b = W              (eigenA/eigenb rows 0-5, main.cpp:1580-1587)
  * G = blkdiag4(cfr), h = 0     (friction pyramid mu=0.5, main.cpp:1603-1625)
  * m = 21.261 kg (sum of <mass> in DogBotV4 dogbot.urdf)
with Jc,i = [I3, -[r_i]x] and W = [m a; m(9.81 + a_z); tau].
"""
from __future__ import annotations

import numpy as np

ROBOT_MASS = 21.261
MU = 0.5
X_NOM = 0.186571
Y_NOM = 0.289186
# BR, BL, FL, FR (main.cpp:438-441)
FOOT_SIGNS = np.array([[+1.0, -1.0], [-1.0, -1.0], [-1.0, +1.0], [+1.0, +1.0]])
FOOT_NAMES = ("BR", "BL", "FL", "FR")

# Stance sets of the controller's gait phases.
STANCE_SETS = {
    "stance4": (0, 1, 2, 3),           # all feet (main.cpp:1471-1668)
    "trot_blfr": (1, 3),               # BL + FR stance (main.cpp:1730-1733)
    "trot_brfl": (0, 2),               # BR + FL stance (main.cpp:2486-2489)
    "crawl_blflfr": (1, 2, 3),         # BR swing (main.cpp:2919-2922)
}

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def uniforms(seed: int, qp_ids: np.ndarray, ndraw: int) -> np.ndarray:
    """[len(qp_ids), ndraw] uniforms in [0, 1) from a counter-based hash."""
    ids = np.asarray(qp_ids, dtype=np.uint64)
    with np.errstate(over="ignore"):
        key = _splitmix64(np.uint64(seed & 0xFFFFFFFFFFFFFFFF) ^ np.uint64(0xD1B54A32D192ED03))
        ctr = ids[:, None] * np.uint64(ndraw) + np.arange(ndraw, dtype=np.uint64)[None, :]
        h = _splitmix64(ctr ^ key)
        h = _splitmix64(h + key)
    return (h >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def _skew(r: np.ndarray) -> np.ndarray:
    """[..., 3] -> [..., 3, 3] cross-product matrices [r]x."""
    z = np.zeros(r.shape[:-1])
    rx, ry, rz = r[..., 0], r[..., 1], r[..., 2]
    return np.stack([np.stack([z, -rz, ry], -1),
                     np.stack([rz, z, -rx], -1),
                     np.stack([-ry, rx, z], -1)], -2)


def friction_block(mu: float = MU) -> np.ndarray:
    """cfr (main.cpp:1610-1615): rows (t1-mu n), (t2-mu n), -(t1+mu n), -(t2+mu n), -n."""
    return np.array([[1.0, 0.0, -mu],
                     [0.0, 1.0, -mu],
                     [-1.0, 0.0, -mu],
                     [0.0, -1.0, -mu],
                     [0.0, 0.0, -1.0]])


def contact_inputs(seed: int, qp_ids: np.ndarray):
    """Per-QP robot terms: foot positions relative to the CoM r [B,4,3] (BR, BL,
    FL, FR) and desired wrench W [B,6] (the inputs of qpb_assemble_contact)."""
    u = uniforms(seed, qp_ids, 19)
    h_com = 0.36 + 0.06 * u[:, 0]
    jit = (0.06 * u[:, 1:13] - 0.03).reshape(-1, 4, 3)
    r = np.empty((len(u), 4, 3))
    r[..., 0] = FOOT_SIGNS[None, :, 0] * X_NOM
    r[..., 1] = FOOT_SIGNS[None, :, 1] * Y_NOM
    r[..., 2] = -h_com[:, None]
    r = r + jit
    acc = np.stack([4.0 * u[:, 13] - 2.0, 4.0 * u[:, 14] - 2.0, 2.0 * u[:, 15] - 1.0], -1)
    tau = 4.0 * u[:, 16:19] - 2.0
    W = np.concatenate([ROBOT_MASS * acc[:, :2],
                        (ROBOT_MASS * (9.81 + acc[:, 2]))[:, None], tau], -1)
    return r, W


def contact_terms(seed: int, qp_ids: np.ndarray):
    """Per-QP contact Jacobian Jc [B,12,6] and desired wrench W [B,6]."""
    r, W = contact_inputs(seed, qp_ids)
    Jc = np.zeros((len(r), 12, 6))
    eye = np.eye(3)
    sk = _skew(r)
    for i in range(4):
        Jc[:, 3 * i:3 * i + 3, 0:3] = eye
        Jc[:, 3 * i:3 * i + 3, 3:6] = -sk[:, i]
    return Jc, W


def contact_force_qp(seed: int, qp_ids, stance=(0, 1, 2, 3), mu: float = MU,
                     feasible_wrench: bool = False):
    """Dense contact-force QPs (12 vars, 5*len(stance) ineq, 6 eq).

    feasible_wrench=False: W from random CoM accelerations/torques.
    feasible_wrench=True: W = sum_i Jc,i^T f_i for random ground-reaction forces
    f_i strictly inside the friction pyramid of each stance foot, so that QPs with
    two or three stance feet (6 / 9 force unknowns against 6 wrench equalities)
    stay feasible (config 3, mixed gait patterns).

    Returns dict with P [B,12,12], c [B,12], A [B,6,12], b [B,6], G [B,m,12],
    h [B,m]; row-major numpy arrays (dense; the solver converts them to CSC by
    dropping exact zeros, as QP_SETUP_dense does)."""
    qp_ids = np.atleast_1d(np.asarray(qp_ids, dtype=np.int64))
    Jc, W = contact_terms(seed, qp_ids)
    swing = [i for i in range(4) if i not in stance]
    for i in swing:                    # swing legs carry no force: zero their rows of Jc
        Jc[:, 3 * i:3 * i + 3, :] = 0.0
    B = len(qp_ids)
    if feasible_wrench:
        u = uniforms(seed ^ 0x0F0ECE, qp_ids, 12).reshape(B, 4, 3)
        fz = 40.0 + 80.0 * u[..., 2]
        f = np.stack([(0.8 * u[..., 0] - 0.4) * mu * 2 * fz * 0.5,
                      (0.8 * u[..., 1] - 0.4) * mu * 2 * fz * 0.5, fz], -1)
        W = np.einsum("bfij,bfi->bj", Jc.reshape(B, 4, 3, 6), f)
    return _contact_qp(Jc, W, stance, mu)


def _contact_qp(Jc, W, stance, mu):
    B = len(W)
    P = 50.0 * np.einsum("bij,bkj->bik", Jc, Jc) + np.eye(12)[None]
    c = -50.0 * np.einsum("bij,bj->bi", Jc, W)
    A = np.ascontiguousarray(np.transpose(Jc, (0, 2, 1)))
    b = np.array(W, dtype=np.float64, copy=True)
    cfr = friction_block(mu)
    m = 5 * len(stance)
    G = np.zeros((B, m, 12))
    for k, foot in enumerate(stance):
        G[:, 5 * k:5 * k + 5, 3 * foot:3 * foot + 3] = cfr
    h = np.zeros((B, m))
    return dict(n=12, m=m, p=6, P=P, c=c, A=A, b=b, G=G, h=h)


def contact_qp_from_terms(r: np.ndarray, W: np.ndarray, stance=(0, 1, 2, 3), mu: float = MU):
    """Dense contact-force QPs from given robot terms: foot positions relative to
    the CoM r [B,4,3] (BR, BL, FL, FR) and wrench W [B,6] (e.g. from recorded
    traces, traces.py) -- the host restatement of qpb_assemble_contact."""
    r = np.asarray(r, dtype=np.float64).reshape(-1, 4, 3)
    Jc = np.zeros((len(r), 12, 6))
    sk = _skew(r)
    for i in stance:
        Jc[:, 3 * i:3 * i + 3, 0:3] = np.eye(3)
        Jc[:, 3 * i:3 * i + 3, 3:6] = -sk[:, i]
    return _contact_qp(Jc, np.asarray(W, dtype=np.float64), stance, mu)


def mpc_qp(seed: int, qp_ids, horizon: int = 10, mu: float = MU):
    """Build-defined MPC contact-force QP.

    u_k in R^12 per stage (n = 12*horizon); P = blkdiag(50 Jk Jk^T + I);
    20 friction rows per stage (m = 20*horizon); 6 wrench-rate equality rows per
    stage, Jk^T u_k - J(k-1)^T u_(k-1) = W_k - W_(k-1) (p = 6*horizon)."""
    qp_ids = np.atleast_1d(np.asarray(qp_ids, dtype=np.int64))
    B, H = len(qp_ids), horizon
    n, m, p = 12 * H, 20 * H, 6 * H
    stage_ids = (qp_ids[:, None] * H + np.arange(H)[None, :]).reshape(-1)
    Jc, W = contact_terms(seed ^ 0x5EED_0004, stage_ids)
    Jc = Jc.reshape(B, H, 12, 6)
    W = W.reshape(B, H, 6)
    P = np.zeros((B, n, n)); c = np.zeros((B, n))
    A = np.zeros((B, p, n)); b = np.zeros((B, p))
    G = np.zeros((B, m, n)); h = np.zeros((B, m))
    cfr = friction_block(mu)
    for k in range(H):
        J = Jc[:, k]
        sl = slice(12 * k, 12 * k + 12)
        P[:, sl, sl] = 50.0 * np.einsum("bij,bkj->bik", J, J) + np.eye(12)[None]
        c[:, sl] = -50.0 * np.einsum("bij,bj->bi", J, W[:, k])
        A[:, 6 * k:6 * k + 6, sl] = np.transpose(J, (0, 2, 1))
        b[:, 6 * k:6 * k + 6] = W[:, k]
        if k > 0:
            A[:, 6 * k:6 * k + 6, 12 * (k - 1):12 * k] = -np.transpose(Jc[:, k - 1], (0, 2, 1))
            b[:, 6 * k:6 * k + 6] = W[:, k] - W[:, k - 1]
        for f in range(4):
            G[:, 20 * k + 5 * f:20 * k + 5 * f + 5, 12 * k + 3 * f:12 * k + 3 * f + 3] = cfr
    return dict(n=n, m=m, p=p, P=P, c=c, A=A, b=b, G=G, h=h)


# swing phases of the controller (SURVEY §8a shape table): the legs in stance,
# the swing legs and the slack count (x = [ddx 6; ddq 12; f_st 3k; slack 12-3k])
SWING_PHASES = {
    "trot": dict(stance=(1, 3), swing=(0, 2), w_slack=1e8),         # 30/70/12, main.cpp:1730-2005
    "crawl": dict(stance=(1, 2, 3), swing=(0,), w_slack=1e4),       # 30/69/15, main.cpp:2919-3232
}


def controller_swing_qp(seed: int, qp_ids, phase: str = "trot"):
    """Controller-shape swing-phase QPs: trot (two stance legs, 30/70/12,
    main.cpp:1730-2005) and crawl (three stance legs, 30/69/15, main.cpp:2919-3232).

    x = [ddx_com (6); ddq (12); f_st (3k); slack (12 - 3k)] with k stance legs:
      Q = 50 T_s' T_s + R, T_s = Jst(:, 0:6)' Sigma (f_st columns), R = I with
          w_slack on the slack block (1e8 trot :1751, 1e4 crawl :2976)
      c = -50 T_s' W_des
      A = [M_com 0 -Jst_com' 0; Jst_com Jst_q 0 0] (3k + 6 rows; :1844-1848, :3021-3044)
      D = friction (5 per stance foot) | tau_max [0 M_jj -Jst_q' 0] | tau_min (negated)
          | swing task [Jsw_com Jsw_q 0 -I] | -[Jsw_com Jsw_q 0 I] | ddq_max [0 I] | ddq_min [0 -I]
          (:1857-1992, :3048-3230)
    Synthetic robot terms as controller_qp; Jst / Jsw rows are the contact
    Jacobian rows [I3, -[r_i]x] of the stance / swing feet w.r.t. the CoM plus
    leg-dominant joint blocks.  b and the swing-task bounds are consistent with a
    random state (ddx*, ddq*, f* inside the friction pyramids, slack 0), so every
    QP is feasible (the controller's trot right-hand side is identically zero,
    main.cpp:1851-1854, which the synthetic state replaces)."""
    ph = SWING_PHASES[phase]
    st, sw = ph["stance"], ph["swing"]
    qp_ids = np.atleast_1d(np.asarray(qp_ids, dtype=np.int64))
    B = len(qp_ids)
    Jc, W = contact_terms(seed, qp_ids)                    # [B, 12, 6] rows per foot coordinate
    u = uniforms(seed ^ 0x5E1F, qp_ids, 144 + 144 + 12 + 12 + 12 + 12 + 6 + 12 + 12 + 12)
    k = 0

    def take(cnt):
        nonlocal k
        v = u[:, k:k + cnt]
        k += cnt
        return v
    Mcom = np.zeros((B, 6, 6))
    Mcom[:, [0, 1, 2], [0, 1, 2]] = ROBOT_MASS
    Mcom[:, 3:, 3:] = np.diag([0.35, 0.85, 0.95])[None]
    Lm = 0.02 * take(144).reshape(B, 12, 12) - 0.01 + 0.25 * np.eye(12)[None]
    Mjj = np.einsum("bij,bkj->bik", Lm, Lm)
    Jq = 0.004 * take(144).reshape(B, 12, 12) - 0.002           # foot-coordinate x joint (leg-dominant)
    jb = 0.7 * take(12).reshape(B, 4, 3) - 0.35
    for leg in range(4):
        blk = np.einsum("bi,ij->bij", jb[:, leg], np.ones((3, 3))) * np.array([[1, .5, .3], [.4, 1, .6], [.2, .5, 1]])
        Jq[:, 3 * leg:3 * leg + 3, 3 * leg:3 * leg + 3] += blk + 0.3 * np.eye(3)[None]
    bias_j = 4.0 * take(12) - 2.0
    q = take(12) - 0.5
    dq = 0.4 * take(12) - 0.2
    ddx = 2.0 * take(6) - 1.0
    ddq = 2.0 * take(12) - 1.0
    uf = take(12).reshape(B, 4, 3)
    tol_sw = 0.5 + take(12)                                      # swing-task tolerances
    rows = lambda legs: np.concatenate([np.arange(3 * i, 3 * i + 3) for i in legs])
    Jst_c, Jst_q = Jc[:, rows(st), :], Jq[:, rows(st), :]        # [B, 3k, 6], [B, 3k, 12]
    Jsw_c, Jsw_q = Jc[:, rows(sw), :], Jq[:, rows(sw), :]
    ns, nw = 3 * len(st), 3 * len(sw)
    n, p = 30, 6 + ns
    o_f, o_s = 18, 18 + ns
    fz = 40.0 + 60.0 * uf[:, list(st), 2]
    f = np.stack([(0.8 * uf[:, list(st), 0] - 0.4) * MU * fz, (0.8 * uf[:, list(st), 1] - 0.4) * MU * fz, fz],
                 -1).reshape(B, ns)
    Ts = np.zeros((B, 6, n))
    Ts[:, :, o_f:o_s] = np.transpose(Jst_c, (0, 2, 1))
    R = np.eye(n)
    R[o_s:, o_s:] *= ph["w_slack"]
    P = 50.0 * np.einsum("bki,bkj->bij", Ts, Ts) + R[None]
    c = -50.0 * np.einsum("bki,bk->bi", Ts, W)
    A = np.zeros((B, p, n))
    A[:, 0:6, 0:6] = Mcom
    A[:, 0:6, o_f:o_s] = -np.transpose(Jst_c, (0, 2, 1))
    A[:, 6:, 0:6] = Jst_c
    A[:, 6:, 6:18] = Jst_q
    xs = np.concatenate([ddx, ddq, f, np.zeros((B, n - o_s))], 1)
    b = np.einsum("bij,bj->bi", A, xs)
    m = 5 * len(st) + 24 + 2 * nw + 24
    G = np.zeros((B, m, n))
    h = np.zeros((B, m))
    cfr = friction_block(MU)
    for i in range(len(st)):
        G[:, 5 * i:5 * i + 5, o_f + 3 * i:o_f + 3 * i + 3] = cfr
    r0 = 5 * len(st)
    JqT = np.transpose(Jst_q, (0, 2, 1))                        # [B, 12, 3k]
    G[:, r0:r0 + 12, 6:18] = Mjj
    G[:, r0:r0 + 12, o_f:o_s] = -JqT
    G[:, r0 + 12:r0 + 24, 6:18] = -Mjj
    G[:, r0 + 12:r0 + 24, o_f:o_s] = JqT
    h[:, r0:r0 + 12] = 60.0 - bias_j
    h[:, r0 + 12:r0 + 24] = 60.0 + bias_j
    r1 = r0 + 24
    sw_acc = np.einsum("bij,bj->bi", Jsw_c, ddx) + np.einsum("bij,bj->bi", Jsw_q, ddq)
    G[:, r1:r1 + nw, 0:6] = Jsw_c
    G[:, r1:r1 + nw, 6:18] = Jsw_q
    G[:, r1:r1 + nw, o_s:o_s + nw] = -np.eye(nw)[None]
    h[:, r1:r1 + nw] = sw_acc + tol_sw[:, :nw]
    G[:, r1 + nw:r1 + 2 * nw, 0:6] = -Jsw_c
    G[:, r1 + nw:r1 + 2 * nw, 6:18] = -Jsw_q
    G[:, r1 + nw:r1 + 2 * nw, o_s:o_s + nw] = -np.eye(nw)[None]
    h[:, r1 + nw:r1 + 2 * nw] = -sw_acc + tol_sw[:, :nw]
    r2 = r1 + 2 * nw
    dt = 0.025
    G[:, r2:r2 + 12, 6:18] = np.eye(12)[None]
    G[:, r2 + 12:r2 + 24, 6:18] = -np.eye(12)[None]
    h[:, r2:r2 + 12] = (2 / dt ** 2) * (1.5 - q - dt * dq)
    h[:, r2 + 12:r2 + 24] = -(2 / dt ** 2) * (-1.5 - q - dt * dq)
    return dict(n=n, m=m, p=p, P=P, c=c, A=A, b=b, G=G, h=h)


def to_colmajor(M: np.ndarray) -> np.ndarray:
    """[B, r, c] row-major -> [B, r*c] column-major (QP_SETUP_dense, ordering 30)."""
    return np.ascontiguousarray(np.transpose(M, (0, 2, 1))).reshape(M.shape[0], -1)


# Per-QP robot terms of the controller's stance QP, in the layout of
# qpb_assemble_controller (include/qpswift_hip.h): the quantities main.cpp:1471-1647
# reads from iDynTree / the planner each tick.
ROBOT_TERMS = (("Jst", 12 * 18),     # JacCOM_lin: foot rows BR BL FL FR x [CoM 6 | joints 12], row-major
               ("Mcom", 36),         # MassMatrixCOM(0:6, 0:6), row-major
               ("Mjj", 144),         # MassMatrixCOM(6:18, 6:18), row-major
               ("bias", 18),         # BiasCOM
               ("jdqd", 12),         # JdqdCOM_lin
               ("wdes", 6),          # Wcom_des (main.cpp:1571)
               ("q", 12), ("dq", 12), ("qmin", 12), ("qmax", 12))
ROBOT_NV = sum(k for _, k in ROBOT_TERMS)


def pack_terms(t: dict) -> np.ndarray:
    """terms dict -> [B, ROBOT_NV] rows in the ROBOT_TERMS layout."""
    B = t["Jst"].shape[0]
    return np.concatenate([np.asarray(t[k], np.float64).reshape(B, -1) for k, _ in ROBOT_TERMS], 1)


def controller_terms(seed: int, qp_ids):
    """The synthetic robot state behind controller_qp (stance): contact Jacobian
    [Jc | J_j], M_com = blkdiag(m I3, I_c), dense SPD M_jj, biases, joint state and
    limits, desired wrench.  BiasCOM(0:6) and JdqdCOM_lin are chosen so that the
    equality right-hand side b = -[BiasCOM(0:6); Jdqd] (main.cpp:1584-1587) is
    consistent with a random state (ddx*, ddq*, f* inside the friction pyramids),
    so every QP is feasible."""
    qp_ids = np.atleast_1d(np.asarray(qp_ids, dtype=np.int64))
    B = len(qp_ids)
    Jc, W = contact_terms(seed, qp_ids)
    u = uniforms(seed ^ 0xC30C30, qp_ids, 3 + 3 + 144 + 144 + 12 + 12 + 12 + 12 + 6 + 12 + 12)
    k = 0

    def take(cnt):
        nonlocal k
        v = u[:, k:k + cnt]
        k += cnt
        return v
    Ic = np.zeros((B, 3, 3))
    Ic[:, [0, 1, 2], [0, 1, 2]] = np.array([0.35, 0.85, 0.95]) * (1.0 + 0.2 * take(3))
    off = 0.02 * take(3) - 0.01
    Ic[:, 0, 1] = Ic[:, 1, 0] = off[:, 0]
    Ic[:, 0, 2] = Ic[:, 2, 0] = off[:, 1]
    Ic[:, 1, 2] = Ic[:, 2, 1] = off[:, 2]
    Mcom = np.zeros((B, 6, 6))
    Mcom[:, [0, 1, 2], [0, 1, 2]] = ROBOT_MASS
    Mcom[:, 3:, 3:] = Ic
    Lm = 0.02 * take(144).reshape(B, 12, 12) - 0.01 + 0.25 * np.eye(12)[None]
    Mjj = np.einsum("bij,bkj->bik", Lm, Lm)                       # dense SPD
    Jj = 0.004 * take(144).reshape(B, 12, 12) - 0.002               # weak off-block coupling
    jb = 0.7 * take(12).reshape(B, 4, 3) - 0.35
    for leg in range(4):                                            # leg-dominant 3x3 blocks
        blk = np.einsum("bi,ij->bij", jb[:, leg], np.ones((3, 3))) * np.array([[1, .5, .3], [.4, 1, .6], [.2, .5, 1]])
        Jj[:, 3 * leg:3 * leg + 3, 3 * leg:3 * leg + 3] += blk + 0.3 * np.eye(3)[None]
    bias_j = 4.0 * take(12) - 2.0
    q = take(12) - 0.5
    dq = 0.4 * take(12) - 0.2
    ddx = 2.0 * take(6) - 1.0
    ddq = 2.0 * take(12) - 1.0
    uf = take(12).reshape(B, 4, 3)
    fz = 40.0 + 60.0 * uf[..., 2]
    f = np.stack([(0.8 * uf[..., 0] - 0.4) * MU * fz, (0.8 * uf[..., 1] - 0.4) * MU * fz, fz], -1).reshape(B, 12)
    Jst = np.concatenate([Jc, Jj], 2)
    A = _controller_A(Jst, Mcom)
    b = np.einsum("bij,bj->bi", A, np.concatenate([ddx, ddq, f], 1))  # consistent with (ddx*, ddq*, f*)
    bias = np.concatenate([-b[:, 0:6], bias_j], 1)
    return dict(Jst=Jst, Mcom=Mcom, Mjj=Mjj, bias=bias, jdqd=-b[:, 6:18], wdes=W, q=q, dq=dq,
                qmin=np.full((B, 12), -1.5), qmax=np.full((B, 12), 1.5))


def _controller_A(Jst, Mcom):
    """eigenA (main.cpp:1579-1582): [M_com 0 -Jstcom'; Jstcom Jstj 0]."""
    B = Jst.shape[0]
    A = np.zeros((B, 18, 30))
    A[:, 0:6, 0:6] = Mcom
    A[:, 0:6, 18:30] = -np.transpose(Jst[:, :, 0:6], (0, 2, 1))
    A[:, 6:18, 0:18] = Jst
    return A


def controller_qp_from_terms(t: dict, mu: float = MU):
    """The controller's stance QP 30/68/18 from its robot terms, restating
    main.cpp:1471-1647 (the numpy reference of qpb_assemble_controller):
      Q = 50 T_s' T_s + I, T_s = Jstcom' Sigma_st;  c = -T_s' (50 I)' W
      A = [M_com 0 -Jstcom'; Jstcom Jstj 0], b = [-BiasCOM(0:6); -Jdqd]
      D = friction | [0 M_jj -Jstj'] | -(same) | [0 I 0] | [0 -I 0]
      C = 0 | tau_max - bias_j | -(tau_min - bias_j) | ddq_max | -ddq_min, tau = 60,
          ddq_lim = (2 / dt^2)(q_lim - q - dt dq), dt = 0.025."""
    Jst, Mcom, Mjj = (np.asarray(t[k], np.float64) for k in ("Jst", "Mcom", "Mjj"))
    B = Jst.shape[0]
    n, m, p = 30, 68, 18
    Jc, Jj = Jst[:, :, 0:6], Jst[:, :, 6:18]
    Ts = np.zeros((B, 6, n))
    Ts[:, :, 18:30] = np.transpose(Jc, (0, 2, 1))
    P = 50.0 * np.einsum("bki,bkj->bij", Ts, Ts) + np.eye(n)[None]
    c = -50.0 * np.einsum("bki,bk->bi", Ts, np.asarray(t["wdes"], np.float64))
    A = _controller_A(Jst, Mcom)
    bias = np.asarray(t["bias"], np.float64)
    b = np.concatenate([-bias[:, 0:6], -np.asarray(t["jdqd"], np.float64)], 1)
    G = np.zeros((B, m, n))
    cfr = friction_block(mu)
    for i in range(4):
        G[:, 5 * i:5 * i + 5, 18 + 3 * i:18 + 3 * i + 3] = cfr
    JjT = np.transpose(Jj, (0, 2, 1))
    G[:, 20:32, 6:18] = Mjj
    G[:, 20:32, 18:30] = -JjT
    G[:, 32:44, 6:18] = -Mjj
    G[:, 32:44, 18:30] = JjT
    G[:, 44:56, 6:18] = np.eye(12)[None]
    G[:, 56:68, 6:18] = -np.eye(12)[None]
    dt = 0.025
    q, dq = np.asarray(t["q"], np.float64), np.asarray(t["dq"], np.float64)
    ddq_max = (2 / dt ** 2) * (np.asarray(t["qmax"], np.float64) - q - dt * dq)
    ddq_min = (2 / dt ** 2) * (np.asarray(t["qmin"], np.float64) - q - dt * dq)
    h = np.zeros((B, m))
    bias_j = bias[:, 6:18]
    h[:, 20:32] = 60.0 - bias_j
    h[:, 32:44] = -(-60.0 - bias_j)
    h[:, 44:56] = ddq_max
    h[:, 56:68] = -ddq_min
    return dict(n=n, m=m, p=p, P=P, c=c, A=A, b=b, G=G, h=h)


def controller_qp(seed: int, qp_ids, phase: str = "stance"):
    """Controller-shape stance QP "C30" (30 vars / 68 ineq / 18 eq), following
    dogbot_controller/src/client/main.cpp:1471-1647 (SURVEY §8a shape table):
    controller_qp_from_terms of the synthetic robot state controller_terms (no
    rigid-body model here: M_com = blkdiag(m I3, I_c), dense SPD M_jj,
    leg-dominant dense J_j, bias ~ U(-2, 2), q ~ U(-0.5, 0.5), dq ~ U(-0.2, 0.2),
    joint limits +-1.5 rad, an equality right-hand side consistent with a random
    feasible state).  Swing phases: controller_swing_qp.  Returns dense row-major
    [B, r, c] arrays like contact_force_qp."""
    if phase != "stance":
        return controller_swing_qp(seed, qp_ids, phase)
    return controller_qp_from_terms(controller_terms(seed, qp_ids))


def _apf_state_draw(seed: int, rep_field: bool, min_exit: bool) -> dict:
    """One random APF tick state (the fields of qpb_apf_state): stance feet around
    the CoM with jitter, small CoM motion, the controller's nominal versors
    (main.cpp:440-458), M_com = blkdiag(m I3, I_c), a 0.03 rad yaw."""
    rng = np.random.default_rng(seed)
    com = np.array([0.1, -0.05, 0.39, 0.01, -0.02, 0.03]) + rng.uniform(-0.01, 0.01, 6)
    nom = FOOT_SIGNS * np.array([X_NOM, Y_NOM])
    ee = com[None, :2] + nom + rng.uniform(-0.03, 0.03, (4, 2))
    versor = nom / np.linalg.norm(nom, axis=1, keepdims=True)
    M = np.zeros((6, 6))
    M[:3, :3] = ROBOT_MASS * np.eye(3)
    M[3:, 3:] = np.diag([0.35, 0.85, 0.95])
    th = 0.03
    R = np.array([[np.cos(th), -np.sin(th), 0], [np.sin(th), np.cos(th), 0], [0, 0, 1]])
    return dict(ee=ee, com=com, com_vel=rng.uniform(-0.1, 0.1, 6), acc_des=rng.uniform(-0.5, 0.5, 6),
                des_orient=np.array([0.0, 0.0]), rob_foot=rng.uniform(0.0, 0.5, 4), versor=versor,
                lat_versor=np.array([1.0, 0.0]), R_wb=R, Mcom=M, mass=ROBOT_MASS, rep_field=rep_field,
                min_exit=min_exit, fake_crawl=False)


def apf_tick_state(seed: int = 7, rep_field: bool = True, min_exit: bool = False, fake_crawl: bool = False) -> dict:
    """A plausible synthetic APF tick for the bench and the tests.  The robustness
    indices are carried as the controller carries them from one gait step to the
    next -- rob_foot = 0.35 rob_foot + 0.65 h_prev / period_st over a 0.4 s step
    (main.cpp:1273-1276) -- and fake_crawl is what main.cpp:1307-1321 derives from
    them (mean of the four < 0.34); states are drawn until it equals the requested
    fake_crawl."""
    for k in range(1000):
        s = _apf_state_draw(seed + 7919 * k, rep_field, min_exit)
        prev = np.random.default_rng(seed + 7919 * k + 1)
        rob = prev.uniform(0.0, 0.6, 4)
        h_prev = prev.uniform(0.0, 0.25, 4)
        rf = [0.35 * float(rob[i]) + 0.65 * float(h_prev[i]) / 0.4 for i in range(4)]
        s["rob_foot"] = np.asarray(rf)
        s["fake_crawl"] = bool((rf[1] + rf[3] + rf[0] + rf[2]) / 4.0 < 0.34)
        if s["fake_crawl"] == bool(fake_crawl):
            return s
    raise RuntimeError("no state with the requested fake_crawl")

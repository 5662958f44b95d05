"""Recorded Gazebo state traces as a QP-input source.

The reference ships gzserver state logs of DogBot runs
(DogBotV4/log/<date>/gzserver/state.log): a Gazebo 7 `<gazebo_log>` whose
`<chunk>`s (zlib + base64, or plain) hold one `<state>` per recorded step with
the pose (x y z roll pitch yaw) and twist of every link of model `dogbot`; the
first state also holds the model's SDF insertion, i.e. each link's mass and
inertial offset and the foot spheres lumped into the lower legs
(`*_lowerleg_fixed_joint_lump__*_foot_collision_5`, pose 0 -0.035 -0.3 in the
lower-leg frame, radius 0.028).

`parse_state_log` reads such a file (host tooling; only
scripts/extract_gazebo_traces.py runs it, in the container that holds the
reference).  The parsed link states are kept as the data file
apf_quadruped_amd/data/gazebo_traces.npz (numbers only: link poses as written
in the log, i.e. exactly representable as integers of 1e-5 m / rad).
`contact_inputs_from_trace` turns them into the inputs of the contact-force QP
(qpb_assemble_contact): per recorded step the whole-body CoM
(sum_l m_l (p_l + R_l c_l) / M), the foot centres relative to it (BR, BL, FL,
FR, the controller's Jacobian order, main.cpp:825-837), the stance set (feet
whose sphere touches the ground plane, within a contact margin) and the wrench
W = [M a_com; M (9.81 + a_z); I_b alpha_b] from central differences of the CoM
position and of the base angular velocity over the step's neighbours.
"""
from __future__ import annotations

import base64
import os
import re
import zlib

import numpy as np

from . import workloads as W

LINKS = ("base_link",
         "back_right_hip", "back_right_upperleg", "back_right_lowerleg",
         "back_left_hip", "back_left_upperleg", "back_left_lowerleg",
         "front_left_hip", "front_left_upperleg", "front_left_lowerleg",
         "front_right_hip", "front_right_upperleg", "front_right_lowerleg")
FEET = ("back_right", "back_left", "front_left", "front_right")   # BR, BL, FL, FR
DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "gazebo_traces.npz")
SCALE = 1e5               # poses are printed with 5 decimals (model pose: 3)
FOOT_RADIUS = 0.028
CONTACT_MARGIN = 0.004    # sphere bottom within 4 mm of the ground plane = stance


def _chunks(text: str):
    for enc, data in re.findall(r"<chunk encoding='(\w+)'>\s*<!\[CDATA\[(.*?)\]\]>", text, re.S):
        yield zlib.decompress(base64.b64decode(data)).decode() if enc == "zlib" else data


def _vec(s: str) -> np.ndarray:
    return np.array([float(v) for v in s.split()])


def parse_state_log(path: str) -> dict:
    """One gzserver state.log -> dict(t [F], pose [F, L, 6] int64 (1e-5 units),
    twist_base [F, 6] int64 (1e-4 units), mass [L], com [L, 3], foot [3], names)
    for the links of LINKS; steps missing a link are dropped."""
    text = open(path).read()
    mass, com, foot = {}, {}, None
    ts, poses, twists = [], [], []
    for chunk in _chunks(text):
        for m in re.finditer(r"<link name='([^']*)'>\s*<pose frame=''>[^<]*</pose>\s*<inertial>\s*"
                             r"<pose frame=''>([^<]*)</pose>\s*<mass>([^<]*)</mass>", chunk):
            mass[m.group(1)] = float(m.group(3))
            com[m.group(1)] = _vec(m.group(2))[:3]
        fm = re.search(r"lowerleg_fixed_joint_lump__\w+_foot_collision_5'>\s*<pose frame=''>([^<]*)</pose>", chunk)
        if fm and foot is None:
            foot = _vec(fm.group(1))[:3]
        for st in chunk.split("<state ")[1:]:
            tm = re.search(r"<sim_time>(\d+) (\d+)</sim_time>", st)
            mm = st.find("<model name='dogbot'>")
            if not tm or mm < 0:
                continue
            body = st[mm:]
            links = {a: (b, c) for a, b, c in re.findall(
                r"<link name='([^']*)'><pose>([^<]*)</pose><velocity>([^<]*)</velocity>", body)}
            if not all(n in links for n in LINKS):
                continue
            ts.append(int(tm.group(1)) + int(tm.group(2)) * 1e-9)
            poses.append([np.rint(_vec(links[n][0]) * SCALE).astype(np.int64) for n in LINKS])
            twists.append(np.rint(_vec(links["base_link"][1]) * 1e4).astype(np.int64))
    if not ts:
        return dict(t=np.zeros(0), pose=np.zeros((0, len(LINKS), 6), np.int64),
                    twist_base=np.zeros((0, 6), np.int64), mass=np.zeros(0), com=np.zeros((0, 3)),
                    foot=np.zeros(3))
    t = np.array(ts)
    order = np.argsort(t, kind="stable")
    keep = order[np.concatenate([[True], np.diff(t[order]) > 0])]     # one state per sim time
    return dict(t=t[keep], pose=np.array(poses)[keep], twist_base=np.array(twists)[keep],
                mass=np.array([mass[n] for n in LINKS]), com=np.array([com[n] for n in LINKS]),
                foot=foot)


def load(path: str = DATA) -> list:
    """The recorded runs in the data file: a list of dicts as parse_state_log's
    (plus 'run', the log directory name)."""
    z = np.load(path, allow_pickle=False)
    runs = []
    for name in [str(s) for s in z["runs"]]:
        runs.append(dict(run=name, t=z[f"{name}/t"], pose=z[f"{name}/pose"], twist_base=z[f"{name}/twist_base"],
                         mass=z["mass"], com=z["com"], foot=z["foot"]))
    return runs


def _rot(rpy: np.ndarray) -> np.ndarray:
    """Gazebo pose roll/pitch/yaw -> rotation matrices [..., 3, 3] (R = Rz Ry Rx)."""
    r, p, y = rpy[..., 0], rpy[..., 1], rpy[..., 2]
    cr, sr, cp, sp, cy, sy = np.cos(r), np.sin(r), np.cos(p), np.sin(p), np.cos(y), np.sin(y)
    R = np.empty(rpy.shape[:-1] + (3, 3))
    R[..., 0, 0] = cy * cp; R[..., 0, 1] = cy * sp * sr - sy * cr; R[..., 0, 2] = cy * sp * cr + sy * sr
    R[..., 1, 0] = sy * cp; R[..., 1, 1] = sy * sp * sr + cy * cr; R[..., 1, 2] = sy * sp * cr - cy * sr
    R[..., 2, 0] = -sp;     R[..., 2, 1] = cp * sr;                R[..., 2, 2] = cp * cr
    return R


BASE_INERTIA = np.diag([0.41, 0.091, 0.482])     # base_link <inertia> (insertion SDF)


def contact_inputs_from_trace(run: dict, k: int = 5, margin: float = CONTACT_MARGIN):
    """Recorded run -> (r [F,4,3] foot centres relative to the CoM, Wr [F,6]
    wrench, stance [F] bitmask (bit i = foot i of BR, BL, FL, FR), t [F]) for the
    steps with k neighbours on each side (central differences over +-k steps)."""
    pose = run["pose"].astype(np.float64) / SCALE
    pos, rpy = pose[..., :3], pose[..., 3:]
    R = _rot(rpy)                                                   # [F, L, 3, 3]
    mass, com = run["mass"], run["com"]
    M = mass.sum()
    cw = pos + np.einsum("flij,lj->fli", R, com)                    # link CoMs, world
    C = np.einsum("l,fli->fi", mass, cw) / M                        # whole-body CoM
    feet = []
    for f in FEET:
        li = LINKS.index(f + "_lowerleg")
        feet.append(pos[:, li] + R[:, li] @ run["foot"])
    feet = np.stack(feet, 1)                                        # [F, 4, 3]
    t = run["t"]
    F = len(t)
    if F < 2 * k + 1:
        z = np.zeros(0)
        return np.zeros((0, 4, 3)), np.zeros((0, 6)), np.zeros(0, np.int64), z
    i = np.arange(k, F - k)
    dt = (t[i + k] - t[i - k]) / 2
    acc = (C[i + k] - 2 * C[i] + C[i - k]) / dt[:, None] ** 2
    w = run["twist_base"][:, 3:].astype(np.float64) * 1e-4          # base angular velocity (world)
    alpha = (w[i + k] - w[i - k]) / (2 * dt[:, None])
    Rb = R[i, LINKS.index("base_link")]
    Iw = Rb @ BASE_INERTIA @ np.transpose(Rb, (0, 2, 1))
    tau = np.einsum("fij,fj->fi", Iw, alpha)
    Wr = np.concatenate([M * acc[:, :2], (M * (9.81 + acc[:, 2]))[:, None], tau], 1)
    r = feet[i] - C[i][:, None, :]
    bottom = feet[i, :, 2] - FOOT_RADIUS
    stance = ((bottom <= margin).astype(np.int64) << np.arange(4)).sum(1)
    return r, Wr, stance, t[i]


def stance_tuple(mask: int) -> tuple:
    return tuple(i for i in range(4) if mask >> i & 1)


def trace_qps(run: dict, mu: float = W.MU, k: int = 5):
    """Dense contact-force QPs of a recorded run, grouped by stance set:
    {mask: dict(frames, r, Wr, qp)} with qp as workloads.contact_force_qp's
    (stance sets of fewer than two feet are skipped: no stance QP there)."""
    r, Wr, stance, t = contact_inputs_from_trace(run, k=k)
    out = {}
    for mask in sorted(set(stance.tolist())):
        if bin(mask).count("1") < 2:
            continue
        sel = np.flatnonzero(stance == mask)
        out[mask] = dict(frames=sel, t=t[sel], r=r[sel], Wr=Wr[sel],
                         qp=W.contact_qp_from_terms(r[sel], Wr[sel], stance_tuple(mask), mu))
    return out


def stance_batches(runs=None, min_feet: int = 2):
    """Every recorded step of `runs` (default: the data file's) grouped by stance
    set: [(mask, r [B,4,3], Wr [B,6])] in ascending mask order -- one member plan
    per stance set of a plan group (qpb_group_solve)."""
    if runs is None:
        runs = load()
    acc = {}
    for run in runs:
        r, Wr, st, _ = contact_inputs_from_trace(run)
        for mask in set(st.tolist()):
            if bin(mask).count("1") >= min_feet:
                sel = st == mask
                a = acc.setdefault(mask, ([], []))
                a[0].append(r[sel])
                a[1].append(Wr[sel])
    return [(mask, np.concatenate(acc[mask][0]), np.concatenate(acc[mask][1])) for mask in sorted(acc)]


def stance_plans(batches, mu: float = W.MU):
    """One Plan (own ordering, row-form kernel) per stance set of `batches`."""
    from .batch import Plan
    out = []
    for mask, r, Wr in batches:
        q = W.contact_qp_from_terms(r[:1], Wr[:1], stance_tuple(mask), mu)
        out.append(Plan.from_dense(12, q["m"], 6, q["P"][0], q["A"][0], q["G"][0]))
    return out

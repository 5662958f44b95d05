"""The wide row kernel's LDS layout, checked on the host from its generated source
(qpb_wave.cpp generate_rowx_kernel; no GPU): every CSC -> LDS scatter slot of P (both
triangles of an upper-triangle P), A and G lands inside its own dense copy of the
QP's LDS block, the staged area is covered exactly by the zero-fill of both row
alignments, and four QPs' blocks fit a CU's LDS.  Shapes: the round-5 fault case
(17 / 20 / 6, dense upper-triangle P past 16 variables), the variable limit 32 / 48 / 16,
the controller's three shapes and 17 / 40 / 5 with a structurally absent P(16, 16)
(STG_END = 1122 = 2 mod 32: the zero-fill's last pair)."""
import re

import numpy as np
import pytest

from rowx_cases import dense_qp
from test_gpu_limits import random_qps


def _defs(src):
    d = {}
    for name in ("LDG", "LDA", "LDP", "OFF_G", "OFF_A", "OFF_P", "STG_END", "OFF_H0", "OFF_L", "O_DUMP", "LDS_QP"):
        m = re.search(r"^#define %s (\d+)$" % name, src, re.M)
        assert m, name
        d[name] = int(m.group(1))
    return d


def _table(src, name):
    m = re.search(r"static __device__ const int %s\[(\d+)\] = \{([^}]*)\}" % name, src)
    assert m, name
    return np.array([int(v) for v in m.group(2).split(",")])


def _cases():
    from apf_quadruped_amd import plans, workloads as W
    out = []
    for n, m, p in ((17, 20, 6), (32, 48, 16)):
        d = random_qps(n, m, p, 1, seed=1000 * n + m + p)
        out.append((f"dense{n}_{m}_{p}", d, True))
    for ph in ("stance", "trot", "crawl"):
        out.append((f"c30_{ph}", W.controller_qp(plans.SEED + 30, np.arange(1), phase=ph), True))
    out.append(("lin17_40_5", dense_qp(17, 40, 5, B=1, seed=7 * 17 + 40, linear_var=16), True))
    out.append(("full24_40_8", dense_qp(24, 40, 8, B=1, seed=5), False))
    return out


@pytest.mark.parametrize("idx", range(7))
def test_rowx_scatter_slots_inside_the_qp_block(idx):
    from apf_quadruped_amd.batch import Plan
    name, d, upper = _cases()[idx]
    n, m, p = d["n"], d["m"], d["p"]
    plan = Plan.from_dense(n, m, p, d["P"][0], d["A"][0] if p else None, d["G"][0], p_upper=upper)
    assert plan.kernel_name(65).startswith("qpb_rowx_"), (name, plan.kernel_name(65))
    src = plan.wave_source()
    L = _defs(src)
    scP, scP2, scG = _table(src, "qpb_scP"), _table(src, "qpb_scP2"), _table(src, "qpb_scG")
    nnzP, nnzA, nnzG = plan.nnz
    assert len(scP) == nnzP and len(scP2) == nnzP and len(scG) == nnzG
    # dense column-major copies: G at OFF_G (n columns of LDG), A at OFF_A, P at OFF_P
    assert ((scP >= 0) & (scP < n * L["LDP"])).all(), name
    assert ((scP2 == -1) | ((scP2 >= 0) & (scP2 < n * L["LDP"]))).all(), name
    assert (scP2 != -1).any() == (upper and any(scP % L["LDP"] != scP // L["LDP"])), name
    assert ((scG >= 0) & (scG < n * L["LDG"])).all() and (scG % L["LDG"] < m).all(), name
    if p:
        scA = _table(src, "qpb_scA")
        assert len(scA) == nnzA and ((scA >= 0) & (scA < n * L["LDA"])).all() and (scA % L["LDA"] < p).all()
        assert L["OFF_A"] + n * L["LDA"] <= L["OFF_P"]
    # both triangles of P inside the P copy; no two entries share a slot
    slots = np.concatenate([scP, scP2[scP2 >= 0]])
    assert len(np.unique(slots)) == len(slots), name
    assert L["OFF_G"] + n * L["LDG"] <= (L["OFF_A"] if p else L["OFF_P"])
    assert L["OFF_P"] + n * L["LDP"] <= L["STG_END"] and L["STG_END"] % 2 == 0
    rows = 17 * n if n <= 16 else 17 * 16 + 33 * (n - 16)
    assert L["OFF_H0"] == L["STG_END"] and L["OFF_L"] == L["OFF_H0"] + rows and L["O_DUMP"] == L["OFF_L"] + rows
    assert L["O_DUMP"] + 16 <= L["LDS_QP"] and 4 * L["LDS_QP"] * 8 <= 160 * 1024
    # the staging zero-fill (qpb_rowx.hip): row r starts at r LDS_QP doubles; 16-byte stores
    # from its first 16-byte aligned double, lane c storing pair c + 16 i while
    # 2 (c + 16 i) + 1 < STG_END - a0, plus Ls[0] and Ls[STG_END - 1] singly
    S = L["STG_END"]
    assert "for (int i = 0; i < (STG_END / 2 + 15) / 16; i++)" in src
    for row in range(4):
        a0 = (row * L["LDS_QP"]) & 1
        hit = np.zeros(S + 2, bool)
        for i in range((S // 2 + 15) // 16):
            for c in range(16):
                k = c + 16 * i
                if 2 * k + 1 < S - a0:
                    hit[a0 + 2 * k] = hit[a0 + 2 * k + 1] = True
        hit[0] = hit[S - 1] = True
        assert hit[:S].all() and not hit[S:].any(), (name, row, np.flatnonzero(~hit[:S])[:4])

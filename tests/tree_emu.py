"""CPU emulation of the tree kernel's gather programs (test tool, no GPU).

Parses the tables the generator prepends to qpb_tree.hip (Plan.tree_source())
and executes the programs step by step with the kernel's semantics (lane l of a
step sums terms l%G, l%G+G, ... of task l/G; the task's epilogue applies the
sum).  Used to check the generated KKT assembly, LDL', solves and residual
products against dense numpy linear algebra on the CPU."""
from __future__ import annotations

import re

import numpy as np

FB = 16
FM = (1 << FB) - 1


def parse_tables(src: str, blob: bytes) -> dict:
    """Sizes and table offsets from the generated source's macros; tables from
    the plan's table blob (u64 descriptors, then int32 tables)."""
    out = {}
    for m in re.finditer(r"#define (QPB_\w+) (-?\d+)\n", src):
        out[m.group(1)] = int(m.group(2))
    nd, nd32 = out["QPB_NDESC"], out["QPB_NDESC32"]
    D = np.frombuffer(blob[:8 * nd], dtype=np.uint64)
    D32 = np.frombuffer(blob[8 * nd:8 * nd + 4 * nd32], dtype=np.uint32).astype(np.uint64)
    I = np.frombuffer(blob[8 * nd + 4 * nd32:], dtype=np.int32).astype(np.int64)
    names = ["fac", "fwd", "bwd", "mv", "obj"]
    for k, name in enumerate(names):
        ns = out[f"QPB_{name}_NSTEPS"]
        d0 = out[f"QPB_D_{name}"]
        out[f"qpb_{name}_desc"] = D[d0:] if name == "fac" else D32[d0:]
        s0 = out[f"QPB_I_{name}_steps"]
        out[f"qpb_{name}_steps"] = I[s0:s0 + 4 * ns]
        h0 = out[f"QPB_I_{name}_hdr"]
        out[f"qpb_{name}_hdr"] = I[h0:]
    for name in ("pinv", "asrc_i", "asrc_l"):
        out[f"qpb_{name}"] = I[out[f"QPB_I_{name}"]:]
    out["I"] = I
    return out


PANEL = 1 << 17


def run_prog(T, name, term, epi, wg, panel=None):
    """Execute a program; panel(record) runs a supernode panel (qpb_tree.hip)."""
    steps = T[f"qpb_{name}_steps"].reshape(-1, 4)[:T[f"QPB_{name}_NSTEPS"]]
    hdr, desc = T[f"qpb_{name}_hdr"], T[f"qpb_{name}_desc"]
    I = T["I"]
    for doff, toff, ntg, rb in steps:
        if int(rb) & PANEL:
            for k in range(int(toff)):
                r0 = int(I[int(doff) + k])
                w = int(I[r0 + 1])
                panel(int(I[r0]), w, int(I[r0 + 2]), [int(v) for v in I[r0 + 3:r0 + 3 + w]])
            continue
        g = int(ntg) & 15
        G, nt, R = 1 << g, int(ntg) >> 4, int(rb) & 0xFFFF
        act = nt * G
        assert act <= wg
        acc = np.zeros(act)
        for r in range(R):
            for lane in range(act):
                d = int(desc[doff + r * act + lane])     # LDS byte offsets -> element indices
                acc[lane] = term(acc[lane], (d & FM) >> 3, ((d >> FB) & FM) >> 3, ((d >> (2 * FB)) & FM) >> 3)
        for t in range(nt):
            epi(int(hdr[toff + t]), float(acc[t * G:(t + 1) * G].sum()))


def rcp_reg(d):
    if abs(d) <= 1e-14:
        return 1e7 if d > 0 else -1e7
    return 1.0 / d


class TreeEmu:
    def __init__(self, plan):
        self.plan = plan
        self.src = plan.tree_source()
        self.T = parse_tables(self.src, plan.tree_tables())
        T = self.T
        self.n, self.m, self.p, self.N = T["QPB_NX"], T["QPB_NZ"], T["QPB_NY"], T["QPB_N"]
        self.lnz, self.wg = T["QPB_LNZ"], T["QPB_WG"]
        self.pinv = T["qpb_pinv"][:self.N]

    def assemble(self, pag, loop, s=None, z=None):
        src = self.T["qpb_asrc_l" if loop else "qpb_asrc_i"][: self.lnz + self.N]
        LD = np.zeros(self.lnz + 1)
        rD = np.zeros(self.N)
        for e, sc in enumerate(src):
            v = pag[sc] if sc >= 0 else 0.0 if sc == -1 else -1.0 if sc == -2 else -s[-3 - sc] / z[-3 - sc]
            if e < self.lnz:
                LD[e] = v
            else:
                rD[e - self.lnz] = v
        return LD, rD

    def factor(self, LD, rD):
        N = self.N

        def term(acc, a, b, k):
            return acc - LD[a] * rD[k] * LD[b]

        def epi(out, acc):
            if out >= 0:
                LD[out] += acc
            elif out >= -N:
                j = -1 - out
                rD[j] = rcp_reg(rD[j] + acc)
            else:
                rD[-1 - N - out] += acc          # supernode diagonal: raw

        def panel(j0, w, R, lp):
            # dense right-looking LDL' of the R x w panel (qpb_pfac)
            P = np.zeros((R, w))
            for c in range(w):
                P[c, c] = rD[j0 + c]
                for r in range(c + 1, R):
                    P[r, c] = LD[lp[c] + r - c - 1]
            for k in range(w):
                rk = rcp_reg(P[k, k])
                rD[j0 + k] = rk
                for c in range(k + 1, w):
                    P[c:, c] -= P[c:, k] * rk * P[c, k]
            for c in range(w):
                for r in range(c + 1, R):
                    LD[lp[c] + r - c - 1] = P[r, c]
        run_prog(self.T, "fac", term, epi, self.wg, panel)

    def solve(self, LD, rD, rhs_natural):
        W = np.zeros(self.N)
        W[self.pinv] = rhs_natural

        def tf(acc, a, k, _):
            return acc - LD[a] * W[k]

        def ef(i, acc):
            if i >= 0:
                W[i] = rD[i] * (W[i] + acc)
            else:
                W[-1 - i] += acc                 # supernode row: raw

        def eb(k, acc):
            W[k] = W[k] + rD[k] * acc

        def pf(j0, w, R, lp):                    # qpb_pfwd
            for k in range(w):
                W[j0 + k] *= rD[j0 + k]
                for c in range(k + 1, w):
                    W[j0 + c] -= LD[lp[k] + c - k - 1] * W[j0 + k]

        def pb(j0, w, R, lp):                    # qpb_pbwd
            for k in range(w - 1, -1, -1):
                for c in range(k):
                    W[j0 + c] -= rD[j0 + c] * LD[lp[c] + k - c - 1] * W[j0 + k]
        run_prog(self.T, "fwd", tf, ef, self.wg, pf)
        run_prog(self.T, "bwd", tf, eb, self.wg, pb)
        return W[self.pinv]

    def products(self, pag, v, prog="mv"):
        R = np.zeros(self.N)

        def term(acc, a, j, _):
            return acc + pag[a] * v[j]

        def epi(r, acc):
            R[r] = acc
        run_prog(self.T, prog, term, epi, self.wg)
        return R

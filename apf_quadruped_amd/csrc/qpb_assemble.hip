// qpb_assemble.hip -- on-device assembly of contact-force QPs.
//
// The controller builds its stance QP on the CPU from the robot terms every tick
// (dogbot_controller/src/client/main.cpp:1471-1647); for the contact-force block
// that is, with the feet ordered BR, BL, FL, FR (main.cpp:825-837) and
// Jc,i = [I3, -[r_i]x] for a stance foot i (zero rows for a swing foot):
//     P = 50 Jc Jc' + I              (main.cpp:1476-1480)
//     c = -50 Jc W                   (main.cpp:1573)
//     A = Jc',  b = W                (main.cpp:1580-1587)
//     G = blkdiag(cfr of the stance feet), h = 0   (main.cpp:1603-1625)
// qpb_assemble_contact evaluates this for B QPs at once -- one lane per (QP, output
// value), the tile's 18 input doubles per QP (foot positions relative to the CoM
// and the desired wrench) staged in LDS --
// writing straight into the plan's tiled SoA input arrays -- so APF / footstep
// samples generated on the device never round-trip through the host.
#include <hip/hip_runtime.h>

#include <mutex>

#include <cstring>
#include <string>
#include <vector>

#include "../../include/qpswift_hip.h"
#include "qpb_runtime.hpp"

namespace {

struct AsmMap {
    int nP, nA, nG, m;
    unsigned char Pr[144], Pc[144];   // (row, column) of every P value slot, CSC order
    unsigned char Ar[72], Ac[72];
    unsigned char Gr[240], Gc[240];
    signed char foot_of[4];           // stance feet in G-row-block order
    int stance;                       // bit i: foot i in contact
    double mu;
};

// J(u, j) of the contact Jacobian (12 x 6) of QP lane `ql`, foot positions in
// LDS (sr[3 i + a][ql]); u, j are wave-uniform, so every branch is uniform
__device__ __forceinline__ double qpb_jc(const double (*sr)[64], int ql, int stance, int u, int j) {
    const int i = u / 3, a = u - 3 * i;
    if (!((stance >> i) & 1)) return 0.0;
    if (j < 3) return a == j ? 1.0 : 0.0;
    // -[r]x, row a, column j - 3
    const int k = j - 3;
    if (a == k) return 0.0;
    const int o = 3 - a - k;                  // the remaining axis
    const double v = sr[3 * i + o][ql];
    // -[r]x = [[0, rz, -ry], [-rz, 0, rx], [ry, -rx, 0]]
    return ((a + 1) % 3 == k) ? v : -v;
}

// One block per tile of 64 QPs and slot chunk (blockIdx.y): the tile's foot
// positions and wrenches are staged in LDS once, then wave g of the block writes
// output slots s = blockIdx.y * 4 + g, + 4 gridDim.y, ... of all 64 QPs -- every
// store a coalesced 512-B row of the tiled layout.  Slots: P values, A, G, c, h, b.
__global__ void __launch_bounds__(256) qpb_assemble_contact_k(long B, const double *__restrict__ feet,
                                                              const double *__restrict__ wrench, AsmMap mp,
                                                              double *__restrict__ P, double *__restrict__ A,
                                                              double *__restrict__ G, double *__restrict__ c,
                                                              double *__restrict__ h, double *__restrict__ b) {
    __shared__ double sr[12][64], sw[6][64];
    const long tile = blockIdx.x;
    const int ql = threadIdx.x & 63, g = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < 18 * 64; i += 256) {
        const int j = i >> 6, l = i & 63;
        if (j < 12) sr[j][l] = feet[tile * (12 * 64) + i];
        else sw[j - 12][l] = wrench[tile * (6 * 64) + (i - 12 * 64)];
    }
    __syncthreads();
    if (tile * 64 + ql >= B) return;
    const int oA = mp.nP, oG = oA + mp.nA, oc = oG + mp.nG, oh = oc + 12, ob = oh + mp.m, S = ob + 6;
    for (int s = blockIdx.y * 4 + g; s < S; s += gridDim.y * 4) {
        if (s < oA) {
            const int u = mp.Pr[s], v = mp.Pc[s];
            double d = 0.0;
            for (int j = 0; j < 6; j++) d += qpb_jc(sr, ql, mp.stance, u, j) * qpb_jc(sr, ql, mp.stance, v, j);
            P[tile * ((long)mp.nP * 64) + s * 64 + ql] = 50.0 * d + (u == v ? 1.0 : 0.0);
        } else if (s < oG) {
            const int k = s - oA;
            A[tile * ((long)mp.nA * 64) + k * 64 + ql] = qpb_jc(sr, ql, mp.stance, mp.Ac[k], mp.Ar[k]);
        } else if (s < oc) {
            const int k = s - oG;
            const int row = mp.Gr[k], col = mp.Gc[k], blk = row / 5, t = row - 5 * blk;
            const int j = col - 3 * mp.foot_of[blk];
            // cfr (main.cpp:1610-1615): t1 - mu n, t2 - mu n, -t1 - mu n, -t2 - mu n, -n
            double v = 0.0;
            if (j == 2) v = t == 4 ? -1.0 : -mp.mu;
            else if (j == 0) v = t == 0 ? 1.0 : (t == 2 ? -1.0 : 0.0);
            else if (j == 1) v = t == 1 ? 1.0 : (t == 3 ? -1.0 : 0.0);
            G[tile * ((long)mp.nG * 64) + k * 64 + ql] = v;
        } else if (s < oh) {
            const int u = s - oc;
            double d = 0.0;
            for (int j = 0; j < 6; j++) d += qpb_jc(sr, ql, mp.stance, u, j) * sw[j][ql];
            c[tile * (12 * 64) + u * 64 + ql] = -50.0 * d;
        } else if (s < ob) {
            h[tile * ((long)mp.m * 64) + (s - oh) * 64 + ql] = 0.0;
        } else {
            b[tile * (6 * 64) + (s - ob) * 64 + ql] = sw[s - ob][ql];
        }
    }
}

// Structural pattern of a generic contact-force QP for `stance` (the exact zeros
// QP_SETUP_dense would drop): dense P of the stance feet plus the identity, A =
// Jc' (force columns: one entry, moment columns: the two off-axis arms), G the
// friction blocks.
void contact_pattern(int stance, bool upper, std::vector<std::vector<char>> &Pn, std::vector<std::vector<char>> &An,
                     std::vector<std::vector<char>> &Gn, int *m_out) {
    Pn.assign(12, std::vector<char>(12, 0));
    An.assign(6, std::vector<char>(12, 0));
    int m = 0;
    for (int i = 0; i < 4; i++) m += (stance >> i) & 1;
    m *= 5;
    Gn.assign(m, std::vector<char>(12, 0));
    auto jnz = [&](int u, int j) {
        const int i = u / 3, a = u - 3 * i;
        if (!((stance >> i) & 1)) return false;
        if (j < 3) return a == j;
        return (j - 3) != a;      // -[r]x: zero on the diagonal, generic elsewhere
    };
    for (int u = 0; u < 12; u++)
        for (int v = 0; v < 12; v++) {
            bool nz = u == v;
            for (int j = 0; j < 6 && !nz; j++) nz = jnz(u, j) && jnz(v, j);
            Pn[u][v] = nz && (!upper || u <= v);
        }
    for (int l = 0; l < 6; l++)
        for (int u = 0; u < 12; u++) An[l][u] = jnz(u, l);
    int blk = 0;
    for (int i = 0; i < 4; i++) {
        if (!((stance >> i) & 1)) continue;
        const int nzc[5][3] = {{1, 0, 1}, {0, 1, 1}, {1, 0, 1}, {0, 1, 1}, {0, 0, 1}};
        for (int t = 0; t < 5; t++)
            for (int j = 0; j < 3; j++) Gn[5 * blk + t][3 * i + j] = (char)nzc[t][j];
        blk++;
    }
    *m_out = m;
}

bool same_pattern(const qpb::Pattern &pt, const std::vector<std::vector<char>> &dense, unsigned char *rows,
                  unsigned char *cols, int cap, int *nnz) {
    const long R = (long)dense.size(), Cn = R ? (long)dense[0].size() : 0;
    if (pt.rows != R || pt.cols != Cn || pt.nnz() > cap) return false;
    long k = 0;
    for (long j = 0; j < Cn; j++)
        for (long i = 0; i < R; i++) {
            if (!dense[i][j]) continue;
            if (k >= pt.nnz() || pt.ir[k] != i || k < pt.jc[j] || k >= pt.jc[j + 1]) return false;
            rows[k] = (unsigned char)i;
            cols[k] = (unsigned char)j;
            k++;
        }
    *nnz = (int)k;
    return k == pt.nnz();
}

}  // namespace

extern "C" int qpb_assemble_contact(const qpb_plan *plan, long B, const double *feet, const double *wrench,
                                    int stance, double mu, double *P, double *A, double *G, double *c, double *h,
                                    double *b, void *stream) {
    if (!plan) return qpb::set_error(QPB_EINVAL, "NULL plan");
    if (B < 0) return qpb::set_error(QPB_EINVAL, "need B >= 0");
    if (stance <= 0 || stance > 15) return qpb::set_error(QPB_EINVAL, "stance: bitmask of 1-4 feet (bits 0-3)");
    const qpb::Plan &pl = plan->pl;
    std::vector<std::vector<char>> Pn, An, Gn;
    int m = 0;
    contact_pattern(stance, pl.pmode == qpb::P_UPPER, Pn, An, Gn, &m);
    AsmMap mp;
    std::memset(&mp, 0, sizeof mp);
    if (pl.n != 12 || pl.p != 6 || pl.m != m || !same_pattern(pl.Pin, Pn, mp.Pr, mp.Pc, 144, &mp.nP) ||
        !same_pattern(pl.A, An, mp.Ar, mp.Ac, 72, &mp.nA) || !same_pattern(pl.G, Gn, mp.Gr, mp.Gc, 240, &mp.nG))
        return qpb::set_error(QPB_ESHAPE, "plan is not the pattern of a contact-force QP with this stance");
    mp.m = m;
    mp.stance = stance;
    mp.mu = mu;
    for (int i = 0, k = 0; i < 4; i++)
        if ((stance >> i) & 1) mp.foot_of[k++] = (signed char)i;
    if (B == 0) return QPB_OK;
    if (!feet || !wrench || !P || !A || !G || !c || !h || !b) return qpb::set_error(QPB_EINVAL, "NULL data pointer");
    // one block per 64-QP tile x 4 slot chunks (16 waves share a tile's ~190 slots)
    const unsigned tiles = (unsigned)((B + 63) / 64);
    (void)hipGetLastError();   // a stale error of an earlier API call is not this launch's
    hipLaunchKernelGGL(qpb_assemble_contact_k, dim3(tiles, 4), dim3(256), 0, (hipStream_t)stream, B, feet, wrench, mp,
                       P, A, G, c, h, b);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return qpb::set_error(QPB_EHIP, (std::string("assemble: ") + hipGetErrorString(e)).c_str());
    return QPB_OK;
}

// ---------------------------------------------------------------------------
// The controller's own 30-variable stance QP (30/68/18) from its robot terms,
// main.cpp:1471-1647 (numpy restatement: workloads.controller_qp_from_terms):
//   Q = 50 T_s' T_s + I, T_s = Jstcom' Sigma_st        c = -T_s' (50 I)' Wcom_des
//   A = [M_com 0 -Jstcom'; Jstcom Jstj 0]              b = [-BiasCOM(0:6); -Jdqd]
//   D = friction(mu) | [0 M_jj -Jstj'] | -(same) | [0 I 0] | [0 -I 0]
//   C = 0 | 60 - bias_j | -(-60 - bias_j) | ddq_max | -ddq_min,
//       ddq_lim = (2 / dt^2)(q_lim - q - dt dq), dt = 0.025
// Robot terms per QP (QPB_ROBOT_NV doubles, tiled or one shared copy):
//   Jst[12][18] Mcom[6][6] Mjj[12][12] bias[18] jdqd[12] wdes[6] q dq qmin qmax[12].
// The host builds one entry per (matrix, row, column) of the dense QP (plus the
// c / h / b rows) with the plan's CSC slot, or -1 for a position outside the
// pattern; such positions must evaluate to exactly 0 -- QP_SETUP_dense would
// drop them -- which `check` records per QP.
namespace {

enum : int { T_JST = 0, T_MCOM = 216, T_MJJ = 252, T_BIAS = 396, T_JDQD = 414, T_WDES = 426, T_Q = 432, T_DQ = 444,
             T_QMIN = 456, T_QMAX = 468, T_NV = 480 };
enum : int { M_P = 0, M_A = 1, M_G = 2, M_C = 3, M_H = 4, M_B = 5 };

struct CtlArgs {
    const double *terms;
    long tstride;          // 0: one shared copy; 1: tiled SoA (nv = T_NV)
    const double *wdes;    // tiled nv = 6 or NULL (terms' wdes)
    const int *ent;        // pairs {code = mat << 16 | row << 8 | col, slot}
    int nent, nP, nA, nG;
    double mu;
    double *P, *A, *G, *c, *h, *b;
    int *check;
    long B;
};

#pragma clang fp contract(off)
struct CtlQP {
    const CtlArgs &a;
    long tile;
    int ql;
    __device__ double T(int i) const {
        return a.tstride ? a.terms[tile * (T_NV * 64) + (long)i * 64 + ql] : a.terms[i];
    }
    __device__ double W(int k) const { return a.wdes ? a.wdes[tile * (6 * 64) + k * 64 + ql] : T(T_WDES + k); }
    __device__ double J(int r, int col) const { return T(T_JST + r * 18 + col); }   // Jst(r, col)
    __device__ double value(int mat, int i, int j) const {
        switch (mat) {
        case M_P: {
            if (i >= 18 && j >= 18) {
                double d = 0.0;
                for (int k = 0; k < 6; k++) d = d + J(i - 18, k) * J(j - 18, k);
                return 50.0 * d + (i == j ? 1.0 : 0.0);
            }
            return i == j ? 1.0 : 0.0;
        }
        case M_A:
            if (i < 6) return j < 6 ? T(T_MCOM + 6 * i + j) : (j >= 18 ? -J(j - 18, i) : 0.0);
            return j < 18 ? J(i - 6, j) : 0.0;
        case M_G: {
            if (i < 20) {
                const int blk = i / 5, t = i - 5 * blk, jj = j - 18 - 3 * blk;
                if (jj < 0 || jj > 2) return 0.0;
                // cfr (main.cpp:1610-1615): t1 - mu n, t2 - mu n, -(t1 + mu n), -(t2 + mu n), -n
                if (jj == 2) return t == 4 ? -1.0 : -a.mu;
                if (jj == 0) return t == 0 ? 1.0 : (t == 2 ? -1.0 : 0.0);
                return t == 1 ? 1.0 : (t == 3 ? -1.0 : 0.0);
            }
            if (i < 44) {
                const double sg = i < 32 ? 1.0 : -1.0;
                const int l = i < 32 ? i - 20 : i - 32;
                if (j >= 6 && j < 18) return sg * T(T_MJJ + 12 * l + (j - 6));
                if (j >= 18) return -sg * J(j - 18, 6 + l);
                return 0.0;
            }
            const int l = i < 56 ? i - 44 : i - 56;
            return j == 6 + l ? (i < 56 ? 1.0 : -1.0) : 0.0;
        }
        case M_C: {
            if (i < 18) return 0.0;
            double d = 0.0;
            for (int k = 0; k < 6; k++) d = d + J(i - 18, k) * W(k);
            return -50.0 * d;
        }
        case M_H: {
            if (i < 20) return 0.0;
            if (i < 32) return 60.0 - T(T_BIAS + 6 + (i - 20));
            if (i < 44) return -(-60.0 - T(T_BIAS + 6 + (i - 32)));
            const double dt = 0.025, k2 = 2.0 / (dt * dt);
            const int l = i < 56 ? i - 44 : i - 56;
            const double lim = i < 56 ? T(T_QMAX + l) : T(T_QMIN + l);
            const double v = k2 * ((lim - T(T_Q + l)) - dt * T(T_DQ + l));
            return i < 56 ? v : -v;
        }
        default:
            return i < 6 ? -T(T_BIAS + i) : -T(T_JDQD + (i - 6));
        }
    }
};
#pragma clang fp contract(on)

// one block per 64-QP tile x entry chunk (blockIdx.y); wave g handles entries
// blockIdx.y * 4 + g, + 4 gridDim.y, ...: lane = QP, every store a coalesced row
__global__ void __launch_bounds__(256) qpb_assemble_controller_k(CtlArgs a) {
    const long tile = blockIdx.x;
    const int ql = threadIdx.x & 63, g = threadIdx.x >> 6;
    if (tile * 64 + ql >= a.B) return;
    const CtlQP qp{a, tile, ql};
    bool ok = true;
    for (int e = blockIdx.y * 4 + g; e < a.nent; e += gridDim.y * 4) {
        const int code = a.ent[2 * e], slot = a.ent[2 * e + 1];
        const int mat = code >> 16, i = (code >> 8) & 255, j = code & 255;
        const double v = qp.value(mat, i, j);
        if (slot < 0) { ok = ok && v == 0.0; continue; }
        double *dst = mat == M_P ? a.P + tile * ((long)a.nP * 64) : mat == M_A ? a.A + tile * ((long)a.nA * 64)
                    : mat == M_G ? a.G + tile * ((long)a.nG * 64) : mat == M_C ? a.c + tile * (30 * 64)
                    : mat == M_H ? a.h + tile * (68 * 64) : a.b + tile * (18 * 64);
        dst[(long)slot * 64 + ql] = v;
    }
    if (!ok && a.check) a.check[tile * 64 + ql] = 0;
}

__global__ void __launch_bounds__(256) qpb_fill_int_k(int *p, long n, int v) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i < n) p[i] = v;
}

// entries of the controller stance QP for this plan (see CtlArgs); empty if the
// plan's shape is not 30/68/18
std::vector<int> controller_entries(const qpb::Plan &pl) {
    std::vector<int> ent;
    if (pl.n != 30 || pl.m != 68 || pl.p != 18) return ent;
    auto slot_of = [](const qpb::Pattern &pt, int i, int j) {
        for (long k = pt.jc[j]; k < pt.jc[j + 1]; k++)
            if (pt.ir[k] == i) return (int)k;
        return -1;
    };
    const bool upper = pl.pmode == qpb::P_UPPER;
    for (int j = 0; j < 30; j++)
        for (int i = 0; i < 30; i++) {
            if (upper && i > j) continue;
            ent.push_back(M_P << 16 | i << 8 | j);
            ent.push_back(slot_of(pl.Pin, i, j));
        }
    for (int j = 0; j < 30; j++)
        for (int i = 0; i < 18; i++) { ent.push_back(M_A << 16 | i << 8 | j); ent.push_back(slot_of(pl.A, i, j)); }
    for (int j = 0; j < 30; j++)
        for (int i = 0; i < 68; i++) { ent.push_back(M_G << 16 | i << 8 | j); ent.push_back(slot_of(pl.G, i, j)); }
    for (int i = 0; i < 30; i++) { ent.push_back(M_C << 16 | i << 8); ent.push_back(i); }
    for (int i = 0; i < 68; i++) { ent.push_back(M_H << 16 | i << 8); ent.push_back(i); }
    for (int i = 0; i < 18; i++) { ent.push_back(M_B << 16 | i << 8); ent.push_back(i); }
    return ent;
}

// ---------------------------------------------------------------------------
// APF-sampled CoM targets (main.cpp:1263-1422) and the desired wrench the QP
// tracks (main.cpp:1484-1571), one lane per candidate target point:
//   per foot i: goal_i = target + (+-0.186571, +-0.289186)       (main.cpp:1171-1174)
//     e_a = sat2(ee_i - goal_i), K_pa = compute_Kpa(e_a), f_a = -K_pa e_a
//     f_r = 5 rob_i versor_i  (MIN_EXIT: 9 rob_i versor_i + 2.2 comb_rob lat_versor)
//     des_i = ee_i + 0.5 f_a (+ 0.5 f_r with REP_FIELD)
//   com_des = mean des_i; CoMPosDes = (sat_step(x), sat_step(y), 0.38, roll*, pitch*, 0)
//   deltax = CoMPosDes - CoM with deltax(3:6) rotated by world_H_base, deltav = -CoM_vel
//   Wcom_des = 3000 deltax + 50 deltav + m g e_z + M_com CoMAccD
// (the per-step TOWR spline between the target and the tick, out of scope here,
// is replaced by its target: CoMPosD = CoMPosDes, CoMVelD = 0).
struct ApfArgs {
    qpb_apf_state st;
    const double *targets;   // tiled nv = 2
    double *wrench;          // tiled nv = 6
    double *com_des;         // tiled nv = 6 or NULL
    long K;
};

__device__ __forceinline__ double apf_sat(double v, double lim) { return fabs(v) > lim ? copysign(lim, v) : v; }

#pragma clang fp contract(off)
__global__ void __launch_bounds__(256) qpb_apf_wrench_k(ApfArgs a) {
    const long k = (long)blockIdx.x * 256 + threadIdx.x;
    if (k >= a.K) return;
    const long tile = k >> 6;
    const int ql = (int)(k & 63);
    const qpb_apf_state &s = a.st;
    const double tx = a.targets[tile * 128 + ql], ty = a.targets[tile * 128 + 64 + ql];
    const double sx[4] = {+1.0, -1.0, -1.0, +1.0}, sy[4] = {-1.0, -1.0, +1.0, +1.0};   // BR BL FL FR
    auto fr = [](double v) { return fabs(v) < 0.07 ? 0.0 : fabs(v); };                   // compute_fr
    const double comb = fr(s.rob_foot[0] - s.rob_foot[1]) + fr(s.rob_foot[3] - s.rob_foot[2]) +
                        fr(fabs(s.rob_foot[0] - s.rob_foot[3])) + fr(fabs(s.rob_foot[1] - s.rob_foot[2]));
    double cx = 0.0, cy = 0.0;
    for (int i = 0; i < 4; i++) {
        const double ex = apf_sat(s.ee[i][0] - (tx + sx[i] * 0.186571), 2.0);
        const double ey = apf_sat(s.ee[i][1] - (ty + sy[i] * 0.289186), 2.0);
        // compute_Kpa (main.cpp:2803-2843)
        const double kx = fabs(ex) < 0.4 ? (s.fake_crawl ? 0.01 : 0.3) : (s.min_exit ? 0.1 : (s.fake_crawl ? 0.01 : 0.3));
        const double ky = fabs(ey) < 0.4 ? (s.fake_crawl ? 0.01 : 0.4) : (s.min_exit ? 0.2 : (s.fake_crawl ? 0.01 : 0.4));
        const double fax = -kx * ex, fay = -ky * ey;
        double frx, fry;
        if (s.min_exit) {
            frx = 9 * s.rob_foot[i] * s.versor[i][0] + 2.2 * comb * s.lat_versor[0];
            fry = 9 * s.rob_foot[i] * s.versor[i][1] + 2.2 * comb * s.lat_versor[1];
        } else {
            frx = 5 * s.rob_foot[i] * s.versor[i][0];
            fry = 5 * s.rob_foot[i] * s.versor[i][1];
        }
        double dx = s.ee[i][0] + 0.5 * fax, dy = s.ee[i][1] + 0.5 * fay;
        if (s.rep_field) { dx = dx + 0.5 * frx; dy = dy + 0.5 * fry; }
        cx = cx + dx;
        cy = cy + dy;
    }
    cx = cx / 4;
    cy = cy / 4;
    // saturate_xstep / saturate_ystep (main.cpp:2767-2790): at most 6 cm from the CoM
    const double stx = s.com[0] - cx, sty = s.com[1] - cy;
    const double px = fabs(stx) > 0.06 ? s.com[0] - copysign(0.06, stx) : cx;
    const double py = fabs(sty) > 0.06 ? s.com[1] - copysign(0.06, sty) : cy;
    const double pd[6] = {px, py, 0.38, s.des_orient[0], s.des_orient[1], 0.0};
    double dxv[6];
    for (int r = 0; r < 6; r++) dxv[r] = pd[r] - s.com[r];
    double rot[3];
    for (int r = 0; r < 3; r++) rot[r] = s.R_wb[3 * r] * dxv[3] + s.R_wb[3 * r + 1] * dxv[4] + s.R_wb[3 * r + 2] * dxv[5];
    for (int r = 0; r < 3; r++) dxv[3 + r] = rot[r];
    for (int r = 0; r < 6; r++) {
        double mac = 0.0;
        for (int c = 0; c < 6; c++) mac = mac + s.Mcom[6 * r + c] * s.acc_des[c];
        const double w = 3000.0 * dxv[r] + 50.0 * (0.0 - s.com_vel[r]) + (r == 2 ? s.mass * 9.81 : 0.0) + mac;
        a.wrench[tile * 384 + r * 64 + ql] = w;
        if (a.com_des) a.com_des[tile * 384 + r * 64 + ql] = pd[r];
    }
}
#pragma clang fp contract(on)

}  // namespace

extern "C" int qpb_assemble_controller(const qpb_plan *plan_c, long B, const double *terms, int terms_shared,
                                       const double *wdes, double mu, double *P, double *A, double *G, double *c,
                                       double *h, double *b, int *check, void *stream) {
    qpb_plan *plan = const_cast<qpb_plan *>(plan_c);
    if (!plan) return qpb::set_error(QPB_EINVAL, "NULL plan");
    if (B < 0) return qpb::set_error(QPB_EINVAL, "need B >= 0");
    // the plan's entry table (host, then per device) is built once, under a lock:
    // concurrent callers on one plan must not build or upload it twice
    void *tab = nullptr;
    size_t nent = 0;
    {
        static std::mutex mu;
        std::lock_guard<std::mutex> lk(mu);
        if (plan->ctl_table.empty()) plan->ctl_table = controller_entries(plan->pl);
        if (plan->ctl_table.empty()) return qpb::set_error(QPB_ESHAPE, "plan is not a 30/68/18 controller stance QP");
        if (B == 0) return QPB_OK;
        if (!terms || !P || !A || !G || !c || !h || !b) return qpb::set_error(QPB_EINVAL, "NULL data pointer");
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess) return qpb::set_error(QPB_EHIP, "hipGetDevice failed (no GPU?)");
        nent = plan->ctl_table.size();
        auto it = plan->ctl_dev.find(dev);
        if (it != plan->ctl_dev.end()) tab = it->second;
        else {
            const size_t bytes = nent * sizeof(int);
            if (hipMalloc(&tab, bytes) != hipSuccess) return qpb::set_error(QPB_ENOMEM, "assembly table");
            if (hipMemcpy(tab, plan->ctl_table.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) {
                (void)hipFree(tab);     // nothing half-uploaded stays in the cache
                return qpb::set_error(QPB_EHIP, "assembly table upload");
            }
            plan->ctl_dev[dev] = tab;
        }
    }
    const qpb::Plan &pl = plan->pl;
    CtlArgs a{terms, terms_shared ? 0L : 1L, wdes, (const int *)tab, (int)(nent / 2),
              (int)pl.Pin.nnz(), (int)pl.A.nnz(), (int)pl.G.nnz(), mu, P, A, G, c, h, b, check, B};
    (void)hipGetLastError();   // a stale error of an earlier API call is not these launches'
    if (check)
        hipLaunchKernelGGL(qpb_fill_int_k, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, (hipStream_t)stream, check,
                           B, 1);
    const unsigned tiles = (unsigned)((B + 63) / 64);
    hipLaunchKernelGGL(qpb_assemble_controller_k, dim3(tiles, 8), dim3(256), 0, (hipStream_t)stream, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return qpb::set_error(QPB_EHIP, (std::string("assemble: ") + hipGetErrorString(e)).c_str());
    return QPB_OK;
}

// main.cpp:1273-1276 (the smoothing, per foot, in BR BL FL FR order of the state)
// and :1307-1321 (robf_to_mean = (bl + fr + br + fl) / 4, fake_crawl below 0.34)
extern "C" int qpb_apf_update(qpb_apf_state *st, const double h_prev[4], double period_st, double *robf_mean) {
    if (!st || !h_prev) return qpb::set_error(QPB_EINVAL, "bad APF update arguments");
    for (int i = 0; i < 4; i++) st->rob_foot[i] = 0.35 * st->rob_foot[i] + 0.65 * h_prev[i] / period_st;
    const double *rf = st->rob_foot;        // 0 BR, 1 BL, 2 FL, 3 FR
    const double mean = (rf[1] + rf[3] + rf[0] + rf[2]) / 4.0;
    st->fake_crawl = mean < 0.34 ? 1 : 0;
    if (robf_mean) *robf_mean = mean;
    return QPB_OK;
}

extern "C" int qpb_apf_wrench(long K, const qpb_apf_state *st, const double *targets, double *wrench,
                              double *com_des, void *stream) {
    if (K < 0 || !st) return qpb::set_error(QPB_EINVAL, "bad APF arguments");
    if (K == 0) return QPB_OK;
    if (!targets || !wrench) return qpb::set_error(QPB_EINVAL, "NULL data pointer");
    ApfArgs a{*st, targets, wrench, com_des, K};
    (void)hipGetLastError();   // a stale error of an earlier API call is not this launch's
    hipLaunchKernelGGL(qpb_apf_wrench_k, dim3((unsigned)((K + 255) / 256)), dim3(256), 0, (hipStream_t)stream, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return qpb::set_error(QPB_EHIP, (std::string("apf: ") + hipGetErrorString(e)).c_str());
    return QPB_OK;
}

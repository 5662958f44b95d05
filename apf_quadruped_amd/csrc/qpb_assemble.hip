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
    hipLaunchKernelGGL(qpb_assemble_contact_k, dim3(tiles, 4), dim3(256), 0, (hipStream_t)stream, B, feet, wrench, mp,
                       P, A, G, c, h, b);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return qpb::set_error(QPB_EHIP, (std::string("assemble: ") + hipGetErrorString(e)).c_str());
    return QPB_OK;
}

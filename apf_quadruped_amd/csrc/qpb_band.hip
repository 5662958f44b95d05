// qpb_band.hip -- multi-stage (block-tridiagonal) IPM kernel: ONE QP per wavefront.
//
// Template source like qpb_row.hip (the host prepends the row template's common
// helpers, then sizes, the CSC -> LDS scatter tables and the stage patterns;
// qpb_wave.cpp generate_band_kernel).  For plans whose variables split into NS
// stages of NB (x), MZ (z) and MY (y) rows with
//   P block diagonal,  G row group k on stage k only,  A row group k on stages k-1, k
// -- a horizon QP such as the MPC contact-force problem of configs[3] (12 / 20 / 6 per
// stage) -- ordered leaves first (z rows, y rows, x in natural order:
// qpb_plan.cpp ORDER_LEAVES, which the plan takes for such patterns).  Every z / y
// row is then a leaf, and the x block of the KKT Schur complement is block
// tridiagonal over the stages:
//   H_kk     = P_k + G_k' W_k G_k + 1e7 (AR_k' AR_k + AL_{k+1}' AL_{k+1})
//   H_k,k-1  = X_k = 1e7 AR_k' AL_k            (AR_k / AL_k: A row group k on stage k / k-1)
// whose LDL' in natural order is the block recurrence
//   Z_k = X_k L_{k-1}^-T,  S_k = H_kk - Z_k D_{k-1}^-1 Z_k',  S_k = L_k D_k L_k'
// -- the same factor as the reference's up-looking LDL' of the permuted KKT matrix
// (ldl.c:253-326, pivot regularisation ldl.c:273-274), in block form, and the same
// triangular solves (kktsolve, Auxilary.c:471-564) as block forward / backward sweeps.
//
// Lanes: x quantities of the current stage live in lane c = lane & 15 of EVERY 16-lane
// DPP row (four identical copies), so a z row r (lane r < MZ <= 64) or a y row
// (lane l < MY <= 64) reads x_j of its stage with a DPP row_newbcast:j in any row;
// the 12 x 12 stage blocks are the row kernel's DPP products and pivot chain.  z / y
// values reach the x lanes through LDS (same-address broadcast reads).  All of the
// QP's state -- P, G, A stage blocks, the factor's L_k (with 1/D_k) and -Z_k rows, the
// iterate, residuals and directions -- stays in the workgroup's LDS for the whole
// solve (79 KB for MPC: two QPs per CU); inputs are read once, outputs written once.
//
// The loop is the row kernel's (qpSWIFT.c:473-644): kkt_initialize as iteration -1,
// residuals + exit test, factor, predictor, corrector, step lengths (Auxilary.c:359-393),
// update; fast mode (FMA contraction, reciprocal pivots).
#pragma clang fp contract(fast)

#define NB QPB_BNB
#define NS QPB_BNS
#define MZ QPB_BMZ
#define MY QPB_BMY
#define MY1 (MY > 0 ? MY : 1)
#define BNX (NB * NS)
#define BNZ (MZ * NS)
#define BNY (MY * NS)
#define BNY1 (BNY > 0 ? BNY : 1)
// per-stage blocks and vectors (doubles; offsets emitted by the generator, qpb_wave.cpp
// band_layout): O_P P_k rows (stride NB), O_L rows of -L_k at stride RS = NB + 1 (zeros
// from the diagonal on, 1 / D_c at column NB), O_Z rows of -Z_k (stride NB), O_G G_k rows,
// O_AR / O_AL the A row groups' stage-k / stage-(k-1) parts (stride NB); the vectors
// x, rx, dx | y, ry, dy | z, s, rz, dz, ds, w in natural order; V_Q one stage's w o bz.
#define BLKP (NB * NB)
#define BLKL (NB * RS)
static_assert(NB >= 1 && NB <= 16 && MZ >= 1 && MZ <= 64 && MY <= 64 && NS >= 2, "band kernel sizes");

// 64-lane sums / maxima: the row butterfly, then the four row results (fixed order)
static __device__ __forceinline__ double qpb_bsum(double v) {
    double t[1] = {v};
    qpb_rsum<1>(t);
    return (qpb_rl64(t[0], 0) + qpb_rl64(t[0], 16)) + (qpb_rl64(t[0], 32) + qpb_rl64(t[0], 48));
}
static __device__ __forceinline__ double qpb_bmax(double v) {
    double t[1] = {v};
    qpb_rmax<1>(t);
    return __builtin_fmax(__builtin_fmax(qpb_rl64(t[0], 0), qpb_rl64(t[0], 16)),
                          __builtin_fmax(qpb_rl64(t[0], 32), qpb_rl64(t[0], 48)));
}

#ifndef QPB_B_TIMING
#define QPB_B_TIMING 0    // 1: cycles per phase (w + residuals, factor, predictor, corrector, steps +
                          // updates, staging) into stats instead of the statistics
#endif
#if QPB_B_TIMING
#define QPB_BT(k) { const long t2_ = (long)__builtin_readcyclecounter(); tph[k] += (double)(t2_ - tcy); tcy = t2_; }
#else
#define QPB_BT(k)
#endif

// solve modes: the right-hand side's z part (bx = RX, by = RY in every mode)
enum { BM_SETUP = 0, BM_PRED = 1, BM_CORR = 2 };

static __device__ __forceinline__ void qpb_band_body(const qpb_args &a, long q, double *__restrict__ Ls) {
    const int lane = threadIdx.x & 63, c = lane & 15;
    if (q >= a.B) return;                      // grid padding (XCD order): wave-uniform
#if QPB_B_TIMING
    double tph[6] = {0, 0, 0, 0, 0, 0};
    long tcy = (long)__builtin_readcyclecounter();
#endif
    const long tile = q >> 6;
    const int ql = (int)(q & 63);
    const int xc = c < NB ? c : NB - 1;        // x lane (clamped: lanes NB..15 compute copies)
    const bool x0 = lane < NB;                 // the x lanes that store / count (row 0)
    const bool isz = lane < MZ, isy = lane < MY;
    const int zr = isz ? lane : MZ - 1, yl = isy ? lane : (MY > 0 ? MY - 1 : 0);
    constexpr double RDY = 1.0 / -1e-7;        // leaf y pivots: D = 0 regularised to -1e-7

    // ---- stage P, G, A into the per-stage dense blocks; c, b, h into RX, RY, RZ
    for (int i = lane; i < O_STATIC_END; i += 64) Ls[i] = 0.0;
    qpb_wsync();
    {
        const double *tP = a.P + tile * (QPB_NNZP * QPB_TSTR) + ql;
        for (int k = lane; k < QPB_NNZP; k += 64) {
            const double v = QPB_LDS(&tP[k * QPB_TSTR]);
            Ls[qpb_bsP[k]] = v;
            if (qpb_bsP2[k] >= 0) Ls[qpb_bsP2[k]] = v;
        }
        const double *tG = a.G + tile * (QPB_NNZG * QPB_TSTR) + ql;
        for (int k = lane; k < QPB_NNZG; k += 64) Ls[qpb_bsG[k]] = QPB_LDS(&tG[k * QPB_TSTR]);
#if MY > 0
        const double *tA = a.A + tile * (QPB_NNZA * QPB_TSTR) + ql;
        for (int k = lane; k < QPB_NNZA; k += 64) Ls[qpb_bsA[k]] = QPB_LDS(&tA[k * QPB_TSTR]);
#endif
        for (int i = lane; i < BNX; i += 64) Ls[V_RX + i] = -QPB_LDS(&a.c[tile * (BNX * QPB_TSTR) + i * QPB_TSTR + ql]);
#if MY > 0
        for (int i = lane; i < BNY; i += 64) Ls[V_RY + i] = QPB_LDS(&a.b[tile * (BNY * QPB_TSTR) + i * QPB_TSTR + ql]);
#endif
        for (int i = lane; i < BNZ; i += 64) {
            Ls[V_RZ + i] = QPB_LDS(&a.h[tile * (BNZ * QPB_TSTR) + i * QPB_TSTR + ql]);
            Ls[V_Z + i] = 1.0;
            Ls[V_S + i] = 1.0;
        }
        for (int i = lane; i < BNX; i += 64) Ls[V_X + i] = 0.0;
        for (int i = lane; i < BNY; i += 64) Ls[V_Y + i] = 0.0;
    }
    qpb_wsync();
    QPB_BT(5);

    // per-element helpers (z lanes): 1 / z, the KKT diagonal's w = -1 / regularise(-s / z)
    auto wz = [](double s, double z) { return -qpb_rcp_reg(-s * qpb_rcp(z)); };
    auto w_pass = [&](bool setup) {
        for (int i = lane; i < BNZ; i += 64)
            Ls[V_W + i] = setup ? 1.0 : wz(Ls[V_S + i], Ls[V_Z + i]);   // kkt_initialize: -I (w = 1)
        qpb_wsync();
    };

    // ---- factor: block LDL' of the x block, stage by stage
    double nLp[NB], rdp = 0.0;                 // previous stage: row xc of -L, 1 / D_xc
#pragma unroll
    for (int f = 0; f < NB; f++) nLp[f] = 0.0;
    auto factor = [&]() {
#pragma unroll 1
        for (int k = 0; k < NS; k++) {
            const double *Pr = Ls + O_P + k * BLKP + xc * NB;
            const double *Gk = Ls + O_G + k * (MZ * NB);
            const double *Wk = Ls + V_W + k * MZ;
            double H[NB];
#pragma unroll
            for (int j = 0; j < NB; j++) H[j] = Pr[j];
            // + G_k' W_k G_k: per row r, lane j's G(r, j) broadcast against G(r, c) w_r
            qpb_for<0, MZ>([&](auto rc) {
                constexpr int r = decltype(rc)::value;
                const double g = Gk[r * NB + xc];
                const double t = g * Wk[r];
                qpb_fence(g, t);
                qpb_for<0, NB>([&](auto jc) {
                    constexpr int j = decltype(jc)::value;
                    if constexpr ((qpb_bGm[r] >> j) & 1) qpb_fx<j>(H[j], g, t);
                });
            });
#if MY > 0
            // + 1e7 AR_k' AR_k + 1e7 AL_{k+1}' AL_{k+1}
            const double *ARk = Ls + O_AR + k * (MY * NB);
            qpb_for<0, MY>([&](auto lc) {
                constexpr int l = decltype(lc)::value;
                const double av = ARk[l * NB + xc];
                const double t = -RDY * av;
                qpb_fence(av, t);
                qpb_for<0, NB>([&](auto jc) {
                    constexpr int j = decltype(jc)::value;
                    if constexpr ((qpb_bARm[l] >> j) & 1) qpb_fx<j>(H[j], av, t);
                });
            });
            if (k + 1 < NS) {
                const double *ALn = Ls + O_AL + (k + 1) * (MY * NB);
                qpb_for<0, MY>([&](auto lc) {
                    constexpr int l = decltype(lc)::value;
                    const double av = ALn[l * NB + xc];
                    const double t = -RDY * av;
                    qpb_fence(av, t);
                    qpb_for<0, NB>([&](auto jc) {
                        constexpr int j = decltype(jc)::value;
                        if constexpr ((qpb_bALm[l] >> j) & 1) qpb_fx<j>(H[j], av, t);
                    });
                });
            }
            if (k > 0) {
                // X_k(c, j) = 1e7 sum_l AR_k(l, c) AL_k(l, j); Z_k = X_k L_{k-1}^-T
                const double *ALk = Ls + O_AL + k * (MY * NB);
                double Zr[NB];
#pragma unroll
                for (int j = 0; j < NB; j++) Zr[j] = 0.0;
                qpb_for<0, MY>([&](auto lc) {
                    constexpr int l = decltype(lc)::value;
                    const double al = ALk[l * NB + xc];
                    const double t = -RDY * ARk[l * NB + xc];
                    qpb_fence(al, t);
                    qpb_for<0, NB>([&](auto jc) {
                        constexpr int j = decltype(jc)::value;
                        if constexpr ((qpb_bALm[l] >> j) & 1) qpb_fx<j>(Zr[j], al, t);
                    });
                });
                // Z(c, e) = X(c, e) - sum_{f<e} L_{k-1}(e, f) Z(c, f): lane e's -L row broadcast,
                // right-looking (column f of Z final -> every later column), so consecutive
                // FMAs are independent; each Z(c, e) still sums over f in ascending order
                qpb_for<0, NB - 1>([&](auto fc) {
                    constexpr int f = decltype(fc)::value;
                    qpb_for<f + 1, NB>([&](auto ec) {
                        constexpr int e = decltype(ec)::value;
                        qpb_fx<e>(Zr[e], nLp[f], Zr[f]);
                    });
                });
                // H -= Z D_{k-1}^-1 Z'; -Z rows to LDS (the solves' coupling terms)
                double *Zs = Ls + O_Z + k * BLKP + xc * NB;
                qpb_for<0, NB>([&](auto ec) {
                    constexpr int e = decltype(ec)::value;
                    const double t = -(Zr[e] * qpb_nb<e>(rdp));
                    qpb_fence(t);
                    qpb_for<0, NB>([&](auto jc) {
                        constexpr int j = decltype(jc)::value;
                        qpb_fx<j>(H[j], Zr[e], t);
                    });
                });
                if (x0) {
#pragma unroll
                    for (int e = 0; e < NB; e++) Zs[e] = -Zr[e];
                }
            }
#endif
            // LDL' of the stage block in natural order (the row kernel's pivot chain)
            double rDd = 0.0;
            double dpiv = qpb_nb<0>(H[0]);
            qpb_for<0, NB>([&](auto kc) {
                constexpr int kk = decltype(kc)::value;
                const double rd = qpb_rcp_reg(dpiv);
                double nl = H[kk] * -rd;
                asm volatile("" : "+v"(nl));
                if constexpr (kk + 1 < NB) {
                    const double h = qpb_nb<kk + 1>(H[kk]), hkk = qpb_nb<kk + 1>(H[kk + 1]);
                    dpiv = __builtin_fma(-(h * h), rd, hkk);
                }
                rDd = xc == kk ? rd : rDd;
                qpb_for<kk + 1, NB>([&](auto jc) {
                    constexpr int j = decltype(jc)::value;
                    qpb_fxs<j>(H[j], H[kk], nl);
                });
                H[kk] = xc > kk ? nl : 0.0;
            });
            double *Lr = Ls + O_L + k * BLKL + xc * RS;
            if (x0) {
#pragma unroll
                for (int f = 0; f < NB; f++) Lr[f] = H[f];
                Lr[NB] = rDd;
            }
#pragma unroll
            for (int f = 0; f < NB; f++) nLp[f] = H[f];
            rdp = rDd;
        }
        qpb_wsync();
    };

    // ---- solve K [dx; dy; dz] = [RX; RY; bz] (bz per mode) into DX, DY, DZ (+ DS)
    // smu, pcd: the corrector's sigma mu and whether the predictor ran (its dz in DZ)
    auto bz_of = [&](int mode, int i, double smu, bool pcd, double *cc_out) -> double {
        const double rz = Ls[V_RZ + i];
        if (mode == BM_SETUP) return rz;
        const double s = Ls[V_S + i];
        if (mode == BM_PRED) return rz + s;
        const double rzi = qpb_rcp(Ls[V_Z + i]);
        double cc = smu;
        if (pcd) {
            const double dzp = Ls[V_DZ + i];
            const double dslp = -s * __builtin_fma(dzp, rzi, 1.0);
            cc = __builtin_fma(-dslp, dzp, smu);
        }
        *cc_out = cc;
        return __builtin_fma(-cc, rzi, rz + s);
    };
    auto solve = [&](int mode, double smu, bool pcd) {
        // forward: u_k = L_k^-1 (t_k - Z_k v_{k-1}), v_k = D_k^-1 u_k -> DX
        double vprev = 0.0;
#pragma unroll 1
        for (int k = 0; k < NS; k++) {
            // leaf values of the stage's z rows: w_r bz_r (LDS, read by every x lane)
            if (isz) {
                double cc;
                const int i = k * MZ + lane;
                Ls[V_Q + lane] = Ls[V_W + i] * bz_of(mode, i, smu, pcd, &cc);
            }
            qpb_wsync();
            const double *Gk = Ls + O_G + k * (MZ * NB);
            double ta[4] = {Ls[V_RX + k * NB + xc], 0.0, 0.0, 0.0};
#pragma unroll
            for (int r = 0; r < MZ; r++) ta[r & 3] = __builtin_fma(Gk[r * NB + xc], Ls[V_Q + r], ta[r & 3]);
#if MY > 0
            const double *ARk = Ls + O_AR + k * (MY * NB);
#pragma unroll
            for (int l = 0; l < MY; l++)
                ta[(MZ + l) & 3] = __builtin_fma(ARk[l * NB + xc] * -RDY, Ls[V_RY + k * MY + l], ta[(MZ + l) & 3]);
            if (k + 1 < NS) {
                const double *ALn = Ls + O_AL + (k + 1) * (MY * NB);
#pragma unroll
                for (int l = 0; l < MY; l++)
                    ta[(MZ + MY + l) & 3] =
                        __builtin_fma(ALn[l * NB + xc] * -RDY, Ls[V_RY + (k + 1) * MY + l], ta[(MZ + MY + l) & 3]);
            }
#endif
            double t = (ta[0] + ta[1]) + (ta[2] + ta[3]);
            const double *Zr = Ls + O_Z + k * BLKP + xc * NB;
            const double *Lr = Ls + O_L + k * BLKL + xc * RS;
            if (k > 0) {
                double nz[NB];
#pragma unroll
                for (int e = 0; e < NB; e++) nz[e] = Zr[e];
                qpb_fence(vprev);
                qpb_for<0, NB>([&](auto ec) { qpb_fx<decltype(ec)::value>(t, vprev, nz[decltype(ec)::value]); });
            }
            double nl[NB];
#pragma unroll
            for (int f = 0; f < NB; f++) nl[f] = Lr[f];
            const double rd = Lr[NB];
            qpb_fence(t);
            qpb_for<0, NB>([&](auto fc) { qpb_fxd<decltype(fc)::value>(t, nl[decltype(fc)::value]); });
            vprev = t * rd;
            if (x0) Ls[V_DX + k * NB + c] = vprev;
            qpb_wsync();
        }
        // backward: dx_k = L_k^-T (v_k - D_k^-1 Z_{k+1}' dx_{k+1}); dz, dy of the stages
        double dxn = 0.0;
#pragma unroll 1
        for (int k = NS - 1; k >= 0; k--) {
            const double *Lk = Ls + O_L + k * BLKL;
            double r = Ls[V_DX + k * NB + xc];
            if (k + 1 < NS) {
                const double *Zn = Ls + O_Z + (k + 1) * BLKP;    // -Z_{k+1}, read by columns
                double zt[NB];
#pragma unroll
                for (int j = 0; j < NB; j++) zt[j] = Zn[j * NB + xc];
                double acc = 0.0;
                qpb_fence(dxn);
                qpb_for<0, NB>([&](auto jc) { qpb_fx<decltype(jc)::value>(acc, dxn, zt[decltype(jc)::value]); });
                r = __builtin_fma(acc, Lk[xc * RS + NB], r);
            }
            double lt[NB];
#pragma unroll
            for (int e = 0; e < NB; e++) lt[e] = Lk[e * RS + xc];      // -L(e, c): column c
            qpb_fence(r);
            qpb_for<0, NB>([&](auto ec) {
                constexpr int e = NB - 1 - decltype(ec)::value;
                qpb_fxd<e>(r, lt[e]);
            });
            const double dx = r;
            if (x0) Ls[V_DX + k * NB + c] = dx;
            // z rows of stage k: dz = w (G dx - bz)
            {
                const double *Gr = Ls + O_G + k * (MZ * NB) + zr * NB;
                double g[NB];
#pragma unroll
                for (int j = 0; j < NB; j++) g[j] = Gr[j];
                double gs = 0.0;
                qpb_fence(dx);
                qpb_for<0, NB>([&](auto jc) {
                    constexpr int j = decltype(jc)::value;
                    if constexpr ((qpb_bGu >> j) & 1) qpb_fx<j>(gs, dx, g[j]);
                });
                if (isz) {
                    const int i = k * MZ + lane;
                    double cc = 0.0;
                    const double bz = bz_of(mode, i, smu, pcd, &cc);
                    const double w = Ls[V_W + i];
                    const double dz = w * (gs - bz);
                    Ls[V_DZ + i] = dz;
                    if (mode == BM_CORR) {
                        const double s = Ls[V_S + i], rzi = qpb_rcp(Ls[V_Z + i]);
                        Ls[V_DS + i] = __builtin_fma(__builtin_fma(-s, dz, cc), rzi, -s);
                    }
                }
            }
#if MY > 0
            // y rows of stage k + 1 (their x neighbours dx_{k+1}, dx_k are known now)
            if (k + 1 < NS) {
                const double *ARn = Ls + O_AR + (k + 1) * (MY * NB) + yl * NB;
                const double *ALn = Ls + O_AL + (k + 1) * (MY * NB) + yl * NB;
                double ar[NB], al[NB];
#pragma unroll
                for (int j = 0; j < NB; j++) { ar[j] = ARn[j]; al[j] = ALn[j]; }
                double gy = 0.0;
                qpb_fence(dxn, dx);
                qpb_for<0, NB>([&](auto jc) {
                    constexpr int j = decltype(jc)::value;
                    if constexpr ((qpb_bARu >> j) & 1) qpb_fx<j>(gy, dxn, ar[j]);
                    if constexpr ((qpb_bALu >> j) & 1) qpb_fx<j>(gy, dx, al[j]);
                });
                if (isy) {
                    const int i = (k + 1) * MY + lane;
                    Ls[V_DY + i] = RDY * (Ls[V_RY + i] - gy);
                }
            }
            if (k == 0) {
                const double *AR0 = Ls + O_AR + yl * NB;
                double ar[NB];
#pragma unroll
                for (int j = 0; j < NB; j++) ar[j] = AR0[j];
                double gy = 0.0;
                qpb_fence(dx);
                qpb_for<0, NB>([&](auto jc) {
                    constexpr int j = decltype(jc)::value;
                    if constexpr ((qpb_bARu >> j) & 1) qpb_fx<j>(gy, dx, ar[j]);
                });
                if (isy) Ls[V_DY + lane] = RDY * (Ls[V_RY + lane] - gy);
            }
#endif
            dxn = dx;
        }
        qpb_wsync();
    };

    // ---- residuals (Auxilary.c:745-786) of the iterate in LDS; returns the objective
    // and the four sums rx'rx, ry'ry, rz'rz, s'z
    auto residuals = [&](double (&red)[4]) -> double {
        double srx = 0.0, sry = 0.0, srz = 0.0, ssz = 0.0, sfv = 0.0;
        double xprev = 0.0;
        // c of the next stage, prefetched (the only input the loop reads from memory)
        double cnext = QPB_LDS(&a.c[tile * (BNX * QPB_TSTR) + xc * QPB_TSTR + ql]);
        double hnext = QPB_LDS(&a.h[tile * (BNZ * QPB_TSTR) + zr * QPB_TSTR + ql]);
#if MY > 0
        double bnext = QPB_LDS(&a.b[tile * (BNY * QPB_TSTR) + yl * QPB_TSTR + ql]);
#endif
#pragma unroll 1
        for (int k = 0; k < NS; k++) {
            const double cx = cnext, hz = hnext;
#if MY > 0
            const double by = bnext;
#endif
            if (k + 1 < NS) {
                cnext = QPB_LDS(&a.c[tile * (BNX * QPB_TSTR) + ((k + 1) * NB + xc) * QPB_TSTR + ql]);
                hnext = QPB_LDS(&a.h[tile * (BNZ * QPB_TSTR) + ((k + 1) * MZ + zr) * QPB_TSTR + ql]);
#if MY > 0
                bnext = QPB_LDS(&a.b[tile * (BNY * QPB_TSTR) + ((k + 1) * MY + yl) * QPB_TSTR + ql]);
#endif
            }
            const double xk = Ls[V_X + k * NB + xc];
            const double *Pr = Ls + O_P + k * BLKP + xc * NB;
            const double *Gk = Ls + O_G + k * (MZ * NB);
            double pr[NB], gr[NB];
#pragma unroll
            for (int j = 0; j < NB; j++) { pr[j] = Pr[j]; gr[j] = Gk[zr * NB + j]; }
            // x lanes: P x (DPP), G'z and A'y (LDS broadcast reads of z, y)
            double px = 0.0, ta[4] = {cx, 0.0, 0.0, 0.0};
#pragma unroll
            for (int r = 0; r < MZ; r++) ta[r & 3] = __builtin_fma(Gk[r * NB + xc], Ls[V_Z + k * MZ + r], ta[r & 3]);
#if MY > 0
            const double *ARk = Ls + O_AR + k * (MY * NB);
#pragma unroll
            for (int l = 0; l < MY; l++)
                ta[(MZ + l) & 3] = __builtin_fma(ARk[l * NB + xc], Ls[V_Y + k * MY + l], ta[(MZ + l) & 3]);
            if (k + 1 < NS) {
                const double *ALn = Ls + O_AL + (k + 1) * (MY * NB);
#pragma unroll
                for (int l = 0; l < MY; l++)
                    ta[(MZ + MY + l) & 3] =
                        __builtin_fma(ALn[l * NB + xc], Ls[V_Y + (k + 1) * MY + l], ta[(MZ + MY + l) & 3]);
            }
#endif
            // z lanes: G x;  y lanes: AR_k x_k + AL_k x_{k-1}
            double gx = 0.0;
            qpb_fence(xk);
            qpb_for<0, NB>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                qpb_fx<j>(px, xk, pr[j]);
                if constexpr ((qpb_bGu >> j) & 1) qpb_fx<j>(gx, xk, gr[j]);
            });
            const double rx = -(((ta[0] + ta[1]) + (ta[2] + ta[3])) + px);
            if (x0) {
                Ls[V_RX + k * NB + c] = rx;
                srx = __builtin_fma(rx, rx, srx);
                sfv = __builtin_fma(xk, __builtin_fma(0.5, px, cx), sfv);   // objective (Auxilary.c:1133-1141)
            }
            if (isz) {
                const int i = k * MZ + lane;
                const double s = Ls[V_S + i];
                const double rz = (hz - s) - gx;
                Ls[V_RZ + i] = rz;
                srz = __builtin_fma(rz, rz, srz);
                ssz = __builtin_fma(s, Ls[V_Z + i], ssz);
            }
#if MY > 0
            {
                const double *ARr = Ls + O_AR + k * (MY * NB) + yl * NB;
                const double *ALr = Ls + O_AL + k * (MY * NB) + yl * NB;
                double ar[NB], al[NB];
#pragma unroll
                for (int j = 0; j < NB; j++) { ar[j] = ARr[j]; al[j] = ALr[j]; }
                double ax = 0.0;
                qpb_fence(xk, xprev);
                qpb_for<0, NB>([&](auto jc) {
                    constexpr int j = decltype(jc)::value;
                    if constexpr ((qpb_bARu >> j) & 1) qpb_fx<j>(ax, xk, ar[j]);
                    if constexpr ((qpb_bALu >> j) & 1) qpb_fx<j>(ax, xprev, al[j]);
                });
                if (isy) {
                    const double ry = by - ax;
                    Ls[V_RY + k * MY + lane] = ry;
                    sry = __builtin_fma(ry, ry, sry);
                }
            }
#endif
            xprev = xk;
        }
        qpb_wsync();
        red[0] = qpb_bsum(srx);
        red[1] = qpb_bsum(sry);
        red[2] = qpb_bsum(srz);
        red[3] = qpb_bsum(ssz);
        return qpb_bsum(sfv);
    };

    // step lengths (Auxilary.c:359-393): alpha = 1 / max(-d / v) over d < 0, 1 if none
    auto step_length = [&](bool corr, double &ap, double &ad) {
        double bp = 0.0, bd = 0.0;
        for (int i = lane; i < BNZ; i += 64) {
            const double s = Ls[V_S + i], z = Ls[V_Z + i], dz = Ls[V_DZ + i];
            const double rzi = qpb_rcp(z);
            const double dsl = corr ? Ls[V_DS + i] : -s * __builtin_fma(dz, rzi, 1.0);
            bp = __builtin_fmax(bp, -dsl * __builtin_amdgcn_rcp(s));
            bd = __builtin_fmax(bd, -dz * rzi);
        }
        bp = qpb_bmax(bp);
        bd = qpb_bmax(bd);
        ap = bp > 1e-10 ? __builtin_amdgcn_rcp(bp) : 1.0;
        ad = bd > 1e-10 ? __builtin_amdgcn_rcp(bd) : 1.0;
    };

    // ---- kkt_initialize (Auxilary.c:992-1089) as iteration -1, then QP_SOLVE (qpSWIFT.c:502-602)
    const double tol2 = a.tol > 0.0 ? a.tol * a.tol : -1.0;
    double sigma = 100.0;      // options->sigma (GlobalOptions.h:49)
    long it = -1, itq = 0;
    int flag = 3;
    double fv = 0.0, st_rx2 = 0.0, st_ry2 = 0.0, st_rz2 = 0.0, st_mu = 0.0, ap = 0.0, ad = 0.0;
    for (;;) {
        if (it >= 0 && it >= a.maxit) { itq = it; flag = 2; break; }
        w_pass(it < 0);
        double red[4] = {0.0, 0.0, 0.0, 1.0};
        double mu = 0.0;
        bool pc = true;
        if (it >= 0) {
            fv = residuals(red);
            const double mu_it = red[3] * (1.0 / BNZ);
            st_rx2 = red[0]; st_ry2 = BNY > 0 ? red[1] : 0.0; st_rz2 = red[2]; st_mu = mu_it;
            if (red[0] < tol2 && red[2] < tol2 && (BNY == 0 || red[1] < tol2) && mu_it < a.abstol) {
                itq = it;
                flag = 0;
                break;
            }
            mu = mu_it;
            pc = sigma > a.sigma_d;
        }
        const double rsz = qpb_rcp(red[3]);
        QPB_BT(0);
        factor();
        QPB_BT(1);
        if (it < 0) {
            // setup solve, rhs [-c; b; h]: x0, y0; s0, z0 from -dz (Auxilary.c:1010-1040)
            solve(BM_SETUP, 0.0, false);
            double mx0 = -1e300, mx1 = -1e300;
            for (int i = lane; i < BNZ; i += 64) {
                const double zi = -Ls[V_DZ + i];
                mx0 = __builtin_fmax(mx0, -zi);
                mx1 = __builtin_fmax(mx1, zi);
            }
            const double sh = qpb_bmax(mx0), hi = qpb_bmax(mx1);
            for (int i = lane; i < BNZ; i += 64) {
                const double zi = -Ls[V_DZ + i];
                Ls[V_S + i] = sh < 0 ? zi : zi + (1 + sh);
                Ls[V_Z + i] = hi < 0 ? -zi : -zi + (1 + hi);
            }
            for (int i = lane; i < BNX; i += 64) Ls[V_X + i] = Ls[V_DX + i];
            for (int i = lane; i < BNY; i += 64) Ls[V_Y + i] = Ls[V_DY + i];
            qpb_wsync();
            QPB_BT(2);
            it = 0;
            continue;
        }
        if (!pc) sigma = a.sigma_d;
        bool pcd = false;
        if (pc) {
            // predictor (kktsolve_1, Auxilary.c:471-515), ds = -s o z
            solve(BM_PRED, 0.0, false);
            step_length(false, ap, ad);
            double rr = 0.0;
            for (int i = lane; i < BNZ; i += 64) {
                const double s = Ls[V_S + i], z = Ls[V_Z + i], dz = Ls[V_DZ + i];
                const double dsl = -s * __builtin_fma(dz, qpb_rcp(z), 1.0);
                rr += (s + ap * dsl) * (z + ad * dz);
            }
            const double rho = qpb_bsum(rr) * rsz;      // formrho
            const double r1 = 1 > rho ? rho : 1;
            const double cube = r1 * r1 * r1;
            sigma = a.sigma_d < cube ? cube : a.sigma_d;
            pcd = true;
        }
        QPB_BT(2);
        // corrector / centering (kktsolve_2, Auxilary.c:524-564)
        solve(BM_CORR, sigma * mu, pcd);
        QPB_BT(3);
        step_length(true, ap, ad);
        ap = 0.99 * ap > 1.0 ? 1.0 : 0.99 * ap;
        ad = 0.99 * ad > 1.0 ? 1.0 : 0.99 * ad;
        for (int i = lane; i < BNX; i += 64) Ls[V_X + i] = __builtin_fma(Ls[V_DX + i], ap, Ls[V_X + i]);
        for (int i = lane; i < BNY; i += 64) Ls[V_Y + i] = __builtin_fma(Ls[V_DY + i], ad, Ls[V_Y + i]);
        for (int i = lane; i < BNZ; i += 64) {
            Ls[V_S + i] = __builtin_fma(Ls[V_DS + i], ap, Ls[V_S + i]);
            Ls[V_Z + i] = __builtin_fma(Ls[V_DZ + i], ad, Ls[V_Z + i]);
        }
        qpb_wsync();
        QPB_BT(4);
        it++;
    }

    // ---- outputs (tiled SoA)
    for (int i = lane; i < BNX; i += 64) QPB_STS(&a.x[tile * (BNX * QPB_TSTR) + i * QPB_TSTR + ql], Ls[V_X + i]);
    for (int i = lane; i < BNY; i += 64) QPB_STS(&a.y[tile * (BNY * QPB_TSTR) + i * QPB_TSTR + ql], Ls[V_Y + i]);
    for (int i = lane; i < BNZ; i += 64) {
        QPB_STS(&a.z[tile * (BNZ * QPB_TSTR) + i * QPB_TSTR + ql], Ls[V_Z + i]);
        QPB_STS(&a.s[tile * (BNZ * QPB_TSTR) + i * QPB_TSTR + ql], Ls[V_S + i]);
    }
    if (lane == 0) {
        QPB_STS(&a.flag[q], flag);
        QPB_STS(&a.iters[q], (int)itq);
        QPB_STS(&a.fval[q], fv);
        if (a.sig) QPB_STS(&a.sig[q], sigma);
#if QPB_B_TIMING
        if (a.stats) {
            double *o = a.stats + tile * 6 * QPB_TSTR + ql;
            for (int k = 0; k < 6; k++) o[k * QPB_TSTR] = tph[k];
        }
#else
        if (a.stats) {
            double *o = a.stats + tile * 6 * QPB_TSTR + ql;
            o[0] = __builtin_sqrt(st_rx2); o[QPB_TSTR] = __builtin_sqrt(st_ry2); o[2 * QPB_TSTR] = __builtin_sqrt(st_rz2);
            o[3 * QPB_TSTR] = st_mu; o[4 * QPB_TSTR] = ap; o[5 * QPB_TSTR] = ad;
        }
#endif
    }
}

extern "C" __global__ void __launch_bounds__(64, 1) QPB_KERNEL_NAME(qpb_args a) {
    __shared__ __attribute__((aligned(16))) double qpb_lds[LDS_QP];
    qpb_band_body(a, qpb_xcd_block(), qpb_lds);
}

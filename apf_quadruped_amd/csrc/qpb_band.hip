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
//   S_k = H_kk - X_k S_{k-1}^-1 X_k' = L_k D_k L_k'
// -- the same factor as the reference's up-looking LDL' of the permuted KKT matrix
// (ldl.c:253-326, pivot regularisation ldl.c:273-274), in block form, and the same
// triangular solves (kktsolve, Auxilary.c:471-564) as block forward / backward sweeps.
//
// Lanes.  Work that is independent across stages (residuals, the blocks H_kk, the
// solves' right-hand sides t_k, the triangular chains S_k^-1 r_k, dz / dy) runs stage-parallel: DPP row R of
// the wavefront takes stage 4 i + R, lane c holding x_c, y_c and the z rows c + 16 u of
// it -- the row kernel's layout, one stage per row, products as DPP row_newbcast FMAs,
// the neighbouring stages' x / y values loaded per lane.  The recurrences (the Schur
// update and pivots of each stage, the sweeps' short coupling products) run stage by
// stage.  The coupling X_k = 1e7 AR_k'AL_k has rank <= MY, so the factor keeps
// Y_k = S_{k-1}^-1 AL_k' (NB x MY) instead of the NB x NB block L_{k,k-1}: the sweeps'
// recursions become short products and their triangular chains run stage-parallel.
// All of the QP's state -- P, G, A stage blocks, the factor's L_k, 1/D_k and Y_k, the
// iterate, residuals and directions -- stays in the workgroup's LDS for the whole
// solve, packed by pattern; inputs are read once, outputs written once.
//
// The loop is the row kernel's (qpSWIFT.c:473-644): kkt_initialize as iteration -1 (the
// warm variant, QPB_WARM = 1, continues from the QP object's state instead),
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
#define ZS ((MZ + 15) / 16)       // z sub-rows of a DPP row (z rows c, c + 16, ..)
#define NR ((NS + 3) / 4)         // rounds of the stage-parallel passes (four stages each)
// per-stage blocks and vectors (doubles; offsets emitted by the generator, qpb_wave.cpp
// band_layout), packed by pattern so that four QPs share a CU (MPC: 40.8 KB): O_P P_k's upper triangle
// (PP per stage, (i, j) at j (j + 1) / 2 + i), O_L -L_k's strict lower triangle (LP per
// stage, row c from c (c - 1) / 2), O_RD 1 / D_k, O_Y Y_k by columns (MY x NB), O_G G_k on
// the union of the stages' G patterns (GS per stage, the last slot zero; per-lane
// position tables qpb_bgc / qpb_bgr), O_AR / O_AL the A row groups' stage-k /
// stage-(k-1) parts (dense rows); the vectors x, dx | y, ry | z, s, rz, dz in natural
// order.  rx is not kept (the solves' right-hand side re-forms it inside its own
// products); the corrector's dy and ds overwrite ry and rz once these are consumed;
// O_DUMP (one slot per lane for masked stores) lies in dz, dead while the factor runs;
// w = -1 / reg(-s/z) is formed where it is used.
#define BLKP (NB * NB)
// A row group k: its stage-k part AR_k, its stage-(k-1) part AL_k (k >= 1; stage 0 has none:
// ALB(0) points at finite data that is only ever multiplied by zero); Y_k (k >= 1)
#define ARB(k) (O_AR + (k) * (MY * NB))
#define ALB(k) (O_AL + ((k) - 1) * (MY * NB))
#define YB(k) (O_Y + ((k) - 1) * (MY * NB))
static_assert(NB >= 1 && NB <= 16 && MZ >= 1 && MZ <= 64 && MY <= 16 && NS >= 2, "band kernel sizes");

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
// 2: cycles per part instead: factor stage-parallel / sequential, solve right-hand sides /
//    forward sweep / backward sweep / directions
#if QPB_B_TIMING == 1
#define QPB_BT(k) { const long t2_ = (long)__builtin_readcyclecounter(); tph[k] += (double)(t2_ - tcy); tcy = t2_; }
#else
#define QPB_BT(k)
#endif
#if QPB_B_TIMING == 2
#define QPB_BT0() { tcy = (long)__builtin_readcyclecounter(); }
#define QPB_BT2(k) { const long t2_ = (long)__builtin_readcyclecounter(); tph[k] += (double)(t2_ - tcy); tcy = t2_; }
#else
#define QPB_BT0()
#define QPB_BT2(k)
#endif

#ifndef QPB_B_NV
#define QPB_B_NV 0        // 1: the stage-parallel passes issue their DPP FMAs as non-volatile asm (the
                          // compiler may interleave rounds / hoist loads; the hazard pass pads)
#endif
#ifndef QPB_B_UNR
#define QPB_B_UNR 1       // rounds of the stage-parallel passes unrolled by this factor
#endif
#define QPB_PRAGMA_(x) _Pragma(#x)
#define QPB_PRAGMA(x) QPB_PRAGMA_(x)
// the rows lane, lane + 64, .. (< N) of a per-row pass, unrolled, each index clamped to N - 1
// (ok_ false on the clamped ones) so that every LDS access is unconditional: a rolled
// `for (i = lane; i < N; i += 64)` waited for each row's loads in turn
#ifndef QPB_B_PREF
#define QPB_B_PREF 0      // 1: each stage's static A slices loaded during the previous stage's pivots (measured: noise)
#endif
#ifndef QPB_B_VFORM
#define QPB_B_VFORM 1     // 1: the rank-MY Schur update as (AR' M) AR; 0: AR' (M AR) (round 5)
#endif
#ifndef QPB_B_ROWS
#define QPB_B_ROWS 1      // 0: the rolled per-row loops (round 5)
#endif
#if QPB_B_ROWS
#define QPB_BROWS(N, i, ...)                                                            \
    do {                                                                                \
        QPB_PRAGMA(unroll)                                                              \
        for (int k_ = 0; k_ < ((N) + 63) / 64; k_++) {                                  \
            const bool ok_ = lane + 64 * k_ < (N);                                      \
            const int i = ok_ ? lane + 64 * k_ : (N) - 1;                               \
            (void)ok_;                                                                  \
            __VA_ARGS__                                                                 \
        }                                                                               \
    } while (0)
#else
#define QPB_BROWS(N, i, ...)                                                            \
    do {                                                                                \
        for (int i = lane; i < (N); i += 64) {                                          \
            const bool ok_ = true;                                                      \
            (void)ok_;                                                                  \
            __VA_ARGS__                                                                 \
        }                                                                               \
    } while (0)
#endif
template <int J> static __device__ __forceinline__ void qpb_bfx(double &acc, double src, double m) {
    if constexpr (QPB_B_NV) qpb_fxs<J>(acc, src, m);
    else qpb_fx<J>(acc, src, m);
}
template <int J> static __device__ __forceinline__ void qpb_bfxd(double &t, double m) {
    if constexpr (QPB_B_NV)
        asm("v_fmac_f64_dpp %0, %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf bound_ctrl:1"
            : "+v"(t) : "v"(m), "i"(J));
    else qpb_fxd<J>(t, m);
}

// solve modes: the right-hand side's z part (bx = RX, by = RY in every mode)
enum { BM_SETUP = 0, BM_PRED = 1, BM_CORR = 2 };

// union of the structural columns of the G rows of z sub-row u (rows 16u .. 16u + 15)
static constexpr unsigned qpb_bgsub(int u) {
    unsigned m = 0;
    for (int r = 16 * u; r < 16 * u + 16 && r < MZ; r++) m |= qpb_bGm[r];
    return m;
}

static __device__ __forceinline__ void qpb_band_body(const qpb_args &a, long q, double *__restrict__ Ls) {
    const int lane = threadIdx.x & 63, R = lane >> 4, c = lane & 15;
    if (q >= a.B) return;                      // grid padding (XCD order): wave-uniform
#if QPB_B_TIMING
    double tph[6] = {0, 0, 0, 0, 0, 0};
    long tcy = (long)__builtin_readcyclecounter();
#endif
    const long tile = q >> 6;
    const int ql = (int)(q & 63);
    // Lanes.  Stage-parallel passes: DPP row R works on stage 4 i + R, lane c holds x_c,
    // y_c (c < MY) and z rows c + 16 u (u < ZS) of it -- the row kernel's layout per stage.
    // Sequential passes (the block factor's Schur complements and pivots, the triangular
    // sweeps): every row computes the same stage (row 0 stores), except the factor, whose
    // rows each hold their own stage's block from the stage-parallel part.
    const int xc = c < NB ? c : NB - 1;
    const bool isx = c < NB, isy = c < MY;
    const int yc = isy ? c : (MY > 0 ? MY - 1 : 0);
    int zrc[ZS];
    bool isz[ZS];
#pragma unroll
    for (int u = 0; u < ZS; u++) {
        isz[u] = c + 16 * u < MZ;
        zrc[u] = isz[u] ? c + 16 * u : MZ - 1;
    }
    const bool st0 = R == 0 && isx;            // the x lanes that store in sequential passes
    // per-lane positions in the packed blocks: P_k row xc, G_k column xc (x lanes) and
    // rows zrc[u] (z lanes), -L_k row xc from lb
    int pidx[NB], gic[MZ], gir[ZS][NB];
#pragma unroll
    for (int j = 0; j < NB; j++) pidx[j] = xc <= j ? j * (j + 1) / 2 + xc : xc * (xc + 1) / 2 + j;
#pragma unroll
    for (int r = 0; r < MZ; r++) gic[r] = qpb_bgc[xc][r];
#pragma unroll
    for (int u = 0; u < ZS; u++)
#pragma unroll
        for (int j = 0; j < NB; j++) gir[u][j] = qpb_bgr[zrc[u]][j];
    const int lb = xc * (xc - 1) / 2;
    constexpr double RDY = 1.0 / -1e-7;        // leaf y pivots: D = 0 regularised to -1e-7
    const double *gc = a.c + tile * (BNX * QPB_TSTR) + ql;
    const double *gh = a.h + tile * (BNZ * QPB_TSTR) + ql;
    const double *gb = a.b + tile * (BNY1 * QPB_TSTR) + ql;

    // ---- stage P, G, A into the per-stage dense blocks; -c, b, h into RX, RY, RZ
    for (int i = 2 * lane; i < O_STATIC_END; i += 128)      // O_STATIC_END even, 16-byte aligned base
        *reinterpret_cast<double2 *>(Ls + i) = double2{0.0, 0.0};
    qpb_wsync();
    {
        // eight values per lane in flight per round (their loads issued before the stores)
        auto scatter = [&](const double *src, auto nnzc, const int *slot, const int *slot2) {
            constexpr int NNZ = decltype(nnzc)::value;
#pragma unroll 1
            for (int k0 = 0; k0 < NNZ; k0 += 512) {
                double v[8];
                int s1[8], s2[8];
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const int k = k0 + 64 * u + lane;
                    const bool ok = k < NNZ;
                    v[u] = ok ? QPB_LDS(&src[k * QPB_TSTR]) : 0.0;
                    s1[u] = ok ? slot[k] : -1;
                    s2[u] = (ok && slot2) ? slot2[k] : -1;
                }
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    if (s1[u] >= 0) Ls[s1[u]] = v[u];
                    if (s2[u] >= 0) Ls[s2[u]] = v[u];
                }
            }
        };
        scatter(a.P + tile * (QPB_NNZP * QPB_TSTR) + ql, qpb_ic<QPB_NNZP>{}, qpb_bsP, nullptr);
        scatter(a.G + tile * (QPB_NNZG * QPB_TSTR) + ql, qpb_ic<QPB_NNZG>{}, qpb_bsG, nullptr);
#if MY > 0
        scatter(a.A + tile * (QPB_NNZA * QPB_TSTR) + ql, qpb_ic<QPB_NNZA>{}, qpb_bsA, nullptr);
#endif
#if MY > 0
        for (int i = lane; i < BNY; i += 64) Ls[V_RY + i] = QPB_LDS(&gb[i * QPB_TSTR]);
#endif
#if QPB_WARM
        // warm variant (qpb_solve_warm): QP_SOLVE continues from the object's iterate
        // (qpSWIFT.c:502-596 never re-initialises); rz / ry are formed by the first pass
        for (int i = lane; i < BNZ; i += 64) {
            Ls[V_Z + i] = QPB_LDS(&a.z[tile * (BNZ * QPB_TSTR) + i * QPB_TSTR + ql]);
            Ls[V_S + i] = QPB_LDS(&a.s[tile * (BNZ * QPB_TSTR) + i * QPB_TSTR + ql]);
        }
        for (int i = lane; i < BNX; i += 64) Ls[V_X + i] = QPB_LDS(&a.x[tile * (BNX * QPB_TSTR) + i * QPB_TSTR + ql]);
        for (int i = lane; i < BNY; i += 64) Ls[V_Y + i] = QPB_LDS(&a.y[tile * (BNY * QPB_TSTR) + i * QPB_TSTR + ql]);
#else
        for (int i = lane; i < BNZ; i += 64) {
            Ls[V_RZ + i] = QPB_LDS(&gh[i * QPB_TSTR]);
            Ls[V_Z + i] = 1.0;
            Ls[V_S + i] = 1.0;
        }
        for (int i = lane; i < BNX; i += 64) Ls[V_X + i] = 0.0;
        for (int i = lane; i < BNY; i += 64) Ls[V_Y + i] = 0.0;
#endif
    }
    qpb_wsync();
    QPB_BT(5);

    // the KKT diagonal's w = -1 / regularise(-s / z) of z row iz (kkt_initialize: -I, w = 1)
    bool wset = true;
    auto wz = [&](int iz) -> double {
        return wset ? 1.0 : -qpb_rcp_reg(-Ls[V_S + iz] * qpb_rcp(Ls[V_Z + iz]));
    };

    // this row's stage slices (stage kc): column xc of G_k, AR_k, AL_k, AL_{k+1} (the last
    // zero when k + 1 = NS), rows zrc[u] of G_k, row yc of AR_k and AL_k
    auto col_G = [&](int kc, double (&g)[MZ]) {
        const double *Gk = Ls + O_G + kc * GS;
#pragma unroll
        for (int r = 0; r < MZ; r++) g[r] = Gk[gic[r]];
    };
    auto row_G = [&](int kc, double (&g)[ZS][NB]) {
        const double *Gk = Ls + O_G + kc * GS;
#pragma unroll
        for (int u = 0; u < ZS; u++)
#pragma unroll
            for (int j = 0; j < NB; j++) g[u][j] = Gk[gir[u][j]];
    };
    auto row_P = [&](int kc, double (&pr)[NB]) {
        const double *Pk = Ls + O_P + kc * PP;
#pragma unroll
        for (int j = 0; j < NB; j++) pr[j] = Pk[pidx[j]];
    };
    // row xc / column xc of -L_k (zero from the diagonal on)
    auto row_L = [&](int k, double (&nl)[NB]) {
        const double *Lk = Ls + O_L + k * LP + lb;
#pragma unroll
        for (int f = 0; f < NB; f++) nl[f] = f < xc ? Lk[f] : 0.0;
    };
    auto col_L = [&](int k, double (&lt)[NB]) {
        const double *Lk = Ls + O_L + k * LP + xc;
#pragma unroll
        for (int e = 0; e < NB; e++) lt[e] = e > xc ? Lk[e * (e - 1) / 2] : 0.0;
    };
    auto col_A = [&](int base, double (&v)[MY1]) {
        const double *Ak = Ls + base + xc;
#pragma unroll
        for (int l = 0; l < MY1; l++) v[l] = MY > 0 ? Ak[l * NB] : 0.0;
    };

    // ---- residuals (Auxilary.c:745-786), stage-parallel; returns the objective and the
    // four sums rx'rx, ry'ry, rz'rz, s'z
    auto residuals = [&](double (&red)[4]) -> double {
        double srx = 0.0, sry = 0.0, srz = 0.0, ssz = 0.0, sfv = 0.0;
QPB_PRAGMA(unroll QPB_B_UNR)
        for (int i = 0; i < NR; i++) {
            const int k = 4 * i + R;
            const bool act = k < NS;
            const int kc = act ? k : NS - 1;
            const bool nxt = kc + 1 < NS;
            const double cx = QPB_LDS(&gc[(kc * NB + xc) * QPB_TSTR]);
            double hz[ZS], zk[ZS], sk[ZS];
#pragma unroll
            for (int u = 0; u < ZS; u++) {
                hz[u] = QPB_LDS(&gh[(kc * MZ + zrc[u]) * QPB_TSTR]);
                zk[u] = Ls[V_Z + kc * MZ + zrc[u]];
                sk[u] = Ls[V_S + kc * MZ + zrc[u]];
            }
            const double xk = Ls[V_X + kc * NB + xc];
            const double xp = kc > 0 ? Ls[V_X + (kc - 1) * NB + xc] : 0.0;
            double pr[NB], gr[ZS][NB], gcl[MZ];
            row_P(kc, pr);
            row_G(kc, gr);
            col_G(kc, gcl);
            double ta[4] = {cx, 0.0, 0.0, 0.0}, px = 0.0, gx[ZS];
#pragma unroll
            for (int u = 0; u < ZS; u++) gx[u] = 0.0;
#if MY > 0
            const double by = QPB_LDS(&gb[(kc * MY + yc) * QPB_TSTR]);
            const double yk = Ls[V_Y + kc * MY + yc];
            const double yn = nxt ? Ls[V_Y + (kc + 1) * MY + yc] : 0.0;
            double arc[MY1], alnc[MY1], arr[NB], alr[NB];
            col_A(ARB(kc), arc);
            col_A(ALB(nxt ? kc + 1 : kc), alnc);
            const double *ARr = Ls + ARB(kc) + yc * NB, *ALr = Ls + ALB(kc) + yc * NB;
#pragma unroll
            for (int j = 0; j < NB; j++) { arr[j] = ARr[j]; alr[j] = ALr[j]; }
            double ay = 0.0, ay2 = 0.0;
#endif
            qpb_fence(xk, xp);
            qpb_for<0, NB>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                qpb_bfx<j>(px, xk, pr[j]);                                   // P x
                qpb_for<0, ZS>([&](auto uc) {
                    constexpr int u = decltype(uc)::value;
                    if constexpr ((qpb_bgsub(u) >> j) & 1) qpb_bfx<j>(gx[u], xk, gr[u][j]);    // G x
                });
#if MY > 0
                if constexpr ((qpb_bARu >> j) & 1) qpb_bfx<j>(ay, xk, arr[j]);       // AR_k x_k
                if constexpr ((qpb_bALu >> j) & 1) qpb_bfx<j>(ay2, xp, alr[j]);      // AL_k x_{k-1}
#endif
            });
            // G'z, AR_k' y_k, AL_{k+1}' y_{k+1}: z / y lanes of the row by DPP broadcast
            qpb_fence(zk[0]);
            qpb_for<0, MZ>([&](auto rc) {
                constexpr int r = decltype(rc)::value;
                qpb_bfx<(r & 15)>(ta[r & 3], zk[r >> 4], gcl[r]);
            });
#if MY > 0
            qpb_fence(yk, yn);
            qpb_for<0, MY>([&](auto lc) {
                constexpr int l = decltype(lc)::value;
                qpb_bfx<l>(ta[(MZ + l) & 3], yk, arc[l]);
                qpb_bfx<l>(ta[(MZ + MY + l) & 3], yn, nxt ? alnc[l] : 0.0);
            });
#endif
            const double rx = -(((ta[0] + ta[1]) + (ta[2] + ta[3])) + px);
            if (act && isx) {
                srx = __builtin_fma(rx, rx, srx);
                sfv = __builtin_fma(xk, __builtin_fma(0.5, px, cx), sfv);   // objective (Auxilary.c:1133-1141)
            }
#pragma unroll
            for (int u = 0; u < ZS; u++) {
                if (act && isz[u]) {
                    const double rz = (hz[u] - sk[u]) - gx[u];
                    Ls[V_RZ + k * MZ + c + 16 * u] = rz;
                    srz = __builtin_fma(rz, rz, srz);
                    ssz = __builtin_fma(sk[u], zk[u], ssz);
                }
            }
#if MY > 0
            if (act && isy) {
                const double ry = by - (ay + ay2);
                Ls[V_RY + k * MY + c] = ry;
                sry = __builtin_fma(ry, ry, sry);
            }
#endif
        }
        qpb_wsync();
        red[0] = qpb_bsum(srx);
        red[1] = qpb_bsum(sry);
        red[2] = qpb_bsum(srz);
        red[3] = qpb_bsum(ssz);
        return qpb_bsum(sfv);
    };

    // ---- factor: block LDL' of the x block.  Every fourth stage a stage-parallel part
    // forms H_kk = P_k + G_k'W_k G_k + 1e7 (AR_k'AR_k + AL_{k+1}'AL_{k+1}) and X_k for the
    // four stages of the round (row R: stage k + R, in registers); then the stages'
    // sequential parts: Z_k = X_k L_{k-1}^-T, H_kk -= Z_k D_{k-1}^-1 Z_k', the pivots.
    // reg: pivots regularised inline (ldl.c:273-274).  The fast pass (reg = false) takes
    // every 1/D as v_rcp_f64 + Newton; the caller redoes the factor with reg = true when
    // a stored 1/D shows a pivot |D| <= 1e-14 (rare) -- otherwise the same operations,
    // so the same bits.
    auto factor = [&](auto regc) {
        constexpr bool REG = decltype(regc)::value != 0;
        double H[NB];
#if QPB_B_PREF && MY > 0
        double pYr[MY1], parc[MY1], palr[NB];   // stage k's static slices, loaded during stage k - 1
#pragma unroll
        for (int l = 0; l < MY1; l++) pYr[l] = parc[l] = 0.0;
#pragma unroll
        for (int j = 0; j < NB; j++) palr[j] = 0.0;
#endif
#pragma unroll 1
        for (int k = 0; k < NS; k++) {
            QPB_BT0();
            if ((k & 3) == 0) {
                const int ks = k + R;
                const int kc = ks < NS ? ks : NS - 1;
                const bool nxt = kc + 1 < NS;
                row_P(kc, H);
                double gcl[MZ], wr[ZS];
                col_G(kc, gcl);
#pragma unroll
                for (int u = 0; u < ZS; u++) wr[u] = wz(kc * MZ + zrc[u]);
                // + G_k' W_k G_k: four rows' products G(r, c) w_r first, then their DPP FMAs
                qpb_for<0, (MZ + 3) / 4>([&](auto qc4) {
                    constexpr int r0 = 4 * decltype(qc4)::value;
                    double cr[4];
                    qpb_for<0, 4>([&](auto uc) {
                        constexpr int r = r0 + decltype(uc)::value;
                        if constexpr (r < MZ) cr[decltype(uc)::value] = gcl[r] * qpb_nb<(r & 15)>(wr[r >> 4]);
                        else cr[decltype(uc)::value] = 0.0;
                    });
                    asm volatile("" : "+v"(cr[0]), "+v"(cr[1]), "+v"(cr[2]), "+v"(cr[3]));
                    qpb_for<0, 4>([&](auto uc) {
                        constexpr int r = r0 + decltype(uc)::value;
                        if constexpr (r < MZ) {
                            qpb_for<0, NB>([&](auto jc) {
                                constexpr int j = decltype(jc)::value;
                                if constexpr ((qpb_bGm[r] >> j) & 1) qpb_bfx<j>(H[j], gcl[r], cr[decltype(uc)::value]);
                            });
                        }
                    });
                });
#if MY > 0
                double arc[MY1], alnc[MY1];
                col_A(ARB(kc), arc);
                col_A(ALB(nxt ? kc + 1 : kc), alnc);
                qpb_for<0, MY>([&](auto lc) {
                    constexpr int l = decltype(lc)::value;
                    const double tr = -RDY * arc[l], an = nxt ? alnc[l] : 0.0, tn = -RDY * an;
                    qpb_fence(tr, an, tn);
                    // the two products' FMAs on one H(c, j) NB instructions apart (not back to back)
                    qpb_for<0, NB>([&](auto jc) {
                        constexpr int j = decltype(jc)::value;
                        if constexpr ((qpb_bARm[l] >> j) & 1) qpb_bfx<j>(H[j], arc[l], tr);    // 1e7 AR_k'AR_k
                    });
                    qpb_for<0, NB>([&](auto jc) {
                        constexpr int j = decltype(jc)::value;
                        if constexpr ((qpb_bALm[l] >> j) & 1) qpb_bfx<j>(H[j], an, tn);        // 1e7 AL_{k+1}'AL_{k+1}
                    });
                });
#endif
            }
            QPB_BT2(0);
            const int kr = k & 3;                   // the row holding stage k's block
            double Hs[NB];
#pragma unroll
            for (int j = 0; j < NB; j++) Hs[j] = H[j];
#if MY > 0
            if (k > 0) {
                // H_kk -= X_k S_{k-1}^-1 X_k' with X_k = 1e7 AR_k' AL_k (rank <= MY):
                //   Y_k = S_{k-1}^-1 AL_k' = L^-T D^-1 L^-1 AL_k'   (x lanes: row c of Y_k)
                //   M = AL_k Y_k, T = M AR_k                          (y lanes: rows l)
                //   H(c, j) -= 1e14 sum_l AR_k(l, c) T(l, j)          (x lanes)
                double nlr[NB], nlc[NB], Yr[MY1], arc[MY1], alr[NB];
                row_L(k - 1, nlr);
                col_L(k - 1, nlc);
                const double rdp = Ls[O_RD + (k - 1) * NB + xc];
#if QPB_B_PREF
#pragma unroll
                for (int l = 0; l < MY; l++) { Yr[l] = pYr[l]; arc[l] = parc[l]; }
#pragma unroll
                for (int j = 0; j < NB; j++) alr[j] = palr[j];
#else
                col_A(ALB(k), Yr);
                col_A(ARB(k), arc);
                const double *ALr = Ls + ALB(k) + yc * NB;
#pragma unroll
                for (int j = 0; j < NB; j++) alr[j] = ALr[j];
#endif
                qpb_for<0, NB>([&](auto fc) {
                    constexpr int f = decltype(fc)::value;
                    qpb_for<0, MY>([&](auto lc) { qpb_fxd<f>(Yr[decltype(lc)::value], nlr[f]); });
                });
#pragma unroll
                for (int l = 0; l < MY; l++) Yr[l] *= rdp;
                qpb_for<0, NB>([&](auto ec) {
                    constexpr int e = NB - 1 - decltype(ec)::value;
                    qpb_for<0, MY>([&](auto lc) { qpb_fxd<e>(Yr[decltype(lc)::value], nlc[e]); });
                });
                if (R == kr && isx) {
#pragma unroll
                    for (int l = 0; l < MY; l++) Ls[YB(k) + l * NB + c] = Yr[l];
                }
                double M[MY1];
#pragma unroll
                for (int l = 0; l < MY; l++) M[l] = 0.0;
                qpb_for<0, NB>([&](auto jc) {
                    constexpr int j = decltype(jc)::value;
                    if constexpr ((qpb_bALu >> j) & 1)
                        qpb_for<0, MY>([&](auto lc) { qpb_fx<j>(M[decltype(lc)::value], Yr[decltype(lc)::value], alr[j]); });
                });
#if QPB_B_VFORM
                // V = AR_k' M (x lanes: row c, MY wide), then H(c, j) -= 1e14 sum_l V(c, l) AR_k(l, j):
                // MY * MY + MY * NB DPP FMAs instead of T = M AR_k's MY * NB + the same MY * NB
                double V[MY1];
#pragma unroll
                for (int l = 0; l < MY; l++) V[l] = 0.0;
                qpb_for<0, MY>([&](auto vc) {
                    constexpr int v = decltype(vc)::value;
                    qpb_for<0, MY>([&](auto lc) {
                        constexpr int l = decltype(lc)::value;
                        qpb_fx<l>(V[v], M[v], arc[l]);          // += AR(l, c) M(l, v)
                    });
                });
#pragma unroll
                for (int l = 0; l < MY; l++) V[l] *= -1e14;
                qpb_for<0, MY>([&](auto lc) {
                    constexpr int l = decltype(lc)::value;
                    qpb_for<0, NB>([&](auto jc) {
                        constexpr int j = decltype(jc)::value;
                        if constexpr ((qpb_bARu >> j) & 1) qpb_fx<j>(Hs[j], arc[l], V[l]);   // AR(l, j): lane j
                    });
                });
#else
                double T[NB], arr[NB];
                const double *ARr = Ls + ARB(k) + yc * NB;
#pragma unroll
                for (int j = 0; j < NB; j++) { T[j] = 0.0; arr[j] = ARr[j]; }
                qpb_for<0, MY>([&](auto lc) {
                    constexpr int l = decltype(lc)::value;
                    qpb_for<0, NB>([&](auto jc) {
                        constexpr int j = decltype(jc)::value;
                        if constexpr ((qpb_bARu >> j) & 1) qpb_fx<l>(T[j], arr[j], M[l]);
                    });
                });
                qpb_for<0, MY>([&](auto lc) {
                    constexpr int l = decltype(lc)::value;
                    const double m = -1e14 * arc[l];
                    qpb_fence(m);
                    qpb_for<0, NB>([&](auto jc) {
                        constexpr int j = decltype(jc)::value;
                        if constexpr ((qpb_bARu >> j) & 1) qpb_fx<l>(Hs[j], T[j], m);
                    });
                });
#endif
            }
#endif
#if QPB_B_PREF && MY > 0
            // the next stage's static slices (AL_{k+1}, AR_{k+1} columns, AL_{k+1} row), loaded
            // here so that they arrive under the pivot chain, which reads no LDS
            {
                const int kn = k + 1 < NS ? k + 1 : NS - 1;
                col_A(ALB(kn), pYr);
                col_A(ARB(kn), parc);
                const double *ALr = Ls + ALB(kn) + yc * NB;
#pragma unroll
                for (int j = 0; j < NB; j++) palr[j] = ALr[j];
            }
#endif
            // LDL' of the stage block in natural order (the row kernel's pivot chain)
            double rDd = 0.0;
            double dpiv = qpb_nb<0>(Hs[0]);
            qpb_for<0, NB>([&](auto kc2) {
                constexpr int kk = decltype(kc2)::value;
                const double rd = REG ? qpb_rcp_reg(dpiv) : qpb_rcp_nr(dpiv);
                double nl = Hs[kk] * -rd;
                asm volatile("" : "+v"(nl));
                if constexpr (kk + 1 < NB) {
                    const double h = qpb_nb<kk + 1>(Hs[kk]), hkk = qpb_nb<kk + 1>(Hs[kk + 1]);
                    dpiv = __builtin_fma(-(h * h), rd, hkk);
                }
                rDd = xc == kk ? rd : rDd;
                qpb_for<kk + 1, NB>([&](auto jc) {
                    constexpr int j = decltype(jc)::value;
                    qpb_fxs<j>(Hs[j], Hs[kk], nl);
                });
                Hs[kk] = nl;        // -L(c, kk) for c > kk; the rest never reaches the packed -L rows
            });
            if (R == kr && isx) {
                const int lrow = O_L + k * LP + c * (c - 1) / 2;
#pragma unroll
                for (int f = 0; f < NB; f++) Ls[f < c ? lrow + f : O_DUMP + lane] = Hs[f];
                Ls[O_RD + k * NB + c] = rDd;
            }
            qpb_wsync();
            QPB_BT2(1);
        }
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
        QPB_BT0();
        // stage-parallel: t_k = bx_k + G_k'(w o bz) + 1e7 (AR_k' by_k + AL_{k+1}' by_{k+1}) -> DX
QPB_PRAGMA(unroll QPB_B_UNR)
        for (int i = 0; i < NR; i++) {
            const int k = 4 * i + R;
            const bool act = k < NS;
            const int kc = act ? k : NS - 1;
            const bool nxt = kc + 1 < NS;
            // t = bx + G'(w o bz) + 1e7 A' by with bx = rx = -c - P x - G'z - A'y (-c at
            // kkt_initialize): rx is not kept, its G' / A' terms fold into the same products
            const bool it0 = mode == BM_SETUP;
            double v[ZS], gcl[MZ];
#pragma unroll
            for (int u = 0; u < ZS; u++) {
                double cc;
                const int iz = kc * MZ + zrc[u];
                v[u] = wz(iz) * bz_of(mode, iz, smu, pcd, &cc) - (it0 ? 0.0 : Ls[V_Z + iz]);
            }
            col_G(kc, gcl);
            double ta[4] = {-QPB_LDS(&gc[(kc * NB + xc) * QPB_TSTR]), 0.0, 0.0, 0.0};
            if (!it0) {
                double pr[NB], px = 0.0;
                row_P(kc, pr);
                const double xk = Ls[V_X + kc * NB + xc];
                qpb_fence(xk);
                qpb_for<0, NB>([&](auto jc) { qpb_bfx<decltype(jc)::value>(px, xk, pr[decltype(jc)::value]); });
                ta[1] = -px;
            }
            qpb_fence(v[0]);
            qpb_for<0, MZ>([&](auto rc) {
                constexpr int r = decltype(rc)::value;
                qpb_bfx<(r & 15)>(ta[r & 3], v[r >> 4], gcl[r]);
            });
#if MY > 0
            double arc[MY1], alnc[MY1];
            col_A(ARB(kc), arc);
            col_A(ALB(nxt ? kc + 1 : kc), alnc);
            const double yr = -RDY * Ls[V_RY + kc * MY + yc] - (it0 ? 0.0 : Ls[V_Y + kc * MY + yc]);
            const double yrn = nxt ? -RDY * Ls[V_RY + (kc + 1) * MY + yc] - (it0 ? 0.0 : Ls[V_Y + (kc + 1) * MY + yc])
                                   : 0.0;
            qpb_fence(yr, yrn);
            qpb_for<0, MY>([&](auto lc) {
                constexpr int l = decltype(lc)::value;
                qpb_bfx<l>(ta[(MZ + l) & 3], yr, arc[l]);
                qpb_bfx<l>(ta[(MZ + MY + l) & 3], yrn, alnc[l]);
            });
#endif
            if (act && isx) Ls[V_DX + k * NB + c] = (ta[0] + ta[1]) + (ta[2] + ta[3]);
        }
        qpb_wsync();
        QPB_BT2(2);
        // block forward / backward substitution (block Thomas) with X_k S_{k-1}^-1 = U_k Y_k',
        // U_k = 1e7 AR_k':  r_0 = t_0, r_k = t_k - U_k (Y_k' r_{k-1});  g_k = S_k^-1 r_k
        // (stage-parallel: two triangular chains per stage);  dx_{NS-1} = g_{NS-1},
        // dx_k = g_k - Y_{k+1} (U_{k+1}' dx_{k+1}).  The recursions are short products.
#if MY > 0
        {
            double rprev = Ls[V_DX + xc];
#pragma unroll 1
            for (int k = 1; k < NS; k++) {
                double yt[NB], arc[MY1];
                const double *Yk = Ls + YB(k) + yc * NB;                    // Y_k(:, yc)
#pragma unroll
                for (int j = 0; j < NB; j++) yt[j] = Yk[j];
                col_A(ARB(k), arc);
                double t = Ls[V_DX + k * NB + xc];
                double q[2] = {0.0, 0.0};
                qpb_for<0, NB>([&](auto jc) {
                    constexpr int j = decltype(jc)::value;
                    qpb_fx<j>(q[j & 1], rprev, yt[j]);
                });
                const double nq = RDY * (q[0] + q[1]);
                double t2 = 0.0;
                qpb_fence(nq);
                qpb_for<0, MY>([&](auto lc) {
                    constexpr int l = decltype(lc)::value;
                    if constexpr (l & 1) qpb_fx<l>(t2, nq, arc[l]);
                    else qpb_fx<l>(t, nq, arc[l]);
                });
                t += t2;
                if (st0) Ls[V_DX + k * NB + c] = t;
                rprev = t;
            }
            qpb_wsync();
        }
#endif
        QPB_BT2(3);
QPB_PRAGMA(unroll QPB_B_UNR)
        for (int i = 0; i < NR; i++) {
            const int k = 4 * i + R;
            const bool act = k < NS;
            const int kc = act ? k : NS - 1;
            double r = Ls[V_DX + kc * NB + xc];
            double nl[NB], lt[NB];
            row_L(kc, nl);
            col_L(kc, lt);
            const double rd = Ls[O_RD + kc * NB + xc];
            qpb_fence(r);
            qpb_for<0, NB>([&](auto fc) { qpb_bfxd<decltype(fc)::value>(r, nl[decltype(fc)::value]); });
            r *= rd;
            qpb_fence(r);
            qpb_for<0, NB>([&](auto ec) {
                constexpr int e = NB - 1 - decltype(ec)::value;
                qpb_bfxd<e>(r, lt[e]);
            });
            if (act && isx) Ls[V_DX + k * NB + c] = r;
        }
        qpb_wsync();
#if MY > 0
        {
            double dxn = Ls[V_DX + (NS - 1) * NB + xc];
#pragma unroll 1
            for (int k = NS - 2; k >= 0; k--) {
                double arr[NB], ycl[MY1];
                const double *ARr = Ls + ARB(k + 1) + yc * NB;
#pragma unroll
                for (int j = 0; j < NB; j++) arr[j] = ARr[j];
                const double *Yn = Ls + YB(k + 1) + xc;                         // Y_{k+1}(xc, :)
#pragma unroll
                for (int l = 0; l < MY; l++) ycl[l] = Yn[l * NB];
                double g = Ls[V_DX + k * NB + xc];
                double p[2] = {0.0, 0.0};
                qpb_for<0, NB>([&](auto jc) {
                    constexpr int j = decltype(jc)::value;
                    if constexpr ((qpb_bARu >> j) & 1) qpb_fx<j>(p[j & 1], dxn, arr[j]);
                });
                const double np = RDY * (p[0] + p[1]);
                double g2 = 0.0;
                qpb_fence(np);
                qpb_for<0, MY>([&](auto lc) {
                    constexpr int l = decltype(lc)::value;
                    if constexpr (l & 1) qpb_fx<l>(g2, np, ycl[l]);
                    else qpb_fx<l>(g, np, ycl[l]);
                });
                g += g2;
                if (st0) Ls[V_DX + k * NB + c] = g;
                dxn = g;
            }
            qpb_wsync();
        }
#endif
        QPB_BT2(4);
        // stage-parallel: dz = w (G dx - bz) (+ ds in the corrector), dy = -1e7 (by - A dx)
QPB_PRAGMA(unroll QPB_B_UNR)
        for (int i = 0; i < NR; i++) {
            const int k = 4 * i + R;
            const bool act = k < NS;
            const int kc = act ? k : NS - 1;
            const double dxk = Ls[V_DX + kc * NB + xc];
            double gr[ZS][NB], gz[ZS];
            row_G(kc, gr);
#pragma unroll
            for (int u = 0; u < ZS; u++) gz[u] = 0.0;
#if MY > 0
            const double dxp = kc > 0 ? Ls[V_DX + (kc - 1) * NB + xc] : 0.0;
            double arr[NB], alr[NB], gy = 0.0, gy2 = 0.0;
            const double *ARr = Ls + ARB(kc) + yc * NB, *ALr = Ls + ALB(kc) + yc * NB;
#pragma unroll
            for (int j = 0; j < NB; j++) { arr[j] = ARr[j]; alr[j] = ALr[j]; }
            qpb_fence(dxk, dxp);
#else
            qpb_fence(dxk);
#endif
            qpb_for<0, NB>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                qpb_for<0, ZS>([&](auto uc) {
                    constexpr int u = decltype(uc)::value;
                    if constexpr ((qpb_bgsub(u) >> j) & 1) qpb_bfx<j>(gz[u], dxk, gr[u][j]);
                });
#if MY > 0
                if constexpr ((qpb_bARu >> j) & 1) qpb_bfx<j>(gy, dxk, arr[j]);
                if constexpr ((qpb_bALu >> j) & 1) qpb_bfx<j>(gy2, dxp, alr[j]);
#endif
            });
#pragma unroll
            for (int u = 0; u < ZS; u++) {
                if (act && isz[u]) {
                    const int iz = k * MZ + c + 16 * u;
                    double cc = 0.0;
                    const double bz = bz_of(mode, iz, smu, pcd, &cc);
                    const double dz = wz(iz) * (gz[u] - bz);
                    Ls[V_DZ + iz] = dz;
                    if (mode == BM_CORR) {      // ds replaces rz (read above, dead from here on)
                        const double s = Ls[V_S + iz], rzi = qpb_rcp(Ls[V_Z + iz]);
                        Ls[V_RZ + iz] = __builtin_fma(__builtin_fma(-s, dz, cc), rzi, -s);
                    }
                }
            }
#if MY > 0
            if (act && isy && mode != BM_PRED) {    // dy replaces ry (the predictor's dy is unused)
                const int iy = k * MY + c;
                Ls[V_RY + iy] = RDY * (Ls[V_RY + iy] - (gy + gy2));
            }
#endif
        }
        qpb_wsync();
        QPB_BT2(5);
    };

    // step lengths (Auxilary.c:359-393): alpha = 1 / max(-d / v) over d < 0, 1 if none
    auto step_length = [&](bool corr, double &ap, double &ad) {
        double bp = 0.0, bd = 0.0;
        // unrolled over the lane's rows with the index clamped (QPB_BROWS): the loads of all
        // rows issue together; a clamped row repeats row BNZ - 1, harmless in a maximum
        QPB_BROWS(BNZ, i, {
            const double s = Ls[V_S + i], z = Ls[V_Z + i], dz = Ls[V_DZ + i];
            const double rzi = qpb_rcp(z);
            const double dsl = corr ? Ls[V_RZ + i] : -s * __builtin_fma(dz, rzi, 1.0);
            bp = __builtin_fmax(bp, -dsl * __builtin_amdgcn_rcp(s));
            bd = __builtin_fmax(bd, -dz * rzi);
        });
        bp = qpb_bmax(bp);
        bd = qpb_bmax(bd);
        ap = bp > 1e-10 ? __builtin_amdgcn_rcp(bp) : 1.0;
        ad = bd > 1e-10 ? __builtin_amdgcn_rcp(bd) : 1.0;
    };

    // ---- kkt_initialize (Auxilary.c:992-1089) as iteration -1, then QP_SOLVE (qpSWIFT.c:502-602)
    const double tol2 = a.tol > 0.0 ? a.tol * a.tol : -1.0;
    double sigma = 100.0;      // options->sigma (GlobalOptions.h:49)
    long it = -1, itq = 0;
#if QPB_WARM
    // the warm variant: IterationCount, stats->Flag and options->sigma the QP enters with
    // (the row kernels' semantics: QP_MAXIT only when IterationCount reaches maxit,
    // qpSWIFT.c:598-601), and the drop-in's timers / per-iteration trace (KernelArgs::trace)
    const long it_in = QPB_LDS(&a.iters[q]);
    const int flag_in = QPB_LDS(&a.flag[q]);
    sigma = QPB_LDS(&a.sig[q]);
    it = 0;
    double sigf = sigma;
    double *const trc = (a.trace && lane == 0) ? a.trace + q * QPB_TRACE_STRIDE : nullptr;
    long t_fac = 0, t_kkt = 0, n_top = 0, n_it = 0;
#define QPB_BSIGF sigf = sigma
#define QPB_BCLK() ((long)__builtin_amdgcn_s_memrealtime())
#else
    constexpr long it_in = 0;
    constexpr int flag_in = 3;
#define QPB_BSIGF (void)0
#endif
    int flag = flag_in;
    double fv = 0.0, st_rx2 = 0.0, st_ry2 = 0.0, st_rz2 = 0.0, st_mu = 0.0, ap = 0.0, ad = 0.0;
    for (;;) {
        if ((QPB_WARM || it >= 0) && it >= a.maxit) {
            itq = it_in + it;
            flag = (!QPB_WARM || itq == a.maxit) ? 2 : flag_in;
            QPB_BSIGF;
            break;
        }
        wset = it < 0;
        double red[4] = {0.0, 0.0, 0.0, 1.0};
        double mu = 0.0;
        bool pc = true;
        if (it >= 0) {
            fv = residuals(red);
            const double mu_it = red[3] * (1.0 / BNZ);
            st_rx2 = red[0]; st_ry2 = BNY > 0 ? red[1] : 0.0; st_rz2 = red[2]; st_mu = mu_it;
#if QPB_WARM
            if (trc && it < QPB_TRACE_MAX) {
                double *e = trc + 4 + 7 * it;
                e[0] = fv; e[1] = __builtin_sqrt(red[0]); e[2] = BNY > 0 ? __builtin_sqrt(red[1]) : 0.0;
                e[3] = __builtin_sqrt(red[2]); e[4] = mu_it;
                n_top = it + 1;
            }
#endif
            if (red[0] < tol2 && red[2] < tol2 && (BNY == 0 || red[1] < tol2) && mu_it < a.abstol) {
                itq = it_in + it;
                flag = (QPB_WARM && itq == a.maxit) ? 2 : 0;
                QPB_BSIGF;
                break;
            }
            mu = mu_it;
            pc = sigma > a.sigma_d;
        }
        const double rsz = qpb_rcp(red[3]);
        QPB_BT(0);
#if QPB_WARM
        const long tf0 = QPB_BCLK();
#endif
        factor(qpb_ic<0>{});
        {
            bool tiny = false;      // any |D| <= 1e-14: |1/D| >= 1e14 (or not finite)
            QPB_BROWS(BNX, i, { tiny |= !(__builtin_fabs(Ls[O_RD + i]) < 1e14); });
            if (qpb_any(tiny)) factor(qpb_ic<1>{});
        }
#if QPB_WARM
        { const long d_ = QPB_BCLK() - tf0; t_fac += d_; t_kkt += d_; }
#endif
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
            for (int i = lane; i < BNY; i += 64) Ls[V_Y + i] = Ls[V_RY + i];
            qpb_wsync();
            QPB_BT(2);
            it = 0;
            continue;
        }
        if (!pc) sigma = a.sigma_d;
        bool pcd = false;
        if (pc) {
            // predictor (kktsolve_1, Auxilary.c:471-515), ds = -s o z
#if QPB_WARM
            const long ts0 = QPB_BCLK();
            solve(BM_PRED, 0.0, false);
            t_kkt += QPB_BCLK() - ts0;
#else
            solve(BM_PRED, 0.0, false);
#endif
            step_length(false, ap, ad);
            double rr = 0.0;
            QPB_BROWS(BNZ, i, {
                const double s = Ls[V_S + i], z = Ls[V_Z + i], dz = Ls[V_DZ + i];
                const double dsl = -s * __builtin_fma(dz, qpb_rcp(z), 1.0);
                const double t = (s + ap * dsl) * (z + ad * dz);
                if (ok_) rr += t;                   // a sum: the clamped repeat is left out
            });
            const double rho = qpb_bsum(rr) * rsz;      // formrho
            const double r1 = 1 > rho ? rho : 1;
            const double cube = r1 * r1 * r1;
            sigma = a.sigma_d < cube ? cube : a.sigma_d;
            pcd = true;
        }
        QPB_BT(2);
        // corrector / centering (kktsolve_2, Auxilary.c:524-564)
#if QPB_WARM
        const long tc0 = QPB_BCLK();
        solve(BM_CORR, sigma * mu, pcd);
        t_kkt += QPB_BCLK() - tc0;
#else
        solve(BM_CORR, sigma * mu, pcd);
#endif
        QPB_BT(3);
        step_length(true, ap, ad);
        ap = 0.99 * ap > 1.0 ? 1.0 : 0.99 * ap;
        ad = 0.99 * ad > 1.0 ? 1.0 : 0.99 * ad;
#if QPB_WARM
        if (trc && it < QPB_TRACE_MAX) {
            trc[4 + 7 * it + 5] = ap;
            trc[4 + 7 * it + 6] = ad;
            n_it = it + 1;
        }
#endif
        // (a clamped row stores the value its own lane stores: the same inputs, loaded by the
        // same instruction before either store)
        QPB_BROWS(BNX, i, { Ls[V_X + i] = __builtin_fma(Ls[V_DX + i], ap, Ls[V_X + i]); });
        if constexpr (BNY > 0) QPB_BROWS(BNY, i, { Ls[V_Y + i] = __builtin_fma(Ls[V_RY + i], ad, Ls[V_Y + i]); });
        QPB_BROWS(BNZ, i, {
            const double sn = __builtin_fma(Ls[V_RZ + i], ap, Ls[V_S + i]);
            const double zn = __builtin_fma(Ls[V_DZ + i], ad, Ls[V_Z + i]);
            Ls[V_S + i] = sn;
            Ls[V_Z + i] = zn;
        });
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
#if QPB_WARM
        QPB_STS(&a.sig[q], sigf);
        if (trc) { trc[0] = (double)t_fac; trc[1] = (double)t_kkt; trc[2] = (double)n_top; trc[3] = (double)n_it; }
#else
        if (a.sig) QPB_STS(&a.sig[q], sigma);
#endif
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
#undef QPB_BSIGF
#undef QPB_BCLK

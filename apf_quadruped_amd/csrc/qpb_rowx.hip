// qpb_rowx.hip -- the row form for plans of up to 32 variables: ONE 16-lane DPP row
// per QP, four QPs per wavefront, x rows c and 16 + c in lane c.
//
// Template source like qpb_row.hip (the host prepends the row template's common
// helpers, then sizes, the CSC -> LDS scatter tables and the structural patterns;
// qpb_wave.cpp generate_rowx_kernel).  Same algorithm and the same elimination as the
// row kernel -- every z and y row a leaf, the x block factored in natural order
// (plan order leaves first) -- for plans beyond the row kernel's n, p <= 16, m <= 32:
// the controller's 30-variable whole-body QPs (30 / 68 / 18 stance, 30 / 70 / 12 trot,
// 30 / 69 / 15 crawl; main.cpp:1649, 2005, 3232).
//
// Lanes.  Lane c of a row holds x rows c + 16 s (slots s < XS), y rows c + 16 v and z
// rows c + 16 u.  Every cross-lane move is a DPP row_newbcast folded into the consuming
// v_fmac_f64, every reduction a row butterfly.  The rows of the KKT Schur complement
// H = P + G'WG + 1e7 A'A (slot s: the lower triangle of its rows, columns 0 .. 16 s + 15)
// are factored in registers and stay there as rows of -L for the forward solves; -L is
// parked in LDS once per factor (packed strictly lower) for the backward solves, which
// read its columns.  P, A, G and H0 = P + 1e7 A'A stay in the row's LDS as dense
// column-major copies: every access is lane-linear with a compile-time offset, so no
// index tables live in registers (the row kernel keeps its slices in registers; at
// 30 / 68 / 18 they would be ~400 of them).
//
// Reference: qpSWIFT's Mehrotra predictor-corrector (qpSWIFT.c:473-644,
// kkt_initialize Auxilary.c:992-1089), LDL' with dynamic regularisation
// (ldl.c:253-326), residuals (Auxilary.c:745-786), step length
// (Auxilary.c:359-393).  Fast mode: FMA contraction, reciprocal pivots.
#pragma clang fp contract(fast)

#define NX QPB_NX
#define NZ QPB_NZ
#define NY QPB_NY
#define NY1 (NY > 0 ? NY : 1)
#define XS ((NX + 15) / 16)
#define YS ((NY + 15) / 16)
#define YS1 (YS > 0 ? YS : 1)
#define ZS ((NZ + 15) / 16)
static_assert(NX >= 1 && NX <= 32 && NY <= 32 && NZ >= 1 && NZ <= 128, "rowx kernel sizes");

#ifndef QPB_X_LAZYREG
#define QPB_X_LAZYREG 1   // pivot regularisation checked once per factor (the factor redone when needed,
                          // same bits), as the row kernel's QPB_R_LAZYREG
#endif
#ifndef QPB_X_TIMING
#define QPB_X_TIMING 0    // 3: cycles per phase (H0 + setup solve, residuals, factor, predictor,
                          //    corrector + tail, staging) into stats, as QPB_R_TIMING = 3;
                          // 2: cycles per part instead (G'WG, pivots, -L parking, the solves'
                          //    right-hand sides, triangular chains, dz / dy)
#endif
#ifndef QPB_X_GWGP
#define QPB_X_GWGP 1      // 1: G'WG issues each row's FMAs one row behind its products (0: right behind)
#endif
#ifndef QPB_X_PINH0
#define QPB_X_PINH0 1     // 1: H0's rows and A's columns loaded before the first DPP FMA (0: round 5's
                          // schedule, one LDS round trip per FMA)
#endif
#ifndef QPB_X_DBG
#define QPB_X_DBG 0       // (diagnostic: stop after the setup factor, its pivots D in x)
#endif
#ifndef QPB_WARM
#define QPB_WARM 0
#endif
#ifndef QPB_SERVE
#define QPB_SERVE 0
#endif
#define QPB_TRACE_MAX 256                       // = qpb::QPB_TRACE_MAX (qpb_codegen.hpp)
#define QPB_TRACE_STRIDE (4 + 7 * QPB_TRACE_MAX)

// columns held by x slot s: 0 .. qpb_xhw(s) - 1 (the lower triangle of its rows)
static constexpr int qpb_xhw(int s) { return 16 * s + 16 < NX ? 16 * s + 16 : NX; }
// G row r has a structural entry in a column of x slot s
static constexpr bool qpb_gxs(int r, int s) {
    for (int j = 16 * s; j < 16 * s + 16 && j < NX; j++)
        if (qpb_Gnz[r][j]) return true;
    return false;
}
// column j has a structural entry in a G row of z slot u
static constexpr bool qpb_gzs(int j, int u) {
    for (int r = 16 * u; r < 16 * u + 16 && r < NZ; r++)
        if (qpb_Gnz[r][j]) return true;
    return false;
}
static constexpr bool qpb_axs(int l, int s) {
    for (int j = 16 * s; j < 16 * s + 16 && j < NX; j++)
        if (NY > 0 && qpb_Anz[l][j]) return true;
    return false;
}
static constexpr bool qpb_ays(int j, int v) {
    for (int l = 16 * v; l < 16 * v + 16 && l < NY; l++)
        if (qpb_Anz[l][j]) return true;
    return false;
}
// a row of x slot s has P(row, j) != 0
static constexpr bool qpb_pxs(int j, int s) {
    for (int i = 16 * s; i < 16 * s + 16 && i < NX; i++)
        if (qpb_Pnz[i][j]) return true;
    return false;
}
// the forward solve's step k reaches a row of slot s: some row i > k of it has L(i, k) != 0
static constexpr bool qpb_lks(int k, int s) {
    for (int i = 16 * s; i < 16 * s + 16 && i < NX; i++)
        if (i > k && qpb_lnz[i][k]) return true;
    return false;
}
// the backward solve's step e reaches a column of slot s: some column k < e of it has L(e, k) != 0
static constexpr bool qpb_lcs(int e, int s) {
    for (int k = 16 * s; k < 16 * s + 16 && k < NX; k++)
        if (k < e && qpb_lnz[e][k]) return true;
    return false;
}

// LDS position of row e of -L (padded rows: 17 doubles for e < 16, 33 after)
static constexpr int qpb_lrow(int e) { return OFF_L + (e < 16 ? 17 * e : 17 * 16 + 33 * (e - 16)); }
// ... and of row i of H0 (the same padded rows; a factor that starts from upper parts holding
// other rows' values diverged on the 30 / 24 / 30 test shape -- an unexplained interaction,
// DESIGN §4c'; zeros there, as in the row kernel's H0, pass)
static constexpr int qpb_hrow(int i) { return OFF_H0 + (i < 16 ? 17 * i : 17 * 16 + 33 * (i - 16)); }
// the backward solve's terms in chain order: (e descending, x slot s) with a column of
// slot s below e structurally in row e of L
static constexpr int qpb_bk_n() {
    int n = 0;
    for (int e = NX - 1; e >= 0; e--)
        for (int s = 0; s < XS; s++) n += (e > 16 * s && qpb_lcs(e, s));
    return n;
}
static constexpr int qpb_bk_at(int k) {
    for (int e = NX - 1; e >= 0; e--)
        for (int s = 0; s < XS; s++)
            if (e > 16 * s && qpb_lcs(e, s) && k-- == 0) return (s << 12) | e;
    return 0;
}

// ---- sparse products as software pipelines.  A product's terms are the structural
// (slot, coefficient) pairs of its pattern; each term is one LDS load of the lane's
// coefficient and one DPP FMA.  The loads run QPB_X_CH terms ahead of their FMAs, with
// scheduling barriers between the groups, so the ~60-cycle LDS latency is paid once per
// product instead of once per term (the compiler otherwise sinks each load next to its
// FMA).  Term code: slot << 12 | family << 8 | index.
#ifndef QPB_X_CH
#define QPB_X_CH 12       // terms per pipeline group (<= 15: the LDS counter's range)
#endif
enum { QF_P = 0, QF_G = 1, QF_A = 2, QF_GZ = 3, QF_AY = 4 };
// does family f hold term (s, i)?  x-side families: P column i / G row i / A row i touches
// a row of x slot s; z / y side: column i touches a G row of z slot s / an A row of y slot s
static constexpr bool qpb_has(int f, int s, int i) {
    return f == QF_P ? (i < NX && qpb_pxs(i, s)) : f == QF_G ? (i < NZ && qpb_gxs(i, s))
         : f == QF_A ? (i < NY && qpb_axs(i, s)) : f == QF_GZ ? (i < NX && qpb_gzs(i, s))
         : (i < NX && NY > 0 && qpb_ays(i, s));
}
static constexpr int qpb_fslots(int f) { return f <= QF_A ? XS : f == QF_GZ ? ZS : YS; }
static constexpr int qpb_flen(int f) { return f == QF_P ? NX : f == QF_G ? NZ : f == QF_A ? NY : NX; }
// the list of families `fams` (bit mask), slot-major: for each slot, families in order
static constexpr int qpb_lst_n(int fams) {
    int n = 0;
    for (int f = 0; f < 5; f++)
        if ((fams >> f) & 1)
            for (int s = 0; s < qpb_fslots(f); s++)
                for (int i = 0; i < qpb_flen(f); i++) n += qpb_has(f, s, i);
    return n;
}
static constexpr int qpb_lst_at(int fams, int k) {
    for (int s = 0; s < 8; s++)
        for (int f = 0; f < 5; f++)
            if (((fams >> f) & 1) && s < qpb_fslots(f))
                for (int i = 0; i < qpb_flen(f); i++)
                    if (qpb_has(f, s, i) && k-- == 0) return (s << 12) | (f << 8) | i;
    return 0;
}
#ifndef QPB_X_WLDS
#define QPB_X_WLDS 0      // 1: G'WG reads w_r from LDS (the -L area, dead while H is formed) as a
                          // row-uniform load in its pipeline instead of a DPP broadcast per G row
#endif
static_assert(!QPB_X_WLDS || NZ <= O_DUMP - OFF_L, "QPB_X_WLDS: w does not fit the -L area");
// G'WG's terms, row-major: (row r, x slot s) with G(r, .) structural in slot s's columns
// (QPB_X_WLDS: each row led by its w term, slot code 7)
static constexpr int qpb_gw_n() {
    int n = 0;
    for (int r = 0; r < NZ; r++) {
        n += QPB_X_WLDS ? 1 : 0;
        for (int s = 0; s < XS; s++) n += qpb_gxs(r, s);
    }
    return n;
}
static constexpr int qpb_gw_at(int k) {
    for (int r = 0; r < NZ; r++) {
        if (QPB_X_WLDS && k-- == 0) return (7 << 12) | r;
        for (int s = 0; s < XS; s++)
            if (qpb_gxs(r, s) && k-- == 0) return (s << 12) | r;
    }
    return -1;
}
// the G'WG term list's row groups: group of term k (rows with terms, in order), row of group g
static constexpr int qpb_gw_grp(int k) {
    int g = 0, last = -1;
    for (int i = 0; i <= k; i++) {
        const int r = qpb_gw_at(i) & 4095;
        if (i > 0 && r != last) g++;
        last = r;
    }
    return g;
}
static constexpr int qpb_gw_row(int g) {
    int gi = 0, last = -1;
    for (int i = 0; i < qpb_gw_n(); i++) {
        const int r = qpb_gw_at(i) & 4095;
        if (i > 0 && r != last) gi++;
        if (gi == g) return r;
        last = r;
    }
    return 0;
}
// for k in [0, N): coef_k = ld(k) (an LDS load), fx(k, coef_k); loads CH terms ahead
template <int N, class LD, class FX>
static __device__ __forceinline__ void qpb_xpipe(LD &&ld, FX &&fx) {
    if constexpr (N > 0) {
        constexpr int CH = QPB_X_CH, NC = (N + CH - 1) / CH;
        double b0[CH], b1[CH];
        qpb_for<0, CH>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            if constexpr (i < N) b0[i] = ld(qpb_ic<i>{});
        });
        qpb_for<0, NC>([&](auto cc) {
            constexpr int ch = decltype(cc)::value;
            double(&cur)[CH] = (ch & 1) ? b1 : b0;
            double(&nxt)[CH] = (ch & 1) ? b0 : b1;
            __builtin_amdgcn_sched_barrier(0);
            qpb_for<0, CH>([&](auto ic) {
                constexpr int k = (ch + 1) * CH + decltype(ic)::value;
                if constexpr (k < N) nxt[decltype(ic)::value] = ld(qpb_ic<k>{});
            });
            __builtin_amdgcn_sched_barrier(0);
            qpb_for<0, CH>([&](auto ic) {
                constexpr int k = ch * CH + decltype(ic)::value;
                if constexpr (k < N) fx(qpb_ic<k>{}, cur[decltype(ic)::value]);
            });
        });
        __builtin_amdgcn_sched_barrier(0);
    }
}
#define QPB_TERM(fams, kc) constexpr int t_ = qpb_lst_at((fams), decltype(kc)::value); \
    constexpr int ts_ = t_ >> 12, tf_ = (t_ >> 8) & 15, ti_ = t_ & 255; (void)ts_; (void)tf_; (void)ti_

// one logical block `lb` of the plan's batch (QPs 4 lb .. 4 lb + 3)
// the value is needed here (an empty asm that reads and writes it: its load is issued and
// waited for before this point, not sunk next to a later use)
static __device__ __forceinline__ void qpb_xpin(double &v) { asm volatile("" : "+v"(v)); }

static __device__ __forceinline__ void qpb_rowx_body(const qpb_args &a, long lb, double *qpb_lds) {
    const int lane = threadIdx.x & 63, row = lane >> 4, c = lane & 15;
#if QPB_X_TIMING
    double tph[6] = {0, 0, 0, 0, 0, 0};
    long tcy = (long)__builtin_readcyclecounter();
#endif
#if QPB_X_TIMING == 3
#define QPB_TM(k) { const long t2_ = (long)__builtin_readcyclecounter(); tph[k] += (double)(t2_ - tcy); tcy = t2_; }
#else
#define QPB_TM(k)
#endif
#if QPB_X_TIMING == 2
#define QPB_TM0() { tcy = (long)__builtin_readcyclecounter(); }
#define QPB_TM2(k) { const long t2_ = (long)__builtin_readcyclecounter(); tph[k] += (double)(t2_ - tcy); tcy = t2_; }
#else
#define QPB_TM0()
#define QPB_TM2(k)
#endif
    const long q0 = lb * 4;
    if (q0 >= a.B) {                           // wave-uniform
        if (a.best) qpb_argmin_arrive(a, __builtin_huge_val(), -1);
        return;
    }
    const long q = q0 + row;
    const bool valid = q < a.B;
    const long qc = valid ? q : a.B - 1;       // rows past the batch solve a copy, write nothing
    const long tile = qc >> 6;
    const int ql = (int)(qc & 63);
    double *__restrict__ Ls = qpb_lds + row * LDS_QP;
    bool isx[XS], isz[ZS], isy[YS1];
    int ixc[XS], izc[ZS], iyc[YS1];
#pragma unroll
    for (int s = 0; s < XS; s++) {
        isx[s] = 16 * s + c < NX;
        ixc[s] = isx[s] ? 16 * s + c : NX - 1;
    }
#pragma unroll
    for (int u = 0; u < ZS; u++) {
        isz[u] = 16 * u + c < NZ;
        izc[u] = isz[u] ? 16 * u + c : NZ - 1;
    }
#pragma unroll
    for (int v = 0; v < YS1; v++) {
        isy[v] = 16 * v + c < NY;
        iyc[v] = isy[v] ? 16 * v + c : (NY > 0 ? NY - 1 : 0);
    }
    constexpr double RDY = 1.0 / -1e-7;        // leaf y pivots: D = 0 regularised to -1e-7

    // ---- stage this QP's P, A, G as dense column-major matrices in the row's LDS
    {
        constexpr int NPL = (QPB_NNZP + 15) / 16, NGL = (QPB_NNZG + 15) / 16, NAL = (QPB_NNZA + 15) / 16;
        double vP[NPL], vG[NGL], vA[NAL > 0 ? NAL : 1];
        int iP[NPL], iP2[NPL], iG[NGL], iA[NAL > 0 ? NAL : 1];
        const double *tP = a.P + tile * (QPB_NNZP * QPB_TSTR) + ql;
        const double *tG = a.G + tile * (QPB_NNZG * QPB_TSTR) + ql;
#pragma unroll
        for (int u = 0; u < NPL; u++) {
            const int k = c + 16 * u;
            const bool ok = k < QPB_NNZP;
            vP[u] = ok ? QPB_LDS(&tP[(ok ? k : QPB_NNZP - 1) * QPB_TSTR]) : 0.0;   // in-bounds address either way
            iP[u] = ok ? qpb_scP[k] : -1;
            iP2[u] = ok ? qpb_scP2[k] : -1;
        }
#pragma unroll
        for (int u = 0; u < NGL; u++) {
            const int k = c + 16 * u;
            const bool ok = k < QPB_NNZG;
            vG[u] = ok ? QPB_LDS(&tG[(ok ? k : QPB_NNZG - 1) * QPB_TSTR]) : 0.0;   // in-bounds address either way
            iG[u] = ok ? qpb_scG[k] : -1;
        }
#if NY > 0
        const double *tA = a.A + tile * (QPB_NNZA * QPB_TSTR) + ql;
#pragma unroll
        for (int u = 0; u < NAL; u++) {
            const int k = c + 16 * u;
            const bool ok = k < QPB_NNZA;
            vA[u] = ok ? QPB_LDS(&tA[(ok ? k : QPB_NNZA - 1) * QPB_TSTR]) : 0.0;   // in-bounds address either way
            iA[u] = ok ? qpb_scA[k] : -1;
        }
#endif
        // zero-fill of the staged matrices: 16-byte stores from the row's first 16-byte
        // aligned double (LDS_QP is odd: rows 1 and 3 start 8 bytes past one), the
        // leading / trailing doubles singly
        {
            const int a0 = (row * LDS_QP) & 1;
            double2 *z2 = reinterpret_cast<double2 *>(Ls + a0);
            // (STG_END is even: rows with a0 = 0 need STG_END / 2 pairs -- one more than the
            // (STG_END - 1) / 2 round 5 sized the loop for, which missed the last pair when
            // STG_END = 2 mod 32)
            static_assert(STG_END % 2 == 0, "staged area ends on a pair");
#pragma unroll
            for (int i = 0; i < (STG_END / 2 + 15) / 16; i++) {
                const int k = c + 16 * i;
                if (2 * k + 1 < STG_END - a0) z2[k] = double2{0.0, 0.0};
            }
            if (c == 0) {
                Ls[0] = 0.0;
                Ls[STG_END - 1] = 0.0;
            }
        }
        qpb_wsync();
#pragma unroll
        for (int u = 0; u < NPL; u++) {
            if (iP[u] >= 0) Ls[OFF_P + iP[u]] = vP[u];
            if (iP2[u] >= 0) Ls[OFF_P + iP2[u]] = vP[u];
        }
#pragma unroll
        for (int u = 0; u < NGL; u++)
            if (iG[u] >= 0) Ls[OFF_G + iG[u]] = vG[u];
#pragma unroll
        for (int u = 0; u < NAL; u++)
            if (iA[u] >= 0) Ls[OFF_A + iA[u]] = vA[u];
        qpb_wsync();
    }
    double cx[XS], hz[ZS], by[YS1];
#pragma unroll
    // (clamped row indices: every address in bounds even if the load is issued for a masked lane)
    for (int s = 0; s < XS; s++) cx[s] = isx[s] ? QPB_LDS(&a.c[tile * (NX * QPB_TSTR) + ixc[s] * QPB_TSTR + ql]) : 0.0;
#pragma unroll
    for (int u = 0; u < ZS; u++) hz[u] = isz[u] ? QPB_LDS(&a.h[tile * (NZ * QPB_TSTR) + izc[u] * QPB_TSTR + ql]) : 0.0;
#pragma unroll
    for (int v = 0; v < YS1; v++)
        by[v] = (NY > 0 && isy[v]) ? QPB_LDS(&a.b[tile * (NY1 * QPB_TSTR) + iyc[v] * QPB_TSTR + ql]) : 0.0;
    QPB_TM(5);
    const double *const Pd = Ls + OFF_P, *const Ad = Ls + OFF_A, *const Gd = Ls + OFF_G;
    // Pd[j LDP + i] = P(i, j) (both triangles); Ad[j LDA + l] = A(l, j); Gd[j LDG + r] = G(r, j)

    // rows of H (then of -L): slot s holds columns 0 .. qpb_xhw(s) - 1
    double H[XS][NX];
    // ---- H0 = P + 1e7 A'A (the leaf y rows folded into the x block), once: rows of
    // this lane's slots to LDS (H0(i, j) at OFF_H0 + j LDP + i)
    {
        qpb_for<0, XS>([&](auto sc) {
            constexpr int s = decltype(sc)::value;
            qpb_for<0, qpb_xhw(s)>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                H[s][j] = Pd[j * LDP + ixc[s]];
            });
        });
        // every load of the H0 rows and A columns issued before the first DPP FMA (one
        // LDS wait): left to the scheduler each load sat in front of its own FMA, some
        // 45 round trips in series
        double al0[NY > 0 ? NY : 1][XS];
        qpb_for<0, NY>([&](auto lc) {
            constexpr int l = decltype(lc)::value;
            qpb_for<0, XS>([&](auto sc) {
                constexpr int s = decltype(sc)::value;
                if constexpr (qpb_axs(l, s)) al0[l][s] = Ad[ixc[s] * LDA + l];
            });
        });
#if QPB_X_PINH0
#pragma unroll
        for (int s = 0; s < XS; s++)
#pragma unroll
            for (int j = 0; j < NX; j++)
                if (j < qpb_xhw(s)) qpb_xpin(H[s][j]);
        qpb_for<0, NY>([&](auto lc) {
            constexpr int l = decltype(lc)::value;
            qpb_for<0, XS>([&](auto sc) {
                constexpr int s = decltype(sc)::value;
                if constexpr (qpb_axs(l, s)) qpb_xpin(al0[l][s]);
            });
        });
#endif
        qpb_for<0, NY>([&](auto lc) {
            constexpr int l = decltype(lc)::value;
            double al[XS], qa[XS];
            qpb_for<0, XS>([&](auto sc) {
                constexpr int s = decltype(sc)::value;
                if constexpr (qpb_axs(l, s)) {
                    al[s] = al0[l][s];
                    qa[s] = -RDY * al[s];                  // 1e7 A(l, row)
                }
            });
            qpb_for<0, XS>([&](auto sc) {
                constexpr int s = decltype(sc)::value;
                if constexpr (qpb_axs(l, s)) {
                    qpb_for<0, qpb_xhw(s)>([&](auto jc) {
                        constexpr int j = decltype(jc)::value;
                        if constexpr (qpb_Anz[l][j]) qpb_fxs<(j & 15)>(H[s][j], al[j >> 4], qa[s]);
                    });
                }
            });
        });
        // padded rows (qpb_hrow): row i's entries j <= i, zeros up to its slot's last column
#pragma unroll
        for (int s = 0; s < XS; s++) {
            if (isx[s]) {
                const int rw = 16 * s + c, base = qpb_hrow(rw);
#pragma unroll
                for (int j = 0; j < qpb_xhw(s); j++) Ls[base + j] = j <= rw ? H[s][j] : 0.0;
            }
        }
        qpb_wsync();
    }

    // ---- factor with z diagonal -s/z: H = H0 + G' diag(w) G, then its LDL' in place
    // (rows of -L in H, 1/D in rDd), -L parked for the backward solves
    double rDd[XS];
    auto gwg = [&](const double (&w)[ZS]) {
        qpb_for<0, XS>([&](auto sc) {
            constexpr int s = decltype(sc)::value;
            qpb_for<0, qpb_xhw(s)>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                H[s][j] = Ls[qpb_hrow(ixc[s]) + j];     // zero beyond the diagonal
            });
        });
        // += G(r, row) w_r G(r, j): lane j's G(r, j) by DPP broadcast against the lane's own
        // G(r, row) w_r -- the same LDS values serve as source and coefficient; the loads
        // pipelined ahead of the rows' FMAs
        double gc[XS], wl = 0.0;
#if QPB_X_GWGP
        double gcb[2][XS], crb[2][XS];
#endif
        (void)gc;
        // row R's FMAs: += G(R, row) w_R G(R, j), lane j's G(R, j) (gcv) by DPP broadcast
        auto gw_row = [&](auto rc, const double (&gcv)[XS], const double (&crv)[XS]) {
            constexpr int R = decltype(rc)::value;
            qpb_for<0, XS>([&](auto sc) {
                constexpr int s2 = decltype(sc)::value;
                if constexpr (qpb_gxs(R, s2)) {
                    qpb_for<0, qpb_xhw(s2)>([&](auto jc) {
                        constexpr int j = decltype(jc)::value;
                        if constexpr (qpb_Gnz[R][j]) qpb_fxs<(j & 15)>(H[s2][j], gcv[j >> 4], crv[s2]);
                    });
                }
            });
        };
        if constexpr (QPB_X_WLDS) {
#pragma unroll
            for (int u = 0; u < ZS; u++)
                if (isz[u]) Ls[OFF_L + 16 * u + c] = w[u];
            qpb_wsync();
        }
        qpb_xpipe<qpb_gw_n()>(
            [&](auto kc) -> double {
                constexpr int t = qpb_gw_at(decltype(kc)::value), ts = t >> 12, r = t & 4095;
                if constexpr (ts == 7) return Ls[OFF_L + r];
                else return Gd[ixc[ts] * LDG + r];
            },
            [&](auto kc, double cf) {
                constexpr int k = decltype(kc)::value, t = qpb_gw_at(k), ts = t >> 12, r = t & 4095;
#if QPB_X_GWGP
                // one row behind: row g's products G(r, row) w_r are formed, then row g-1's
                // FMAs issue -- no FMA right behind the multiply that feeds it (a DPP
                // operand written by the previous VALU waits); buffers by row parity, so
                // each H entry still takes its rows in order (the same bits)
                constexpr int g = qpb_gw_grp(k);
                if constexpr (ts == 7) wl = cf;
                else gcb[g & 1][ts] = cf;
                if constexpr (k + 1 == qpb_gw_n() || (qpb_gw_at(k + 1) & 4095) != r) {   // the row's last term
                    const double wr = QPB_X_WLDS ? wl : qpb_nb<(r & 15)>(w[r >> 4]);
                    qpb_for<0, XS>([&](auto sc) {
                        constexpr int s2 = decltype(sc)::value;
                        if constexpr (qpb_gxs(r, s2)) crb[g & 1][s2] = gcb[g & 1][s2] * wr;
                    });
                    if constexpr (g > 0) gw_row(qpb_ic<qpb_gw_row(g - 1)>{}, gcb[(g - 1) & 1], crb[(g - 1) & 1]);
                    if constexpr (k + 1 == qpb_gw_n()) gw_row(qpb_ic<r>{}, gcb[g & 1], crb[g & 1]);
                }
#else
                if constexpr (ts == 7) wl = cf;
                else gc[ts] = cf;
                if constexpr (k + 1 == qpb_gw_n() || (qpb_gw_at(k + 1) & 4095) != r) {   // the row's last term
                    const double wr = QPB_X_WLDS ? wl : qpb_nb<(r & 15)>(w[r >> 4]);
                    double cr[XS];
                    qpb_for<0, XS>([&](auto sc) {
                        constexpr int s2 = decltype(sc)::value;
                        if constexpr (qpb_gxs(r, s2)) cr[s2] = gc[s2] * wr;
                    });
                    gw_row(qpb_ic<r>{}, gc, cr);
                }
#endif
            });
    };
    // right-looking LDL' in natural order; the pivot recurrence is the critical path:
    // D_{k+1} from H'(k+1, k) and H'(k+1, k+1) ahead of pivot k's own update (the row
    // kernel's lookahead).  REG: every pivot regularised inline (ldl.c:273-274); the fast
    // pass returns min |D| so the caller can redo the factor with REG when needed.
    auto pivots = [&](auto regc) -> double {
        constexpr bool REG = decltype(regc)::value != 0;
        double dmin = __builtin_huge_val();
        double dpiv = qpb_nb<0>(H[0][0]);
#pragma unroll
        for (int s = 0; s < XS; s++) rDd[s] = 0.0;
        qpb_for<0, NX>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            double rd;
            if constexpr (REG || !QPB_X_LAZYREG) {
                rd = qpb_rcp_reg(dpiv);
            } else {
                rd = qpb_rcp_nr(dpiv);
                dmin = __builtin_fmin(dmin, __builtin_fabs(dpiv));
            }
            double nl[XS];
            qpb_for<0, XS>([&](auto sc) {
                constexpr int s = decltype(sc)::value;
                if constexpr (k + 1 < qpb_xhw(s)) {           // slot s has rows below the pivot
                    nl[s] = H[s][k] * -rd;                     // -L(row, k)
                    asm volatile("" : "+v"(nl[s]));
                }
            });
            if constexpr (k + 1 < NX) {
                constexpr int s1 = (k + 1) >> 4;
                const double h = qpb_nb<((k + 1) & 15)>(H[s1][k]), hkk = qpb_nb<((k + 1) & 15)>(H[s1][k + 1]);
                dpiv = __builtin_fma(-(h * h), rd, hkk);
            }
            rDd[k >> 4] = c == (k & 15) ? rd : rDd[k >> 4];
            qpb_for<0, XS>([&](auto sc) {
                constexpr int s = decltype(sc)::value;
                if constexpr (k + 1 < qpb_xhw(s)) {
                    qpb_for<k + 1, qpb_xhw(s)>([&](auto jc) {
                        constexpr int j = decltype(jc)::value;
                        if constexpr (qpb_lnz[j][k]) qpb_fxs<(j & 15)>(H[s][j], H[j >> 4][k], nl[s]);   // -= L(row,k) H(j,k)
                    });
                }
            });
            qpb_for<0, XS>([&](auto sc) {
                constexpr int s = decltype(sc)::value;
                if constexpr (k + 1 < qpb_xhw(s)) {
                    if constexpr (k < 16 * s) H[s][k] = nl[s];
                    else H[s][k] = c > k - 16 * s ? nl[s] : 0.0;
                }
            });
        });
        return dmin;
    };
    auto factor = [&](const double (&w)[ZS]) {
        QPB_TM0();
        gwg(w);
        QPB_TM2(0);
        const double dmin = pivots(qpb_ic<0>{});
        QPB_TM2(1);
        if (QPB_X_LAZYREG && qpb_any(dmin <= 1e-14)) {     // wave-uniform, rare
            gwg(w);
            pivots(qpb_ic<1>{});
        }
        // rows of -L to LDS, padded (qpb_lrow): the entries from the diagonal on are zero
        // (the pivots' selects; the slot's last column zeroed here)
        qpb_for<0, XS>([&](auto sc) {
            constexpr int s = decltype(sc)::value;
            if (isx[s]) {
                const int base = qpb_lrow(16 * s + c);
                qpb_for<0, qpb_xhw(s)>([&](auto kc) {
                    constexpr int k = decltype(kc)::value;
                    Ls[base + k] = k + 1 == qpb_xhw(s) ? 0.0 : H[s][k];
                });
            }
        });
        qpb_wsync();
        QPB_TM2(2);
    };

    // ---- solve K [dx; dy; dz] = [bx; by; bz] with the current factor and w
    auto solve = [&](const double (&w)[ZS], const double (&bx)[XS], const double (&byv)[YS1], const double (&bz)[ZS],
                     double (&dx)[XS], double (&dy)[YS1], double (&dz)[ZS]) {
        QPB_TM0();
        double v[ZS], yr[YS1];
#pragma unroll
        for (int u = 0; u < ZS; u++) v[u] = w[u] * bz[u];                 // leaf eliminations
#pragma unroll
        for (int l = 0; l < YS1; l++) yr[l] = -RDY * byv[l];
        double t[XS], ta[XS][4];
#pragma unroll
        for (int s = 0; s < XS; s++) { ta[s][0] = bx[s]; ta[s][1] = ta[s][2] = ta[s][3] = 0.0; }
        constexpr int FR = (1 << QF_G) | (1 << QF_A);
        qpb_xpipe<qpb_lst_n(FR)>(
            [&](auto kc) -> double {
                QPB_TERM(FR, kc);
                if constexpr (tf_ == QF_G) return Gd[ixc[ts_] * LDG + ti_];
                else return Ad[ixc[ts_] * LDA + ti_];
            },
            [&](auto kc, double cf) {
                QPB_TERM(FR, kc);
                if constexpr (tf_ == QF_G) qpb_fxs<(ti_ & 15)>(ta[ts_][ti_ & 3], v[ti_ >> 4], cf);
                else qpb_fxs<(ti_ & 15)>(ta[ts_][(NZ + ti_) & 3], yr[ti_ >> 4], cf);
            });
#pragma unroll
        for (int s = 0; s < XS; s++) t[s] = (ta[s][0] + ta[s][1]) + (ta[s][2] + ta[s][3]);
        QPB_TM2(3);
        // forward: t(row) += -L(row, k) t(k)
        qpb_for<0, NX>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            qpb_for<0, XS>([&](auto sc) {
                constexpr int s = decltype(sc)::value;
                if constexpr (qpb_lks(k, s)) {
                    if constexpr (s == (k >> 4)) qpb_fxd<(k & 15)>(t[s], H[s][k]);
                    else qpb_fx<(k & 15)>(t[s], t[k >> 4], H[s][k]);
                }
            });
        });
#pragma unroll
        for (int s = 0; s < XS; s++) t[s] *= rDd[s];
        // backward: t(col) += -L(e, col) t(e), e > col; the -L columns streamed from LDS
        // ahead of the chain
        qpb_xpipe<qpb_bk_n()>(
            [&](auto kc) -> double {
                constexpr int bt = qpb_bk_at(decltype(kc)::value), e = bt & 255, s2 = bt >> 12;
                return Ls[qpb_lrow(e) + ixc[s2]];       // zero where e <= the column
            },
            [&](auto kc, double lt) {
                constexpr int bt = qpb_bk_at(decltype(kc)::value), e = bt & 255, s2 = bt >> 12;
                if constexpr (s2 == (e >> 4)) qpb_fxd<(e & 15)>(t[s2], lt);
                else qpb_fx<(e & 15)>(t[s2], t[e >> 4], lt);
            });
#pragma unroll
        for (int s = 0; s < XS; s++) dx[s] = t[s];
        QPB_TM2(4);
        // dz = w (G dx - bz), dy = -1e7 (by - A dx)
        double gz[ZS][2], gy[YS1][2];
#pragma unroll
        for (int u = 0; u < ZS; u++) gz[u][0] = gz[u][1] = 0.0;
#pragma unroll
        for (int l = 0; l < YS1; l++) gy[l][0] = gy[l][1] = 0.0;
        constexpr int FD = (1 << QF_GZ) | (1 << QF_AY);
        qpb_xpipe<qpb_lst_n(FD)>(
            [&](auto kc) -> double {
                QPB_TERM(FD, kc);
                if constexpr (tf_ == QF_GZ) return Gd[ti_ * LDG + izc[ts_]];
                else return Ad[ti_ * LDA + iyc[ts_]];
            },
            [&](auto kc, double cf) {
                QPB_TERM(FD, kc);
                if constexpr (tf_ == QF_GZ) qpb_fxs<(ti_ & 15)>(gz[ts_][ti_ & 1], t[ti_ >> 4], cf);
                else qpb_fxs<(ti_ & 15)>(gy[ts_][ti_ & 1], t[ti_ >> 4], cf);
            });
#pragma unroll
        for (int u = 0; u < ZS; u++) dz[u] = w[u] * ((gz[u][0] + gz[u][1]) - bz[u]);
#pragma unroll
        for (int l = 0; l < YS; l++) dy[l] = RDY * (byv[l] - (gy[l][0] + gy[l][1]));
        QPB_TM2(5);
    };

    // ---- kkt_initialize (Auxilary.c:992-1089) as iteration -1, then the QP_SOLVE
    // loop (qpSWIFT.c:502-602); the wave runs until all four rows stop
    double x[XS], y[YS1], z[ZS], sl[ZS];
#pragma unroll
    for (int s = 0; s < XS; s++) x[s] = 0.0;
#pragma unroll
    for (int v = 0; v < YS1; v++) y[v] = 0.0;
#pragma unroll
    for (int u = 0; u < ZS; u++) { z[u] = 1.0; sl[u] = 1.0; }
    bool act = valid;
    long itq = 0;
    double st_rx2 = 0.0, st_ry2 = 0.0, st_rz2 = 0.0, st_mu = 0.0, ap = 0.0, ad = 0.0, fv = 0.0;
    const double tol2 = a.tol > 0.0 ? a.tol * a.tol : -1.0;
    double sigma = 100.0;      // options->sigma (SIGMA, GlobalOptions.h:49)
    long it = -1;
#if QPB_WARM
    // warm variant (qpb_solve_warm): QP_SOLVE continues from the object's iterate,
    // IterationCount and options->sigma (qpSWIFT.c:502-596 never re-initialises)
#if QPB_SERVE
    const double *wi = a.win;                  // the host's block (KernelArgs::win, QP 0)
#pragma unroll
    for (int s = 0; s < XS; s++) if (isx[s]) x[s] = QPB_LDS(&wi[ixc[s]]);
#pragma unroll
    for (int v = 0; v < YS; v++) if (isy[v]) y[v] = QPB_LDS(&wi[NX + iyc[v]]);
#pragma unroll
    for (int u = 0; u < ZS; u++)
        if (isz[u]) { z[u] = QPB_LDS(&wi[NX + NY + izc[u]]); sl[u] = QPB_LDS(&wi[NX + NY + NZ + izc[u]]); }
    const int *wfl = reinterpret_cast<const int *>(wi + NX + NY + 2 * NZ);
    const long it0 = QPB_LDS(&wfl[1]);
    const int flag0 = QPB_LDS(&wfl[0]);
    sigma = QPB_LDS(&wi[NX + NY + 2 * NZ + 1]);
#else
#pragma unroll
    for (int s = 0; s < XS; s++) if (isx[s]) x[s] = QPB_LDS(&a.x[tile * (NX * 64) + ixc[s] * 64 + ql]);
#pragma unroll
    for (int v = 0; v < YS; v++) if (isy[v]) y[v] = QPB_LDS(&a.y[tile * (NY1 * 64) + iyc[v] * 64 + ql]);
#pragma unroll
    for (int u = 0; u < ZS; u++)
        if (isz[u]) {
            z[u] = QPB_LDS(&a.z[tile * (NZ * 64) + izc[u] * 64 + ql]);
            sl[u] = QPB_LDS(&a.s[tile * (NZ * 64) + izc[u] * 64 + ql]);
        }
    const long it0 = QPB_LDS(&a.iters[qc]);   // IterationCount the QP enters with
    const int flag0 = QPB_LDS(&a.flag[qc]);   // stats->Flag it enters with (QP_FATAL after setup)
    sigma = QPB_LDS(&a.sig[qc]);
#endif
    it = 0;
    double sigf = sigma;       // options->sigma when this row's loop ends
#define QPB_SIGF sigf = sigma
    // the drop-in's timers and verbose trace (KernelArgs::trace, qpb_codegen.hpp)
    double *const trc = (a.trace && valid && c == 0) ? a.trace + qc * QPB_TRACE_STRIDE : nullptr;
    long t_fac = 0, t_kkt = 0, n_top = 0, n_it = 0;
#define QPB_CLK() ((long)__builtin_amdgcn_s_memrealtime())
#else
    constexpr long it0 = 0;
    constexpr int flag0 = 3;
#define QPB_SIGF (void)0
#endif
    int flag = flag0;
    QPB_TM(0);
    for (;;) {
        if ((QPB_WARM || it >= 0) && it >= a.maxit) {
            // qpSWIFT.c:598-601: QP_MAXIT only when IterationCount == maxit
            if (act) { itq = it0 + it; flag = (!QPB_WARM || itq == a.maxit) ? 2 : flag0; QPB_SIGF; }
            break;
        }
        // updatekktmatrix (Auxilary.c:211-215): z diagonal -s/z (-I at setup, s = z = 1)
        double rzi[ZS], rsi[ZS], w[ZS];
#pragma unroll
        for (int u = 0; u < ZS; u++) {
            rzi[u] = qpb_rcp(z[u]);
            rsi[u] = __builtin_amdgcn_rcp(sl[u]);     // step length
            const double kd = isz[u] ? -sl[u] * rzi[u] : -1.0;
            w[u] = -qpb_rcp_reg(kd);
        }
        // residuals (Auxilary.c:745-786): rx = -c - P x - G'z - A'y, ry = b - A x, rz = h - s - G x
        double rx[XS], ry[YS1], rz[ZS], red[4] = {0.0, 0.0, 0.0, 1.0}, fq = 0.0;
#pragma unroll
        for (int l = 0; l < YS1; l++) ry[l] = 0.0;
        if (QPB_WARM || it >= 0) {
            // x side: rx = -c - P x - G'z - A'y;  z / y side: G x, A x
            double ta[XS][4], px[XS][2], gz[ZS][2], gy[YS1][2];
#pragma unroll
            for (int s = 0; s < XS; s++) {
                ta[s][0] = cx[s]; ta[s][1] = ta[s][2] = ta[s][3] = 0.0;
                px[s][0] = px[s][1] = 0.0;
            }
#pragma unroll
            for (int u = 0; u < ZS; u++) gz[u][0] = gz[u][1] = 0.0;
#pragma unroll
            for (int l = 0; l < YS1; l++) gy[l][0] = gy[l][1] = 0.0;
            constexpr int FX_ = (1 << QF_P) | (1 << QF_G) | (1 << QF_A), FZ_ = (1 << QF_GZ) | (1 << QF_AY);
            qpb_xpipe<qpb_lst_n(FX_)>(
                [&](auto kc) -> double {
                    QPB_TERM(FX_, kc);
                    if constexpr (tf_ == QF_P) return Pd[ti_ * LDP + ixc[ts_]];
                    else if constexpr (tf_ == QF_G) return Gd[ixc[ts_] * LDG + ti_];
                    else return Ad[ixc[ts_] * LDA + ti_];
                },
                [&](auto kc, double cf) {
                    QPB_TERM(FX_, kc);
                    if constexpr (tf_ == QF_P) qpb_fxs<(ti_ & 15)>(px[ts_][ti_ & 1], x[ti_ >> 4], cf);
                    else if constexpr (tf_ == QF_G) qpb_fxs<(ti_ & 15)>(ta[ts_][ti_ & 3], z[ti_ >> 4], cf);
                    else qpb_fxs<(ti_ & 15)>(ta[ts_][(NZ + ti_) & 3], y[ti_ >> 4], cf);
                });
            qpb_xpipe<qpb_lst_n(FZ_)>(
                [&](auto kc) -> double {
                    QPB_TERM(FZ_, kc);
                    if constexpr (tf_ == QF_GZ) return Gd[ti_ * LDG + izc[ts_]];
                    else return Ad[ti_ * LDA + iyc[ts_]];
                },
                [&](auto kc, double cf) {
                    QPB_TERM(FZ_, kc);
                    if constexpr (tf_ == QF_GZ) qpb_fxs<(ti_ & 15)>(gz[ts_][ti_ & 1], x[ti_ >> 4], cf);
                    else qpb_fxs<(ti_ & 15)>(gy[ts_][ti_ & 1], x[ti_ >> 4], cf);
                });
            red[3] = 0.0;
#pragma unroll
            for (int s = 0; s < XS; s++) {
                const double pxs = px[s][0] + px[s][1];
                rx[s] = -(((ta[s][0] + ta[s][1]) + (ta[s][2] + ta[s][3])) + pxs);
                if (isx[s]) {
                    red[0] = __builtin_fma(rx[s], rx[s], red[0]);
                    fq = __builtin_fma(x[s], __builtin_fma(0.5, pxs, cx[s]), fq);   // objective (Auxilary.c:1133-1141)
                }
            }
#pragma unroll
            for (int u = 0; u < ZS; u++) {
                rz[u] = (hz[u] - sl[u]) - (gz[u][0] + gz[u][1]);
                if (isz[u]) {
                    red[2] = __builtin_fma(rz[u], rz[u], red[2]);
                    red[3] = __builtin_fma(sl[u], z[u], red[3]);
                }
            }
#pragma unroll
            for (int l = 0; l < YS; l++) {
                ry[l] = by[l] - (gy[l][0] + gy[l][1]);
                if (isy[l]) red[1] = __builtin_fma(ry[l], ry[l], red[1]);
            }
            qpb_rsum<4>(red);
        } else {
            // kkt_initialize's pass (iteration -1) has no exit test: no residuals
#pragma unroll
            for (int s = 0; s < XS; s++) rx[s] = 0.0;
#pragma unroll
            for (int v = 0; v < YS1; v++) ry[v] = 0.0;
#pragma unroll
            for (int u = 0; u < ZS; u++) rz[u] = 0.0;
        }
        const double sz = red[3];
        const double rsz = qpb_rcp(sz);            // formrho's 1 / s'z
        QPB_TM(1);
        bool pc = true;
        double mu = 0.0;
        if (QPB_WARM || it >= 0) {
            const double mu_it = sz * (1.0 / NZ);
            double fr[1] = {fq};
            qpb_rsum<1>(fr);
#if QPB_WARM
            if (trc && act && it < QPB_TRACE_MAX) {
                double *e = trc + 4 + 7 * it;
                e[0] = fr[0]; e[1] = __builtin_sqrt(red[0]); e[2] = NY > 0 ? __builtin_sqrt(red[1]) : 0.0;
                e[3] = __builtin_sqrt(red[2]); e[4] = mu_it;
                n_top = it + 1;
            }
#endif
            if (act) {
                fv = fr[0];
                st_rx2 = red[0];
                st_ry2 = NY > 0 ? red[1] : 0.0;
                st_rz2 = red[2];
                st_mu = mu_it;
                if (red[0] < tol2 && red[2] < tol2 && (NY == 0 || red[1] < tol2) && mu_it < a.abstol) {
                    itq = it0 + it;
                    flag = (QPB_WARM && itq == a.maxit) ? 2 : 0;
                    QPB_SIGF;
                    act = false;
                }
            }
            if (!qpb_any(act)) break;
            mu = mu_it;
            pc = sigma > a.sigma_d;
        }
        // factor after the exit test: the wave's last pass skips it
#if QPB_WARM
        const long tf0 = QPB_CLK();
#endif
        factor(w);
#if QPB_WARM
        { const long d_ = QPB_CLK() - tf0; t_fac += d_; t_kkt += d_; }
#endif
        QPB_TM(2);
        if (!pc) sigma = a.sigma_d;
        double dx[XS], dy[YS1], dz[ZS], dsl[ZS], cc[ZS], bz[ZS];
        auto step_length = [&]() {
            // alpha = min over d < 0 of v/(-d) == 1 / max(-d/v); 1 if none (Auxilary.c:359-393)
            double bm[2] = {0.0, 0.0};
#pragma unroll
            for (int u = 0; u < ZS; u++) {
                if (isz[u]) {
                    bm[0] = __builtin_fmax(bm[0], -dsl[u] * rsi[u]);
                    bm[1] = __builtin_fmax(bm[1], -dz[u] * rzi[u]);
                }
            }
            qpb_rmax<2>(bm);
            ap = bm[0] > 1e-10 ? __builtin_amdgcn_rcp(bm[0]) : 1.0;
            ad = bm[1] > 1e-10 ? __builtin_amdgcn_rcp(bm[1]) : 1.0;
        };
#if QPB_X_DBG == 1
        // (diagnostic: the setup factor's pivots D into x, then stop)
        if (!QPB_WARM && it < 0) {
#pragma unroll
            for (int s = 0; s < XS; s++)
                if (valid && isx[s]) QPB_STS(&a.x[tile * (NX * QPB_TSTR) + (16 * s + c) * QPB_TSTR + ql], 1.0 / rDd[s]);
            if (valid && c == 0) QPB_STS(&a.flag[q], 99);
            return;
        }
#endif
        if (!QPB_WARM && it < 0) {
            // setup solve, rhs [-c; b; h] (Auxilary.c:1010-1040): x0, y0; then
            // s0, z0 from r = h - G x0 = -dz (w = 1 exactly here)
            double mcx[XS];
#pragma unroll
            for (int s = 0; s < XS; s++) mcx[s] = -cx[s];
            solve(w, mcx, by, hz, dx, dy, dz);
#if QPB_X_DBG == 2
            // (diagnostic: the setup solve's x0 into x, then stop)
#pragma unroll
            for (int s = 0; s < XS; s++)
                if (valid && isx[s]) QPB_STS(&a.x[tile * (NX * QPB_TSTR) + (16 * s + c) * QPB_TSTR + ql], dx[s]);
            if (valid && c == 0) QPB_STS(&a.flag[q], 98);
            return;
#endif
#pragma unroll
            for (int s = 0; s < XS; s++) x[s] = isx[s] ? dx[s] : 0.0;
#pragma unroll
            for (int v = 0; v < YS1; v++) y[v] = isy[v] ? dy[v] : 0.0;
            double lh[2] = {-1e300, -1e300};
#pragma unroll
            for (int u = 0; u < ZS; u++) {
                if (isz[u]) {
                    lh[0] = __builtin_fmax(lh[0], dz[u]);     // -zi
                    lh[1] = __builtin_fmax(lh[1], -dz[u]);    // zi
                }
            }
            qpb_rmax<2>(lh);
            const double sh = lh[0], hi = lh[1];          // sh = -min(zi)
#pragma unroll
            for (int u = 0; u < ZS; u++) {
                const double zi = -dz[u];
                sl[u] = isz[u] ? (sh < 0 ? zi : zi + (1 + sh)) : 1.0;
                z[u] = isz[u] ? (hi < 0 ? -zi : -zi + (1 + hi)) : 1.0;
            }
            it = 0;
            QPB_TM(0);
            continue;
        }
#pragma unroll
        for (int u = 0; u < ZS; u++) cc[u] = sigma * mu;
        if (qpb_any(act && pc)) {
            // predictor (kktsolve_1, Auxilary.c:471-515), ds = -s.*z
#if QPB_WARM
            const long ts0 = QPB_CLK();
#endif
#pragma unroll
            for (int u = 0; u < ZS; u++) bz[u] = rz[u] + sl[u];
            solve(w, rx, ry, bz, dx, dy, dz);
#if QPB_WARM
            t_kkt += QPB_CLK() - ts0;
#endif
#pragma unroll
            for (int u = 0; u < ZS; u++) dsl[u] = -sl[u] * __builtin_fma(dz[u], rzi[u], 1.0);
            step_length();
            double rr[1] = {0.0};
#pragma unroll
            for (int u = 0; u < ZS; u++)
                if (isz[u]) rr[0] = __builtin_fma(sl[u] + ap * dsl[u], z[u] + ad * dz[u], rr[0]);
            qpb_rsum<1>(rr);
            const double rho = rr[0] * rsz;             // formrho
            const double r1 = 1 > rho ? rho : 1;
            const double cube = r1 * r1 * r1;
            if (pc) {
                sigma = a.sigma_d < cube ? cube : a.sigma_d;
#pragma unroll
                for (int u = 0; u < ZS; u++) cc[u] = __builtin_fma(-dsl[u], dz[u], sigma * mu);
            }
        }
        QPB_TM(3);
        // corrector / centering (kktsolve_2, Auxilary.c:524-564)
#if QPB_WARM
        const long tc0 = QPB_CLK();
#endif
#pragma unroll
        for (int u = 0; u < ZS; u++) bz[u] = __builtin_fma(-cc[u], rzi[u], rz[u] + sl[u]);
        solve(w, rx, ry, bz, dx, dy, dz);
#if QPB_WARM
        t_kkt += QPB_CLK() - tc0;
#endif
#pragma unroll
        for (int u = 0; u < ZS; u++) dsl[u] = __builtin_fma(__builtin_fma(-sl[u], dz[u], cc[u]), rzi[u], -sl[u]);
        step_length();
        ap = 0.99 * ap > 1.0 ? 1.0 : 0.99 * ap;
        ad = 0.99 * ad > 1.0 ? 1.0 : 0.99 * ad;
#if QPB_WARM
        if (trc && act && it < QPB_TRACE_MAX) {
            trc[4 + 7 * it + 5] = ap;
            trc[4 + 7 * it + 6] = ad;
            n_it = it + 1;
        }
#endif
        if (act) {
#pragma unroll
            for (int s = 0; s < XS; s++) if (isx[s]) x[s] = __builtin_fma(dx[s], ap, x[s]);
#pragma unroll
            for (int v = 0; v < YS; v++) if (isy[v]) y[v] = __builtin_fma(dy[v], ad, y[v]);
#pragma unroll
            for (int u = 0; u < ZS; u++)
                if (isz[u]) { sl[u] = __builtin_fma(dsl[u], ap, sl[u]); z[u] = __builtin_fma(dz[u], ad, z[u]); }
        }
        it++;
        QPB_TM(4);
#if QPB_X_DBG >= 3
        // (diagnostic: the iterate x after QPB_X_DBG - 2 passes, then stop)
        if (it == QPB_X_DBG - 2) {
#pragma unroll
            for (int s = 0; s < XS; s++)
                if (valid && isx[s]) QPB_STS(&a.x[tile * (NX * QPB_TSTR) + (16 * s + c) * QPB_TSTR + ql], x[s]);
            if (valid && c == 0) QPB_STS(&a.flag[q], 97);
            return;
        }
#endif
    }
    // fused argmin first: the arrival's store -> s_waitcnt vmcnt(0) -> atomic round
    // trip then waits for the wave's partial only, not for its output stores
    if (a.best) {
        double bv = __builtin_huge_val();
        long bi = -1;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const double v = qpb_rl64(fv, 16 * r);
            const int f = __builtin_amdgcn_readlane(valid && flag == 0 ? 0 : 1, 16 * r);
            if (f == 0 && qpb_better(v, q0 + r, bv, bi)) { bv = v; bi = q0 + r; }
        }
        qpb_argmin_arrive(a, bv, bi);
    }
    // ---- outputs (tiled SoA)
    if (valid) {
#pragma unroll
        for (int s = 0; s < XS; s++)
            if (isx[s]) QPB_STS(&a.x[tile * (NX * QPB_TSTR) + (16 * s + c) * QPB_TSTR + ql], x[s]);
#pragma unroll
        for (int v = 0; v < YS; v++)
            if (isy[v]) QPB_STS(&a.y[tile * (NY1 * QPB_TSTR) + (16 * v + c) * QPB_TSTR + ql], y[v]);
#pragma unroll
        for (int u = 0; u < ZS; u++)
            if (isz[u]) {
                QPB_STS(&a.z[tile * (NZ * QPB_TSTR) + (16 * u + c) * QPB_TSTR + ql], z[u]);
                QPB_STS(&a.s[tile * (NZ * QPB_TSTR) + (16 * u + c) * QPB_TSTR + ql], sl[u]);
            }
        if (c == 0) {
            QPB_STS(&a.flag[q], flag);
            QPB_STS(&a.iters[q], (int)itq);
            QPB_STS(&a.fval[q], fv);
#if QPB_WARM
            QPB_STS(&a.sig[q], sigf);
            if (trc) { trc[0] = (double)t_fac; trc[1] = (double)t_kkt; trc[2] = (double)n_top; trc[3] = (double)n_it; }
#else
            if (a.sig) QPB_STS(&a.sig[q], sigma);
#endif
#if QPB_X_TIMING
            QPB_TM(4);
            if (a.stats) {
                double *o = a.stats + tile * 384 + ql;
                for (int k = 0; k < 6; k++) o[64 * k] = tph[k];
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
}

#if QPB_SERVE
// persistent form (the drop-in's QP_SOLVE, qpb::serve_ex): one wave, QP 0, one
// solve per request posted in the mailbox (qpb_serve_wait, runtime prelude)
extern "C" __global__ void __launch_bounds__(64, 1)
QPB_KERNEL_NAME(qpb_args a, qpb_mailbox *mb, unsigned long long last, unsigned long long idle,
                unsigned long long life) {
    __shared__ __attribute__((aligned(16))) double qpb_lds[4 * LDS_QP];
    const unsigned long long t_launch = __builtin_amdgcn_s_memrealtime();
    unsigned long long t_seen = 0;
    while (qpb_serve_wait(mb, &last, idle, life, t_launch, &t_seen)) {
        qpb_rowx_body(a, 0, qpb_lds);
        qpb_serve_done(mb, last, t_seen);
        if (life == 0) break;
    }
}
#else
extern "C" __global__ void __launch_bounds__(64, 1) QPB_KERNEL_NAME(qpb_args a) {
    __shared__ __attribute__((aligned(16))) double qpb_lds[4 * LDS_QP];
    qpb_rowx_body(a, qpb_xcd_block(), qpb_lds);
}
#endif
#undef QPB_TM
#undef QPB_TM0
#undef QPB_TM2
#undef QPB_SIGF
#undef QPB_CLK

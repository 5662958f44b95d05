// qpb_tree.hip -- tree kernel: ONE QP per workgroup, any sparsity pattern.
//
// Template source: the host (qpb_tree.cpp generate_tree_kernel) prepends the
// sizes, the KKT assembly tables and five gather programs (fac, fwd, bwd, mv,
// obj), each a list of steps; see qpb_tree.cpp for their meaning.  Everything a
// QP needs lives in the workgroup's LDS for the whole solve: the P/A/G values,
// the factor (stored as LD = L*D, plus 1/D), and every IPM vector.  Global
// memory is touched to stage the inputs, to read the (plan-wide, cache-resident)
// program tables, and to write the outputs.
//
// A program step: lane l < ntask*G works on task l/G and sums that task's terms
// l%G, l%G+G, ...; a DPP butterfly over the G lanes completes the sum; the
// task's last lane applies the epilogue.  A workgroup barrier closes each level.
//
// Reference: qpSWIFT's Mehrotra predictor-corrector (qpSWIFT.c:473-644,
// kkt_initialize Auxilary.c:992-1089), LDL' with dynamic regularisation
// (ldl.c:253-326), triangular solves (ldl.c:495-557), residuals
// (Auxilary.c:745-786), step length (Auxilary.c:359-393), formrho
// (Auxilary.c:879-892).  Fast mode: FMA contraction, reciprocal pivots.
#pragma clang fp contract(fast)

struct qpb_args {
    const double *P, *A, *G, *c, *h, *b;
    double *x, *y, *z, *s;
    int *flag, *iters;
    double *fval;
    double *stats;
    long B;
    double tol, abstol, sigma_d;
    long maxit;
    const void *tab;        // plan tables (qpb_tree.cpp Blob): u64 descriptors, then int32 tables
    double *best;           // (row kernel's fused argmin; unused here)
    unsigned long long *part;
    unsigned *ctr;
    double *sig;            // per-QP sigma: in (warm) / out (NULL: not tracked)
    long warm;              // 1: continue from x, y, z, s, iters, flag, sig (no kkt_initialize)
    double *trace;            // warm variant: per-QP timers + per-iteration statistics (or NULL)
};

#ifndef QPB_WARM
#define QPB_WARM 0              // 1: the warm-solve variant (qpb_solve_warm), compiled on demand
#endif
#define QPB_TRACE_MAX 256                       // = qpb::QPB_TRACE_MAX (qpb_codegen.hpp)
#define QPB_TRACE_STRIDE (4 + 7 * QPB_TRACE_MAX)

#define NX QPB_NX
#define NY QPB_NY
#define NZ QPB_NZ
#define NN QPB_N
#define LNZ QPB_LNZ
#define NY1 (NY > 0 ? NY : 1)
#define NPAG (QPB_NNZP + QPB_NNZA + QPB_NNZG)
#define NW (QPB_WG / 64)

// LDS layout of a QP (doubles): only what other threads of the workgroup read.
// P / A / G stay in global memory (the tiled inputs, read where a program or the
// KKT assembly needs them: the 8 QPs sharing a cache line run on one XCD, so the
// re-reads hit its L2); c | b | h, pinv and the z-row work vectors (ds, lambda,
// dz, ds~) live in the registers of the thread that owns the KKT row (row r:
// thread r % WG); the step tables are read from the plan tables (scalar loads).
// MPC (N = 380, Lnz 3 000): 66.5 -> 39 KB, four QPs per CU instead of two.
#define O_LD 0                         // factor L*D in L's CSC order, [LNZ] = 0
#define O_RD (O_LD + LNZ + 1)          // 1/D (holds the assembled diagonal before the factor)
#define O_V (O_RD + NN)                // x | y | z
#define O_S (O_V + NN)                 // s
#define O_R (O_S + NZ)                 // residual products / rx | ry | rz
#define O_W (O_R + NN)                 // permuted solve vector
#define O_RED (O_W + NN)               // reduction scratch [NW][8]
#define LDS_QP (O_RED + 64)
#define RU ((NN + QPB_WG - 1) / QPB_WG)   // KKT rows per thread (row t + u WG)
#ifndef QPB_T_MSLDS
#define QPB_T_MSLDS 1   // 1: the programs' step tables staged in LDS (~1 KB): a step's metadata is one
                        // LDS read ahead of its descriptor loads instead of a second global round trip
#endif
// step tables of the five programs in LDS (ints)
#define QPB_MS_FAC 0
#define QPB_MS_FWD (QPB_MS_FAC + 4 * QPB_fac_NSTEPS)
#define QPB_MS_BWD (QPB_MS_FWD + 4 * QPB_fwd_NSTEPS)
#define QPB_MS_MV (QPB_MS_BWD + 4 * QPB_bwd_NSTEPS)
#define QPB_MS_OBJ (QPB_MS_MV + 4 * QPB_mv_NSTEPS)
#define QPB_MS_TOTAL (QPB_MS_OBJ + 4 * QPB_obj_NSTEPS + 4)

// compile-time loop (the owner-row registers are only ever indexed by constants:
// a runtime index would put them in scratch memory)
template <int V> struct qpb_tic { static constexpr int value = V; };
template <int J0, int J1, class F> static __device__ __forceinline__ void qpb_tfor(F &&f) {
    if constexpr (J0 < J1) {
        f(qpb_tic<J0>{});
        qpb_tfor<J0 + 1, J1>(f);
    }
}

static __device__ __forceinline__ double qpb_rcp(double v) {
    double r = __builtin_amdgcn_rcp(v);
    double e = __builtin_fma(-v, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-v, r, 1.0);
    return __builtin_fma(r, e, r);
}

// 1 / regularise(d) (ldl.c:273-274, 319-320): |d| <= 1e-14 -> d = +-1e-7 (sign: d > 0)
static __device__ __forceinline__ double qpb_rcp_reg(double d) {
    const double r = qpb_rcp(d);
    const double reg = d > 0.0 ? 1e7 : -1e7;
    return __builtin_fabs(d) <= 1e-14 ? reg : r;
}

// descriptor fields: LDS byte offsets from a region base (qpb_tree.cpp pk)
static __device__ __forceinline__ unsigned qpb_lo16(unsigned w) { return w & 0xffffu; }
static __device__ __forceinline__ unsigned qpb_hi16(unsigned w) { return w >> 16; }
#define QPB_AT(region, byteoff) (*(const double *)((const char *)(L + (region)) + (byteoff)))

// DPP move with a row mask (rows outside it read 0)
template <int CTRL, int RM = 0xf> static __device__ __forceinline__ double qpb_dpp(double v) {
    return __builtin_amdgcn_update_dpp(0.0, v, CTRL, RM, 0xf, false);
}
// sum over aligned groups of 2^g lanes (g uniform, 0..6), all DPP: butterflies
// inside a row (quad_perm, row_half_mirror, row_mirror) leave the group sum in
// every lane of a <= 16-lane group; row_bcast15 / row_bcast31 then fold rows
// upwards, so the LAST lane of every group holds its sum
static __device__ __forceinline__ double qpb_gsum(double v, int g) {
    if (g >= 1) v += qpb_dpp<0xB1>(v);          // quad_perm [1,0,3,2]
    if (g >= 2) v += qpb_dpp<0x4E>(v);          // quad_perm [2,3,0,1]
    if (g >= 3) v += qpb_dpp<0x141>(v);         // row_half_mirror
    if (g >= 4) v += qpb_dpp<0x140>(v);         // row_mirror
    if (g >= 5) v += qpb_dpp<0x142, 0xA>(v);    // row_bcast15 into rows 1, 3
    if (g >= 6) v += qpb_dpp<0x143, 0xC>(v);    // row_bcast31 into rows 2, 3
    return v;
}
// as qpb_gsum, called by the active lanes only: every group is fully active,
// and no butterfly stage reads across a group boundary
static __device__ __forceinline__ double qpb_gsum_act(double v, int g) { return qpb_gsum(v, g); }
static __device__ __forceinline__ double qpb_wmin(double v) {
    v = __builtin_fmin(v, qpb_dpp<0xB1>(v));
    v = __builtin_fmin(v, qpb_dpp<0x4E>(v));
    v = __builtin_fmin(v, qpb_dpp<0x141>(v));
    v = __builtin_fmin(v, qpb_dpp<0x140>(v));
    const double u = __builtin_amdgcn_update_dpp(v, v, 0x142, 0xA, 0xf, false);
    v = __builtin_fmin(v, u);
    const double w = __builtin_amdgcn_update_dpp(v, v, 0x143, 0xC, 0xf, false);
    return __builtin_fmin(v, w);                // lane 63 holds the wave minimum
}

#ifndef QPB_T_TIMING
#define QPB_T_TIMING 0  // 1: per-phase cycle counts (s_memtime) into stats instead of the residual norms
#endif
#if QPB_T_TIMING == 2
// in-step segments (wave 0, lane 0 accumulates): [0] waiting for the step's
// descriptors, [1] terms + group sum, [2] epilogue, [3] barrier; [4] step count
__shared__ double qpb_seg[8];
#define QPB_SEG(k, ...) do { asm volatile("" ::__VA_ARGS__); const long qpb_now = (long)__builtin_readcyclecounter(); \
    if (threadIdx.x == 0) qpb_seg[k] += (double)(qpb_now - qpb_seg_t); qpb_seg_t = qpb_now; } while (0)
#else
#define QPB_SEG(k, ...) do { } while (0)
#endif
#if QPB_T_TIMING
#define QPB_TIC() const long qpb_t0 = (long)__builtin_readcyclecounter()
#define QPB_TOC(v) (v) += (double)((long)__builtin_readcyclecounter() - qpb_t0)
#else
#define QPB_TIC()
#define QPB_TOC(v)
#endif

#ifndef QPB_T_EXP
#define QPB_T_EXP 0     // timing experiments only (wrong results): 2 no barriers, 3 no terms,
                        // 4 no group sums, 5 no epilogue
#endif
#ifndef QPB_T_DEPTH
#define QPB_T_DEPTH 2   // register sets of prefetched steps (2 or 4): a step's tables are loaded DEPTH steps ahead
#endif
#ifndef QPB_T_XR
#define QPB_T_XR 8      // extra rounds a step loads at its start (beyond the prefetched ones;
                        // 24 -> 8: -16 KB of code, same speed)
#endif
#ifndef QPB_T_PF
#define QPB_T_PF 8      // descriptor rounds prefetched per step
#endif

// Workgroup barrier that waits for LDS traffic only: descriptor prefetches
// (global loads of plan constants) stay in flight across it.  The "memory"
// clobber keeps the compiler from moving LDS accesses across.
static __device__ __forceinline__ void qpb_bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Run one gather program.  ms: the program's step table, staged in LDS (4 ints
// per step: descriptor offset, output-code offset, ntask << 4 | log2 G, rounds
// | barrier << 16).  term(acc, desc) -> acc; pre(code) -> the epilogue's own
// operands (loaded before the terms are summed); post(code, acc, pre) writes the
// result.  D: descriptor word (u64 for the factor, u32 otherwise).
//
// Descriptors, output codes and step metadata are prefetched QPB_T_DEPTH steps
// ahead into as many register sets (the loop is unrolled by the depth, so no set
// is ever copied).  Every prefetch issues the same loads (rounds past
// a step's count re-read round 0, lanes past its active count read padding), so
// the compiler waits with vmcnt(N) for the set a step consumes instead of
// vmcnt(0); the step metadata is uniform (readfirstlane) so each load is an
// SGPR base + the lane's offset.  Round counts are padded to 1, 2, 4 or 8 with
// dummy terms (they read the zero entries), so a step sums its terms without
// branches and their LDS reads issue back to back.
struct qpb_pre { double a, b; };
template <class D> struct qpb_set { D d[QPB_T_PF]; int h, doff, toff, ntg, rb; };
template <class D, class Term, class Pre, class Post, class Panel>
static __device__ __forceinline__ void qpb_run(const int *ms, int nsteps, const int *__restrict__ hdr,
                                               const D *__restrict__ desc, Term term, Pre pre, Post post,
                                               Panel panel) {
    if (nsteps <= 0) return;
    // the lane index, opaque here: the per-lane table addresses below are formed per
    // run instead of being hoisted out of the IPM loop and held (spilled) across it
    int l = threadIdx.x;
    asm volatile("" : "+v"(l));
    qpb_set<D> A, B;
    auto prefetch = [&](int st, qpb_set<D> &S) {
        st = st < nsteps ? st : nsteps - 1;
        const int4 m = *(const int4 *)(ms + 4 * st);
        S.doff = __builtin_amdgcn_readfirstlane(m.x);
        const int toff = __builtin_amdgcn_readfirstlane(m.y);
        S.toff = toff;
        S.ntg = __builtin_amdgcn_readfirstlane(m.z);
        S.rb = __builtin_amdgcn_readfirstlane(m.w);
        const int g = S.ntg & 15, act = (S.ntg >> 4) << g, R = S.rb & 0xffff;
        const D *base = desc + (act ? S.doff : 0);       // panel steps have no gather lanes
#pragma unroll
        for (int r = 0; r < QPB_T_PF; r++) S.d[r] = base[(r < R ? r : 0) * act + l];
        S.h = hdr[act ? toff + (l >> g) : 0];
    };
#if QPB_T_TIMING == 2
    long qpb_seg_t = (long)__builtin_readcyclecounter();
#endif
    auto step = [&](const qpb_set<D> &S) {
        const int g = S.ntg & 15, act = (S.ntg >> 4) << g, R = S.rb & 0xffff;
        QPB_SEG(0, "v"(S.d[0]), "v"(S.h));
        if (l < act) {
#if QPB_T_EXP == 5
            const qpb_pre e{0.0, 1.0};
#else
            const qpb_pre e = pre(S.h);
#endif
            double acc;
#if QPB_T_EXP == 3
            if (true) {
                acc = 0.0;
            } else
#endif
            if (R == 1) {
                acc = term(0.0, S.d[0]);
            } else if (R == 2) {
                acc = term(term(0.0, S.d[0]), S.d[1]);
            } else if (R == 4) {
                acc = term(term(0.0, S.d[0]), S.d[1]) + term(term(0.0, S.d[2]), S.d[3]);
            } else if (R == QPB_T_PF) {
                double u = 0.0, v = 0.0;
#pragma unroll
                for (int r = 0; r < QPB_T_PF; r += 2) { u = term(u, S.d[r]); v = term(v, S.d[r + 1]); }
                acc = u + v;
            } else {
                // more rounds than prefetched: load up to QPB_T_XR more at once (one
                // memory latency, overlapped with the prefetched rounds' terms), a
                // rolled loop beyond that
                D dx[QPB_T_XR];
#pragma unroll
                for (int r = 0; r < QPB_T_XR; r++)
                    if (QPB_T_PF + r < R) dx[r] = desc[S.doff + (QPB_T_PF + r) * act + l];
                double u = 0.0, v = 0.0;
#pragma unroll
                for (int r = 0; r < QPB_T_PF; r += 2) { u = term(u, S.d[r]); v = term(v, S.d[r + 1]); }
#pragma unroll
                for (int r = 0; r < QPB_T_XR; r += 2) {
                    if (QPB_T_PF + r < R) u = term(u, dx[r]);
                    if (QPB_T_PF + r + 1 < R) v = term(v, dx[r + 1]);
                }
                for (int r = QPB_T_PF + QPB_T_XR; r < R; r++) u = term(u, desc[S.doff + r * act + l]);   // rare
                acc = u + v;
            }
#if QPB_T_EXP != 4
            acc = qpb_gsum(acc, g);
#endif
            QPB_SEG(1, "v"(acc));
#if QPB_T_EXP != 5
            if ((l & ((1 << g) - 1)) == (1 << g) - 1) post(S.h, acc, e);
#else
            asm volatile("" ::"v"(acc), "v"(e.a));
#endif
        }
        // a use of every prefetched value on every path: otherwise the compiler
        // sinks each load into the one branch that reads it, right before its use,
        // and the prefetch no longer runs ahead
        static_assert(QPB_T_PF == 8 || QPB_T_PF == 4, "qpb_keep lists four or eight descriptor slots");
        if constexpr (QPB_T_PF == 8)
            asm volatile("" ::"v"(S.h), "v"(S.d[0]), "v"(S.d[1]), "v"(S.d[2]), "v"(S.d[3]), "v"(S.d[4]), "v"(S.d[5]),
                         "v"(S.d[6]), "v"(S.d[7]));
        else
            asm volatile("" ::"v"(S.h), "v"(S.d[0]), "v"(S.d[1]), "v"(S.d[2]), "v"(S.d[3]));
        QPB_SEG(2, "s"(0));
        if (S.rb & (1 << 17)) {
            panel(S.doff, S.toff);                      // supernode panels of this level (list, count)
            QPB_SEG(5, "s"(0));
#if QPB_T_TIMING == 2
            if (threadIdx.x == 0) qpb_seg[6] += 1.0;
#endif
        }
#if QPB_T_EXP != 2
        if (S.rb & (1 << 16)) qpb_bar();
#endif
        QPB_SEG(3, "s"(0));
#if QPB_T_TIMING == 2
        if (threadIdx.x == 0) qpb_seg[4] += 1.0;
#endif
    };
#if QPB_T_DEPTH == 4
    qpb_set<D> C, E;
    prefetch(0, A);
    prefetch(1, B);
    prefetch(2, C);
    prefetch(3, E);
    for (int st = 0; st < nsteps; st += 4) {
        step(A);
        prefetch(st + 4, A);
        if (st + 1 < nsteps) step(B);
        prefetch(st + 5, B);
        if (st + 2 < nsteps) step(C);
        prefetch(st + 6, C);
        if (st + 3 < nsteps) step(E);
        prefetch(st + 7, E);
    }
#else
    prefetch(0, A);
    prefetch(1, B);
    for (int st = 0; st < nsteps; st += 2) {
        step(A);
        prefetch(st + 2, A);
        if (st + 1 < nsteps) step(B);
        prefetch(st + 3, B);
    }
#endif
}

// K-value sums over the workgroup (result in every thread)
template <int K>
static __device__ __forceinline__ void qpb_bsum(double (&v)[K], double *red) {
#pragma unroll
    for (int k = 0; k < K; k++) v[k] = qpb_gsum(v[k], 6);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 63)
#pragma unroll
        for (int k = 0; k < K; k++) red[w * 8 + k] = v[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; k++) {
        v[k] = red[k];
        for (int ww = 1; ww < NW; ww++) v[k] += red[ww * 8 + k];
    }
    __syncthreads();
}
template <int K>
static __device__ __forceinline__ void qpb_bmin(double (&v)[K], double *red) {
#pragma unroll
    for (int k = 0; k < K; k++) v[k] = qpb_wmin(v[k]);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 63)
#pragma unroll
        for (int k = 0; k < K; k++) red[w * 8 + k] = v[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; k++) {
        v[k] = red[k];
        for (int ww = 1; ww < NW; ww++) v[k] = __builtin_fmin(v[k], red[ww * 8 + k]);
    }
    __syncthreads();
}


// ---- supernode panels (qpb_tree.cpp Snode): one wavefront per supernode, one
// panel row per lane, the panel's columns in registers (W is a compile-time
// width; the plan's widths are listed in QPB_PANEL_WIDTHS).  Record layout in the
// int tables: j0, W, R (rows), then Lp of the W columns; column c's entries are
// the panel rows after c, so row r of column c sits at LD[Lp(j0+c) + r - c - 1].

// value of lane `lane` (a compile-time constant after unrolling), in every lane
static __device__ __forceinline__ double qpb_rl(double v, int lane) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, lane);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), lane);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// value of lane J of this lane's 16-lane row (DPP row_newbcast): a panel's solve
// runs on its first W <= 16 lanes, all in row 0, so this is lane J's value there
// -- one VALU operation instead of two v_readlane and a move
template <int J> static __device__ __forceinline__ double qpb_nb(double v) {
    return __builtin_amdgcn_update_dpp(0.0, v, 0x150 + J, 0xf, 0xf, true);
}

// right-looking LDL' of the panel (the supernode's external updates are already
// applied; its diagonal arrives raw in rD): pivot k -> 1/D_k with the reference's
// regularisation (ldl.c:273-274, 319-320), then A(r,c) -= A(r,k) A(c,k) / D_k for
// k < c <= r.  LD keeps the unscaled column (A(r,k) at pivot k), as the gather
// programs do.  Lanes above a column's diagonal compute values never stored.
//
// Panels with W <= 16 and R <= W + 4 (16 - W) rows (every MPC panel: 12 x 24) are
// factored with the top W rows copied into every 16-lane DPP row (QPB_T_PDUP):
// lane L holds panel row L & 15 if that is < W (the same row, the same operations,
// the same bits in all four DPP rows), else row W + (L >> 4)(16 - W) + (L & 15) - W.
// A(c, k) for c < W is then lane c of the lane's own DPP row: one row_newbcast
// instead of two v_readlane through SGPRs per update, and the pivot chain has no
// VALU -> SGPR -> VALU round trip.  Only DPP row 0 stores the top rows.
// Off in the 192-thread form (168 registers for three waves per SIMD): there it
// spills more (148 vs 108 B of scratch per lane) for the same time, and the spill
// traffic of 1 024 MPC QPs grows from 93 to 166 MB written per launch.
// a pivot reciprocal: regularised (REG), or v_rcp_f64 + Newton with min |d| tracked
// for the caller's one check per factor (QPB_T_LAZYREG)
template <bool REG> static __device__ __forceinline__ double qpb_piv_rcp(double d, double &dmin) {
    if constexpr (REG) return qpb_rcp_reg(d);
    dmin = __builtin_fmin(dmin, __builtin_fabs(d));
    return qpb_rcp(d);
}
#ifndef QPB_T_LAZYREG
#define QPB_T_LAZYREG 0   // 1: measured slower on 1 024 MPC QPs (1.48 vs 1.46 ms: 3 spilled registers)
#endif

#ifndef QPB_T_PDUP
#define QPB_T_PDUP (QPB_WG != 192)
#endif
template <int W, bool REG>
static __device__ __forceinline__ void qpb_pfac(double *__restrict__ L, const int *__restrict__ rec, int lane,
                                                double &dmin) {
    const int j0 = rec[0], R = rec[2];
    const int *lp = rec + 3;
    if constexpr (QPB_T_PDUP && W <= 16) {
        if (R <= W + 4 * (16 - W)) {                   // uniform
            const int c16 = lane & 15, dr = lane >> 4;
            const int pr = c16 < W ? c16 : W + dr * (16 - W) + (c16 - W);
            const bool on = pr < R, st = on && (pr >= W || dr == 0);
            double P[W];
#pragma unroll
            for (int c = 0; c < W; c++)
                P[c] = L[pr == c ? O_RD + j0 + c : O_LD + ((on && pr > c) ? lp[c] + pr - c - 1 : LNZ)];
            double myr = 0.0;
            qpb_tfor<0, W>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                const double rk = qpb_piv_rcp<REG>(qpb_nb<k>(P[k]), dmin);
                myr = pr == k ? rk : myr;
                const double f = -P[k] * rk;
                qpb_tfor<k + 1, W>([&](auto cc) {
                    constexpr int c = decltype(cc)::value;
                    P[c] = __builtin_fma(f, qpb_nb<c>(P[k]), P[c]);
                });
            });
#pragma unroll
            for (int c = 0; c < W; c++)
                if (st && pr > c) L[O_LD + lp[c] + pr - c - 1] = P[c];
            if (lane < W) L[O_RD + j0 + lane] = myr;
            return;
        }
    }
    const bool on = lane < R;
    double P[W];
#pragma unroll
    for (int c = 0; c < W; c++)
        P[c] = L[lane == c ? O_RD + j0 + c : O_LD + ((on && lane > c) ? lp[c] + lane - c - 1 : LNZ)];
    double myr = 0.0;
#pragma unroll
    for (int k = 0; k < W; k++) {
        const double rk = qpb_piv_rcp<REG>(qpb_rl(P[k], k), dmin);
        myr = lane == k ? rk : myr;
        const double f = -P[k] * rk;
#pragma unroll
        for (int c = k + 1; c < W; c++) P[c] = __builtin_fma(f, qpb_rl(P[k], c), P[c]);
    }
#pragma unroll
    for (int c = 0; c < W; c++)
        if (on && lane > c) L[O_LD + lp[c] + lane - c - 1] = P[c];
    if (lane < W) L[O_RD + j0 + lane] = myr;
}

// forward solve inside the supernode: W holds b minus the external terms (raw);
// w_k = t_k / D_k, then t_c -= LD(c,k) w_k for c > k
template <int W>
static __device__ __forceinline__ void qpb_pfwd(double *__restrict__ L, const int *__restrict__ rec, int lane) {
    const int j0 = rec[0];
    const int *lp = rec + 3;
    const bool on = lane < W;
    double Lr[W];
#pragma unroll
    for (int k = 0; k < W; k++) Lr[k] = -L[O_LD + ((on && lane > k) ? lp[k] + lane - k - 1 : LNZ)];
    double t = L[O_W + j0 + (on ? lane : 0)];
    const double rd = L[O_RD + j0 + (on ? lane : 0)];
    if constexpr (W <= 16) {
        // (t_k rd_k formed on every lane, lane k's taken: the same product)
        qpb_tfor<0, W>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            const double u = t * rd;
            t = __builtin_fma(Lr[k], qpb_nb<k>(u), t);
        });
    } else {
#pragma unroll
        for (int k = 0; k < W; k++) t = __builtin_fma(Lr[k], qpb_rl(t, k) * qpb_rl(rd, k), t);
    }
    if (on) L[O_W + j0 + lane] = rd * t;
}

// backward solve inside the supernode: W holds w minus D^-1 times the terms of
// the rows below; x_k final in descending k, then v_c -= LD(k,c) x_k / D_c for c < k
template <int W>
static __device__ __forceinline__ void qpb_pbwd(double *__restrict__ L, const int *__restrict__ rec, int lane) {
    const int j0 = rec[0];
    const int *lp = rec + 3;
    const bool on = lane < W;
    const int lpl = lp[on ? lane : 0];
    const double rd = L[O_RD + j0 + (on ? lane : 0)];
    double Lc[W];
#pragma unroll
    for (int i = 0; i < W; i++) Lc[i] = -rd * L[O_LD + ((on && i > lane) ? lpl + i - lane - 1 : LNZ)];
    double v = L[O_W + j0 + (on ? lane : 0)];
    if constexpr (W <= 16) {
        qpb_tfor<0, W>([&](auto kc) {
            constexpr int k = W - 1 - decltype(kc)::value;
            v = __builtin_fma(Lc[k], qpb_nb<k>(v), v);
        });
    } else {
#pragma unroll
        for (int k = W - 1; k >= 0; k--) v = __builtin_fma(Lc[k], qpb_rl(v, k), v);
    }
    if (on) L[O_W + j0 + lane] = v;
}

#ifndef QPB_PANEL_WIDTHS
#define QPB_PANEL_WIDTHS(X)
#endif

// XCD-aware block order: blocks b and b + 8 share an XCD (and its L2), so
// logical block (b % 8) * (nb / 8) + b / 8 gives each XCD a contiguous run of
// QPs -- the 64 QPs of a tile, whose values share cache lines, stay on one L2.
// The host pads the grid to a multiple of 8 (surplus blocks find no QPs).
static __device__ __forceinline__ long qpb_xcd_block() {
    const unsigned b = blockIdx.x, nb = gridDim.x;
    return (nb & 7) ? (long)b : (long)(b & 7) * (nb >> 3) + (b >> 3);
}

#ifndef QPB_T_WPE
#define QPB_T_WPE 2     // waves per SIMD the register allocation must allow (launch bound): two
                        // 256-thread or four 128-thread workgroups per CU need <= 256 registers
                        // (VGPRs + AGPRs); above that one wave per SIMD halves the QPs per CU
#endif
extern "C" __global__ void __launch_bounds__(QPB_WG, QPB_T_WPE) QPB_KERNEL_NAME(qpb_args a) {
    __shared__ __attribute__((aligned(16))) double L[LDS_QP];
    __shared__ int SN[QPB_PANEL_INTS > 0 ? QPB_PANEL_INTS : 1];       // supernode records + panel lists
#if QPB_T_MSLDS
    __shared__ __attribute__((aligned(16))) int MS[QPB_MS_TOTAL];
#endif
    int t = threadIdx.x;                         // opaque at every stage (the loop below)
    const long q = qpb_xcd_block();
    if (q >= a.B) return;                        // workgroup-uniform
    const long tile = q >> 6;
    const int ql = (int)(q & 63);
    double tm_fac = 0.0, tm_sol = 0.0, tm_mv = 0.0, tm_all = 0.0;
    (void)tm_fac; (void)tm_sol; (void)tm_mv; (void)tm_all;
    const unsigned long long *__restrict__ TD = (const unsigned long long *)a.tab;
    const unsigned *__restrict__ TD32 = (const unsigned *)(TD + QPB_NDESC);
    const int *__restrict__ TI = (const int *)(TD32 + QPB_NDESC32);
#define qpb_asrc_i (TI + QPB_I_asrc_i)
#define qpb_asrc_l (TI + QPB_I_asrc_l)
    double *__restrict__ LD = L + O_LD;
    double *__restrict__ rD = L + O_RD;
    double *__restrict__ V = L + O_V;
    double *__restrict__ S = L + O_S;
    double *__restrict__ R = L + O_R;
    double *__restrict__ W = L + O_W;
    double *__restrict__ RED = L + O_RED;
    // this QP's P / A / G values in the tiled inputs: entry e of the P | A | G
    // concatenation (e = NPAG: the zero the dummy terms read)
    // (branch-free: one global load per term, the zero entry masked; the address is
    // integer arithmetic -- a choice between pointers becomes a scratch table)
    typedef const double __attribute__((address_space(1))) qpb_gdouble;
    typedef unsigned long long qpb_u64;
    const qpb_u64 bP = (qpb_u64)(a.P + tile * (QPB_NNZP * 64) + ql);
    const qpb_u64 bA = QPB_NNZA > 0 ? (qpb_u64)(a.A + tile * (QPB_NNZA * 64) + ql) : bP;
    const qpb_u64 bG = (qpb_u64)(a.G + tile * (QPB_NNZG * 64) + ql);
    const qpb_u64 dA = bA - bP - (qpb_u64)QPB_NNZP * 512, dG = bG - bA - (qpb_u64)QPB_NNZA * 512;
    auto pag = [&](int e) -> double {
        const bool inA = e >= QPB_NNZP, inG = e >= QPB_NNZP + QPB_NNZA, in = e < NPAG;
        const qpb_u64 ad = bP + (qpb_u64)(in ? e : NPAG - 1) * 512 + (inA ? dA : 0ull) + (inG ? dG : 0ull);
        const double v = *(qpb_gdouble *)ad;
        return in ? v : 0.0;
    };

    // the rows this thread owns: r = t + u WG
    double chb[RU], ds[RU], lam[RU], dzr[RU], dsl[RU], xp[RU];
    int pv[RU];
    qpb_tfor<0, RU>([&](auto uc_) {
        constexpr int u = decltype(uc_)::value;
        const int r = t + u * QPB_WG;
        double v = 0.0;
        if (r < NX) v = a.c[tile * (NX * 64) + r * 64 + ql];
#if NY > 0
        else if (r < NX + NY) v = a.b[tile * (NY * 64) + (r - NX) * 64 + ql];
#endif
        else if (r < NN) v = a.h[tile * (NZ * 64) + (r - NX - NY) * 64 + ql];
        chb[u] = v;
        pv[u] = r < NN ? TI[QPB_I_pinv + r] : 0;
        ds[u] = lam[u] = dzr[u] = dsl[u] = xp[u] = 0.0;
    });
    if (t == 0) LD[LNZ] = 0.0;
#if QPB_T_TIMING == 2
    if (t < 8) qpb_seg[t] = 0.0;
#endif
    for (int j = t; j < QPB_PANEL_INTS; j += QPB_WG) SN[j] = TI[j];
#if QPB_T_MSLDS
    for (int j = t; j < 4 * QPB_fac_NSTEPS; j += QPB_WG) MS[QPB_MS_FAC + j] = TI[QPB_I_fac_steps + j];
    for (int j = t; j < 4 * QPB_fwd_NSTEPS; j += QPB_WG) MS[QPB_MS_FWD + j] = TI[QPB_I_fwd_steps + j];
    for (int j = t; j < 4 * QPB_bwd_NSTEPS; j += QPB_WG) MS[QPB_MS_BWD + j] = TI[QPB_I_bwd_steps + j];
    for (int j = t; j < 4 * QPB_mv_NSTEPS; j += QPB_WG) MS[QPB_MS_MV + j] = TI[QPB_I_mv_steps + j];
    for (int j = t; j < 4 * QPB_obj_NSTEPS; j += QPB_WG) MS[QPB_MS_OBJ + j] = TI[QPB_I_obj_steps + j];
#define QPB_STEPS(name, NAME) (MS + QPB_MS_##NAME)
#else
#define QPB_STEPS(name, NAME) (TI + QPB_I_##name##_steps)
#endif
    __syncthreads();

    // KKT values into the factor layout (init: z diagonal -1; loop: -s/z)
    auto assemble = [&](const int *__restrict__ src) {
        for (int e = t; e < LNZ + NN; e += QPB_WG) {
            const int sc = src[e];
            double v;
            if (sc >= 0) v = pag(sc);
            else if (sc == -1) v = 0.0;
            else if (sc == -2) v = -1.0;
            else { const int r = -3 - sc; v = -S[r] * qpb_rcp(V[NX + NY + r]); }
            L[O_LD + e + (e >= LNZ ? 1 : 0)] = v;      // e >= LNZ: diagonal -> rD[e - LNZ]
        }
        __syncthreads();
    };
    // QPB_T_LAZYREG: the panel pivots skip the regularisation select and track min |D|;
    // the caller re-assembles and refactors with it only when some panel pivot is
    // <= 1e-14 (ldl.c:273-274) -- otherwise the same operations, so the same bits
    auto factor = [&](auto regc) -> double {
        constexpr bool REG = decltype(regc)::value != 0 || !QPB_T_LAZYREG;
        double dmin = __builtin_huge_val();
        QPB_TIC();
        qpb_run(QPB_STEPS(fac, FAC), QPB_fac_NSTEPS, TI + QPB_I_fac_hdr, TD + QPB_D_fac,
                [&](double acc, unsigned long long d) {
                    const unsigned lo = (unsigned)d, hi = (unsigned)(d >> 32);
                    return __builtin_fma(-QPB_AT(O_LD, qpb_lo16(lo)) * QPB_AT(O_RD, qpb_lo16(hi)),
                                         QPB_AT(O_LD, qpb_hi16(lo)), acc);
                },
                // one LDS index, not a choice of pointers (which the compiler turns into a
                // scratch table of generic pointers and a flat load)
                [&](int out) { return qpb_pre{L[out >= 0 ? O_LD + out : O_RD + (out >= -NN ? -1 - out : -1 - NN - out)], 0.0}; },
                [&](int out, double acc, qpb_pre e) {
                    if (out >= 0) LD[out] = e.a + acc;
                    else if (out >= -NN) rD[-1 - out] = qpb_rcp_reg(e.a + acc);
                    else rD[-1 - NN - out] = e.a + acc;          // supernode diagonal: raw, the panel pivots
                },
                [&](int list, int count) {
                    for (int i = threadIdx.x >> 6; i < count; i += NW) {
                        const int *rec = SN + SN[list + i];
                        switch (rec[1]) {
#define QPB_PF(w) case w: qpb_pfac<w, REG>(L, rec, threadIdx.x & 63, dmin); break;
                            QPB_PANEL_WIDTHS(QPB_PF)
#undef QPB_PF
                        }
                    }
                });
        QPB_TOC(tm_fac);
        return dmin;
    };
    // W (permuted rhs) -> W (permuted solution)
    auto solve = [&]() {
        QPB_TIC();
        qpb_run(QPB_STEPS(fwd, FWD), QPB_fwd_NSTEPS, TI + QPB_I_fwd_hdr, TD32 + QPB_D_fwd,
                [&](double acc, unsigned d) {
                    return __builtin_fma(-QPB_AT(O_LD, qpb_lo16(d)), QPB_AT(O_W, qpb_hi16(d)), acc);
                },
                [&](int i) { const int j = i >= 0 ? i : -1 - i; return qpb_pre{W[j], rD[j]}; },
                [&](int i, double acc, qpb_pre e) {
                    if (i >= 0) W[i] = e.b * (e.a + acc);
                    else W[-1 - i] = e.a + acc;                  // supernode row: raw, the panel solves
                },
                [&](int list, int count) {
                    for (int i = threadIdx.x >> 6; i < count; i += NW) {
                        const int *rec = SN + SN[list + i];
                        switch (rec[1]) {
#define QPB_PF(w) case w: qpb_pfwd<w>(L, rec, threadIdx.x & 63); break;
                            QPB_PANEL_WIDTHS(QPB_PF)
#undef QPB_PF
                        }
                    }
                });
        qpb_run(QPB_STEPS(bwd, BWD), QPB_bwd_NSTEPS, TI + QPB_I_bwd_hdr, TD32 + QPB_D_bwd,
                [&](double acc, unsigned d) {
                    return __builtin_fma(-QPB_AT(O_LD, qpb_lo16(d)), QPB_AT(O_W, qpb_hi16(d)), acc);
                },
                [&](int k) { return qpb_pre{W[k], rD[k]}; },
                [&](int k, double acc, qpb_pre e) { W[k] = __builtin_fma(e.b, acc, e.a); },
                [&](int list, int count) {
                    for (int i = threadIdx.x >> 6; i < count; i += NW) {
                        const int *rec = SN + SN[list + i];
                        switch (rec[1]) {
#define QPB_PF(w) case w: qpb_pbwd<w>(L, rec, threadIdx.x & 63); break;
                            QPB_PANEL_WIDTHS(QPB_PF)
#undef QPB_PF
                        }
                    }
                });
        QPB_TOC(tm_sol);
    };
    // R = [P A' G'; A 0 0; G 0 0] V (raw products)
    auto products = [&](const double *__restrict__ vec) {
        QPB_TIC();
        qpb_run(QPB_STEPS(mv, MV), QPB_mv_NSTEPS, TI + QPB_I_mv_hdr, TD32 + QPB_D_mv,
                [&](double acc, unsigned d) {
                    return __builtin_fma(pag((int)(qpb_lo16(d) >> 3)),
                                         *(const double *)((const char *)vec + qpb_hi16(d)), acc);
                },
                [&](int) { return qpb_pre{0.0, 0.0}; },
                [&](int r, double acc, qpb_pre) { R[r] = acc; }, [](int, int) {});
        QPB_TOC(tm_mv);
    };
    // the owner loop: f(u, r) for every KKT row r = t + u WG < NN
#define QPB_ROWS(...) qpb_tfor<0, RU>([&](auto uc_) { constexpr int u = decltype(uc_)::value; \
        const int r = t + u * QPB_WG; if (r < NN) { __VA_ARGS__ } });

    // ---- kkt_initialize (Auxilary.c:992-1089) and the QP_SOLVE loop (qpSWIFT.c:502-602)
    // as one state machine, so that assemble / factor / solve / products each have a
    // single call site: inlined at every use they made a 378 KB kernel, several times
    // the instruction cache
#if QPB_T_TIMING
    const long qpb_tall = (long)__builtin_readcyclecounter();
#endif
    double sigma = 100.0, alpha_p = 0.0, alpha_d = 0.0;
    double n_rx = 0.0, n_ry = 0.0, n_rz = 0.0, n_mu = 0.0, mu = 0.0;
    long it = 0;
    bool conv = false;
    const double invm = 1.0 / (double)NZ;
    // rhs b = [rx; ry; rz - ds/z] (updatekktmatrix_b, Auxilary.c:274-295)
    auto rhs = [&]() {
        QPB_ROWS(
            double v = R[r];
            if (r >= NX + NY) v -= ds[u] * qpb_rcp(V[r]);
            W[pv[u]] = v;
        )
    };
    // kktsolve_2 extraction: dz, ds~ and the step-length minima of this thread's rows
    auto extract = [&](double (&ab)[2]) {
        QPB_ROWS(if (r >= NX + NY) {
            const double si = S[r - NX - NY], zi = V[r], dz = W[pv[u]];
            const double d = (ds[u] - si * dz) * qpb_rcp(zi);
            dzr[u] = dz;
            dsl[u] = d;
            if (d < 0) ab[0] = __builtin_fmin(ab[0], -(si / d));
            if (dz < 0) ab[1] = __builtin_fmin(ab[1], -(zi / dz));
        })
    };
    // stages: INIT the setup solve (rhs [-c; b; h], z block -I), INITZ the initial
    // s / z, TOP an iteration's residuals and exit test, PRED the predictor
    // (kktsolve_1), CORR the corrector on the same factor, CENT pure centering
    // (sigma <= sigma_d: refactor, qpSWIFT.c:572-579)
    enum { ST_INIT, ST_INITZ, ST_TOP, ST_PRED, ST_CORR, ST_CENT };
    int stage = ST_INIT;
#if QPB_WARM
    // warm variant (qpb_solve_warm): QP_SOLVE continues from the object's iterate,
    // IterationCount and options->sigma (qpSWIFT.c:502-596 never re-initialises)
    for (int j = t; j < NX; j += QPB_WG) V[j] = a.x[tile * (NX * 64) + j * 64 + ql];
#if NY > 0
    for (int j = t; j < NY; j += QPB_WG) V[NX + j] = a.y[tile * (NY * 64) + j * 64 + ql];
#endif
    for (int j = t; j < NZ; j += QPB_WG) {
        V[NX + NY + j] = a.z[tile * (NZ * 64) + j * 64 + ql];
        S[j] = a.s[tile * (NZ * 64) + j * 64 + ql];
    }
    const long it0 = a.iters[q];    // IterationCount the QP enters with
    const int flag0 = a.flag[q];    // stats->Flag it enters with (QP_FATAL after setup)
    sigma = a.sig[q];
    __syncthreads();
    QPB_ROWS(if (r < NX) xp[u] = V[r];)
    stage = ST_TOP;
    // the drop-in's timers and verbose trace (KernelArgs::trace, qpb_codegen.hpp):
    // s_memrealtime ticks in the factorisations and in factor + solves, and the
    // statistics the reference prints per iteration (qpSWIFT.c:506-517, 598-600)
    double *const trc = (a.trace && t == 0) ? a.trace + q * QPB_TRACE_STRIDE : nullptr;
    long t_fac = 0, t_kkt = 0, n_top = 0, n_it = 0;
#define QPB_CLK() ((long)__builtin_amdgcn_s_memrealtime())
#else
    constexpr long it0 = 0;
    constexpr int flag0 = 3;
#endif
    int flag = flag0;
    for (;;) {
        // masks and addresses derived from the lane index are formed where used, not
        // hoisted out of the loop (held across it they spill)
        asm volatile("" : "+v"(t));
        if (stage == ST_INITZ || stage == ST_TOP) {
            if (stage == ST_TOP && it >= a.maxit) break;
            products(V);
            if (stage == ST_INITZ) {
                double lo = 1e300, hi = -1e300;
                QPB_ROWS(if (r >= NX + NY) {
                    const double zi = chb[u] - R[r];
                    lo = __builtin_fmin(lo, zi);
                    hi = __builtin_fmax(hi, zi);
                })
                double mm[2] = {lo, -hi};
                qpb_bmin(mm, RED);
                lo = mm[0];
                hi = -mm[1];
                const double shift = -lo;
                QPB_ROWS(if (r >= NX + NY) {
                    const double zi = chb[u] - R[r];
                    S[r - NX - NY] = shift < 0 ? zi : zi + (1.0 + shift);
                    V[r] = hi < 0 ? -zi : -zi + (1.0 + hi);
                })
                __syncthreads();
                stage = ST_TOP;
                continue;
            }
            {
                double acc[4] = {0.0, 0.0, 0.0, 0.0};
                QPB_ROWS(
                    double v;
                    if (r < NX) { v = -R[r] - chb[u]; xp[u] = V[r]; acc[0] = __builtin_fma(v, v, acc[0]); }
                    else if (r < NX + NY) { v = chb[u] - R[r]; acc[1] = __builtin_fma(v, v, acc[1]); }
                    else {
                        const double si = S[r - NX - NY];
                        v = chb[u] - R[r] - si;
                        acc[2] = __builtin_fma(v, v, acc[2]);
                        acc[3] = __builtin_fma(si, V[r], acc[3]);
                    }
                    R[r] = v;
                )
                qpb_bsum(acc, RED);
                n_rx = __builtin_sqrt(acc[0]);
                n_ry = __builtin_sqrt(acc[1]);
                n_rz = __builtin_sqrt(acc[2]);
                n_mu = acc[3] * invm;
            }
#if QPB_WARM
            {
                // (the objective needs its own gather program over R, which holds the
                // residuals here: the tree kernel traces fval only at the end -- NaN)
                if (trc && it < QPB_TRACE_MAX) {
                    double *e = trc + 4 + 7 * it;
                    e[0] = __builtin_nan("");
                    e[1] = n_rx; e[2] = n_ry; e[3] = n_rz; e[4] = n_mu;
                    n_top = it + 1;
                }
            }
#endif
            if (n_rx < a.tol && n_rz < a.tol && (NY == 0 || n_ry < a.tol) && n_mu < a.abstol) {
                flag = 0;
                conv = true;
                break;
            }
            {
                double acc[1] = {0.0};
                QPB_ROWS(if (r >= NX + NY) {
                    const double lm = __builtin_sqrt(S[r - NX - NY] * V[r]);
                    lam[u] = lm;
                    acc[0] = __builtin_fma(lm, lm, acc[0]);
                })
                qpb_bsum(acc, RED);
                mu = acc[0] * invm;
            }
            if (sigma > a.sigma_d) {
                // predictor: ds = -lambda^2 (form_ds, Auxilary.c:319-326)
                qpb_tfor<0, RU>([&](auto uc_) { constexpr int u = decltype(uc_)::value; ds[u] = -lam[u] * lam[u]; });
                stage = ST_PRED;
            } else {
                sigma = a.sigma_d;
                const double smu = sigma * mu;
                qpb_tfor<0, RU>([&](auto uc_) { constexpr int u = decltype(uc_)::value; ds[u] = -(lam[u] * lam[u]) + smu; });
                stage = ST_CENT;
            }
        }
        // this stage's system: K assembled and factored, except for the corrector
        // (same factor as the predictor), then the solve
        const bool fac = stage != ST_CORR;
        if (fac) assemble(stage == ST_INIT ? qpb_asrc_i : qpb_asrc_l);
        if (stage == ST_INIT) {
            QPB_ROWS(W[pv[u]] = r < NX ? -chb[u] : chb[u];)
        } else {
            rhs();
        }
#if QPB_WARM
        const long tk0 = QPB_CLK();
#endif
        if (fac) {                        // its level barriers order the rhs before the solve
            const double dm = factor(qpb_tic<0>{});
            if (QPB_T_LAZYREG && __syncthreads_or(dm <= 1e-14)) {     // a tiny panel pivot: rare
                assemble(stage == ST_INIT ? qpb_asrc_i : qpb_asrc_l);
                factor(qpb_tic<1>{});
            }
        } else {
            __syncthreads();
        }
#if QPB_WARM
        const long tk1 = QPB_CLK();
        if (fac) t_fac += tk1 - tk0;
#endif
        solve();
#if QPB_WARM
        t_kkt += QPB_CLK() - tk0;
#endif
        if (stage == ST_INIT) {
            QPB_ROWS(V[r] = r < NX + NY ? W[pv[u]] : 0.0;)
            __syncthreads();
            stage = ST_INITZ;
            continue;
        }
        double ab[2] = {1e300, 1e300};
        extract(ab);
        qpb_bmin(ab, RED);                // (its barriers also end every read of W above)
        if (stage == ST_PRED) {
            const double ap = ab[0] < 1e10 ? ab[0] : 1.0, ad = ab[1] < 1e10 ? ab[1] : 1.0;
            double rr[2] = {0.0, 0.0};
            QPB_ROWS(if (r >= NX + NY) {
                const double si = S[r - NX - NY], zi = V[r];
                rr[0] = __builtin_fma(__builtin_fma(ap, dsl[u], si), __builtin_fma(ad, dzr[u], zi), rr[0]);
                rr[1] = __builtin_fma(si, zi, rr[1]);
            })
            qpb_bsum(rr, RED);
            const double rho = rr[0] / rr[1];
            const double r1 = rho < 1.0 ? rho : 1.0, cube = r1 * r1 * r1;
            sigma = a.sigma_d < cube ? cube : a.sigma_d;
            const double smu = sigma * mu;
            qpb_tfor<0, RU>([&](auto uc_) {
                constexpr int u = decltype(uc_)::value;
                ds[u] = -(lam[u] * lam[u]) - dsl[u] * dzr[u] + smu;
            });
            stage = ST_CORR;
            continue;
        }
        // corrector / centering: step length and updates (qpSWIFT.c:583-600)
        alpha_p = ab[0] < 1e10 ? ab[0] : 1.0;
        alpha_d = ab[1] < 1e10 ? ab[1] : 1.0;
        alpha_p = 0.99 * alpha_p > 1.0 ? 1.0 : 0.99 * alpha_p;
        alpha_d = 0.99 * alpha_d > 1.0 ? 1.0 : 0.99 * alpha_d;
#if QPB_WARM
        if (trc && it < QPB_TRACE_MAX) {
            trc[4 + 7 * it + 5] = alpha_p;
            trc[4 + 7 * it + 6] = alpha_d;
            n_it = it + 1;
        }
#endif
        QPB_ROWS(
            if (r < NX) V[r] = __builtin_fma(W[pv[u]], alpha_p, V[r]);
            else if (r < NX + NY) V[r] = __builtin_fma(W[pv[u]], alpha_d, V[r]);
            else {
                S[r - NX - NY] = __builtin_fma(dsl[u], alpha_p, S[r - NX - NY]);
                V[r] = __builtin_fma(dzr[u], alpha_d, V[r]);
            }
        )
        __syncthreads();
        it++;
        stage = ST_TOP;
    }
    if (it0 + it == a.maxit) flag = 2;     // qpSWIFT.c:598-601: IterationCount == maxit

    // ---- objective of the x the last residuals were computed at (qpSWIFT.c:515):
    // V itself after convergence, else the iteration's starting x (owner registers)
    if (!conv) {
        QPB_ROWS(if (r < NX) R[r] = xp[u];)     // R is free here: the objective's x
    } else {
        QPB_ROWS(if (r < NX) R[r] = V[r];)
    }
    __syncthreads();
    qpb_run(QPB_STEPS(obj, OBJ), QPB_obj_NSTEPS, TI + QPB_I_obj_hdr, TD32 + QPB_D_obj,
            [&](double acc, unsigned d) {
                return __builtin_fma(pag((int)(qpb_lo16(d) >> 3)), *(const double *)((const char *)R + qpb_hi16(d)),
                                     acc);
            },
            [&](int) { return qpb_pre{0.0, 0.0}; },
            [&](int r, double acc, qpb_pre) { W[r] = acc; }, [](int, int) {});
    double fv[1] = {0.0};
    QPB_ROWS(if (r < NX) fv[0] += R[r] * (0.5 * W[r] + chb[u]);)
    qpb_bsum(fv, RED);
#undef QPB_ROWS

    // ---- outputs
    for (int j = t; j < NX; j += QPB_WG) a.x[tile * (NX * 64) + j * 64 + ql] = V[j];
#if NY > 0
    for (int j = t; j < NY; j += QPB_WG) a.y[tile * (NY * 64) + j * 64 + ql] = V[NX + j];
#endif
    for (int j = t; j < NZ; j += QPB_WG) {
        a.z[tile * (NZ * 64) + j * 64 + ql] = V[NX + NY + j];
        a.s[tile * (NZ * 64) + j * 64 + ql] = S[j];
    }
    if (t == 0) {
        a.flag[q] = flag;
        a.iters[q] = (int)(it0 + it);
        a.fval[q] = fv[0];
#if QPB_WARM
        a.sig[q] = sigma;
        if (trc) { trc[0] = (double)t_fac; trc[1] = (double)t_kkt; trc[2] = (double)n_top; trc[3] = (double)n_it; }
#else
        if (a.sig) a.sig[q] = sigma;            // options->sigma after a cold QP_SOLVE (drop-in)
#endif
        if (a.stats) {
            double *st = a.stats + tile * (6 * 64) + ql;
#if QPB_T_TIMING == 2
            st[0] = qpb_seg[0]; st[64] = qpb_seg[1]; st[128] = qpb_seg[2]; st[192] = qpb_seg[3]; st[256] = qpb_seg[4];
            st[320] = qpb_seg[5] + 1e9 * qpb_seg[6];     // panel cycles + 1e9 x panel steps
#elif QPB_T_TIMING
            tm_all = (double)((long)__builtin_readcyclecounter() - qpb_tall);
            st[0] = tm_fac; st[64] = tm_sol; st[128] = tm_mv; st[192] = tm_all; st[256] = (double)QPB_fac_NSTEPS;
            st[320] = (double)(QPB_fwd_NSTEPS + QPB_bwd_NSTEPS);
#else
            st[0] = n_rx; st[64] = n_ry; st[128] = n_rz; st[192] = n_mu; st[256] = alpha_p; st[320] = alpha_d;
#endif
        }
    }
}

// qpb_wave.hip -- wave-cooperative IPM kernel: ONE wavefront per QP.
//
// Template source: compiled at run time with hiprtc after the host prepends the
// plan's sizes (QPB_NX = n, QPB_NZ = m, QPB_NY = p), its sparsity tables and the
// kernel name (qpb_wave.cpp).  Algorithm = qpSWIFT's Mehrotra predictor-corrector
// (qpSWIFT.c:473-644, kkt_initialize Auxilary.c:992-1089) with the KKT LDL'
// (ldl.c:253-326, same regularisation) of the PLAN'S permutation, reorganised:
// z and y rows whose neighbours (x rows) all come later in the permutation are
// leaves -- their row of L is empty and their pivot is the diagonal (-s/z, and
// 0 -> -1e-7 for y, the reference's regularisation) -- so they are eliminated
// first, all at once, adding
//     P + G_L' diag(z/s) G_L + 1e7 A_L'A_L          (L = leaf rows)
// onto the x block.  Every other row (x, non-leaf y and z) forms a dense block
// factored right-looking in permutation order, so the pivots, and which of
// them are regularised, are the reference's when it is given the same
// permutation.  Lanes own rows: lane d holds dense row d of H (then of L);
// lane i holds x_i, lane l holds y_l, lane r (+64, ...) holds s_r, z_r.
// Cross-lane traffic: whole vectors are all-gathered through LDS (one store,
// wide same-address loads); the sequential dense factor / triangular solves
// broadcast with DPP row_newbcast (x block within one 16-lane row) or
// v_readlane beyond 16 rows; reductions are DPP row reductions.  Results agree
// with the reference to rounding (fast mode: FMA contraction, reciprocal pivots).
#pragma clang fp contract(fast)
#ifndef QPB_LDS
// Persistent form (QPB_SERVE): the zero-copy slab is re-read and re-written by every
// request, and the host rewrites it in between.  Everything the wave reads from it or
// writes to it goes through system-scope loads / stores (sc0 sc1): a store leaves no
// copy of the line in this XCD's L2 and a load reads past L1, so no request sees a
// line cached for an earlier one (round 3: a warm solve started from the previous
// QP's iterate).  Batched builds keep plain loads and stores.
#if defined(QPB_SERVE) && QPB_SERVE
#ifndef QPB_TSTR          // (QPB_WAVE_OPTS="QPB_TSTR=64": the tiled slab, for A/B -- the host follows)
#define QPB_TSTR 1        // the persistent (drop-in, B = 1) variants: QP 0's values packed in the slab
#endif
#define QPB_LDS(p) __hip_atomic_load((p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
#define QPB_STS(p, v) __hip_atomic_store((p), (v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
#else
#define QPB_LDS(p) (*(p))
#define QPB_STS(p, v) (*(p) = (v))
#endif
#endif
#ifndef QPB_TSTR
#define QPB_TSTR 64       // tiled SoA: value j of QP q at [(q / 64) * n * 64 + j * 64 + q % 64]
#endif

template <int V> struct qpb_ic { static constexpr int value = V; };

struct qpb_args {
    const double *P, *A, *G, *c, *h, *b;
    double *x, *y, *z, *s;
    int *flag, *iters;
    double *fval;
    double *stats;
    long B;
    double tol, abstol, sigma_d;
    long maxit;
    const void *tab;              // (tree kernel tables; unused here)
    double *best;                 // (row kernel's fused argmin; unused here)
    unsigned long long *part;
    unsigned *ctr;
    double *sig;                  // per-QP sigma: in (warm) / out (NULL: not tracked)
    long warm;                    // 1: continue from x, y, z, s, iters, flag, sig (no kkt_initialize)
    double *trace;            // warm variant: per-QP timers + per-iteration statistics (or NULL)
    const double *win;        // persistent warm variants: x y z s {flag, iters} sigma to continue from (or NULL)
};

#ifndef QPB_WARM
#define QPB_WARM 0                // 1: the warm-solve variant (qpb_solve_warm), compiled on demand
#endif
#define QPB_TRACE_MAX 256                       // = qpb::QPB_TRACE_MAX (qpb_codegen.hpp)
#define QPB_TRACE_STRIDE (4 + 7 * QPB_TRACE_MAX)

// tuning knobs (defaults = measured best; scripts/sweep.py "wave:KNOB=V,...")
#ifndef QPB_W_GG           // 1: G(r,i)G(r,j) products in registers; 0: recompute from LDS
#define QPB_W_GG (QPB_NNZG <= 48)
#endif
#ifndef QPB_W_EXECDBG      // 1 (diagnostics): persistent form records each request's starting EXEC mask
#define QPB_W_EXECDBG 0
#endif
#ifndef QPB_W_SIGOUT       // 0 (diagnostics): the cold variants do not report sigma (round 3's code)
#define QPB_W_SIGOUT 1
#endif
#ifndef QPB_W_ASMV         // 1 (diagnostics): every inline asm volatile (no CSE / motion of the DPP asm)
#define QPB_W_ASMV 0
#endif
#if QPB_W_ASMV
#define QPB_W_ASM asm volatile
#else
#define QPB_W_ASM asm
#endif
#ifndef QPB_W_LAZYREG      // 1: pivot regularisation checked once per factor (redone only when needed);
#define QPB_W_LAZYREG 0    // off: AMD-ordered plans regularise their y pivots in most factors, so the
#endif                     // factor ran twice (controller call batched 2.73 -> 24.7 ms, C30 tick 335 -> 520 us)
#ifndef QPB_W_MFMA         // 1: the leaf z rows' G'diag(w)G as an MFMA GEMM (v_mfma_f64_16x16x4f64)
#define QPB_W_MFMA (!QPB_W_GG && QPB_NX <= 64)
#endif
#ifndef QPB_W_LDSB         // 1: LDL' update broadcasts through LDS (dense blocks beyond one DPP row)
#define QPB_W_LDSB (QPB_ND > 16)
#endif
#ifndef QPB_W_LTLDS        // 1: the backward solve reads its column of -L from LDS (no register copy)
#define QPB_W_LTLDS (QPB_ND > 16)
#endif
#ifndef QPB_W_REGS         // 1: this lane's slices of P, A, G in registers; 0: read LDS in place
#define QPB_W_REGS (QPB_NX <= 16 && QPB_NZ <= 32)
#endif
#ifndef QPB_W_BLK          // 1: blocked LDL' -- 16-column panels, rank-16 trailing updates on MFMA
#define QPB_W_BLK 0       // 1 measured slower on 30/68/18 AMD (29.1k vs 22.5k cycles per factor), DESIGN.md
#endif
#ifndef QPB_W_DUP          // 1: dense blocks of 17..32 rows factored with every lane holding two rows
#define QPB_W_DUP (QPB_ND > 16 && QPB_ND <= 32)   // (L & 15 and 16 + (L & 15)): all broadcasts DPP
#endif
#ifndef QPB_W_H0RE         // 1: the static part of the dense row recomputed per factor (not held live)
#define QPB_W_H0RE (QPB_ND > 32)
#endif
#ifndef QPB_W_ABL          // cost attribution only (wrong results): skip 1 LDL' 2 G'WG 4 solve chains
#define QPB_W_ABL 0       // 8 residual products 16 transpose (scripts/lat_bench.py, fixed iteration count)
#endif
#ifndef QPB_W_H0BF         // 1: the static dense-row part H0 formed branch-free (QPB_W_H0RE recomputes
#define QPB_W_H0BF 1       // it at every factor: the divergent loads cost the AMD-ordered C30 kernel)
#endif
#ifndef QPB_W_TRUNM        // 1: the -L transpose stores every row unmasked, in descending column order
#define QPB_W_TRUNM 1
#endif
#ifndef QPB_W_LTZS         // 1: the backward solve's -L column above the diagonal read from the zero
#define QPB_W_LTZS 1       // slot T_SINK (an address select) instead of a value select
#endif
#ifndef QPB_W_LSKIP        // 1: the LDL' skips the updates whose H(j, k) is a structural zero (qpb_lnz)
#define QPB_W_LSKIP 1
#endif
#ifndef QPB_W_LDSB_SYNC     // 1: a wave fence between publishing column k+1 and reading it (diagnostic)
#define QPB_W_LDSB_SYNC 0
#endif
#ifndef QPB_W_KDIAG        // 1: a dense z row's kd on its diagonal before the factor (0: added to the
#define QPB_W_KDIAG 1      // pivot at its step, round 5)
#endif
#ifndef QPB_W_RCH          // residual / solve products G x, A x, P x in chunks of this many columns,
#define QPB_W_RCH 4        // each chunk's LDS loads issued together (0: per column -- the allocator
#endif                     // then kept one load in flight: an LDS round trip per column)
#ifndef QPB_W_TIMING
#define QPB_W_TIMING 0    // 1: phase timestamps (s_memtime) of QP 0 of each tile into stats (debug)
#endif
#ifndef QPB_W_SPLIT
#define QPB_W_SPLIT 1     // independent partial sums per long accumulation (ILP)
#endif

#define NX QPB_NX
#define NZ QPB_NZ
#define NY QPB_NY
#define NY1 (NY > 0 ? NY : 1)
#define WPB (QPB_WG / 64)
#define ND QPB_ND
#define NV (NX + NZ + NY)
// vector exchange area: x | z | y  (residual gather); solve: bx | by | bz | v | out
#define VB_SIZE (((2 * NV + NZ + NX) + 1) & ~1)
// per-wave LDS (doubles): Pd[NX*LDP] Ad[NX*LDY] Gd[NX*LDZ] | T | Vb.  T holds the
// strictly lower triangle of -L, packed by rows (row d at d(d-1)/2), for the
// transpose; between a transpose and the next factor it is scratch for the MFMA
// G'WG tiles (NXP^2) and the LDL' broadcast buffers (2 x 64); its last two slots
// are a read target for masked lanes.  (Packing, instead of ND^2, keeps the
// 30/68/18 QP at 39.6 KB: four QPs per CU.)
// leading dimensions of the staged matrices.  QPB_W_PAD=1 makes them odd (a
// lane-strided access then spreads over all LDS banks) but costs the 16-byte
// alignment of the columns the uniform paired loads read: measured slower
// (30/68/18, 1 024 QPs 380 vs 365 us; one AMD-ordered QP 296 vs 289 us), so off
#ifndef QPB_W_PAD
#define QPB_W_PAD 0       // (the host's scatter tables follow QPB_WAVE_OPTS, qpb_wave.cpp wave_pad)
#endif
#define LDP (QPB_W_PAD ? (NX | 1) : NX)
#define LDY (QPB_W_PAD ? (NY1 | 1) : NY1)
#ifdef QPB_LDZ                // chosen by the host (qpb_wave.cpp wave_ldz): NZ, or NZ padded to 2 mod 4
#define LDZ QPB_LDZ
#else
#define LDZ (QPB_W_PAD ? (NZ | 1) : NZ)
#endif
#define OFF_A (NX * LDP)
#define OFF_G (OFF_A + (NY > 0 ? LDY : 0) * NX)
#define OFF_C (OFF_G + LDZ * NX)
#define OFF_T ((OFF_C + 1) & ~1)
#define QPB_TMAX(a, b) ((a) > (b) ? (a) : (b))
// blocked LDL' scratch (QPB_W_BLK): broadcast buffers 2 x 64 | U panel 48 x 16 | C tile
// column 48 x 16 | the panel's reciprocal pivots 16; panel rows padded to 17 doubles
// (a row per lane: stride 16 would put every lane on one bank)
#define BLK_RS 17
#define BLK_SZ (128 + 2 * 48 * BLK_RS + 16)
#define TSZ (((QPB_TMAX(QPB_TMAX(QPB_TMAX(ND * (ND - 1) / 2, QPB_W_MFMA ? 256 * ((NX + 15) / 16) * ((NX + 15) / 16) : 0), \
                                  QPB_W_BLK ? BLK_SZ : (QPB_W_LDSB ? 128 : 0)), QPB_W_DUP ? ND * ND : 0) + 1) & ~1) + 2)
#define T_SINK (TSZ - 2)
#define OFF_V (OFF_T + TSZ)
#define LDS_WAVE (OFF_V + VB_SIZE)
#define ZC ((NZ + 63) / 64)          // z rows per lane (lane r holds r, r + 64, ...)
#define ROWS_D ((ND + 15) / 16)
#define ROWS_X ((NX + 15) / 16)
#define ROWS_Z (ZC > 1 ? 4 : (NZ + 15) / 16)
#define ROWS_Y ((NY1 + 15) / 16)
#define ROWS_R (ROWS_Z > ROWS_X ? (ROWS_Z > ROWS_Y ? ROWS_Z : ROWS_Y) : (ROWS_X > ROWS_Y ? ROWS_X : ROWS_Y))

static __device__ __forceinline__ double qpb_rcp(double v) {
    double r = __builtin_amdgcn_rcp(v);
    double e = __builtin_fma(-v, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-v, r, 1.0);
    return __builtin_fma(r, e, r);
}

// an opaque copy of v: values derived from it (per-step lane masks, LDS addresses)
// are formed where they are used instead of being hoisted out of the IPM loop and
// held live across it (for large dense blocks they would not fit the registers)
#ifndef QPB_W_OPQ
#define QPB_W_OPQ 1       // 0: plain lane ids (the compiler may hoist what derives from them)
#endif
static __device__ __forceinline__ int qpb_opaque(int v) {
    if constexpr (QPB_W_OPQ) asm volatile("" : "+v"(v));
    return v;
}

// value of lane l (l wave-uniform) in every lane, through an SGPR pair
static __device__ __forceinline__ double qpb_bc(double v, int l) {
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = __builtin_amdgcn_readlane((int)b, l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}

// value of lane J of the dense block in every lane that uses it: one DPP
// row_newbcast when the dense block fits one 16-lane row, else v_readlane
template <int J> static __device__ __forceinline__ double qpb_xb(double v) {
    if constexpr (ND <= 16) return __builtin_amdgcn_update_dpp(0.0, v, 0x150 + J, 0xf, 0xf, true);
    else return qpb_bc(v, J);
}

// acc + (v of dense lane J) * m as ONE v_fmac_f64 with a DPP row_newbcast
// source (the compiler does not fold a 64-bit DPP move into a VOP2 FMA).  The
// DPP read hazard (v written by one of the two preceding VALU instructions) is
// invisible to the compiler's hazard recognizer inside inline asm, and a VALU
// copy placed by the register allocator right before the asm cannot be ruled
// out from the source: the runtime audits every compiled code object
// (qpb_runtime.hip, dpp_audit) and rebuilds with QPB_DPP_NOP = 2 (wait states
// inside every DPP asm) should it find a hazard.
#ifndef QPB_DPP_NOP           // -1: no wait states in the asm text, the post-assembly pass places each one
#define QPB_DPP_NOP -1         // (0: a fixed s_nop 1 in the chained asm, on top of the s_nop 0 LLVM puts
#endif                         // between dependent inline asm on gfx950 -- 3 wait states for 2; -2 % per
                               // headline launch, profiles/r04_dpp_nop_ab.log)
#if QPB_DPP_NOP < 0           // every wait state placed by the post-assembly pass (qpb_hazard asm_fixup)
#define QPB_DPP_PRE ""
#define QPB_DPP_DEP ""
#elif QPB_DPP_NOP >= 2
#define QPB_DPP_PRE "s_nop 4\n\t"
#define QPB_DPP_DEP "s_nop 4\n\t"
#elif QPB_DPP_NOP
#define QPB_DPP_PRE "s_nop 1\n\t"
#define QPB_DPP_DEP "s_nop 1\n\t"
#else
#define QPB_DPP_PRE ""
#define QPB_DPP_DEP "s_nop 1\n\t"
#endif
template <int J> static __device__ __forceinline__ double qpb_fmac_xb(double acc, double v, double m) {
    if constexpr (ND <= 16) {
        QPB_W_ASM(QPB_DPP_PRE "v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf bound_ctrl:1"
            : "+v"(acc) : "v"(v), "v"(m), "i"(J));
        return acc;
    } else {
        return __builtin_fma(qpb_bc(v, J), m, acc);
    }
}

// same, for a chain whose previous step wrote v (the triangular solves): the
// two wait states the DPP read needs are inserted explicitly
template <int J> static __device__ __forceinline__ double qpb_fmac_xb_dep(double acc, double v, double m) {
    if constexpr (ND <= 16) {
        QPB_W_ASM(QPB_DPP_DEP "v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf bound_ctrl:1"
            : "+v"(acc) : "v"(v), "v"(m), "i"(J));
        return acc;
    } else {
        return __builtin_fma(qpb_bc(v, J), m, acc);
    }
}

template <int CTRL> static __device__ __forceinline__ double qpb_dpp(double v) {
    return __builtin_amdgcn_update_dpp(0.0, v, CTRL, 0xf, 0xf, true);
}
// the value is needed here: its load is issued and waited for before this point
static __device__ __forceinline__ void qpb_wpin(double &v) { asm volatile("" : "+v"(v)); }

// sums / maxima over the first R 16-lane rows (result wave-uniform); lanes
// outside the data range must contribute 0 (sum) or a neutral value (max)
template <int R> static __device__ __forceinline__ double qpb_rsum(double v) {
    v += qpb_dpp<0xB1>(v);    // quad_perm [1,0,3,2]
    v += qpb_dpp<0x4E>(v);    // quad_perm [2,3,0,1]
    v += qpb_dpp<0x141>(v);   // row_half_mirror
    v += qpb_dpp<0x140>(v);   // row_mirror
    double r = qpb_bc(v, 0);
#pragma unroll
    for (int k = 1; k < R; k++) r += qpb_bc(v, 16 * k);
    return r;
}
// K independent sums at once, stage-major so the K DPP chains overlap
template <int R, int K> static __device__ __forceinline__ void qpb_rsum_n(double (&v)[K]) {
#pragma unroll
    for (int k = 0; k < K; k++) v[k] += qpb_dpp<0xB1>(v[k]);
#pragma unroll
    for (int k = 0; k < K; k++) v[k] += qpb_dpp<0x4E>(v[k]);
#pragma unroll
    for (int k = 0; k < K; k++) v[k] += qpb_dpp<0x141>(v[k]);
#pragma unroll
    for (int k = 0; k < K; k++) v[k] += qpb_dpp<0x140>(v[k]);
#pragma unroll
    for (int k = 0; k < K; k++) {
        double r = qpb_bc(v[k], 0);
#pragma unroll
        for (int j = 1; j < R; j++) r += qpb_bc(v[k], 16 * j);
        v[k] = r;
    }
}
template <int R> static __device__ __forceinline__ double qpb_rmax(double v) {
    v = __builtin_fmax(v, qpb_dpp<0xB1>(v));
    v = __builtin_fmax(v, qpb_dpp<0x4E>(v));
    v = __builtin_fmax(v, qpb_dpp<0x141>(v));
    v = __builtin_fmax(v, qpb_dpp<0x140>(v));
    double r = qpb_bc(v, 0);
#pragma unroll
    for (int k = 1; k < R; k++) r = __builtin_fmax(r, qpb_bc(v, 16 * k));
    return r;
}

template <int R, int K> static __device__ __forceinline__ void qpb_rmax_n(double (&v)[K]) {
#pragma unroll
    for (int k = 0; k < K; k++) v[k] = __builtin_fmax(v[k], qpb_dpp<0xB1>(v[k]));
#pragma unroll
    for (int k = 0; k < K; k++) v[k] = __builtin_fmax(v[k], qpb_dpp<0x4E>(v[k]));
#pragma unroll
    for (int k = 0; k < K; k++) v[k] = __builtin_fmax(v[k], qpb_dpp<0x141>(v[k]));
#pragma unroll
    for (int k = 0; k < K; k++) v[k] = __builtin_fmax(v[k], qpb_dpp<0x140>(v[k]));
#pragma unroll
    for (int k = 0; k < K; k++) {
        double r = qpb_bc(v[k], 0);
#pragma unroll
        for (int j = 1; j < R; j++) r = __builtin_fmax(r, qpb_bc(v[k], 16 * j));
        v[k] = r;
    }
}

// LDS is shared by the lanes of one wave only: in-order per wave, so a compiler
// fence is all that is needed between a store by one lane and a load by another.
static __device__ __forceinline__ void qpb_wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ldl.c:273-274, 319-320
static __device__ __forceinline__ double qpb_regularise(double d) {
    const double sg = d <= 0.0 ? -1.0 : 1.0;
    return sg * d <= 1e-14 ? sg * 1e-7 : d;
}

// 1 / regularise(d): v_rcp_f64 + one Newton step, computed unconditionally (the
// asm keeps the compiler from turning the rare regularised case into a branch);
// |d| <= 1e-14 -> 1/(+-1e-7), sign as ldl.c:273 (d <= 0 -> negative, NaN kept)
static __device__ __forceinline__ double qpb_rcp_reg(double d) {
    double r = __builtin_amdgcn_rcp(d);
    r = __builtin_fma(__builtin_fma(-d, r, 1.0), r, r);
    QPB_W_ASM("" : "+v"(r));     // opaque but not a scheduling barrier
    const double reg = d > 0.0 ? 1e7 : -1e7;
    return __builtin_fabs(d) <= 1e-14 ? reg : r;
}

// a pivot reciprocal: regularised (REG), or v_rcp_f64 + Newton with min |d| tracked
// for the caller's one check per factor (QPB_W_LAZYREG)
template <bool REG> static __device__ __forceinline__ double qpb_piv_rcp(double d, double &dmin) {
    if constexpr (REG) return qpb_rcp_reg(d);
    dmin = __builtin_fmin(dmin, __builtin_fabs(d));
    const double r = __builtin_amdgcn_rcp(d);
    return __builtin_fma(__builtin_fma(-d, r, 1.0), r, r);
}

template <int J0, int J1, class F> static __device__ __forceinline__ void qpb_for(F &&f) {
    if constexpr (J0 < J1) {
        f(qpb_ic<J0>{});
        qpb_for<J0 + 1, J1>(f);
    }
}

#if QPB_W_TIMING == 2      // per QP: start / end (100 MHz realtime, core cycles) + iterations
#define QPB_TS(k) do { } while (0)
#elif QPB_W_TIMING
#define QPB_TS(k)                                                                      \
    do {                                                                               \
        if (ql == 0 && a.stats && (k) < 384) {                                         \
            const double t_ = (double)__builtin_readcyclecounter();                    \
            if (lane == 0) a.stats[tile * 384 + (k)] = t_;                             \
        }                                                                              \
    } while (0)
#else
#define QPB_TS(k) do { } while (0)
#endif

// XCD-aware block order: blocks b and b + 8 share an XCD (and its L2), so
// logical block (b % 8) * (nb / 8) + b / 8 gives each XCD a contiguous run of
// QPs -- the 64 QPs of a tile, whose values share cache lines, stay on one L2.
// The host pads the grid to a multiple of 8 (surplus blocks find no QPs).
static __device__ __forceinline__ long qpb_xcd_block() {
    const unsigned b = blockIdx.x, nb = gridDim.x;
    return (nb & 7) ? (long)b : (long)(b & 7) * (nb >> 3) + (b >> 3);
}

#if QPB_SERVE
// the persistent form (end of file) runs the body once per request, on QP 0
static __device__ __forceinline__ void qpb_wave_body(const qpb_args &a, double *qpb_lds, unsigned qpb_tid) {
    const long qpb_blk = 0;
#else
extern "C" __global__ void __launch_bounds__(QPB_WG, 1) QPB_KERNEL_NAME(qpb_args a) {
    __shared__ __attribute__((aligned(16))) double qpb_lds[WPB * LDS_WAVE];
    const long qpb_blk = qpb_xcd_block();
    const unsigned qpb_tid = threadIdx.x;
#endif
    const int lane = qpb_tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(qpb_tid >> 6);
    const long q = qpb_blk * WPB + wv;
    if (q >= a.B) return;                    // wave-uniform
    double *__restrict__ Ls = qpb_lds + wv * LDS_WAVE;
    const long tile = q >> 6;
    const int ql = (int)(q & 63);
    const bool isx = lane < NX, isy = lane < NY, isd = lane < ND;
    const int ix = isx ? lane : NX - 1;
    const int iy = isy ? lane : (NY > 0 ? NY - 1 : 0);
    const int id = isd ? lane : ND - 1;
    bool isz[ZC], zleaf[ZC];
    int iz[ZC];
#pragma unroll
    for (int t = 0; t < ZC; t++) {
        isz[t] = lane + 64 * t < NZ;
        iz[t] = isz[t] ? lane + 64 * t : NZ - 1;
        zleaf[t] = qpb_zleaf_d[iz[t]] != 0;
    }
    const bool yleaf = NY > 0 ? qpb_yleaf_d[iy] != 0 : true;
    // this lane's dense row: kind (0 x, 1 y, 2 z) and variable index
    const int dk = qpb_dkind_d[id], di = qpb_didx_d[id];
    const int dvar = dk == 0 ? di : (dk == 1 ? NX + di : NX + NY + di);   // x | y | z numbering
    constexpr double RDY = 1.0 / -1e-7;      // leaf y pivots: D = 0 regularised to -1e-7

#if QPB_W_TIMING == 2
    const double t_rt0 = (double)__builtin_amdgcn_s_memrealtime(), t_cy0 = (double)__builtin_readcyclecounter();
#endif
    QPB_TS(0);
    // ---- stage this QP's inputs as dense matrices in LDS (tiled SoA -> dense):
    // every global load is issued before the first LDS store
    constexpr int NPL = (QPB_NNZP + 63) / 64, NGL = (QPB_NNZG + 63) / 64, NAL = (QPB_NNZA + 63) / 64;
    double vP[NPL], vG[NGL], vA[NAL > 0 ? NAL : 1];
    int iP[NPL], iP2[NPL], iG[NGL], iA[NAL > 0 ? NAL : 1];
    {
        const double *tP = a.P + tile * (QPB_NNZP * QPB_TSTR) + ql;
        const double *tG = a.G + tile * (QPB_NNZG * QPB_TSTR) + ql;
#pragma unroll
        for (int u = 0; u < NPL; u++) {
            const int k = lane + 64 * u;
            const bool ok = k < QPB_NNZP;
            vP[u] = ok ? QPB_LDS(&tP[k * QPB_TSTR]) : 0.0;
            iP[u] = ok ? qpb_scP[k] : -1;
            iP2[u] = ok ? qpb_scP2[k] : -1;
        }
#pragma unroll
        for (int u = 0; u < NGL; u++) {
            const int k = lane + 64 * u;
            const bool ok = k < QPB_NNZG;
            vG[u] = ok ? QPB_LDS(&tG[k * QPB_TSTR]) : 0.0;
            iG[u] = ok ? qpb_scG[k] : -1;
        }
#if NY > 0
        const double *tA = a.A + tile * (QPB_NNZA * QPB_TSTR) + ql;
#pragma unroll
        for (int u = 0; u < NAL; u++) {
            const int k = lane + 64 * u;
            const bool ok = k < QPB_NNZA;
            vA[u] = ok ? QPB_LDS(&tA[k * QPB_TSTR]) : 0.0;
            iA[u] = ok ? qpb_scA[k] : -1;
        }
#endif
    }
    const double cx = isx ? QPB_LDS(&a.c[tile * (NX * QPB_TSTR) + lane * QPB_TSTR + ql]) : 0.0;
    double hz[ZC];
#pragma unroll
    for (int t = 0; t < ZC; t++) hz[t] = isz[t] ? QPB_LDS(&a.h[tile * (NZ * QPB_TSTR) + (lane + 64 * t) * QPB_TSTR + ql]) : 0.0;
#if NY > 0
    const double by = isy ? QPB_LDS(&a.b[tile * (NY * QPB_TSTR) + lane * QPB_TSTR + ql]) : 0.0;
#else
    const double by = 0.0;
#endif
    // the whole per-wave area starts zeroed (staging needs it; the transpose /
    // scratch area and the exchange vectors then never hold stale bits)
#pragma unroll
    for (int i = 0; i < (LDS_WAVE + 63) / 64; i++)      // compile-time trip count: unrolled
        if (lane + 64 * i < LDS_WAVE) Ls[lane + 64 * i] = 0.0;
    qpb_wsync();
#pragma unroll
    for (int u = 0; u < NPL; u++) {
        if (iP[u] >= 0) Ls[iP[u]] = vP[u];
        if (iP2[u] >= 0) Ls[iP2[u]] = vP[u];
    }
#pragma unroll
    for (int u = 0; u < NGL; u++)
        if (iG[u] >= 0) Ls[OFF_G + iG[u]] = vG[u];
#pragma unroll
    for (int u = 0; u < NAL; u++)
        if (iA[u] >= 0) Ls[OFF_A + iA[u]] = vA[u];
    qpb_wsync();
    const double *Pd = Ls, *Ad = Ls + OFF_A, *Gd = Ls + OFF_G;
    double *Tx = Ls + OFF_T, *Vb = Ls + OFF_V;
    // Pd[j*LDP+i] = P(i,j) as given; Ad[j*LDY+l] = A(l,j); Gd[j*LDZ+r] = G(r,j)

    // this lane's slices of the (constant) matrices: registers when small (REGS)
    double Prow[QPB_W_REGS ? NX : 1], Grow[QPB_W_REGS ? ZC * NX : 1], Arow[QPB_W_REGS ? NX : 1];
    if constexpr (QPB_W_REGS) {
#pragma unroll
        for (int j = 0; j < NX; j++) {
            Prow[j] = Pd[j * LDP + ix];
            Arow[j] = NY > 0 ? Ad[j * LDY + iy] : 0.0;
#pragma unroll
            for (int t = 0; t < ZC; t++) Grow[t * NX + j] = Gd[j * LDZ + iz[t]];
        }
    }
    auto PR = [&](int j) { if constexpr (QPB_W_REGS) return Prow[j]; else return Pd[j * LDP + ix]; };   // P(i, j)
    auto GR = [&](int t, int j) { if constexpr (QPB_W_REGS) return Grow[t * NX + j]; else return Gd[j * LDZ + iz[t]]; };  // G(r, j)
    auto AR = [&](int j) { if constexpr (QPB_W_REGS) return Arow[j]; else return Ad[j * LDY + iy]; };   // A(l, j)
    // dense-row slices: G(r, i) / A(l, i) of this lane's dense row when it is x_i, else 0
    const int dxi = dk == 0 ? di : 0;
    const double dxm = dk == 0 ? 1.0 : 0.0;
    double Gcol[QPB_W_REGS ? NZ : 1], Acol[QPB_W_REGS ? NY1 : 1];
    if constexpr (QPB_W_REGS) {
#pragma unroll
        for (int r = 0; r < NZ; r++) Gcol[r] = dxm * Gd[dxi * LDZ + r];
#pragma unroll
        for (int l = 0; l < NY1; l++) Acol[l] = NY > 0 ? dxm * Ad[dxi * LDY + l] : 0.0;
    }
    auto GC = [&](int r) { if constexpr (QPB_W_REGS) return Gcol[r]; else return dxm * Gd[dxi * LDZ + r]; };
    auto AC = [&](int l) { if constexpr (QPB_W_REGS) return Acol[l]; else return dxm * Ad[dxi * LDY + l]; };

    // H0: the static part of this lane's dense row (perm order of the columns):
    //   x_i  : P(i,j) (upper, symmetrised) + 1e7 sum_{leaf y} A(l,i)A(l,j) | A(l,i) | G(r,i)
    //   y_l  : A(l,j) on x columns, 0 elsewhere
    //   z_r  : G(r,j) on x columns, 0 elsewhere (the diagonal -s/z joins at pivot time)
    // (large dense blocks: recomputed from the staged matrices at every factor
    // instead of holding ND more doubles live across the iteration -- QPB_W_H0RE)
    auto h0_row = [&](double *H0) {
#if QPB_W_H0BF
    // branch-free: one LDS read at a selected address per entry, the leaf-y terms with
    // the lane's own 1e7 A(l, i) (0 unless dense row i is x_i) -- no divergent loads
    double aL[NY1];
#pragma unroll
    for (int l = 0; l < NY1; l++) aL[l] = (NY > 0 && qpb_yleaf[l < NY ? l : 0]) ? -RDY * dxm * Ad[dxi * LDY + l] : 0.0;
#endif
    qpb_for<0, ND>([&](auto ec) {
        constexpr int e = decltype(ec)::value;
        constexpr int ke = qpb_dkind[e], je = qpb_didx[e];
        double v = 0.0;
#if QPB_W_H0BF
        if constexpr (ke == 0) {
            const int pa = dxi <= je ? je * LDP + dxi : dxi * LDP + je;
            const int ya = OFF_A + je * LDY + (NY > 0 ? di : 0), za = OFF_G + je * LDZ + di;
            double vx = Ls[dk == 0 ? pa : (dk == 1 ? ya : za)];
#pragma unroll
            for (int l = 0; l < NY; l++)
                if (qpb_yleaf[l]) vx = __builtin_fma(aL[l], Ad[je * LDY + l], vx);
            v = vx;
        } else {
            double u = ke == 1 ? Ad[dxi * LDY + je] : Gd[dxi * LDZ + je];
            asm volatile("" : "+v"(u));        // loaded by every lane, then selected
            v = dk == 0 ? u : 0.0;
        }
#else
        if constexpr (ke == 0) {
            const double px = dxi <= je ? Pd[je * LDP + dxi] : Pd[dxi * LDP + je];
            double vx = px;
#pragma unroll
            for (int l = 0; l < NY; l++)
                if (qpb_yleaf[l]) vx = __builtin_fma(Ad[dxi * LDY + l], -RDY * Ad[je * LDY + l], vx);
            v = dk == 0 ? vx : (dk == 1 ? Ad[je * LDY + (NY > 0 ? di : 0)] : Gd[je * LDZ + di]);
        } else if constexpr (ke == 1) {
            v = dk == 0 ? Ad[dxi * LDY + je] : 0.0;
        } else {
            v = dk == 0 ? Gd[dxi * LDZ + je] : 0.0;
        }
#endif
        H0[e] = isd ? v : 0.0;
    });
    };
    double H0[QPB_W_H0RE ? 1 : ND];
    if constexpr (!QPB_W_H0RE) h0_row(H0);
    // G(r,i) G(r,j) for every structural G(r,j) of a leaf z row (x_i rows only)
    double GG[QPB_W_GG ? QPB_NNZG : 1];
    if constexpr (QPB_W_GG) {
        int e = 0;
#pragma unroll
        for (int r = 0; r < NZ; r++)
#pragma unroll
            for (int j = 0; j < NX; j++)
                if (qpb_Gnz[r][j]) GG[e++] = GC(r) * Gd[j * LDZ + r];
    }

    double H[ND], Lt[QPB_W_LTLDS ? 1 : ND], rDd = 0.0, w[ZC];
    // The factor with z diagonal kd (per z row) in three pieces, so that its
    // register-only part can be scheduled together with the residuals: leaf z
    // rows fold into the x block as G'diag(w)G, w = -1/regularise(kd); dense z
    // rows take kd at their pivot.
    constexpr int VBW = NV;          // w | kd exchange, after the residual's x | z | y
    auto factor_publish = [&](const double *kd) {
#pragma unroll
        for (int t = 0; t < ZC; t++) {
            w[t] = -qpb_rcp_reg(kd[t]);
            if (isz[t]) {
                Vb[VBW + lane + 64 * t] = w[t];
                if constexpr (!QPB_XID) Vb[VBW + NZ + lane + 64 * t] = kd[t];   // dense z rows' diagonals
            }
        }
    };
    // after a wsync: H = H0 + G_L' W G_L, then the right-looking LDL' of the
    // dense block in permutation order (registers and DPP only)
    int fstamp = 0;     // timing build: factor-internal stamps base (0 = off)
    // QPB_W_LAZYREG: the pivot reciprocals skip the regularisation select (ldl.c:273-274)
    // and track min |D|; the caller redoes the factor with it only when some pivot is
    // <= 1e-14 -- otherwise the same operations, so the same bits.
    auto factor_ldl = [&](auto regc) -> double {
        constexpr bool REG = decltype(regc)::value != 0 || !QPB_W_LAZYREG;
        double dmin = __builtin_huge_val();
        const int ln = qpb_opaque(lane);
        if constexpr (QPB_W_H0RE) {
            h0_row(H);
        } else {
#pragma unroll
            for (int e = 0; e < ND; e++) H[e] = H0[e];
        }
        if (fstamp) QPB_TS(fstamp + 0);
        if constexpr (QPB_W_GG) {      // small G: every (r, j) unrolled, products precomputed
            int e = 0;
#pragma unroll
            for (int r = 0; r < NZ; r++) {
                const double wr = Vb[VBW + r];
#pragma unroll
                for (int j = 0; j < NX; j++)
                    if (qpb_Gnz[r][j]) {
                        H[qpb_xpos[j]] = __builtin_fma(GG[e], wr, H[qpb_xpos[j]]);
                        e++;
                    }
            }
        } else if constexpr (QPB_W_ABL & 2) {
        } else if constexpr (QPB_W_MFMA) {
            // C = G_L' diag(w) G_L over the x columns as a dense GEMM on the matrix
            // cores: 16 x 16 output tiles (I <= J; C is symmetric), K = 4 z rows per
            // v_mfma_f64_16x16x4f64.  A operand: lane l holds G(r, 16 I + (l & 15)),
            // r = 4 s + (l >> 4); B operand: w_r G(r, 16 J + (l & 15)) (w_r = 0 for a
            // non-leaf row, which joins the dense block instead).  D: lane l, reg t is
            // C(16 I + (l >> 4) + 4 t, 16 J + (l & 15)).  The tiles go through the L
            // transpose area (dead between the last solve and the next transpose),
            // and each x row adds its row of C.
            typedef double qpb_v4d __attribute__((ext_vector_type(4)));
            constexpr int NT = (NX + 15) / 16, NXP = 16 * NT, NP = NT * (NT + 1) / 2;
            qpb_v4d acc[NP];
#pragma unroll
            for (int p = 0; p < NP; p++) acc[p] = qpb_v4d{0.0, 0.0, 0.0, 0.0};
            const int li = lane & 15, lk = lane >> 4;
            // branch-free operand loads (clamped index x 0/1 mask), so every LDS read
            // of the GEMM can be issued ahead of the MFMA chain
            int gi[NT];
            double gm[NT];
#pragma unroll
            for (int I = 0; I < NT; I++) {
                const int i = 16 * I + li;
                gi[I] = (i < NX ? i : NX - 1) * LDZ;
                gm[I] = i < NX ? 1.0 : 0.0;
            }
            qpb_for<0, (NZ + 3) / 4>([&](auto sc) {
                constexpr int s4 = 4 * decltype(sc)::value;
                constexpr bool l0 = s4 < NZ && qpb_zleaf[s4 < NZ ? s4 : 0];
                constexpr bool l1 = s4 + 1 < NZ && qpb_zleaf[s4 + 1 < NZ ? s4 + 1 : 0];
                constexpr bool l2 = s4 + 2 < NZ && qpb_zleaf[s4 + 2 < NZ ? s4 + 2 : 0];
                constexpr bool l3 = s4 + 3 < NZ && qpb_zleaf[s4 + 3 < NZ ? s4 + 3 : 0];
                const double lm = lk == 0 ? (l0 ? 1.0 : 0.0) : lk == 1 ? (l1 ? 1.0 : 0.0)
                                : lk == 2 ? (l2 ? 1.0 : 0.0) : (l3 ? 1.0 : 0.0);
                const int rr = (s4 + 3 < NZ) ? s4 + lk : (s4 + lk < NZ ? s4 + lk : NZ - 1);
                const double wr = lm * Vb[VBW + rr];
                double g[NT];
#pragma unroll
                for (int I = 0; I < NT; I++) g[I] = gm[I] * Gd[gi[I] + rr];
                int p = 0;
#pragma unroll
                for (int I = 0; I < NT; I++)
#pragma unroll
                    for (int J = I; J < NT; J++, p++)
                        acc[p] = __builtin_amdgcn_mfma_f64_16x16x4f64(g[I], wr * g[J], acc[p], 0, 0, 0);
            });
            double *Sc = Tx;
            {
                int p = 0;
#pragma unroll
                for (int I = 0; I < NT; I++)
#pragma unroll
                    for (int J = I; J < NT; J++, p++)
#pragma unroll
                        for (int t = 0; t < 4; t++) {
                            const int row = 16 * I + lk + 4 * t, col = 16 * J + li;
                            Sc[row * NXP + col] = acc[p][t];
                            if (I != J) Sc[col * NXP + row] = acc[p][t];
                        }
            }
            qpb_wsync();
            if (dk == 0) {
#pragma unroll
                for (int j = 0; j < NX; j++) H[qpb_xpos[j]] += Sc[dxi * NXP + j];
            }
            qpb_wsync();
        } else {                       // per column-pattern group: rows looped, columns unrolled
            qpb_for<0, QPB_NGRP>([&](auto gc) {
                constexpr int g = decltype(gc)::value;
#pragma nounroll
                for (int u = qpb_goff[g]; u < qpb_goff[g + 1]; u++) {
                    const int r = __builtin_amdgcn_readfirstlane(qpb_grow[u]);
                    const double t = dxm * Gd[dxi * LDZ + r] * Vb[VBW + r];     // G(r, i) w_r
                    qpb_for<0, qpb_gncol[g]>([&](auto cc) {
                        constexpr int j = qpb_gcol[g][decltype(cc)::value];
                        H[qpb_xpos[j]] = __builtin_fma(t, Gd[j * LDZ + r], H[qpb_xpos[j]]);
                    });
                }
            });
        }
        if (fstamp) QPB_TS(fstamp + 1);
        double kdz[ND];
#if QPB_W_KDIAG
        // a dense z row's diagonal is kd alone (H0 and G'WG put nothing there): it enters
        // the row before the factor, as in the reference's KKT matrix (ldl.c starts each
        // pivot from the diagonal) -- its loads batched here, not one LDS round trip on
        // the pivot chain per z pivot
        qpb_for<0, ND>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            if constexpr (qpb_dkind[k] == 2) kdz[k] = Vb[VBW + NZ + qpb_didx[k]];
        });
        qpb_for<0, ND>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            if constexpr (qpb_dkind[k] == 2) qpb_wpin(kdz[k]);
        });
        qpb_for<0, ND>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            if constexpr (qpb_dkind[k] == 2) H[k] = ln == k ? H[k] + kdz[k] : H[k];
        });
#else
        qpb_for<0, ND>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            if constexpr (qpb_dkind[k] == 2) kdz[k] = Vb[VBW + NZ + qpb_didx[k]];
        });
#endif
        // The pivot recurrence is the critical path: D_{k+1} is formed from
        // H'(k+1,k) and H'(k+1,k+1) (values before step k) with exactly the
        // operations lane k+1's own update performs, so the trailing updates
        // of step k are off the chain.
#if QPB_W_DUP
        // 17..32 dense rows: lane L holds rows L & 15 (Hlo) and 16 + (L & 15) (Hhi),
        // the same copy in each of the four 16-lane DPP rows, so H(j, k) of any row j
        // is one row_newbcast away (no LDS round trip per pivot, no v_readlane).
        // Every lane updates both of its rows: the same operations, in the same
        // order, as the one-row-per-lane factor -- the same bits.
        double Hlo[ND], Hhi[ND];
        {
            double *Sd = Tx;                     // ND x ND scratch (TSZ >= ND^2)
            if (isd) {
#pragma unroll
                for (int e = 0; e < ND; e++) Sd[ln * ND + e] = H[e];
            }
            qpb_wsync();
            const int rl = ln & 15, rh = 16 + (ln & 15);
            const int rhc = rh < ND ? rh : ND - 1;
#pragma unroll
            for (int e = 0; e < ND; e++) {
                Hlo[e] = Sd[rl * ND + e];
                const double v = Sd[rhc * ND + e];
                Hhi[e] = rh < ND ? v : 0.0;
            }
            qpb_wsync();                         // every read before Tx is reused
        }
        double dpiv = qpb_dpp<0x150>(Hlo[0]);    // row 0's H(0,0): lane 0 of every DPP row
        if constexpr (!QPB_W_KDIAG && qpb_dkind[0] == 2) dpiv += kdz[0];
        const int lr = ln & 15;
        qpb_for<0, ND>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            const double rd = qpb_piv_rcp<REG>(dpiv, dmin);
            if constexpr (k + 1 < ND) {
                constexpr int r1 = k + 1;
                const double h = qpb_dpp<0x150 + (r1 & 15)>(r1 < 16 ? Hlo[k] : Hhi[k]);
                const double hkk = qpb_dpp<0x150 + (r1 & 15)>(r1 < 16 ? Hlo[k + 1] : Hhi[k + 1]);
                dpiv = __builtin_fma(h, h * -rd, hkk);
                if constexpr (!QPB_W_KDIAG && qpb_dkind[k + 1] == 2) dpiv += kdz[k + 1];
            }
            rDd = ln == k ? rd : rDd;
            const double nlo = Hlo[k] * -rd, nhi = Hhi[k] * -rd;
            qpb_for<k + 1, ND>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                if constexpr (!QPB_W_LSKIP || qpb_lnz[j][k]) {
                    const double b = qpb_dpp<0x150 + (j & 15)>(j < 16 ? Hlo[k] : Hhi[k]);   // H(j, k)
                    Hlo[j] = __builtin_fma(b, nlo, Hlo[j]);
                    Hhi[j] = __builtin_fma(b, nhi, Hhi[j]);
                }
            });
            Hlo[k] = lr > k ? nlo : 0.0;
            Hhi[k] = 16 + lr > k ? nhi : 0.0;
        });
        // back to one row per lane: lane d < 16 owns row d (Hlo), 16 <= d < 32 row d (Hhi)
#pragma unroll
        for (int e = 0; e < ND; e++) H[e] = ln < 16 ? Hlo[e] : Hhi[e];
#else
#if QPB_W_LDSB
        // broadcasts of the updates through LDS instead of v_readlane pairs: column
        // k (H(j,k) of every row j) is published by its lanes as soon as step k-1
        // has finalised it, into one of two 64-slot buffers in the L transpose area
        // (free between the G'WG and the transpose); step k reads it as wave-uniform
        // LDS loads, paired by the compiler
        double *Bc = Tx;                         // aliases Tx (no __restrict__: the MFMA tiles and the transpose share it)
        Bc[ln] = H[0];
#endif
        double dpiv = qpb_xb<0>(H[0]);
        if constexpr (!QPB_W_KDIAG && qpb_dkind[0] == 2) dpiv += kdz[0];
#if QPB_W_BLK
        // Blocked right-looking LDL': pivots in permutation order as below, but each
        // step updates only its 16-column panel; after a panel [k0, k1) the rows and
        // columns beyond it get the rank-16 update C(d, j) = sum_k -L(d,k) D_k L(j,k)
        // = sum_k (-1/D_k) U(d,k) U(j,k), U(d,k) = row d's column-k value when step k
        // reads it, as v_mfma_f64_16x16x4f64 tiles: A operand U(16I + (l & 15), kk)
        // * (-1/D_kk), B operand U(16J + (l & 15), kk), kk = 4s + (l >> 4).  The tiles
        // of one column block J go through LDS and each row adds its 16 values.  The
        // pivots (and which are regularised) are those of the unblocked factor; only
        // the summation order of the trailing updates changes.
        double *Up = Tx + 128, *Ct = Tx + 128 + 48 * BLK_RS, *Rv = Tx + 128 + 2 * 48 * BLK_RS;
        typedef double qpb_v4b __attribute__((ext_vector_type(4)));
        constexpr int NTB = (ND + 15) / 16;
#endif
        qpb_for<0, ND>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            if constexpr ((QPB_W_ABL & 1) != 0) return;
#if QPB_W_BLK
            constexpr int k0 = k & ~15, k1 = (k0 + 16 < ND) ? k0 + 16 : ND;
            const double rd = qpb_piv_rcp<REG>(dpiv, dmin);
            if constexpr (k + 1 < k1) {
                const double h = qpb_xb<k + 1>(H[k]), hkk = qpb_xb<k + 1>(H[k + 1]);
                dpiv = __builtin_fma(h, h * -rd, hkk);
                if constexpr (!QPB_W_KDIAG && qpb_dkind[k + 1] == 2) dpiv += kdz[k + 1];
            }
            rDd = ln == k ? rd : rDd;
            if constexpr (k1 < ND) {
                if (ln >= k1) Up[(ln - k1) * BLK_RS + (k - k0)] = H[k];     // U(d, k) of a trailing row
                if (ln == 0) Rv[k - k0] = -rd;
            }
            const double nl = H[k] * -rd;
            constexpr int cb = (k & 1) * 64, nb = ((k + 1) & 1) * 64;
            qpb_for<k + 1, k1>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                H[j] = __builtin_fma(Tx[cb + j], nl, H[j]);
                if constexpr (j == k + 1) Tx[nb + ln] = H[j];       // column k+1 is final
            });
            H[k] = ln > k ? nl : 0.0;
            if constexpr (k == k1 - 1 && k1 < ND) {
                qpb_wsync();
                const int li = lane & 15, lk = lane >> 4;
                double rv[4];
#pragma unroll
                for (int s4 = 0; s4 < 4; s4++) rv[s4] = Rv[4 * s4 + lk];
                qpb_for<k1 / 16, NTB>([&](auto Jc) {
                    constexpr int J = decltype(Jc)::value;
                    constexpr int NI = NTB - k1 / 16;
                    qpb_v4b acc[NI];
#pragma unroll
                    for (int i = 0; i < NI; i++) acc[i] = qpb_v4b{0.0, 0.0, 0.0, 0.0};
#pragma unroll
                    for (int s4 = 0; s4 < 4; s4++) {
                        const double bo = Up[(16 * J + li - k1) * BLK_RS + 4 * s4 + lk];
#pragma unroll
                        for (int i = 0; i < NI; i++) {
                            const double ao = Up[(16 * (k1 / 16 + i) + li - k1) * BLK_RS + 4 * s4 + lk] * rv[s4];
                            acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(ao, bo, acc[i], 0, 0, 0);
                        }
                    }
#pragma unroll
                    for (int i = 0; i < NI; i++)
#pragma unroll
                        for (int t = 0; t < 4; t++) Ct[(16 * i + lk + 4 * t) * BLK_RS + li] = acc[i][t];
                    qpb_wsync();
                    if (ln >= k1) {
                        qpb_for<16 * J, (16 * J + 16 < ND ? 16 * J + 16 : ND)>([&](auto cc) {
                            constexpr int c = decltype(cc)::value;
                            H[c] += Ct[(ln - k1) * BLK_RS + (c - 16 * J)];
                        });
                    }
                    qpb_wsync();
                });
                // the next panel's first pivot, after its row got the trailing update
                dpiv = qpb_xb<k1>(H[k1]);
                if constexpr (!QPB_W_KDIAG && qpb_dkind[k1] == 2) dpiv += kdz[k1];
                Tx[nb + ln] = H[k1];                                  // column k1 for step k1
            }
#else
            const double rd = qpb_piv_rcp<REG>(dpiv, dmin);
            if constexpr (k + 1 < ND) {
                const double h = qpb_xb<k + 1>(H[k]), hkk = qpb_xb<k + 1>(H[k + 1]);
                dpiv = __builtin_fma(h, h * -rd, hkk);
                if constexpr (!QPB_W_KDIAG && qpb_dkind[k + 1] == 2) dpiv += kdz[k + 1];
            }
            rDd = ln == k ? rd : rDd;
            // -L(d,k): kept negated so every update (and the solves) is a plain
            // v_fmac_f64 whose broadcast operand folds into it as DPP row_newbcast
            const double nl = H[k] * -rd;
#if QPB_W_LDSB
            constexpr int cb = (k & 1) * 64, nb = ((k + 1) & 1) * 64;
            qpb_for<k + 1, ND>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                if constexpr (!QPB_W_LSKIP || qpb_lnz[j][k]) H[j] = __builtin_fma(Bc[cb + j], nl, H[j]);
                if constexpr (j == k + 1) Bc[nb + ln] = H[j];      // column k+1 is final
            });
            if constexpr (QPB_W_LDSB_SYNC) qpb_wsync();
#else
            qpb_for<k + 1, ND>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                if constexpr (!QPB_W_LSKIP || qpb_lnz[j][k]) H[j] = qpb_fmac_xb<j>(H[j], H[k], nl);
            });
#endif
            H[k] = ln > k ? nl : 0.0;       // -L(d,k) below the diagonal, 0 elsewhere
#endif
        });
#endif  // QPB_W_DUP
        if (fstamp) QPB_TS(fstamp + 2);
        return dmin;
    };
    // transpose -L through LDS: lane e gets column e (0 on and above the
    // diagonal); the first wsync also orders every earlier Vb read before the
    // solve's stores
    auto factor_transpose = [&]() {
        if constexpr ((QPB_W_ABL & 16) != 0) return;
        {
            // row `lane` of -L: entries e < lane at lane(lane-1)/2 + e (exec-masked
            // stores: a shared sink slot would serialise the masked lanes' writes)
            const int lt = qpb_opaque(lane);
            const int base = isd ? lt * (lt - 1) / 2 : 0;
#if QPB_W_TRUNM
            // unmasked, in descending e: a lane's stores past the end of its row land in
            // later rows' slots BEFORE those rows' own stores (a slot of row r is hit by
            // a lane d < r only at e = slot - base_d, above r's own e), and one wave's LDS
            // stores complete in program order -- the empty asm keeps the compiler from
            // reordering them (per lane the addresses are distinct, so it otherwise may).
            // One divergent region instead of one per store (lane 0 shares base 0 with 1).
            if (isd && lt > 0) {
#pragma unroll
                for (int e = ND - 2; e >= 0; e--) {
                    Tx[base + e] = H[e];
                    asm volatile("" ::: "memory");
                }
            }
#else
#pragma unroll
            for (int e = 0; e < ND - 1; e++)
                if (isd && e < lt) Tx[base + e] = H[e];
#endif
        }
        qpb_wsync();
#if !QPB_W_LTLDS
#pragma unroll
        for (int k = 0; k < ND; k++) {
            const double v = Tx[k > id ? k * (k - 1) / 2 + id : T_SINK];
            Lt[k] = k > id ? v : 0.0;
        }
        qpb_wsync();
#endif
    };

    // solve K [dx; dy; dz] = [bx; byv; bz] with the current factor
    constexpr int VBX = 0, VBY = NX, VBZ = NX + NY, VBV = NX + NY + NZ, VBO = NX + NY + 2 * NZ;
    int sstamp = 0;     // timing build: solve-internal stamps base (0 = off)
    auto solve = [&](double bx, double byv, const double *bz, double &dx, double &dy, double *dz) {
        if (sstamp) QPB_TS(sstamp + 0);
        if constexpr (!QPB_XID) {
            if (lane < NX) Vb[VBX + lane] = bx;
            if (lane < NY) Vb[VBY + lane] = byv;
        }
#pragma unroll
        for (int t = 0; t < ZC; t++)
            if (isz[t]) {
                if constexpr (!QPB_XID) Vb[VBZ + lane + 64 * t] = bz[t];
                Vb[VBV + lane + 64 * t] = w[t] * bz[t];     // -bz / D_z (read for leaf rows only)
            }
        if constexpr (QPB_XID)
            if (lane < NY) Vb[VBY + lane] = byv;
        qpb_wsync();
        if (sstamp) QPB_TS(sstamp + 1);
        // this dense row's right-hand side after the leaves' forward elimination
        double ta[QPB_W_SPLIT];
#pragma unroll
        for (int k = 0; k < QPB_W_SPLIT; k++) ta[k] = 0.0;
#pragma unroll
        for (int r = 0; r < NZ; r++)
            if (qpb_zleaf[r]) ta[r % QPB_W_SPLIT] = __builtin_fma(GC(r), Vb[VBV + r], ta[r % QPB_W_SPLIT]);
#pragma unroll
        for (int l = 0; l < NY; l++)
            if (qpb_yleaf[l])
                ta[(NZ + l) % QPB_W_SPLIT] = __builtin_fma(AC(l), -RDY * Vb[VBY + l], ta[(NZ + l) % QPB_W_SPLIT]);
        double t;
        if constexpr (QPB_XID) t = bx;        // dense row d is x_d
        else t = Vb[dvar];                    // bx_i | by_l | bz_r  (VBX, VBY, VBZ are contiguous)
#pragma unroll
        for (int k = 0; k < QPB_W_SPLIT; k++) t += ta[k];
        qpb_wsync();
        if (sstamp) QPB_TS(sstamp + 2);
        qpb_for<0, ND>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            if constexpr ((QPB_W_ABL & 4) != 0) return;
            t = qpb_fmac_xb_dep<k>(t, t, H[k]);
        });
        t *= rDd;
#if QPB_W_LTLDS
        // column `id` of -L straight from the packed transpose area (intact until
        // the next factor): live only through this chain, not across the iteration
        double Ltl[ND];
        const int ido = qpb_opaque(id);
#pragma unroll
        for (int k = 0; k < ND; k++) {
#if QPB_W_LTZS
            Ltl[k] = Tx[k > ido ? k * (k - 1) / 2 + ido : T_SINK];   // T_SINK: never written, 0
#else
            const double v = Tx[k * (k - 1) / 2 + ido];      // in the area for every k <= ND - 1, id <= ND - 1
            Ltl[k] = k > ido ? v : 0.0;
#endif
        }
        qpb_for<0, ND>([&](auto kc) {
            constexpr int k = ND - 1 - decltype(kc)::value;
            if constexpr ((QPB_W_ABL & 4) != 0) return;
            t = qpb_fmac_xb_dep<k>(t, t, Ltl[k]);
        });
#else
        qpb_for<0, ND>([&](auto kc) {
            constexpr int k = ND - 1 - decltype(kc)::value;
            t = qpb_fmac_xb_dep<k>(t, t, Lt[k]);
        });
#endif
        if (sstamp) QPB_TS(sstamp + 3);
        if constexpr (QPB_XID) {
            if (lane < NX) Vb[VBO + lane] = t;
        } else if (isd) {
            Vb[VBO + dvar] = t;               // dense solution, by variable
        }
        qpb_wsync();
        if (sstamp) QPB_TS(sstamp + 4);
        if constexpr (QPB_XID) dx = t;
        else dx = Vb[VBO + ix];
        double gza[ZC][QPB_W_SPLIT], gya[QPB_W_SPLIT];
#pragma unroll
        for (int k = 0; k < QPB_W_SPLIT; k++) {
            gya[k] = 0.0;
#pragma unroll
            for (int u = 0; u < ZC; u++) gza[u][k] = 0.0;
        }
#if QPB_W_RCH > 0
#pragma unroll
        for (int j0 = 0; j0 < NX; j0 += QPB_W_RCH) {
            double xv[QPB_W_RCH], gv[ZC][QPB_W_RCH], av[QPB_W_RCH];
#pragma unroll
            for (int k = 0; k < QPB_W_RCH; k++)
                if (j0 + k < NX) {
                    xv[k] = Vb[VBO + j0 + k];
#pragma unroll
                    for (int u = 0; u < ZC; u++) gv[u][k] = GR(u, j0 + k);
                    if constexpr (NY > 0) av[k] = AR(j0 + k);
                }
#pragma unroll
            for (int k = 0; k < QPB_W_RCH; k++)
                if (j0 + k < NX) {
                    qpb_wpin(xv[k]);
#pragma unroll
                    for (int u = 0; u < ZC; u++) qpb_wpin(gv[u][k]);
                    if constexpr (NY > 0) qpb_wpin(av[k]);
                }
#pragma unroll
            for (int k = 0; k < QPB_W_RCH; k++)
                if (j0 + k < NX) {
                    const int j = j0 + k;
#pragma unroll
                    for (int u = 0; u < ZC; u++) gza[u][j % QPB_W_SPLIT] = __builtin_fma(gv[u][k], xv[k], gza[u][j % QPB_W_SPLIT]);
                    if constexpr (NY > 0) gya[j % QPB_W_SPLIT] = __builtin_fma(av[k], xv[k], gya[j % QPB_W_SPLIT]);
                }
        }
#else
#pragma unroll
        for (int j = 0; j < NX; j++) {
            const double xj = Vb[VBO + j];
#pragma unroll
            for (int u = 0; u < ZC; u++) gza[u][j % QPB_W_SPLIT] = __builtin_fma(GR(u, j), xj, gza[u][j % QPB_W_SPLIT]);
            if constexpr (NY > 0) gya[j % QPB_W_SPLIT] = __builtin_fma(AR(j), xj, gya[j % QPB_W_SPLIT]);
        }
#endif
        double gy = gya[0];
#pragma unroll
        for (int k = 1; k < QPB_W_SPLIT; k++) gy += gya[k];
#pragma unroll
        for (int u = 0; u < ZC; u++) {
            double gz = gza[u][0];
#pragma unroll
            for (int k = 1; k < QPB_W_SPLIT; k++) gz += gza[u][k];
            if constexpr (QPB_XID) dz[u] = -w[u] * (bz[u] - gz);
            else dz[u] = zleaf[u] ? -w[u] * (bz[u] - gz) : Vb[VBO + NX + NY + iz[u]];
        }
        if constexpr (QPB_XID) dy = RDY * (byv - gy);
        else dy = yleaf ? RDY * (byv - gy) : Vb[VBO + NX + iy];
        qpb_wsync();
        if (sstamp) QPB_TS(sstamp + 5);
    };

    // lane sums over this lane's z slots (0 outside the range)
    auto zsum = [&](auto f) {
        double v = 0.0;
#pragma unroll
        for (int t = 0; t < ZC; t++) v += isz[t] ? f(t) : 0.0;
        return qpb_rsum<ROWS_Z>(v);
    };

    QPB_TS(1);
    // ---- kkt_initialize (Auxilary.c:992-1089) as iteration -1, then the
    // QP_SOLVE loop (qpSWIFT.c:502-602).  One instance of factor() and of
    // solve() serves the setup solve, the predictor and the corrector, which
    // keeps the kernel's code small enough for the instruction cache.
    double x = 0.0, y = 0.0, s[ZC], z[ZC];
#pragma unroll
    for (int t = 0; t < ZC; t++) { s[t] = 1.0; z[t] = 1.0; }
    long it = -1;
    // squared residual norms; the exit test compares them with tol^2 (sqrt is
    // monotone), the norms themselves are taken once, for the statistics
    double st_rx2 = 0.0, st_ry2 = 0.0, st_rz2 = 0.0, st_mu = 0.0, ap = 0.0, ad = 0.0;
    double fv = 0.0;    // this lane's objective term at the last residual evaluation
    const double tol2 = a.tol > 0.0 ? a.tol * a.tol : -1.0;
    double sigma = 100.0;      // options->sigma (SIGMA, GlobalOptions.h:49)
#if QPB_WARM
    // warm variant (qpb_solve_warm): QP_SOLVE continues from the object's iterate,
    // IterationCount and options->sigma (qpSWIFT.c:502-596 never re-initialises)
#if QPB_SERVE
    // the host's block (KernelArgs::win): never a line this wave wrote
    const double *wi = a.win;
    if (isx) x = QPB_LDS(&wi[lane]);
#if NY > 0
    if (isy) y = QPB_LDS(&wi[NX + lane]);
#endif
#pragma unroll
    for (int t = 0; t < ZC; t++)
        if (isz[t]) {
            z[t] = QPB_LDS(&wi[NX + NY + lane + 64 * t]);
            s[t] = QPB_LDS(&wi[NX + NY + NZ + lane + 64 * t]);
        }
    const int *wfl = reinterpret_cast<const int *>(wi + NX + NY + 2 * NZ);
    const long it0 = QPB_LDS(&wfl[1]);
    const int flag0 = QPB_LDS(&wfl[0]);
    sigma = QPB_LDS(&wi[NX + NY + 2 * NZ + 1]);
#else
    if (isx) x = QPB_LDS(&a.x[tile * (NX * 64) + lane * 64 + ql]);
#if NY > 0
    if (isy) y = QPB_LDS(&a.y[tile * (NY * 64) + lane * 64 + ql]);
#endif
#pragma unroll
    for (int t = 0; t < ZC; t++)
        if (isz[t]) {
            z[t] = QPB_LDS(&a.z[tile * (NZ * 64) + (lane + 64 * t) * 64 + ql]);
            s[t] = QPB_LDS(&a.s[tile * (NZ * 64) + (lane + 64 * t) * 64 + ql]);
        }
    const long it0 = QPB_LDS(&a.iters[q]);   // IterationCount the QP enters with
    const int flag0 = QPB_LDS(&a.flag[q]);   // stats->Flag it enters with (QP_FATAL after setup)
    sigma = QPB_LDS(&a.sig[q]);
#endif
    it = 0;
    // the drop-in's timers and verbose trace (KernelArgs::trace, qpb_codegen.hpp):
    // s_memrealtime ticks in the factorisations and in factor + solves, and the
    // statistics the reference prints per iteration (qpSWIFT.c:506-517, 598-600)
    double *const trc = (a.trace && lane == 0) ? a.trace + q * QPB_TRACE_STRIDE : nullptr;
    long t_fac = 0, t_kkt = 0, n_top = 0, n_it = 0;
#define QPB_CLK() ((long)__builtin_amdgcn_s_memrealtime())
#else
    constexpr long it0 = 0;
    constexpr int flag0 = 3;
#endif
    int flag = flag0;
    for (;;) {
        // qpSWIFT.c:598-601: QP_MAXIT only when IterationCount == maxit
        if ((QPB_WARM || it >= 0) && it >= a.maxit) { flag = (!QPB_WARM || it0 + it == a.maxit) ? 2 : flag0; break; }
        QPB_TS(it >= 0 ? 8 + 8 * it : 2);
        // updatekktmatrix (Auxilary.c:211-215): z diagonal -s/z.  The setup
        // system has -I there, which is this with s = z = 1 (iteration -1).
        double rx, ry, rz[ZC], rzi[ZC], kd[ZC], sz, mu = 0.0;
#pragma unroll
        for (int t = 0; t < ZC; t++) {
            rzi[t] = qpb_rcp(z[t]);
            kd[t] = isz[t] ? -s[t] * rzi[t] : -1.0;
        }
        // The factor does not depend on the residuals, so it is formed before
        // the exit test (wasted on the last iteration): one LDS exchange serves
        // both, and the LDL's latency-bound pivot chain is scheduled together
        // with the residual products and reductions.
        if (QPB_W_TIMING) fstamp = it == 1 ? 360 : 0;
#if QPB_WARM
        const long tf0 = QPB_CLK();
#endif
        factor_publish(kd);
        // residuals (Auxilary.c:745-786), objective (Auxilary.c:1133-1141)
        if (lane < NX) Vb[lane] = x;
#pragma unroll
        for (int t = 0; t < ZC; t++)
            if (isz[t]) Vb[NX + lane + 64 * t] = z[t];
        if (lane < NY) Vb[NX + NZ + lane] = y;
        qpb_wsync();
        // (a dense block of <= 16 rows lives in DPP row 0: the other rows' broadcasts
        // are not pivots and do not vote)
        if (QPB_W_LAZYREG && __builtin_amdgcn_ballot_w64(factor_ldl(qpb_ic<0>{}) <= 1e-14 && (ND > 16 || lane < 16)) != 0)
            factor_ldl(qpb_ic<1>{});                        // a tiny pivot: rare, wave-uniform
        else if (!QPB_W_LAZYREG)
            factor_ldl(qpb_ic<1>{});
#if QPB_WARM
        long tf1 = QPB_CLK() - tf0;   // + the transpose below
#endif
        if (QPB_W_TIMING && it == 1) QPB_TS(364);
        double tp = 0.0;
        ry = by;
        rx = -cx;
#pragma unroll
        for (int t = 0; t < ZC; t++) rz[t] = hz[t] - s[t];
        if constexpr (!(QPB_W_ABL & 8)) {
#if QPB_W_RCH > 0
        // chunks of QPB_W_RCH columns: every load of a chunk issued before its first FMA
        // (the same FMAs in the same order)
#pragma unroll
        for (int j0 = 0; j0 < NX; j0 += QPB_W_RCH) {
            double xv[QPB_W_RCH], pv[QPB_W_RCH], gv[ZC][QPB_W_RCH], av[QPB_W_RCH];
#pragma unroll
            for (int k = 0; k < QPB_W_RCH; k++)
                if (j0 + k < NX) {
                    xv[k] = Vb[j0 + k];
                    pv[k] = PR(j0 + k);
#pragma unroll
                    for (int t = 0; t < ZC; t++) gv[t][k] = GR(t, j0 + k);
                    if constexpr (NY > 0) av[k] = AR(j0 + k);
                }
#pragma unroll
            for (int k = 0; k < QPB_W_RCH; k++)
                if (j0 + k < NX) {
                    qpb_wpin(xv[k]);
                    qpb_wpin(pv[k]);
#pragma unroll
                    for (int t = 0; t < ZC; t++) qpb_wpin(gv[t][k]);
                    if constexpr (NY > 0) qpb_wpin(av[k]);
                }
#pragma unroll
            for (int k = 0; k < QPB_W_RCH; k++)
                if (j0 + k < NX) {
                    tp = __builtin_fma(-pv[k], xv[k], tp);
#pragma unroll
                    for (int t = 0; t < ZC; t++) rz[t] = __builtin_fma(-gv[t][k], xv[k], rz[t]);
                    if constexpr (NY > 0) ry = __builtin_fma(-av[k], xv[k], ry);
                }
        }
#else
#pragma unroll
        for (int j = 0; j < NX; j++) {
            const double xj = Vb[j];
            tp = __builtin_fma(-PR(j), xj, tp);
#pragma unroll
            for (int t = 0; t < ZC; t++) rz[t] = __builtin_fma(-GR(t, j), xj, rz[t]);
            if constexpr (NY > 0) ry = __builtin_fma(-AR(j), xj, ry);
        }
#endif
        {
            double ra[QPB_W_SPLIT];
#pragma unroll
            for (int k = 0; k < QPB_W_SPLIT; k++) ra[k] = k ? 0.0 : rx;
#pragma unroll
            for (int r = 0; r < NZ; r++)   // G(r, i): the dense-row slice when dense row i is x_i
                ra[r % QPB_W_SPLIT] = __builtin_fma(-(QPB_XID ? GC(r) : Gd[ix * LDZ + r]), Vb[NX + r], ra[r % QPB_W_SPLIT]);
#pragma unroll
            for (int l = 0; l < NY; l++)
                ra[(NZ + l) % QPB_W_SPLIT] =
                    __builtin_fma(-(QPB_XID ? AC(l) : Ad[ix * LDY + l]), Vb[NX + NZ + l], ra[(NZ + l) % QPB_W_SPLIT]);
            rx = ra[0];
#pragma unroll
            for (int k = 1; k < QPB_W_SPLIT; k++) rx += ra[k];
        }
        }
        rx += tp;
        if (QPB_W_TIMING && it == 1) QPB_TS(365);
        {
            double red[4] = {isx ? rx * rx : 0.0, isy ? ry * ry : 0.0, 0.0, 0.0};
#pragma unroll
            for (int t = 0; t < ZC; t++)
                if (isz[t]) {
                    red[2] = __builtin_fma(rz[t], rz[t], red[2]);
                    red[3] = __builtin_fma(s[t], z[t], red[3]);
                }
            qpb_rsum_n<ROWS_R>(red);
            if (QPB_W_TIMING && it == 1) QPB_TS(366);
            sz = red[3];
            if (QPB_WARM || it >= 0) {
                fv = isx ? x * __builtin_fma(-0.5, tp, cx) : 0.0;      // summed at exit
                st_rx2 = red[0];
                st_ry2 = NY > 0 ? red[1] : 0.0;
                st_rz2 = red[2];
                st_mu = sz * (1.0 / NZ);
            }
        }
        bool pc = true;
#if QPB_WARM
        {
            const double fq = qpb_rsum<ROWS_X>(isx ? x * __builtin_fma(-0.5, tp, cx) : 0.0);
            if (trc && it < QPB_TRACE_MAX) {
                double *e = trc + 4 + 7 * it;
                e[0] = fq; e[1] = __builtin_sqrt(st_rx2); e[2] = __builtin_sqrt(st_ry2); e[3] = __builtin_sqrt(st_rz2);
                e[4] = st_mu;
                n_top = it + 1;
            }
        }
#endif
        if (QPB_WARM || it >= 0) {
            if (st_rx2 < tol2 && st_rz2 < tol2 && (NY == 0 || st_ry2 < tol2) && st_mu < a.abstol) {
                flag = (QPB_WARM && it0 + it == a.maxit) ? 2 : 0;
                break;
            }
            mu = st_mu;
            pc = sigma > a.sigma_d;
        }
        QPB_TS(it >= 0 ? 9 + 8 * it : 5);
#if QPB_WARM
        const long tt0 = QPB_CLK();
#endif
        factor_transpose();
#if QPB_WARM
        tf1 += QPB_CLK() - tt0;
        t_fac += tf1;
        t_kkt += tf1;
#endif
        QPB_TS(it >= 0 ? 10 + 8 * it : 6);
        if (!pc) sigma = a.sigma_d;
        double cc[ZC];
#pragma unroll
        for (int t = 0; t < ZC; t++) cc[t] = sigma * mu;
        double dx, dy, dz[ZC], dsl[ZC];
        auto step_length = [&]() {
            // alpha = min over d < 0 of v/(-d) == 1 / max(-d/v); 1 if none (Auxilary.c:359-393)
            double bm[2] = {0.0, 0.0};
#pragma unroll
            for (int t = 0; t < ZC; t++)
                if (isz[t]) {
                    bm[0] = __builtin_fmax(bm[0], -dsl[t] * __builtin_amdgcn_rcp(s[t]));
                    bm[1] = __builtin_fmax(bm[1], -dz[t] * rzi[t]);
                }
            qpb_rmax_n<ROWS_Z>(bm);
            const double bp = bm[0], bd = bm[1];
            ap = bp > 1e-10 ? __builtin_amdgcn_rcp(bp) : 1.0;
            ad = bd > 1e-10 ? __builtin_amdgcn_rcp(bd) : 1.0;
        };
        // pass 2: setup solve, rhs [-c; b; h]; pass 0: predictor (kktsolve_1,
        // Auxilary.c:471-515), ds = -s.*z; pass 1: corrector / centering
        // (kktsolve_2, Auxilary.c:524-564)
        int pass = (!QPB_WARM && it < 0) ? 2 : (pc ? 0 : 1);
        for (;;) {
            double bxv = rx, byv = ry, bz[ZC];
#pragma unroll
            for (int t = 0; t < ZC; t++)
                bz[t] = pass == 2 ? hz[t] : (pass == 0 ? rz[t] + s[t] : __builtin_fma(-cc[t], rzi[t], rz[t] + s[t]));
            if (pass == 2) { bxv = -cx; byv = by; }
            if (QPB_W_TIMING) sstamp = (it == 1 && pass == 0) ? 300 : 0;
#if QPB_WARM
            const long ts0 = QPB_CLK();
#endif
            solve(bxv, byv, bz, dx, dy, dz);
#if QPB_WARM
            t_kkt += QPB_CLK() - ts0;
#endif
            QPB_TS(it >= 0 ? (pass == 0 ? 11 : 13) + 8 * it : 3);
            if (pass == 2) {
                // initial point: x0, y0 from the solve; s0, z0 from r = h - G x0
                x = isx ? dx : 0.0;
                y = isy ? dy : 0.0;
                if (lane < NX) Vb[lane] = x;
                qpb_wsync();
                double zi[ZC];
#pragma unroll
                for (int t = 0; t < ZC; t++) {
                    double gx = 0.0;
#pragma unroll
                    for (int j = 0; j < NX; j++) gx = __builtin_fma(GR(t, j), Vb[j], gx);
                    zi[t] = hz[t] - gx;
                }
                qpb_wsync();
                double lh[2] = {-1e300, -1e300};
#pragma unroll
                for (int t = 0; t < ZC; t++)
                    if (isz[t]) {
                        lh[0] = __builtin_fmax(lh[0], -zi[t]);
                        lh[1] = __builtin_fmax(lh[1], zi[t]);
                    }
                qpb_rmax_n<ROWS_Z>(lh);
                const double lo = -lh[0], hi = lh[1];
                const double sh = -lo;
#pragma unroll
                for (int t = 0; t < ZC; t++) {
                    s[t] = sh < 0 ? zi[t] : zi[t] + (1 + sh);
                    z[t] = hi < 0 ? -zi[t] : -zi[t] + (1 + hi);
                    if (!isz[t]) { s[t] = 1.0; z[t] = 1.0; }
                }
                QPB_TS(4);
                break;
            }
            if (pass == 0) {
#pragma unroll
                for (int t = 0; t < ZC; t++) dsl[t] = -s[t] * __builtin_fma(dz[t], rzi[t], 1.0);
                step_length();
                const double rho = zsum([&](int t) { return (s[t] + ap * dsl[t]) * (z[t] + ad * dz[t]); }) * qpb_rcp(sz);   // formrho
                const double r1 = 1 > rho ? rho : 1;
                const double cube = r1 * r1 * r1;
                sigma = a.sigma_d < cube ? cube : a.sigma_d;
#pragma unroll
                for (int t = 0; t < ZC; t++) cc[t] = __builtin_fma(-dsl[t], dz[t], sigma * mu);
                QPB_TS(12 + 8 * it);
                pass = 1;
                continue;
            }
#pragma unroll
            for (int t = 0; t < ZC; t++) dsl[t] = __builtin_fma(__builtin_fma(-s[t], dz[t], cc[t]), rzi[t], -s[t]);
            step_length();
            QPB_TS(14 + 8 * it);
            ap = 0.99 * ap > 1.0 ? 1.0 : 0.99 * ap;
            ad = 0.99 * ad > 1.0 ? 1.0 : 0.99 * ad;
#if QPB_WARM
            if (trc && it < QPB_TRACE_MAX) {
                trc[4 + 7 * it + 5] = ap;
                trc[4 + 7 * it + 6] = ad;
                n_it = it + 1;
            }
#endif
            if (isx) x = __builtin_fma(dx, ap, x);
            if (isy) y = __builtin_fma(dy, ad, y);
#pragma unroll
            for (int t = 0; t < ZC; t++)
                if (isz[t]) {
                    s[t] = __builtin_fma(dsl[t], ap, s[t]);
                    z[t] = __builtin_fma(dz[t], ad, z[t]);
                }
            break;
        }
        it++;
    }
    QPB_TS(370);
    const double fval = qpb_rsum<ROWS_X>(fv);
    // ---- outputs (tiled SoA)
    if (isx) QPB_STS(&a.x[tile * (NX * QPB_TSTR) + lane * QPB_TSTR + ql], x);
#if NY > 0
    if (isy) QPB_STS(&a.y[tile * (NY * QPB_TSTR) + lane * QPB_TSTR + ql], y);
#endif
#pragma unroll
    for (int t = 0; t < ZC; t++)
        if (isz[t]) {
            QPB_STS(&a.z[tile * (NZ * QPB_TSTR) + (lane + 64 * t) * QPB_TSTR + ql], z[t]);
            QPB_STS(&a.s[tile * (NZ * QPB_TSTR) + (lane + 64 * t) * QPB_TSTR + ql], s[t]);
        }
    if (lane == 0) {
        QPB_STS(&a.flag[q], flag);
        QPB_STS(&a.iters[q], (int)(it0 + it));
        QPB_STS(&a.fval[q], fval);
#if QPB_WARM
        QPB_STS(&a.sig[q], sigma);
        if (trc) { trc[0] = (double)t_fac; trc[1] = (double)t_kkt; trc[2] = (double)n_top; trc[3] = (double)n_it; }
#elif QPB_W_SIGOUT
        if (a.sig) QPB_STS(&a.sig[q], sigma);   // options->sigma after a cold QP_SOLVE (drop-in)
#endif
        if (a.stats && !QPB_W_TIMING) {
            double *o = a.stats + tile * 6 * QPB_TSTR + ql;
            o[0] = __builtin_sqrt(st_rx2); o[QPB_TSTR] = __builtin_sqrt(st_ry2); o[2 * QPB_TSTR] = __builtin_sqrt(st_rz2); o[3 * QPB_TSTR] = st_mu; o[4 * QPB_TSTR] = ap; o[5 * QPB_TSTR] = ad;
        }
    }
    QPB_TS(371);
#if QPB_W_TIMING == 2
    if (lane == 0 && a.stats) {
        double *o = a.stats + tile * 384 + ql;
        o[0] = t_rt0; o[64] = (double)__builtin_amdgcn_s_memrealtime();
        o[128] = t_cy0; o[192] = (double)__builtin_readcyclecounter(); o[256] = (double)it;
        const unsigned hwid = __builtin_amdgcn_s_getreg(4 | (31 << 11));    // HW_ID (wave, simd, cu, se)
        const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (31 << 11));    // XCC_ID
        o[320] = (double)hwid + 4294967296.0 * (double)(xcc & 0xf);
    }
#endif
}

#if QPB_SERVE
#ifndef QPB_W_SERVE_CALL   // 1 (diagnostics): each request's body is a call (noinline, its own
#define QPB_W_SERVE_CALL 0 // LDS, the kernel arguments re-read per request): nothing of the body's
#endif                     // register allocation spans the request loop
#ifndef QPB_W_SERVE_OPQ    // 1 (diagnostics): body inlined, kernel arguments opaque per request
#define QPB_W_SERVE_OPQ 0
#endif
#if QPB_W_SERVE_CALL
static __device__ __attribute__((noinline)) void qpb_wave_req(const qpb_args *ap, unsigned tid) {
    __shared__ __attribute__((aligned(16))) double req_lds[WPB * LDS_WAVE];
    const qpb_args ra = *ap;
    qpb_wave_body(ra, req_lds, tid);
}
#endif
// persistent form (the drop-in's QP_SOLVE, qpb::serve_ex): one wave, QP 0, one
// solve per request posted in the mailbox (qpb_serve_wait, runtime prelude)
extern "C" __global__ void __launch_bounds__(QPB_WG, 1)
QPB_KERNEL_NAME(qpb_args a, qpb_mailbox *mb, unsigned long long last, unsigned long long idle,
                unsigned long long life) {
    __shared__ __attribute__((aligned(16))) double qpb_lds[WPB * LDS_WAVE];
    const unsigned long long t_launch = __builtin_amdgcn_s_memrealtime();
    unsigned long long t_seen = 0;
    while (qpb_serve_wait(mb, &last, idle, life, t_launch, &t_seen)) {
#if QPB_W_EXECDBG
        {   // diagnostics: the EXEC mask each request starts with -> mailbox word 40
            const unsigned long long ex = __builtin_amdgcn_read_exec();
            if ((threadIdx.x & 63) == 0)
                __hip_atomic_store((unsigned long long *)mb + 40, ex, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
#endif
        // a fresh lane index per request: nothing derived from it is hoisted out of
        // this loop (that would hold extra registers through the solve)
        unsigned tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
#if QPB_W_SERVE_CALL
        (void)qpb_lds;
        qpb_wave_req(&a, tid);
#elif QPB_W_SERVE_OPQ
        // diagnostics: every kernel argument opaque per request, so nothing derived
        // from them is computed once and carried through the request loop
        qpb_args ra = a;
        // (QPB_W_SERVE_OPQ = 1: every field; a larger value is a bit mask over the field
        // groups below, for bisection -- bit k + 1 = group k)
#define QPB_OPQ(k, f) if constexpr (QPB_W_SERVE_OPQ == 1 || ((QPB_W_SERVE_OPQ >> ((k) + 1)) & 1)) \
            asm volatile("" : "+s"(ra.f))
        QPB_OPQ(0, P); QPB_OPQ(0, A); QPB_OPQ(0, G); QPB_OPQ(0, c); QPB_OPQ(0, h); QPB_OPQ(0, b);
        QPB_OPQ(1, x); QPB_OPQ(1, y); QPB_OPQ(1, z); QPB_OPQ(1, s);
        QPB_OPQ(2, flag); QPB_OPQ(2, iters); QPB_OPQ(2, fval); QPB_OPQ(2, stats);
        QPB_OPQ(3, B); QPB_OPQ(4, tol); QPB_OPQ(5, abstol); QPB_OPQ(6, sigma_d);
        QPB_OPQ(7, maxit); QPB_OPQ(8, sig); QPB_OPQ(8, warm); QPB_OPQ(8, trace);
#undef QPB_OPQ
        qpb_wave_body(ra, qpb_lds, tid);
#else
        qpb_wave_body(a, qpb_lds, tid);
#endif
        qpb_serve_done(mb, last, t_seen);
        if (life == 0) break;       // one request per launch (the default; the host pre-launches the next)
    }
}
#endif

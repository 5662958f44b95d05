// qpb_row.hip -- row-cooperative IPM kernel: ONE 16-lane row per QP, four QPs
// per wavefront.
//
// Template source like qpb_wave.hip (the host prepends sizes, tables and the
// kernel name; qpb_wave.cpp generate_row_kernel).  Same algorithm and the same
// elimination as the wave kernel's common case -- every z and y row is a leaf
// and the x block is factored in natural order (QPB_XID) -- for plans small
// enough that one QP fits a 16-lane DPP row: n <= 16, p <= 16, m <= 32.
//
// Lane c of a row holds x_c, y_c, z_c / s_c (c < 16) and z_{16+c} / s_{16+c}
// (second register when m > 16).  Every cross-lane move is inside the row, so
// it is a DPP row_newbcast folded into the consuming v_fmac_f64 (no LDS round
// trips, no SGPR traffic), and every reduction is a 4-stage row butterfly that
// leaves the result in all 16 lanes.  LDS is used once per factorisation, to
// transpose L for the backward solve, and for the input staging.  A QP that
// converges freezes while the other rows of its wave go on.
//
// Reference: qpSWIFT's Mehrotra predictor-corrector (qpSWIFT.c:473-644,
// kkt_initialize Auxilary.c:992-1089), LDL' with dynamic regularisation
// (ldl.c:253-326), residuals (Auxilary.c:745-786), step length
// (Auxilary.c:359-393).  Fast mode: FMA contraction, reciprocal pivots.
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

#ifndef QPB_ROW_COMMON_DONE
#define QPB_ROW_COMMON_DONE
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
    const void *tab;          // (tree kernel tables; unused here)
    double *best;             // fused argmin (qpb_solve_best): {fval, index}, or NULL
    unsigned long long *part; // per-wave partials {fval bits, index}
    unsigned *ctr;            // arrival counter (zero between launches)
    double *sig;              // per-QP sigma: in (warm) / out (NULL: not tracked)
    long warm;                // 1: continue from x, y, z, s, iters, flag, sig (no kkt_initialize)
    double *trace;            // warm variant: per-QP timers + per-iteration statistics (or NULL)
    const double *win;        // persistent warm variants: x y z s {flag, iters} sigma to continue from (or NULL)
};

// Staging / H0 knobs.  Round 1 saw an illegal-address fault with ZF128, AADPP and
// LATEFAC all on; round 3 found no faulting instruction in today's objects.
// ZF128 stays off (the unrolled zero-fill replaced it); AADPP is on since round 4
// (+2 % at 1 024 and 2^20 QPs, profiles/r04_aadpp_ab.jsonl, the GPU suite green).
#ifndef QPB_R_ZF128
#define QPB_R_ZF128 0     // zero-fill the staging area with 16-byte LDS stores
#endif
#ifndef QPB_R_AADPP
#define QPB_R_AADPP 1     // 1e7 A'A of H0 by DPP broadcasts (1) or LDS reads (0)
#endif
#ifndef QPB_R_LATEFAC
#define QPB_R_LATEFAC 1   // factor after the exit test (0: before it, overlapping the reductions)
#endif
#ifndef QPB_R_REGH0
#if defined(QPB_R_WPE) && QPB_R_WPE > 1
#define QPB_R_REGH0 0     // two-wave form: <= 256 registers, H0 / -P rows stay in LDS
#else
#define QPB_R_REGH0 0     // 1: the lane's H0 and -P rows held in registers (no LDS
                          // round trip at the start of every factor and residual pass)
#endif
#endif
#ifndef QPB_R_LAZYREG     // 1: pivot regularisation checked once per factor, the factor redone only
#if defined(QPB_R_WPE) && QPB_R_WPE > 1   // when needed (same bits).  The two-wave form spills 34
#define QPB_R_LAZYREG 0   // more registers with it (2^20 QPs 3.59 -> 3.82 ms); the one-wave kernel
#else                     // gains since the DPP wait states moved to the hazard pass (1 024 QPs
#define QPB_R_LAZYREG 1   // 30.3 -> 29.8 us, profiles/r04_row_knobs2_ab.jsonl; round 3: no gain)
#endif
#endif
#ifndef QPB_R_GWG4
#define QPB_R_GWG4 1      // G'WG four rows at a time, products formed before their DPP FMAs
#endif
#ifndef QPB_R_NLFIRST
#define QPB_R_NLFIRST 1   // each pivot's -L(c,k) formed before the lookahead
#endif
#ifndef QPB_R_EARLYGWG
#define QPB_R_EARLYGWG 0  // 1: H = H0 + G'WG formed before the exit test, between the residual products
                          // and their reductions (independent work in the reductions' latency; wasted on
                          // a wave's last pass), the pivot chain after it
#endif
#ifndef QPB_R_RCP1
#define QPB_R_RCP1 0      // 1: pivot reciprocals without the Newton step (v_rcp_f64 alone, off the chain's
                          // two dependent FMAs per pivot)
#endif
#ifndef QPB_R_SPLIT
#define QPB_R_SPLIT 0     // 1: two waves per four QPs (128-thread workgroups): wave 0 factors, solves and
                          // updates, wave 1 forms the residuals (and the exit test) while wave 0 factors;
                          // they swap residuals and iterate through LDS, two barriers per pass
#endif
#ifndef QPB_R_ALIAS
#define QPB_R_ALIAS 1     // the iteration's LDS areas overlay the staging area (half the LDS per QP)
#endif
#ifndef QPB_R_GATHER
#define QPB_R_GATHER 0    // sparse products with G (and A') as per-lane gathers from the row's LDS vector
                          // area (one ds_read + one FMA per term of the lane's own row / column) instead
                          // of one DPP broadcast per column of the pattern's union (qpb_wave.cpp
                          // row_gather_tables).  Bit mask: 1 the residual products, 2 G'WG's sources,
                          // 4 the solves' leaf eliminations (G'v, A'yr), 8 the solves' G dx / A dx.
                          // Off: measured slower everywhere (profiles/r05_row_gather_ab.jsonl, DESIGN
                          // §4c round 5) -- 18 % fewer VALU instructions per pass, but every gather is an
                          // LDS round trip on the chain (1 024 QPs: 29.5 -> 32.1 us), and at 2^20 QPs the
                          // CU's one LDS pipe serves four SIMDs: 3.58 -> 3.88 ms
#endif
#define GR_RES ((QPB_R_GATHER) & 1)
#define GR_GWG ((QPB_R_GATHER) & 2)
#define GR_SLV ((QPB_R_GATHER) & 4)
#define GR_SLX ((QPB_R_GATHER) & 8)
#ifndef QPB_R_PIVLDS
#define QPB_R_PIVLDS 0    // the factor keeps no zeroed triangle and no 1/D select per pivot: each pivot
                          // goes to an LDS slot (1/D re-formed per lane afterwards, the same bits), -L goes
                          // to LDS under an address mask (strict lower part only; the rest of the area
                          // stays zero), and both triangular solves read their multipliers there.  -48
                          // VALU instructions per factor, but two more LDS round trips per pass: 1 024 QPs
                          // 29.5 -> 30.2 us, 2^20 unchanged (profiles/r05_row_gather_ab.jsonl); off
#endif
#ifndef QPB_R_RDLDS
#define QPB_R_RDLDS 0     // each pivot D_k to an LDS slot (one store per pivot) and 1/D per lane re-formed
                          // from its own D_c after the factor (the same bits) -- no 64-bit select per
                          // pivot; the lazy regularisation check reads the same slots (QPB_R_PIVLDS does
                          // this too, with the -L store masked and the solves reading -L from LDS)
#endif
#ifndef QPB_R_H2
#define QPB_R_H2 1        // the lookahead pivot D_{k+1} = H(k+1,k+1) - H(k+1,k)^2 / D_k with the square formed
                          // off the pivot chain (one dependent FMA after 1/D_k instead of a multiply + FMA)
#endif
#ifndef QPB_WARM
#define QPB_WARM 0        // 1: the warm-solve variant (qpb_solve_warm), compiled on demand
#endif
#define QPB_TRACE_MAX 256                       // = qpb::QPB_TRACE_MAX (qpb_codegen.hpp)
#define QPB_TRACE_STRIDE (4 + 7 * QPB_TRACE_MAX)
#ifndef QPB_R_SELSLICE
#define QPB_R_SELSLICE 1  // 1: the static slices loaded unconditionally + select (0: the round-5 branchy form)
#endif
#ifndef QPB_R_TIMING
#define QPB_R_TIMING 0    // 2: per-QP start / end (realtime, cycles), iterations, hardware ids into stats;
                          // 3: cycles per phase (H0 + setup solve, residuals, factor, predictor,
                          //    corrector + tail, staging) into stats
#endif

static __device__ __forceinline__ double qpb_rcp(double v) {
    double r = __builtin_amdgcn_rcp(v);
    double e = __builtin_fma(-v, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-v, r, 1.0);
    return __builtin_fma(r, e, r);
}

// 1 / regularise(d) (ldl.c:273-274): v_rcp_f64 + one Newton step, computed
// unconditionally; |d| <= 1e-14 -> 1/(+-1e-7), sign as ldl.c:273
static __device__ __forceinline__ double qpb_rcp_reg(double d) {
    double r = __builtin_amdgcn_rcp(d);
    r = __builtin_fma(__builtin_fma(-d, r, 1.0), r, r);
    asm("" : "+v"(r));     // keeps the rare regularised case from becoming a branch
    const double reg = d > 0.0 ? 1e7 : -1e7;
    return __builtin_fabs(d) <= 1e-14 ? reg : r;
}

// the pivot's 1 / regularise(d) (QPB_R_RCP1: the bare v_rcp_f64)
static __device__ __forceinline__ double qpb_rcp_piv(double d) {
    if constexpr (!QPB_R_RCP1) return qpb_rcp_reg(d);
    double r = __builtin_amdgcn_rcp(d);
    asm("" : "+v"(r));
    const double reg = d > 0.0 ? 1e7 : -1e7;
    return __builtin_fabs(d) <= 1e-14 ? reg : r;
}

// the same 1/d without the regularisation select (QPB_R_LAZYREG's fast pass)
static __device__ __forceinline__ double qpb_rcp_nr(double d) {
    double r = __builtin_amdgcn_rcp(d);
    return __builtin_fma(__builtin_fma(-d, r, 1.0), r, r);
}

template <int J0, int J1, class F> static __device__ __forceinline__ void qpb_for(F &&f) {
    if constexpr (J0 < J1) {
        f(qpb_ic<J0>{});
        qpb_for<J0 + 1, J1>(f);
    }
}

// lane J of this row, in every lane of the row (compiler DPP move)
template <int J> static __device__ __forceinline__ double qpb_nb(double v) {
    return __builtin_amdgcn_update_dpp(0.0, v, 0x150 + J, 0xf, 0xf, true);
}
template <int CTRL> static __device__ __forceinline__ double qpb_dpp(double v) {
    return __builtin_amdgcn_update_dpp(0.0, v, CTRL, 0xf, 0xf, true);
}

// acc += (src of row lane J) * m as one v_fmac_f64 with a DPP row_newbcast
// source (the compiler does not fold a 64-bit DPP move into an FMA).  A DPP
// source must not have been written by the two preceding VALU instructions, and
// the compiler's hazard recognizer cannot see into inline asm -- nor can the
// source code rule out a VALU copy the register allocator places right before
// the asm (e.g. out of an AGPR).  So the runtime audits every compiled code
// object (qpb_runtime.hip, dpp_audit: no write of a DPP instruction's VGPR
// operands within 2 wait states, no VALU exec write within 5, across branches)
// and, should it find one, rebuilds the kernel with QPB_DPP_NOP = 2: wait states
// inside every DPP asm (25 % slower, never needed so far).
//  - qpb_fxs: static sources (prologue slices) and the factor's columns;
//  - qpb_fx:  dynamic sources, volatile so a phase keeps its order;
//  - qpb_fxd: the chained triangular solves (src is the accumulator itself).
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
template <int J> static __device__ __forceinline__ void qpb_fxs(double &acc, double src, double m) {
    asm(QPB_DPP_PRE "v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf bound_ctrl:1"
        : "+v"(acc) : "v"(src), "v"(m), "i"(J));
}
template <int J> static __device__ __forceinline__ void qpb_fx(double &acc, double src, double m) {
    asm volatile(QPB_DPP_PRE "v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                 : "+v"(acc) : "v"(src), "v"(m), "i"(J));
}
template <int J> static __device__ __forceinline__ void qpb_fxd(double &t, double m) {
    asm volatile(QPB_DPP_DEP "v_fmac_f64_dpp %0, %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                 : "+v"(t) : "v"(m), "i"(J));
}
static __device__ __forceinline__ void qpb_fence(double a) { asm volatile("s_nop 1" ::"v"(a)); }
static __device__ __forceinline__ void qpb_fence(double a, double b) { asm volatile("s_nop 1" ::"v"(a), "v"(b)); }
static __device__ __forceinline__ void qpb_fence(double a, double b, double c) {
    asm volatile("s_nop 1" ::"v"(a), "v"(b), "v"(c));
}
static __device__ __forceinline__ void qpb_fence(double a, double b, double c, double d) {
    asm volatile("s_nop 1" ::"v"(a), "v"(b), "v"(c), "v"(d));
}

// K sums / maxima over the 16 lanes of each row, stage-major (the K chains
// overlap); the result is in every lane of the row
template <int K> static __device__ __forceinline__ void qpb_rsum(double (&v)[K]) {
#pragma unroll
    for (int k = 0; k < K; k++) v[k] += qpb_dpp<0xB1>(v[k]);    // quad_perm [1,0,3,2]
#pragma unroll
    for (int k = 0; k < K; k++) v[k] += qpb_dpp<0x4E>(v[k]);    // quad_perm [2,3,0,1]
#pragma unroll
    for (int k = 0; k < K; k++) v[k] += qpb_dpp<0x141>(v[k]);   // row_half_mirror
#pragma unroll
    for (int k = 0; k < K; k++) v[k] += qpb_dpp<0x140>(v[k]);   // row_mirror
}
template <int K> static __device__ __forceinline__ void qpb_rmax(double (&v)[K]) {
#pragma unroll
    for (int k = 0; k < K; k++) v[k] = __builtin_fmax(v[k], qpb_dpp<0xB1>(v[k]));
#pragma unroll
    for (int k = 0; k < K; k++) v[k] = __builtin_fmax(v[k], qpb_dpp<0x4E>(v[k]));
#pragma unroll
    for (int k = 0; k < K; k++) v[k] = __builtin_fmax(v[k], qpb_dpp<0x141>(v[k]));
#pragma unroll
    for (int k = 0; k < K; k++) v[k] = __builtin_fmax(v[k], qpb_dpp<0x140>(v[k]));
}

// LDS of a row is touched by the lanes of one wave only: in-order per wave, so
// a compiler fence is all that is needed between a store and another lane's load
static __device__ __forceinline__ void qpb_wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

static __device__ __forceinline__ bool qpb_any(bool v) { return __builtin_amdgcn_ballot_w64(v) != 0; }

// XCD-aware block order: blocks b and b + 8 share an XCD (and its L2), so
// logical block (b % 8) * (nb / 8) + b / 8 gives each XCD a contiguous run of
// QPs -- the 64 QPs of a tile, whose values share cache lines, stay on one L2.
// The host pads the grid to a multiple of 8 (surplus blocks find no QPs).
static __device__ __forceinline__ long qpb_xcd_block() {
    const unsigned b = blockIdx.x, nb = gridDim.x;
    return (nb & 7) ? (long)b : (long)(b & 7) * (nb >> 3) + (b >> 3);
}


// Fused argmin of qpb_solve_best (lowest fval among optimal QPs, ties -> lowest
// index, as qpb_argmin).  Every wave of the grid arrives once with the best of its
// QPs: its partial goes out with agent-scope (write-through) stores, `s_waitcnt
// vmcnt(0)` makes it visible, then an agent-scope add on the arrival counter; the
// wave that arrives last reads every partial with agent-scope loads, reduces them
// and writes {fval, index}, and re-arms the counter.  No cache write-back or
// invalidate is needed (the partials never sit in a non-coherent L2 line).
static __device__ __forceinline__ double qpb_rl64(double v, int lane) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, lane);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), lane);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
static __device__ __forceinline__ bool qpb_better(double va, long ia, double vb, long ib) {
    return ia >= 0 && (ib < 0 || va < vb || (va == vb && ia < ib));
}
static __device__ __forceinline__ void qpb_argmin_arrive(const qpb_args &a, double bv, long bi) {
    const unsigned nw = (gridDim.x * blockDim.x) >> 6, w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    unsigned old = 0;
    if (lane == 0) {
        __hip_atomic_store(&a.part[2 * w], __builtin_bit_cast(unsigned long long, bv), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&a.part[2 * w + 1], (unsigned long long)bi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        old = __hip_atomic_fetch_add(a.ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    old = __builtin_amdgcn_readfirstlane(old);
    if (old != nw - 1) return;                 // wave-uniform: not the last arrival
    asm volatile("" ::: "memory");
    double v = __builtin_huge_val();
    long i = -1;
    // four partials per lane per round, all loads issued before the first compare
    // (one memory latency per 256 waves instead of one per 64)
    for (unsigned k0 = lane; k0 < nw; k0 += 256) {
        double pv[4];
        long pi[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const unsigned k = k0 + 64u * u < nw ? k0 + 64u * u : nw - 1;
            pv[u] = __builtin_bit_cast(double, __hip_atomic_load(&a.part[2 * k], __ATOMIC_RELAXED,
                                                                 __HIP_MEMORY_SCOPE_AGENT));
            pi[u] = (long)__hip_atomic_load(&a.part[2 * k + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
        for (int u = 0; u < 4; u++)
            if (k0 + 64u * u < nw && qpb_better(pv[u], pi[u], v, i)) { v = pv[u]; i = pi[u]; }
    }
    for (int o = 1; o < 64; o <<= 1) {
        const double ov = __shfl_xor(v, o, 64);
        const long oi = __shfl_xor(i, o, 64);
        if (qpb_better(ov, oi, v, i)) { v = ov; i = oi; }
    }
    if (lane == 0) {
        a.best[0] = v;
        a.best[1] = (double)i;
        __hip_atomic_store(a.ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

#endif  // QPB_ROW_COMMON_DONE

#ifndef QPB_ROW_COMMON_ONLY
#define NX QPB_NX
#define NZ QPB_NZ
#define NY QPB_NY
#define NY1 (NY > 0 ? NY : 1)
#define WPB (QPB_WG / 64)
#define ZH (NZ > 16)
// per-row LDS (doubles): staging Pd[NX*NX] Ad[NY1*NX] Gd[NZ*NX] | Tx[NX*NX]
// (columns of -L, one contiguous run per lane) | PR[NX*NX] (-P rows) | H0s[NX*NX]
// With QPB_R_ALIAS the loop's three areas overlay the staging area: the staged
// matrices are read only while the static slices are formed, before PR / H0s are
// written (program order within the wave: LDS operations of one wave stay in order),
// and Tx is first written by the first factor.  Per row 3 NX^2 (or the staging
// area, whichever is larger) instead of both: 7.1 -> 3.6 KB for the 12/20/6 QP.
#define EVEN(v) (((v) + 1) & ~1)
#define OFF_A (NX * NX)
// row stride of the per-lane rows parked in LDS (-P, H0, the -L transpose): lane c reads
// its row at c * RS, 16-byte pieces; RS = 2 mod 4 doubles puts the 16 lanes of a row on
// distinct bank quadruples (RS = NX = 12 pairs them up: 2-way conflicts on every read)
#ifndef QPB_R_RS
#define QPB_R_RS 1
#endif
#define RS (QPB_R_RS ? NX + ((2 - NX % 4) + 4) % 4 : NX)
#define OFF_G (OFF_A + NY1 * NX)
#define STG_END EVEN(OFF_G + NZ * NX)
#define OFF_T (QPB_R_ALIAS ? 0 : STG_END)
#define OFF_PR EVEN(OFF_T + NX * RS)
#define OFF_H0 EVEN(OFF_PR + NX * RS)
#define LOOP_END EVEN(OFF_H0 + NX * RS)
// QPB_R_GATHER: the row's vector area (z / w / v at 0..31, y at 32..47, x / dx at 48..63,
// a zero at 64), after everything else (never overlays the staging)
#define OFF_VEC (LOOP_END > STG_END ? LOOP_END : STG_END)
// + QPB_R_PIVLDS: a dump slot at 65 and the pivots D_k at 66..81
#define LDS_ROW (OFF_VEC + (QPB_R_GATHER || QPB_R_PIVLDS || QPB_R_RDLDS ? 82 : 0))
#ifndef QPB_R_GATHER_A
#define QPB_R_GATHER_A (QPB_AX_LEN + 2 <= QPB_AX_UNION)   // y rows' A products gathered when shorter
#endif
// QPB_R_SPLIT: per row, the iterate wave 0 forms (x y z0 z1 s0 s1: 6 x 16) and the residuals
// wave 1 forms (rx ry rz0 rz1 -P x: 5 x 16, the four row sums)
#define XCH_ROW (6 * 16 + 5 * 16 + 4)
#define LDS_ALL (WPB * 4 * LDS_ROW + (QPB_R_SPLIT ? 4 * XCH_ROW : 0))
#if QPB_R_SPLIT && (QPB_WARM || QPB_SERVE || defined(QPB_GROUP))
#error "the split row form is a cold batched kernel only"
#endif

// one logical block `lb` of the plan's batch (QPs 4 (lb WPB + wave) ..); qoff
// offsets the indices the fused argmin reports (the plan's first QP in a group)
static __device__ __forceinline__ void qpb_row_body(const qpb_args &a, long lb, long qoff, double *qpb_lds) {
    const int lane = threadIdx.x & 63, row = lane >> 4, c = lane & 15;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#if QPB_R_SPLIT
    const int role = wv;                       // 0: factor, solves, updates; 1: residuals
    const long q0 = lb * 4;                    // both waves of the workgroup: the same four QPs
    double *__restrict__ Xc = qpb_lds + WPB * 4 * LDS_ROW + row * XCH_ROW;
#else
    constexpr int role = 0;
    const long q0 = (lb * WPB + wv) * 4;
#endif
#if QPB_R_TIMING == 3
    double tph[6] = {0, 0, 0, 0, 0, 0};
    long tcy = (long)__builtin_readcyclecounter();
#define QPB_TM(k) { const long t2_ = (long)__builtin_readcyclecounter(); tph[k] += (double)(t2_ - tcy); tcy = t2_; }
#else
#define QPB_TM(k)
#endif
    if (q0 >= a.B) {                           // wave-uniform
        if (a.best) qpb_argmin_arrive(a, __builtin_huge_val(), -1);
        return;
    }
#if QPB_R_TIMING == 2
    const double t_rt0 = (double)__builtin_amdgcn_s_memrealtime(), t_cy0 = (double)__builtin_readcyclecounter();
#endif
    const long q = q0 + row;
    const bool valid = q < a.B;
    const long qc = valid ? q : a.B - 1;       // rows past the batch solve a copy, write nothing
    const long tile = qc >> 6;
    const int ql = (int)(qc & 63);
    double *__restrict__ Ls = qpb_lds + (wv * 4 + row) * LDS_ROW;
    const bool isx = c < NX, isy = c < NY, isz0 = c < NZ, isz1 = 16 + c < NZ;
    const int ix = isx ? c : NX - 1, iy = isy ? c : (NY > 0 ? NY - 1 : 0);
    const int iz0 = isz0 ? c : NZ - 1, iz1 = isz1 ? 16 + c : NZ - 1;
    constexpr double RDY = 1.0 / -1e-7;        // leaf y pivots: D = 0 regularised to -1e-7

    // ---- stage this QP's P, A, G as dense matrices in the row's LDS
    constexpr int NPL = (QPB_NNZP + 15) / 16, NGL = (QPB_NNZG + 15) / 16, NAL = (QPB_NNZA + 15) / 16;
    double vP[NPL], vG[NGL], vA[NAL > 0 ? NAL : 1];
    int iP[NPL], iP2[NPL], iG[NGL], iA[NAL > 0 ? NAL : 1];
    {
        const double *tP = a.P + tile * (QPB_NNZP * QPB_TSTR) + ql;
        const double *tG = a.G + tile * (QPB_NNZG * QPB_TSTR) + ql;
#pragma unroll
        for (int u = 0; u < NPL; u++) {
            const int k = c + 16 * u;
            const bool ok = k < QPB_NNZP;
            vP[u] = ok ? QPB_LDS(&tP[k * QPB_TSTR]) : 0.0;
            iP[u] = ok ? qpb_scP[k] : -1;
            iP2[u] = ok ? qpb_scP2[k] : -1;
        }
#pragma unroll
        for (int u = 0; u < NGL; u++) {
            const int k = c + 16 * u;
            const bool ok = k < QPB_NNZG;
            vG[u] = ok ? QPB_LDS(&tG[k * QPB_TSTR]) : 0.0;
            iG[u] = ok ? qpb_scG[k] : -1;
        }
#if NY > 0
        const double *tA = a.A + tile * (QPB_NNZA * QPB_TSTR) + ql;
#pragma unroll
        for (int u = 0; u < NAL; u++) {
            const int k = c + 16 * u;
            const bool ok = k < QPB_NNZA;
            vA[u] = ok ? QPB_LDS(&tA[k * QPB_TSTR]) : 0.0;
            iA[u] = ok ? qpb_scA[k] : -1;
        }
#endif
    }
    const double cx = isx ? QPB_LDS(&a.c[tile * (NX * QPB_TSTR) + c * QPB_TSTR + ql]) : 0.0;
    const double hz0 = isz0 ? QPB_LDS(&a.h[tile * (NZ * QPB_TSTR) + c * QPB_TSTR + ql]) : 0.0;
    const double hz1 = isz1 ? QPB_LDS(&a.h[tile * (NZ * QPB_TSTR) + (16 + c) * QPB_TSTR + ql]) : 0.0;
#if NY > 0
    const double by = isy ? QPB_LDS(&a.b[tile * (NY * QPB_TSTR) + c * QPB_TSTR + ql]) : 0.0;
#else
    const double by = 0.0;
#endif
#if QPB_R_ZF128
    for (int k = 2 * c; k < STG_END; k += 32)
        *reinterpret_cast<double2 *>(Ls + k) = double2{0.0, 0.0};   // 16-byte stores (STG_END, LDS_ROW even)
#else
    // unrolled (a compile-time trip count): the rolled loop cost ~7 instructions per store
#pragma unroll
    for (int i = 0; i < (STG_END + 15) / 16; i++)
        if (c + 16 * i < STG_END) Ls[c + 16 * i] = 0.0;
#endif
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
    QPB_TM(5);    // staging: global loads + LDS scatter
    const double *Pd = Ls, *Ad = Ls + OFF_A, *Gd = Ls + OFF_G;
    double *Tx = Ls + OFF_T, *PR = Ls + OFF_PR, *H0s = Ls + OFF_H0;
    // Pd[j*NX+i] = P(i,j) (both triangles); Ad[j*NY+l] = A(l,j); Gd[j*NZ+r] = G(r,j)

    // this lane's static slices, negated (every product is subtracted):
    //   x_c: -P(c,:), -G(:,c), -A(:,c);  z_c / z_{16+c}: -G(c,:), -G(16+c,:);  y_c: -A(c,:)
    // (-P rows and H0 rows are used once per iteration: parked in LDS, one
    // contiguous run per lane, read where they are needed)
    // Every load unconditional (the indices are clamped in range), then a select: a
    // load under `cond ? -X[i] : 0` became a branch with its own s_waitcnt -- some
    // 40 LDS round trips in series before the setup pass (QPB_R_SELSLICE=0: that form).
    double nGc[NZ], nAc[NY1], nGl[NX], nGh[ZH ? NX : 1], nAr[NX];
#if !QPB_R_SELSLICE
#pragma unroll
    for (int j = 0; j < NX; j++) {
        nGl[j] = isz0 ? -Gd[j * NZ + iz0] : 0.0;
        if constexpr (ZH) nGh[j] = isz1 ? -Gd[j * NZ + iz1] : 0.0;
        nAr[j] = isy ? -Ad[j * NY + iy] : 0.0;
    }
#pragma unroll
    for (int r = 0; r < NZ; r++) nGc[r] = isx ? -Gd[ix * NZ + r] : 0.0;
#pragma unroll
    for (int l = 0; l < NY1; l++) nAc[l] = (isx && NY > 0) ? -Ad[ix * NY + l] : 0.0;
#else
#pragma unroll
    for (int j = 0; j < NX; j++) {
        const double gl = Gd[j * NZ + iz0], ar = Ad[j * NY + iy];
        nGl[j] = isz0 ? -gl : 0.0;
        if constexpr (ZH) {
            const double gh = Gd[j * NZ + iz1];
            nGh[j] = isz1 ? -gh : 0.0;
        }
        nAr[j] = isy ? -ar : 0.0;
    }
#pragma unroll
    for (int r = 0; r < NZ; r++) {
        const double g = Gd[ix * NZ + r];
        nGc[r] = isx ? -g : 0.0;
    }
#pragma unroll
    for (int l = 0; l < NY1; l++) {
        const double av = Ad[ix * NY + (NY > 0 ? l : 0)];
        nAc[l] = (isx && NY > 0) ? -av : 0.0;
    }
    // pinned: otherwise the compiler keeps the loaded value and redoes the negation
    // and select (v_xor + v_mov) in front of every use inside the iteration loop
#pragma unroll
    for (int j = 0; j < NX; j++) {
        asm volatile("" : "+v"(nGl[j]), "+v"(nAr[j]));
        if constexpr (ZH) asm volatile("" : "+v"(nGh[j]));
    }
#pragma unroll
    for (int r = 0; r < NZ; r++) asm volatile("" : "+v"(nGc[r]));
#pragma unroll
    for (int l = 0; l < NY1; l++) asm volatile("" : "+v"(nAc[l]));
#endif
#if QPB_R_GATHER || QPB_R_PIVLDS || QPB_R_RDLDS
    // gathered products: per-lane slot pointers into the vector area and the negated
    // coefficients of this lane's terms (padding: the zero slot, coefficient 0)
    double *const Vr = Ls + OFF_VEC;
    const double *pXT[QPB_XT_LEN > 0 ? QPB_XT_LEN : 1], *pZ0[QPB_ZX0_LEN > 0 ? QPB_ZX0_LEN : 1],
        *pZ1[QPB_ZX1_LEN > 0 ? QPB_ZX1_LEN : 1], *pAX[QPB_AX_LEN > 0 ? QPB_AX_LEN : 1];
    double cXT[QPB_XT_LEN > 0 ? QPB_XT_LEN : 1], cZ0[QPB_ZX0_LEN > 0 ? QPB_ZX0_LEN : 1],
        cZ1[QPB_ZX1_LEN > 0 ? QPB_ZX1_LEN : 1], cAX[QPB_AX_LEN > 0 ? QPB_AX_LEN : 1];
    {
        auto load = [&](auto lc, const auto &slot, const auto &src, const double **pp, double *cc) {
#pragma unroll
            for (int k = 0; k < decltype(lc)::value; k++) {
                const int sr = src[c][k];
                pp[k] = Vr + slot[c][k];
                cc[k] = sr >= 0 ? -Ls[sr] : 0.0;
            }
        };
        load(qpb_ic<QPB_XT_LEN>{}, qpb_slot_XT, qpb_src_XT, pXT, cXT);
        load(qpb_ic<QPB_ZX0_LEN>{}, qpb_slot_ZX0, qpb_src_ZX0, pZ0, cZ0);
        load(qpb_ic<QPB_ZX1_LEN>{}, qpb_slot_ZX1, qpb_src_ZX1, pZ1, cZ1);
        load(qpb_ic<QPB_AX_LEN>{}, qpb_slot_AX, qpb_src_AX, pAX, cAX);
        Vr[64] = 0.0;
    }
    // sum of a gathered list onto acc (two accumulators)
    auto gsum = [&](auto lc, double acc, const double *const *pp, const double *cc) -> double {
        constexpr int L = decltype(lc)::value;
        double a2[2] = {acc, 0.0};
#pragma unroll
        for (int k = 0; k < L; k++) a2[k & 1] = __builtin_fma(cc[k], *pp[k], a2[k & 1]);
        return L > 1 ? a2[0] + a2[1] : a2[0];
    };
#endif
    // H0 = P (upper triangle, symmetrised) + 1e7 A'A (the leaf y rows folded into the x block)
    double nP[NX], H0[NX];
    {
#pragma unroll
        for (int j = 0; j < NX; j++) {
            nP[j] = -Pd[j * NX + ix];
            H0[j] = ix <= j ? Pd[j * NX + ix] : Pd[ix * NX + j];
#if !QPB_R_AADPP
#pragma unroll
            for (int l = 0; l < NY; l++) H0[j] = __builtin_fma(Ad[ix * NY + l], -RDY * Ad[j * NY + l], H0[j]);
#endif
        }
#if QPB_R_AADPP
        // += 1e7 A(l,j) A(l,c): row lane j's 1e7 A(l,j) by DPP broadcast (no LDS
        // reads); per H0[j] the same fma chain over l as the factor's reference order
#pragma unroll
        for (int l = 0; l < NY; l++) {
            const double qs = RDY * nAc[l];      // 1e7 A(l,c)
            qpb_fence(qs);
            qpb_for<0, NX>([&](auto jc) { qpb_fx<decltype(jc)::value>(H0[decltype(jc)::value], qs, -nAc[l]); });
        }
#endif
        if (!QPB_R_REGH0 && isx) {
#pragma unroll
            for (int j = 0; j < NX; j++) { PR[c * RS + j] = nP[j]; H0s[c * RS + j] = H0[j]; }
        }
#if QPB_R_PIVLDS
        // the -L area: the factor writes only its strict lower part, the rest stays 0
        // (the staging it overlays is dead: every static slice was read above)
#pragma unroll
        for (int i = 0; i < (NX * RS + 15) / 16; i++)
            if (c + 16 * i < NX * RS) Tx[c + 16 * i] = 0.0;
#endif
        qpb_wsync();
    }

    QPB_TM(0);
    double H[NX], rDd = 0.0;
    // factor with z diagonal kd: H = H0 + G' diag(w) G, w = -1/regularise(kd),
    // then the LDL' of H (rows of -L in H, 1/D in rDd), -L transposed into Lt.
    // Pivot regularisation off the pivot chain (QPB_R_LAZYREG): the fast pass takes
    // every 1/D as v_rcp_f64 + Newton and tracks min |D|; only when some pivot is
    // <= 1e-14 (ldl.c:273-274) is the factor redone with the regularised reciprocal
    // -- the same operations as the fast pass otherwise, so the same bits.
    // H = H0 + G' diag(w) G
    auto gwg = [&](double w0, double w1) {
#if GR_GWG
        // lane j gathers w_r for the G rows r of its own column and forms -G(r,j) w_r
        // (XG entries); the update of H(c, j) by row r then broadcasts lane j's entry
        // for r (position qpb_xtpos[r][j], a compile-time constant) against the lane's
        // own -G(r, c): += G(r,c) w_r G(r,j), one DPP FMA per structural (r, j)
        Vr[c] = w0;
        if constexpr (ZH) Vr[16 + c] = w1;
        qpb_wsync();
        double gw[QPB_XG_LEN > 0 ? QPB_XG_LEN : 1];
#pragma unroll
        for (int k = 0; k < QPB_XG_LEN; k++) gw[k] = cXT[k] * *pXT[k];
#pragma unroll
        for (int e = 0; e < NX; e++) H[e] = QPB_R_REGH0 ? H0[e] : H0s[ix * RS + e];
        qpb_for<0, NZ>([&](auto rc) {
            constexpr int r = decltype(rc)::value;
            qpb_for<0, NX>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                if constexpr (qpb_Gnz[r][j]) qpb_fxs<j>(H[j], gw[qpb_xtpos[r][j]], nGc[r]);
            });
        });
#else
#pragma unroll
        for (int e = 0; e < NX; e++) H[e] = QPB_R_REGH0 ? H0[e] : H0s[ix * RS + e];
#endif
#if GR_GWG
#elif QPB_R_GWG4
        // four rows at a time: the four products -G(r,c) w_r are formed (in their own
        // registers) before any of their DPP FMAs, so no FMA waits out the DPP operand
        // hazard behind the multiply that feeds it, and the rows do not serialise on
        // one temporary (round 3: 16 such waits of 2 wait states per factor)
        qpb_for<0, (NZ + 3) / 4>([&](auto qc) {
            constexpr int r0 = 4 * decltype(qc)::value;
            double cr[4];
            qpb_for<0, 4>([&](auto uc) {
                constexpr int r = r0 + decltype(uc)::value;
                if constexpr (r < NZ) {
                    const double wr = r < 16 ? qpb_nb<(r & 15)>(w0) : qpb_nb<(r & 15)>(w1);
                    cr[decltype(uc)::value] = nGc[r] * wr;       // -G(r,c) w_r
                } else {
                    cr[decltype(uc)::value] = 0.0;
                }
            });
            asm volatile("" : "+v"(cr[0]), "+v"(cr[1]), "+v"(cr[2]), "+v"(cr[3]));
            qpb_for<0, 4>([&](auto uc) {
                constexpr int r = r0 + decltype(uc)::value;
                if constexpr (r < NZ) {
                    qpb_for<0, NX>([&](auto jc) {
                        constexpr int j = decltype(jc)::value;
                        if constexpr (qpb_Gnz[r][j]) qpb_fxs<j>(H[j], nGc[r], cr[decltype(uc)::value]);
                    });
                }
            });
        });
#else
        qpb_for<0, NZ>([&](auto rc) {
            constexpr int r = decltype(rc)::value;
            const double wr = r < 16 ? qpb_nb<(r & 15)>(w0) : qpb_nb<(r & 15)>(w1);
            const double cr = nGc[r] * wr;        // -G(r,c) w_r
            qpb_for<0, NX>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                if constexpr (qpb_Gnz[r][j]) qpb_fxs<j>(H[j], nGc[r], cr);   // += G(r,c) w_r G(r,j)
            });
        });
#endif
    };
    // LDL' of H in place
    auto pivots = [&](auto regc) -> double {
        constexpr bool REG = decltype(regc)::value != 0;
        double dmin = __builtin_huge_val();
        // right-looking LDL' in natural order; the pivot recurrence is the
        // critical path: D_{k+1} comes from H'(k+1,k) and H'(k+1,k+1) with
        // exactly the operations lane k+1's own update performs
        double dpiv = qpb_nb<0>(H[0]);
        qpb_for<0, NX>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            double rd;
            if constexpr (REG || !QPB_R_LAZYREG) {
                rd = qpb_rcp_piv(dpiv);
            } else {
                rd = qpb_rcp_nr(dpiv);
                if constexpr (!QPB_R_PIVLDS && !QPB_R_RDLDS) dmin = __builtin_fmin(dmin, __builtin_fabs(dpiv));
            }
#if QPB_R_NLFIRST
            // -L(c,k) first: its multiply then sits two instructions ahead of the DPP
            // FMAs that read it (the lookahead's multiply and FMA in between) instead of
            // right before them behind a 2-wait-state pad
            double nl = H[k] * -rd;
            asm volatile("" : "+v"(nl));
#endif
#if QPB_R_PIVLDS || QPB_R_RDLDS
            if (c == 0) Vr[66 + k] = dpiv;        // D_k (one lane per row: a loop-invariant exec mask)
#endif
            if constexpr (k + 1 < NX) {
                const double h = qpb_nb<k + 1>(H[k]), hkk = qpb_nb<k + 1>(H[k + 1]);
#if QPB_R_H2
                dpiv = __builtin_fma(-(h * h), rd, hkk);   // h^2 off the chain: rcp -> 2 Newton FMAs -> this FMA
#else
                dpiv = __builtin_fma(h, h * -rd, hkk);
#endif
            }
#if !QPB_R_PIVLDS && !QPB_R_RDLDS
            rDd = c == k ? rd : rDd;
#endif
#if !QPB_R_NLFIRST
            const double nl = H[k] * -rd;        // -L(c,k)
#endif
            qpb_for<k + 1, NX>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                qpb_fxs<j>(H[j], H[k], nl);        // H(c,j) -= L(c,k) H(j,k)
            });
#if QPB_R_PIVLDS
            H[k] = nl;                              // -L(c,k) for c > k (others: masked at the store)
#else
            H[k] = c > k ? nl : 0.0;
#endif
        });
#if QPB_R_PIVLDS || QPB_R_RDLDS
        // this lane's 1/D: the same function of the same D_c the chain used
        qpb_wsync();
        const double dc = Vr[66 + ix];
        rDd = (REG || !QPB_R_LAZYREG) ? qpb_rcp_piv(dc) : qpb_rcp_nr(dc);
        if constexpr (!REG && QPB_R_LAZYREG) dmin = isx ? __builtin_fabs(dc) : __builtin_huge_val();
#endif
        return dmin;
    };
    auto factor_core = [&](double w0, double w1, auto regc) -> double {
        gwg(w0, w1);
        return pivots(regc);
    };
    // the factor; early: H = H0 + G'WG was formed already (QPB_R_EARLYGWG)
    auto factor = [&](double w0, double w1, bool early = false) {
        const double dmin = early ? pivots(qpb_ic<0>{}) : factor_core(w0, w1, qpb_ic<0>{});
        if (QPB_R_LAZYREG && qpb_any(dmin <= 1e-14)) factor_core(w0, w1, qpb_ic<1>{});   // wave-uniform, rare
        // column c of -L, contiguous for lane c: Tx[c*NX + k] = -L(k, c)
#if QPB_R_PIVLDS
        // strict lower part only (e < c): the rest of the area is 0 from the prologue on
#pragma unroll
        for (int e = 0; e < NX; e++) *((isx && e < c) ? &Tx[e * RS + c] : Vr + 65) = H[e];
#else
        if (isx) {
#pragma unroll
            for (int e = 0; e < NX; e++) Tx[e * RS + c] = H[e];
        }
#endif
        qpb_wsync();
    };

    // solve K [dx; dy; dz] = [bx; by; bz] with the current factor and w
    auto solve = [&](double w0, double w1, double bx, double byv, double bz0, double bz1, double &dx, double &dy,
                     double &dz0, double &dz1) {
        const double v0 = -w0 * bz0, v1 = -w1 * bz1, yr = RDY * byv;   // leaf eliminations
#if GR_SLV
        // the leaf rows' values to the vector area; each x lane gathers its G' / A' terms
        Vr[c] = v0;
        if constexpr (ZH) Vr[16 + c] = v1;
        if constexpr (NY > 0) Vr[32 + c] = yr;
        qpb_wsync();
        double t = gsum(qpb_ic<QPB_XT_LEN>{}, bx, pXT, cXT);
#else
        qpb_fence(v0, v1, yr);
        double ta[4] = {bx, 0.0, 0.0, 0.0};
        qpb_for<0, NZ>([&](auto rc) {
            constexpr int r = decltype(rc)::value;
            qpb_fx<(r & 15)>(ta[r & 3], r < 16 ? v0 : v1, nGc[r]);
        });
        qpb_for<0, NY>([&](auto lc) {
            constexpr int l = decltype(lc)::value;
            qpb_fx<l>(ta[(NZ + l) & 3], yr, nAc[l]);
        });
        double t = (ta[0] + ta[1]) + (ta[2] + ta[3]);
#endif
#if QPB_R_PIVLDS
        double Lf[NX];                              // row c of -L (column c of the area): 0 from k = c on
#pragma unroll
        for (int k = 0; k < NX; k++) Lf[k] = Tx[k * RS + ix];
        qpb_for<0, NX>([&](auto kc) { qpb_fxd<decltype(kc)::value>(t, Lf[decltype(kc)::value]); });
#else
        qpb_for<0, NX>([&](auto kc) { qpb_fxd<decltype(kc)::value>(t, H[decltype(kc)::value]); });
#endif
        t *= rDd;
        double Lt[NX];
#pragma unroll
        for (int k = 0; k < NX; k++) Lt[k] = Tx[ix * RS + k];
        qpb_for<0, NX>([&](auto kc) {
            constexpr int k = NX - 1 - decltype(kc)::value;
            qpb_fxd<k>(t, Lt[k]);
        });
        dx = t;
#if GR_SLX
        // dx to the vector area; z (and y) rows gather their G (A) row terms
        Vr[48 + c] = t;
        qpb_wsync();
        double gy = 0.0;
        if constexpr (NY > 0 && !QPB_R_GATHER_A) {
            qpb_fence(t);
            qpb_for<0, NX>([&](auto jc) { qpb_fx<decltype(jc)::value>(gy, t, nAr[decltype(jc)::value]); });
        }
        const double g0 = gsum(qpb_ic<QPB_ZX0_LEN>{}, 0.0, pZ0, cZ0);
        const double g1 = ZH ? gsum(qpb_ic<QPB_ZX1_LEN>{}, 0.0, pZ1, cZ1) : 0.0;
        if constexpr (NY > 0 && QPB_R_GATHER_A) gy = gsum(qpb_ic<QPB_AX_LEN>{}, 0.0, pAX, cAX);
#else
        qpb_fence(t);
        double g0 = 0.0, g1 = 0.0, gy = 0.0;
        qpb_for<0, NX>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            qpb_fx<j>(g0, t, nGl[j]);
            if constexpr (ZH && qpb_ghmask[j]) qpb_fx<j>(g1, t, nGh[j]);
            if constexpr (NY > 0) qpb_fx<j>(gy, t, nAr[j]);
        });
#endif
        dz0 = -w0 * (bz0 + g0);                   // g = -G dx
        dz1 = -w1 * (bz1 + g1);
        dy = RDY * (byv + gy);
    };

    // ---- kkt_initialize (Auxilary.c:992-1089) as iteration -1, then the
    // QP_SOLVE loop (qpSWIFT.c:502-602); the wave runs until all four rows stop
    double x = 0.0, y = 0.0, s0 = 1.0, s1 = 1.0, z0 = 1.0, z1 = 1.0;
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
    // the host's block (KernelArgs::win, QP 0): never a line this wave wrote
    const double *wi = a.win;
    if (isx) x = QPB_LDS(&wi[c]);
#if NY > 0
    if (isy) y = QPB_LDS(&wi[NX + c]);
#endif
    if (isz0) { z0 = QPB_LDS(&wi[NX + NY + c]); s0 = QPB_LDS(&wi[NX + NY + NZ + c]); }
    if (isz1) { z1 = QPB_LDS(&wi[NX + NY + 16 + c]); s1 = QPB_LDS(&wi[NX + NY + NZ + 16 + c]); }
    const int *wfl = reinterpret_cast<const int *>(wi + NX + NY + 2 * NZ);
    const long it0 = QPB_LDS(&wfl[1]);
    const int flag0 = QPB_LDS(&wfl[0]);
    sigma = QPB_LDS(&wi[NX + NY + 2 * NZ + 1]);
#else
    if (isx) x = QPB_LDS(&a.x[tile * (NX * 64) + c * 64 + ql]);
#if NY > 0
    if (isy) y = QPB_LDS(&a.y[tile * (NY * 64) + c * 64 + ql]);
#endif
    if (isz0) { z0 = QPB_LDS(&a.z[tile * (NZ * 64) + c * 64 + ql]); s0 = QPB_LDS(&a.s[tile * (NZ * 64) + c * 64 + ql]); }
    if (isz1) { z1 = QPB_LDS(&a.z[tile * (NZ * 64) + (16 + c) * 64 + ql]); s1 = QPB_LDS(&a.s[tile * (NZ * 64) + (16 + c) * 64 + ql]); }
    const long it0 = QPB_LDS(&a.iters[qc]);   // IterationCount the QP enters with
    const int flag0 = QPB_LDS(&a.flag[qc]);   // stats->Flag it enters with (QP_FATAL after setup)
    sigma = QPB_LDS(&a.sig[qc]);
#endif
    it = 0;
    double sigf = sigma;       // options->sigma when this row's loop ends (a frozen row's own
                               // sigma keeps being recomputed while the rest of the wave runs)
#define QPB_SIGF sigf = sigma
    // the drop-in's timers and verbose trace (KernelArgs::trace, qpb_codegen.hpp):
    // s_memrealtime ticks in the factorisations and in factor + solves, and the
    // statistics the reference prints per iteration (qpSWIFT.c:506-517, 598-600)
    double *const trc = (a.trace && valid && c == 0) ? a.trace + qc * QPB_TRACE_STRIDE : nullptr;
    long t_fac = 0, t_kkt = 0, n_top = 0, n_it = 0;
#define QPB_CLK() ((long)__builtin_amdgcn_s_memrealtime())
#else
    constexpr long it0 = 0;
    constexpr int flag0 = 3;
#define QPB_SIGF (void)0
#endif
    int flag = flag0;
    for (;;) {
        if ((QPB_WARM || it >= 0) && it >= a.maxit) {
            // qpSWIFT.c:598-601: QP_MAXIT only when IterationCount == maxit
            if (act) { itq = it0 + it; flag = (!QPB_WARM || itq == a.maxit) ? 2 : flag0; QPB_SIGF; }
            break;
        }
        // updatekktmatrix (Auxilary.c:211-215): z diagonal -s/z (-I at setup, s = z = 1)
        const double rzi0 = qpb_rcp(z0), rzi1 = qpb_rcp(z1);
        const double rsi0 = __builtin_amdgcn_rcp(s0), rsi1 = __builtin_amdgcn_rcp(s1);   // step length
        const double kd0 = isz0 ? -s0 * rzi0 : -1.0, kd1 = isz1 ? -s1 * rzi1 : -1.0;
        const double w0 = -qpb_rcp_reg(kd0), w1 = -qpb_rcp_reg(kd1);
        // residuals (Auxilary.c:745-786)
        double tp, ry, rz0, rz1, rx, red[4];
        auto residuals = [&](bool early_gwg) {
            qpb_fence(x, y, z0, z1);
            double nPr[NX];
            tp = 0.0; ry = by; rz0 = hz0 - s0; rz1 = hz1 - s1;
#pragma unroll
            for (int j = 0; j < NX; j++) nPr[j] = QPB_R_REGH0 ? nP[j] : PR[ix * RS + j];
#if GR_RES
            // x, z, y to the vector area; z (y) rows gather their G (A) row terms, x rows
            // their G' / A' column terms; -P x (dense) stays a DPP product, issued while
            // the gathers are in flight
            Vr[48 + c] = x;
            Vr[c] = z0;
            if constexpr (ZH) Vr[16 + c] = z1;
            if constexpr (NY > 0) Vr[32 + c] = y;
            qpb_wsync();
            qpb_for<0, NX>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                if constexpr (NY > 0 && !QPB_R_GATHER_A) qpb_fx<j>(ry, x, nAr[j]);
                qpb_fx<j>(tp, x, nPr[j]);              // -P x
            });
            rz0 = gsum(qpb_ic<QPB_ZX0_LEN>{}, rz0, pZ0, cZ0);
            if constexpr (ZH) rz1 = gsum(qpb_ic<QPB_ZX1_LEN>{}, rz1, pZ1, cZ1);
            if constexpr (NY > 0 && QPB_R_GATHER_A) ry = gsum(qpb_ic<QPB_AX_LEN>{}, ry, pAX, cAX);
            rx = gsum(qpb_ic<QPB_XT_LEN>{}, -cx, pXT, cXT) + tp;
#else
            qpb_for<0, NX>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                qpb_fx<j>(rz0, x, nGl[j]);
                if constexpr (ZH && qpb_ghmask[j]) qpb_fx<j>(rz1, x, nGh[j]);
                if constexpr (NY > 0) qpb_fx<j>(ry, x, nAr[j]);
                qpb_fx<j>(tp, x, nPr[j]);              // -P x
            });
            double ra[4] = {-cx, 0.0, 0.0, 0.0};
            qpb_for<0, NZ>([&](auto rc) {
                constexpr int r = decltype(rc)::value;
                qpb_fx<(r & 15)>(ra[r & 3], r < 16 ? z0 : z1, nGc[r]);
            });
            qpb_for<0, NY>([&](auto lc) {
                constexpr int l = decltype(lc)::value;
                qpb_fx<l>(ra[(NZ + l) & 3], y, nAc[l]);
            });
            rx = ((ra[0] + ra[1]) + (ra[2] + ra[3])) + tp;
#endif
            red[0] = isx ? rx * rx : 0.0;
            red[1] = isy ? ry * ry : 0.0;
            red[2] = (isz0 ? rz0 * rz0 : 0.0) + (isz1 ? rz1 * rz1 : 0.0);
            red[3] = (isz0 ? s0 * z0 : 0.0) + (isz1 ? s1 * z1 : 0.0);
            if (early_gwg) gwg(w0, w1);   // independent of the residuals: issued into the reductions' latency
            qpb_rsum<4>(red);
        };
#if QPB_R_SPLIT
        if (role == 1) {
            residuals(false);
            Xc[96 + c] = rx; Xc[112 + c] = ry; Xc[128 + c] = rz0; Xc[144 + c] = rz1; Xc[160 + c] = tp;
            if (c == 0) { Xc[176] = red[0]; Xc[177] = red[1]; Xc[178] = red[2]; Xc[179] = red[3]; }
        } else {
            factor(w0, w1);              // while wave 1 forms the residuals (wasted on the last pass)
        }
        __syncthreads();
        if (role == 0) {
            rx = Xc[96 + c]; ry = Xc[112 + c]; rz0 = Xc[128 + c]; rz1 = Xc[144 + c]; tp = Xc[160 + c];
            red[0] = Xc[176]; red[1] = Xc[177]; red[2] = Xc[178]; red[3] = Xc[179];
        }
#else
        if (QPB_WARM || it >= 0) {
            residuals(QPB_R_EARLYGWG && QPB_R_LATEFAC);
        } else {
            // kkt_initialize's pass (iteration -1) has no exit test: no residuals
            rx = ry = rz0 = rz1 = tp = 0.0;
            red[0] = red[1] = red[2] = 0.0;
            red[3] = 1.0;
        }
#endif
        const double sz = red[3];
        const double rsz = qpb_rcp(sz);            // formrho's 1 / s'z, off the predictor's chain
        QPB_TM(1);
#if !QPB_R_LATEFAC && !QPB_R_SPLIT
        // the factor does not depend on the residuals: formed before the exit
        // test (wasted on a row's last iteration), overlapping the reductions
        factor(w0, w1);
        QPB_TM(2);
#endif
        bool pc = true;
        double mu = 0.0;
        if (QPB_WARM || it >= 0) {
            const double mu_it = sz * (1.0 / NZ);
#if QPB_WARM
            {
                double fq[1] = {isx ? x * __builtin_fma(-0.5, tp, cx) : 0.0};
                qpb_rsum<1>(fq);
                if (trc && act && it < QPB_TRACE_MAX) {
                    double *e = trc + 4 + 7 * it;
                    e[0] = fq[0]; e[1] = __builtin_sqrt(red[0]); e[2] = NY > 0 ? __builtin_sqrt(red[1]) : 0.0;
                    e[3] = __builtin_sqrt(red[2]); e[4] = mu_it;
                    n_top = it + 1;
                }
            }
#endif
            if (act) {
                fv = isx ? x * __builtin_fma(-0.5, tp, cx) : 0.0;      // objective (Auxilary.c:1133-1141)
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
#if QPB_R_LATEFAC && !QPB_R_SPLIT
        // factor after the exit test: the wave's last pass skips it
#if QPB_WARM
        const long tf0 = QPB_CLK();
#endif
        factor(w0, w1, QPB_R_EARLYGWG != 0);
#if QPB_WARM
        { const long d_ = QPB_CLK() - tf0; t_fac += d_; t_kkt += d_; }
#endif
        QPB_TM(2);
#endif
        if (!pc) sigma = a.sigma_d;
        double cc0 = sigma * mu, cc1 = sigma * mu;
        double dx, dy, dz0, dz1, dsl0, dsl1;
        auto step_length = [&]() {
            // alpha = min over d < 0 of v/(-d) == 1 / max(-d/v); 1 if none (Auxilary.c:359-393)
            double bm[2] = {__builtin_fmax(isz0 ? -dsl0 * rsi0 : 0.0, isz1 ? -dsl1 * rsi1 : 0.0),
                            __builtin_fmax(isz0 ? -dz0 * rzi0 : 0.0, isz1 ? -dz1 * rzi1 : 0.0)};
            bm[0] = __builtin_fmax(bm[0], 0.0);
            bm[1] = __builtin_fmax(bm[1], 0.0);
            qpb_rmax<2>(bm);
            ap = bm[0] > 1e-10 ? __builtin_amdgcn_rcp(bm[0]) : 1.0;
            ad = bm[1] > 1e-10 ? __builtin_amdgcn_rcp(bm[1]) : 1.0;
        };
#if QPB_R_SPLIT
        // wave 0's iterate to wave 1 (its next residuals)
        auto exchange = [&]() {
            if (role == 0) {
                Xc[c] = x; Xc[16 + c] = y; Xc[32 + c] = z0; Xc[48 + c] = z1; Xc[64 + c] = s0; Xc[80 + c] = s1;
            }
            __syncthreads();
            if (role == 1) {
                x = Xc[c]; y = Xc[16 + c]; z0 = Xc[32 + c]; z1 = Xc[48 + c]; s0 = Xc[64 + c]; s1 = Xc[80 + c];
            }
        };
#endif
        if (!QPB_WARM && it < 0) {
            // setup solve, rhs [-c; b; h] (Auxilary.c:1010-1040): x0, y0; then
            // s0, z0 from r = h - G x0 = -dz (w = 1 exactly here)
          if (role == 0) {
            solve(w0, w1, -cx, by, hz0, hz1, dx, dy, dz0, dz1);
            x = isx ? dx : 0.0;
            y = isy ? dy : 0.0;
            const double zi0 = -dz0, zi1 = -dz1;
            double lh[2] = {__builtin_fmax(isz0 ? -zi0 : -1e300, isz1 ? -zi1 : -1e300),
                            __builtin_fmax(isz0 ? zi0 : -1e300, isz1 ? zi1 : -1e300)};
            qpb_rmax<2>(lh);
            const double sh = lh[0], hi = lh[1];    // sh = -min(zi)
            s0 = sh < 0 ? zi0 : zi0 + (1 + sh);
            s1 = sh < 0 ? zi1 : zi1 + (1 + sh);
            z0 = hi < 0 ? -zi0 : -zi0 + (1 + hi);
            z1 = hi < 0 ? -zi1 : -zi1 + (1 + hi);
            if (!isz0) { s0 = 1.0; z0 = 1.0; }
            if (!isz1) { s1 = 1.0; z1 = 1.0; }
          }
#if QPB_R_SPLIT
            exchange();
#endif
            it = 0;
            QPB_TM(0);
            continue;
        }
      if (role == 0) {
        if (qpb_any(act && pc)) {
            // predictor (kktsolve_1, Auxilary.c:471-515), ds = -s.*z
#if QPB_WARM
            const long ts0 = QPB_CLK();
#endif
            solve(w0, w1, rx, ry, rz0 + s0, rz1 + s1, dx, dy, dz0, dz1);
#if QPB_WARM
            t_kkt += QPB_CLK() - ts0;
#endif
            dsl0 = -s0 * __builtin_fma(dz0, rzi0, 1.0);
            dsl1 = -s1 * __builtin_fma(dz1, rzi1, 1.0);
            step_length();
            double rr[1] = {(isz0 ? (s0 + ap * dsl0) * (z0 + ad * dz0) : 0.0) +
                            (isz1 ? (s1 + ap * dsl1) * (z1 + ad * dz1) : 0.0)};
            qpb_rsum<1>(rr);
            const double rho = rr[0] * rsz;             // formrho
            const double r1 = 1 > rho ? rho : 1;
            const double cube = r1 * r1 * r1;
            if (pc) {
                sigma = a.sigma_d < cube ? cube : a.sigma_d;
                cc0 = __builtin_fma(-dsl0, dz0, sigma * mu);
                cc1 = __builtin_fma(-dsl1, dz1, sigma * mu);
            }
        }
        QPB_TM(3);
        // corrector / centering (kktsolve_2, Auxilary.c:524-564)
#if QPB_WARM
        const long tc0 = QPB_CLK();
#endif
        solve(w0, w1, rx, ry, __builtin_fma(-cc0, rzi0, rz0 + s0), __builtin_fma(-cc1, rzi1, rz1 + s1), dx, dy, dz0,
              dz1);
#if QPB_WARM
        t_kkt += QPB_CLK() - tc0;
#endif
        dsl0 = __builtin_fma(__builtin_fma(-s0, dz0, cc0), rzi0, -s0);
        dsl1 = __builtin_fma(__builtin_fma(-s1, dz1, cc1), rzi1, -s1);
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
            if (isx) x = __builtin_fma(dx, ap, x);
            if (isy) y = __builtin_fma(dy, ad, y);
            if (isz0) { s0 = __builtin_fma(dsl0, ap, s0); z0 = __builtin_fma(dz0, ad, z0); }
            if (isz1) { s1 = __builtin_fma(dsl1, ap, s1); z1 = __builtin_fma(dz1, ad, z1); }
        }
      }   // role == 0
#if QPB_R_SPLIT
        exchange();
#endif
        it++;
        QPB_TM(4);
    }
    double fr[1] = {fv};
    qpb_rsum<1>(fr);
    // fused argmin first: the arrival's store -> s_waitcnt vmcnt(0) -> atomic round
    // trip then waits for the wave's partial only, not for its output stores
    if (a.best && role != 0) qpb_argmin_arrive(a, __builtin_huge_val(), -1);   // QPB_R_SPLIT's wave 1
    if (a.best && role == 0) {
        // this wave's best: rows are QPs (fval / flag uniform within a row)
        double bv = __builtin_huge_val();
        long bi = -1;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const double v = qpb_rl64(fr[0], 16 * r);
            const int f = __builtin_amdgcn_readlane(valid && flag == 0 ? 0 : 1, 16 * r);
            if (f == 0 && qpb_better(v, qoff + q0 + r, bv, bi)) { bv = v; bi = qoff + q0 + r; }
        }
        qpb_argmin_arrive(a, bv, bi);
    }
    // ---- outputs (tiled SoA)
    if (valid && role == 0) {
        if (isx) QPB_STS(&a.x[tile * (NX * QPB_TSTR) + c * QPB_TSTR + ql], x);
#if NY > 0
        if (isy) QPB_STS(&a.y[tile * (NY * QPB_TSTR) + c * QPB_TSTR + ql], y);
#endif
        if (isz0) {
            QPB_STS(&a.z[tile * (NZ * QPB_TSTR) + c * QPB_TSTR + ql], z0);
            QPB_STS(&a.s[tile * (NZ * QPB_TSTR) + c * QPB_TSTR + ql], s0);
        }
        if (isz1) {
            QPB_STS(&a.z[tile * (NZ * QPB_TSTR) + (16 + c) * QPB_TSTR + ql], z1);
            QPB_STS(&a.s[tile * (NZ * QPB_TSTR) + (16 + c) * QPB_TSTR + ql], s1);
        }
        if (c == 0) {
            QPB_STS(&a.flag[q], flag);
            QPB_STS(&a.iters[q], (int)itq);
            QPB_STS(&a.fval[q], fr[0]);
#if QPB_WARM
            QPB_STS(&a.sig[q], sigf);
            if (trc) { trc[0] = (double)t_fac; trc[1] = (double)t_kkt; trc[2] = (double)n_top; trc[3] = (double)n_it; }
#else
            // options->sigma after a cold QP_SOLVE: this row's sigma when the wave stops --
            // its own final sigma for the wave's last row to finish, e.g. the drop-in's B = 1
            if (a.sig) QPB_STS(&a.sig[q], sigma);
#endif
#if QPB_R_TIMING == 3
            QPB_TM(4);
            if (a.stats) {
                double *o = a.stats + tile * 384 + ql;
                for (int k = 0; k < 6; k++) o[64 * k] = tph[k];
            }
#else
            if (a.stats && QPB_R_TIMING != 2) {
                double *o = a.stats + tile * 6 * QPB_TSTR + ql;
                o[0] = __builtin_sqrt(st_rx2); o[QPB_TSTR] = __builtin_sqrt(st_ry2); o[2 * QPB_TSTR] = __builtin_sqrt(st_rz2);
                o[3 * QPB_TSTR] = st_mu; o[4 * QPB_TSTR] = ap; o[5 * QPB_TSTR] = ad;
            }
#if QPB_R_TIMING == 2
            if (a.stats) {
                double *o = a.stats + tile * 384 + ql;
                o[0] = t_rt0; o[64] = (double)__builtin_amdgcn_s_memrealtime();
                o[128] = t_cy0; o[192] = (double)__builtin_readcyclecounter(); o[256] = (double)itq;
                const unsigned hwid = __builtin_amdgcn_s_getreg(4 | (31 << 11));
                const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (31 << 11));
                o[320] = (double)hwid + 4294967296.0 * (double)(xcc & 0xf);
            }
#endif
#endif  // QPB_R_TIMING == 3
        }
    }
}

#ifndef QPB_R_WPE
#define QPB_R_WPE 1       // waves per SIMD the register allocation must allow (2: <= 256 VGPRs + AGPRs)
#endif
#ifndef QPB_GROUP
#if QPB_SERVE
// persistent form (the drop-in's QP_SOLVE, qpb::serve_ex): one wave, QP 0, one
// solve per request posted in the mailbox (qpb_serve_wait, runtime prelude)
extern "C" __global__ void __launch_bounds__(QPB_WG, QPB_R_WPE)
QPB_KERNEL_NAME(qpb_args a, qpb_mailbox *mb, unsigned long long last, unsigned long long idle,
                unsigned long long life) {
    __shared__ __attribute__((aligned(16))) double qpb_lds[WPB * 4 * LDS_ROW];
    const unsigned long long t_launch = __builtin_amdgcn_s_memrealtime();
    unsigned long long t_seen = 0;
    while (qpb_serve_wait(mb, &last, idle, life, t_launch, &t_seen)) {
        qpb_row_body(a, 0, 0, qpb_lds);
        qpb_serve_done(mb, last, t_seen);
        if (life == 0) break;       // one request per launch (the default; the host pre-launches the next)
    }
}
#else
extern "C" __global__ void __launch_bounds__(QPB_WG, QPB_R_WPE) QPB_KERNEL_NAME(qpb_args a) {
    __shared__ __attribute__((aligned(16))) double qpb_lds[LDS_ALL];
    qpb_row_body(a, qpb_xcd_block(), 0, qpb_lds);
}
#endif
#endif
#undef QPB_TM
#undef QPB_SIGF
#undef QPB_CLK
#endif  // QPB_ROW_COMMON_ONLY

// qpb_codegen.hpp -- plan -> one straight-line HIP kernel (gfx950).
#pragma once

#include <string>

#include "qpb_plan.hpp"

namespace qpb {

struct GenOptions {
    // exact = true: every floating-point operation is issued in the reference's
    // order with IEEE division and no FMA contraction, so results are
    // bit-identical to qpSWIFT (and to the oracle).  exact = false: FMA
    // contraction, reciprocal-multiply for the pivots and 1/z, division-free step
    // length search (results within rounding of the reference).
    bool exact = false;
    int wg = 256;             // threads per workgroup (one QP per lane)
    int waves_per_eu = 1;     // __launch_bounds__ minimum waves per SIMD
    // Fast mode: which matrix inputs are staged in LDS (each lane owns a private
    // LDS column: no barriers).  0 = none, 1 = A and G, 2 = P, A and G.
    int lds_mode = 1;
    int park_z = 1;           // mode 4: also keep z and 1/z in LDS
};

// Kernel argument block; identical layout in the generated device code.
struct KernelArgs {
    const double *P, *A, *G, *c, *h, *b;   // tiled SoA (see qpswift_hip.h)
    double *x, *y, *z, *s;                  // tiled SoA outputs
    int *flag, *iters;                      // [B]
    double *fval;                           // [B]
    double *stats;                          // optional, tiled with 6 values per QP
    long B;
    double tol;                             // reltol / sqrt(3) (qpSWIFT.c:521)
    double abstol, sigma_d;
    long maxit;
    const void *tab = nullptr;              // tree kernel only: plan tables on the device
    double *best = nullptr;                 // row kernel: fused argmin output {fval, index}
    unsigned long long *part = nullptr;     //   per-wave partials
    unsigned *ctr = nullptr;                //   arrival counter (zero between launches)
    // warm solve (qpb_solve_warm; QP_SOLVE called again on the same QP object,
    // qpSWIFT.c:502-596): warm = 0 is cold (kkt_initialize first); warm = 1
    // continues every QP from x, y, z, s, iters, flag as they are in the output
    // arrays and from sigma = sig[q] (options->sigma).  sig (when not NULL)
    // receives the last sigma.
    double *sig = nullptr;
    long warm = 0;
    // warm variant only (the drop-in's QP_SOLVE): per QP q, at trace + q * QPB_TRACE_STRIDE,
    // [0] s_memrealtime ticks (100 MHz) in the factorisations (LDL_numeric), [1] in the KKT
    // factor + solves (kktsolve_1 / _2), [2] loop-top evaluations recorded, [3] iterations
    // recorded, then per loop pass i < QPB_TRACE_MAX: fval, n_rx, n_ry, n_rz, n_mu
    // (before the exit test) and alpha_p, alpha_d (after the update) at [4 + 7 i ..]
    double *trace = nullptr;
    // persistent (QPB_SERVE) warm variants, one QP: the state to continue from as one
    // contiguous block the host writes and the kernel only reads -- x[n] y[p] z[m] s[m],
    // {flag, iters} (two ints in one double), sigma -- instead of the output slots.  A
    // resident wave re-reading a host-memory line it wrote itself during an earlier
    // request was measured to get its own old bytes, not the host's later write
    // (DESIGN_HISTORY §4i); NULL: read the output slots (launched kernels)
    const double *win = nullptr;
};
constexpr int QPB_TRACE_MAX = 256;
constexpr long QPB_TRACE_STRIDE = 4 + 7L * QPB_TRACE_MAX;

std::string kernel_name(const Plan &pl, const GenOptions &opt);
// Pick workgroup size / LDS placement for a plan (fast mode): keep every matrix
// input on-chip when it fits the 160 KiB LDS of a CU.
GenOptions choose_options(const Plan &pl, bool exact);
std::string generate_kernel(const Plan &pl, const GenOptions &opt);
std::string kernel_name_of(const std::string &src);   // name inside generated source

}  // namespace qpb

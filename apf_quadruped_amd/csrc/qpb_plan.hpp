// qpb_plan.hpp -- host-side plan for one QP sparsity pattern.
//
// A plan is everything about a qpSWIFT solve that depends only on the sparsity
// pattern (and the KKT ordering), never on values:
//   * the full symmetric KKT CSC [P A' G'; A 0 0; G 0 -I] exactly as the
//     reference assembles it (dogbot_controller/src/qpSWIFT/Auxilary.c:71-181),
//     every slot tagged with the input value it comes from;
//   * the KKT permutation: the caller's, the reference's own AMD ordering
//     (qpb_amd.cpp; what qpSWIFT computes every tick when Permut = NULL,
//     qpSWIFT.c:416-440), or one of our orderings (leaves first / min degree);
//   * the elimination tree and column counts (ldl.c:187-240);
//   * the exact operation schedule of the up-looking LDL' numeric factorisation
//     (ldl.c:253-326), obtained by executing its index logic symbolically.
// The code generator (qpb_codegen.cpp) turns a plan into one straight-line HIP
// kernel in which every index is a compile-time constant.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace qpb {

// Where one KKT CSC slot's value comes from.
enum class Src : uint8_t { P, A, G, NegOne, ZDiag };

struct Slot {
    int32_t row;
    Src kind;
    int32_t idx;   // index into the P / A / G value array, or the z index for ZDiag
};

struct Pattern {
    long rows = 0, cols = 0;
    std::vector<long> jc, ir;
    long nnz() const { return jc.empty() ? 0 : jc[cols]; }
};

// One step of the LDL' numeric schedule (ldl.c:276-322).
enum class FacOp : uint8_t {
    RowBegin,   // a = k
    Scatter,    // Y[a] += K[slot b]                 (ldl.c:290)
    Update,     // Y[a] -= L[b] * Y[c]               (ldl.c:311)
    NewL,       // L[b] = Y[a] / D[a]; D[k] -= L[b]*Y[a] (ldl.c:313-316), a = i
    RowEnd,     // D[k] = Y[k] first, regularise     (ldl.c:300, 319-320)
};

struct FacStep {
    FacOp op;
    int32_t a, b, c;
};

enum PModes : int { P_FULL = 0, P_UPPER = 1 };

// Ordering of the KKT rows when the caller gives no permutation.
enum Ordering : int {
    ORDER_CALLER = 0,   // caller's permutation (qpSWIFT's Permut argument)
    ORDER_MINDEG = 1,   // own exact minimum degree, lowest-index ties
    ORDER_AMD = 2,      // the reference's AMD (amd_l_order with amd_l_defaults): Permut = NULL
    ORDER_LEAVES = 3,   // own: z rows, y rows, then x in natural order (small QPs)
    ORDER_OWN = 4,      // request only: ORDER_LEAVES for n, p <= 64, m <= 256 (the wave kernel's
                        // range: its dense block is then the x block) and for multi-stage patterns
                        // (band_shape: the band kernel's elimination), else ORDER_MINDEG.  A plan
                        // in that range that a large batch sends to the lane or tree kernel also
                        // gets the dense x block (more fill than minimum degree; not measured)
};

// amd_l_order's status codes (include/qpSWIFT/amd.h): OK, OK but the columns were
// unsorted / held duplicates (still ordered), invalid input.
enum AmdStatus : int { AMD_STATUS_OK = 0, AMD_STATUS_JUMBLED = 1, AMD_STATUS_INVALID = -2 };

// AMD ordering of the n x n pattern (ap, ai) (CSC; A + A' is ordered, the diagonal
// ignored), written to perm[n]; the same permutation as the reference's
// amd_l_order for the same pattern and control values (qpb_amd.cpp).
int amd_order(long n, const long *ap, const long *ai, long *perm, double dense_ratio = 10.0,
              bool aggressive = true);

struct Plan {
    long n = 0, m = 0, p = 0, N = 0;
    int pmode = P_FULL;
    Pattern Pin, A, G;                       // caller patterns (P full or upper)
    Pattern Pf;  std::vector<long> Pf_src;   // full P pattern -> index into P values
    Pattern At;  std::vector<long> At_src;   // A' -> index into A values
    Pattern Gt;  std::vector<long> Gt_src;   // G' -> index into G values
    Pattern K;                               // KKT CSC (reference layout)
    std::vector<Slot> K_init;                // values as assembled (setup solve)
    std::vector<Slot> K_loop;                // after updatekktmatrix (IPM loop)
    std::vector<long> perm, pinv, parent, Lp, Li;
    long lnz = 0;
    int ordering_kind = 0;                   // ORDER_* below: how perm was chosen
    // multi-stage (block-tridiagonal) structure, 0 if none: x, z, y split into band_ns
    // stages of band_nb / band_mz / band_my rows with P block diagonal, G row group k on
    // stage k, A row group k on stages k-1 and k (band_shape; the band kernel, qpb_band.hip)
    int band_nb = 0, band_ns = 0, band_mz = 0, band_my = 0;
    std::vector<FacStep> fac;                // numeric schedule
    long fac_updates = 0, fac_divs = 0;      // op counts (flop accounting)
    uint64_t hash = 0;
    std::string key;                         // stable text key (hash input)
};

// Error codes: the same values as the QPB_E* macros of include/qpswift_hip.h.
enum Err : int {
    E_OK = 0,
    E_INVAL = -1,
    E_NOMEM = -2,
    E_HIP = -3,
    E_COMPILE = -4,
    E_SHAPE = -5,
};

// Build a plan.  P pattern is either full (both triangles, as QP_SETUP takes it)
// or upper-triangular (pmode = P_UPPER, symmetric semantics).  perm may be null:
// then `order` (ORDER_OWN / ORDER_LEAVES / ORDER_MINDEG: ours, ORDER_AMD: the
// reference's AMD) chooses it.  Returns QPB_OK or an error.
int build_plan(Plan &pl, long n, long m, long p, int pmode,
               const long *Pjc, const long *Pir,
               const long *Ajc, const long *Air,
               const long *Gjc, const long *Gir,
               const long *perm, std::string *err, int order = ORDER_OWN);

// Multi-stage structure of the plan's P / A / G patterns (fills pl.band_*): the
// smallest stage width NB <= 16 with n = NB NS, m = MZ NS, p = MY NS (NS >= 2,
// MZ <= 64, MY <= 16), every P entry inside a stage block, G row r on stage r / MZ
// only, A row l on stages l / MY - 1 and l / MY only, and no empty G row.
void band_shape(Plan &pl);

// Minimum-degree ordering of a symmetric pattern (own implementation; ties go
// to the lowest index).  Exposed for tests.
std::vector<long> min_degree_order(const Pattern &sym);

uint64_t fnv1a(const std::string &s);

}  // namespace qpb

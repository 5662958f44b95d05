// qpb_wave.hpp -- wave-cooperative kernel generator (one wavefront per QP).
#pragma once

#include <string>

#include "qpb_plan.hpp"

#include <vector>

namespace qpb {
// Elimination layout of the wave kernel for the plan's permutation: z / y rows
// whose neighbours all come later ("leaves") are eliminated first, in parallel;
// every other KKT row forms a dense block factored in permutation order.
struct WaveLayout {
    std::vector<int> zleaf, yleaf;   // per z / y row: 1 = leaf
    std::vector<long> dense;         // KKT indices of the dense block, in perm order
};
WaveLayout wave_layout(const Plan &pl);
// Can the plan run on the wave kernel?  (n, p <= 64, m <= 256, <= 64 dense
// rows, no empty G row, LDS fits.)
bool wave_eligible(const Plan &pl, std::string *why);
// Workgroup size: 64 x (QPs per workgroup that fit the LDS), 0 if none fits.
int wave_wg_for(const Plan &pl);
// Full hiprtc source; the kernel name is returned through name_out.
std::string generate_wave_kernel(const Plan &pl, int wg, std::string *name_out);
// Row form (qpb_row.hip, one QP per 16-lane row, four per wavefront): plans
// with every z / y row a leaf, the x block in natural order, n, p <= 16, m <= 32.
bool row_eligible(const Plan &pl);
// wpe: waves per SIMD the register allocation must allow (QPB_R_WPE; 2 for large
// batches, where two waves per SIMD hide the latency the single wave exposes)
std::string generate_row_kernel(const Plan &pl, std::string *name_out, int wpe = 1, bool split = false);
// One kernel for up to QPB_GROUP_MAX row-form plans (qpb_group_*): logical
// blocks [bend[i-1], bend[i]) run member i.
constexpr int QPB_GROUP_MAX = 16;
std::string generate_row_group_kernel(const std::vector<const Plan *> &pls, std::string *name_out);
// Band form (qpb_band.hip, one QP per wavefront): multi-stage plans (Plan::band_*)
// in leaves-first order whose per-QP state fits the LDS of a CU.
bool band_eligible(const Plan &pl, std::string *why);
long band_lds_bytes(const Plan &pl);
std::string generate_band_kernel(const Plan &pl, std::string *name_out);
// Wide row form (qpb_rowx.hip, one QP per 16-lane row, four per wavefront, two x rows
// per lane): the row form's structure for n, p <= 32, m <= 128 (the controller's
// 30-variable QPs).  Per-QP LDS doubles: dense column-major G, A, P, H0 (leading
// dimensions LDG / LDA / LDP), packed strictly-lower -L, 16 dump slots.
struct RowxLayout {
    long LDG, LDA, LDP, OFF_G, OFF_A, OFF_P, STG_END, OFF_H0, OFF_L, O_DUMP, LDS_QP;
};
RowxLayout rowx_layout(const Plan &pl);
bool rowx_eligible(const Plan &pl, std::string *why);
std::string generate_rowx_kernel(const Plan &pl, std::string *name_out);
}  // namespace qpb

// qpb_tree.hpp -- tree kernel generator (one workgroup per QP, any pattern).
#pragma once

#include <string>
#include <vector>

#include "qpb_plan.hpp"

namespace qpb {
// Shape statistics of the level-scheduled programs of a plan's tree kernel.
struct TreeStats {
    long levels = 0;          // height of the (supernodal) elimination tree
    long supernodes = 0;      // relaxed supernodes factored / solved as dense panels
    long fac_steps = 0, fwd_steps = 0, bwd_steps = 0, mv_steps = 0;
    long fac_contrib = 0;     // factor update terms per factorisation
    long desc_words = 0;      // descriptor table size (8-byte words, all programs)
    long lds_bytes = 0;       // LDS per QP (= per workgroup)
};
// Can the plan run on the tree kernel?  (fast mode; LDS footprint <= 160 KiB;
// Lnz, N and nnz below the descriptor field limit.)
bool tree_eligible(const Plan &pl, std::string *why);
// Threads per workgroup (= per QP): 64, 128 or 256 by KKT size (QPB_TREE_WG overrides).
int tree_wg_for(const Plan &pl);
// Kernel source; `tables` receives the plan-wide table blob the kernel reads
// through its `tab` argument (u64 descriptors, then int32 tables).
std::string generate_tree_kernel(const Plan &pl, int wg, std::string *name_out, TreeStats *stats = nullptr,
                                 std::vector<char> *tables = nullptr);
}  // namespace qpb

// qpb_runtime.hpp -- internals shared by the batched C ABI and the qpSWIFT drop-in.
#pragma once

#include <functional>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "qpb_codegen.hpp"
#include "qpb_plan.hpp"

struct qpb_plan {
    qpb::Plan pl;
    qpb::GenOptions gen;
    std::string kname;                          // lane kernel (one QP per lane)
    std::shared_ptr<std::vector<char>> code;
    bool wave_ok = false;                       // wave kernel (one QP per wavefront)
    int wave_wg = 256;
    int wave_qpw = 1;                           // QPs per wavefront: 1 wave form, 4 row form
    long wave_max_batch = 0;                    // auto: wave kernel for B <= this
    int kernel_pref = 0;                        // 0 auto, 1 lane only, 2 wave only
    std::string wave_kname;
    std::shared_ptr<std::vector<char>> wave_code;
    // row form for large batches: the same kernel allocated for two waves per SIMD
    // (<= 256 registers), used from row_occ_batch QPs on (-1: never)
    std::string row2_kname;
    std::shared_ptr<std::vector<char>> row2_code;
    long row_occ_batch = -1;
    bool tree_ok = false;                       // tree kernel (one QP per workgroup, any pattern)
    bool large_tree = false;                    // auto: tree (not lane) kernel beyond the wave kernel's range
    int tree_wg = 256;
    std::string tree_kname;
    std::shared_ptr<std::vector<char>> tree_code;
    std::vector<char> tree_tables;              // plan tables of the tree kernel (host copy)
    std::map<int, void *> tree_dev;             // device -> uploaded tables
    // large batches of N > 160 plans: the 128-thread form (four QPs per CU by LDS
    // and registers instead of two), used beyond tree_occ_batch QPs (-1: never)
    int tree2_wg = 0;
    long tree_occ_batch = -1;
    std::string tree2_kname;
    std::shared_ptr<std::vector<char>> tree2_code;
    std::vector<char> tree2_tables;
    std::map<int, void *> tree2_dev;
    // warm-solve variants (qpb_solve_warm; QPB_WARM = 1), compiled on first use:
    // cold kernel name -> code of "<name>_w"
    std::map<std::string, std::shared_ptr<std::vector<char>>> warm_code;
    std::vector<int> ctl_table;                 // controller-QP assembly entries (qpb_assemble_controller)
    std::map<int, void *> ctl_dev;              // device -> uploaded entries
    ~qpb_plan();
};

namespace qpb {
struct CopySeg {
    const double *src;
    double *dst;
    long n, ss, ds;   // element count, source stride, destination stride
};
struct CopySegs {
    static constexpr int kMax = 16;
    CopySeg seg[kMax];
    int nseg;
};
// Device-side strided copies on `stream` (one launch for all segments).
int strided_copy(const CopySegs &t, void *stream);
int compile_plan(qpb_plan *plan);
int compile_wave(qpb_plan *plan);
int compile_row2(qpb_plan *plan);
int compile_tree2(qpb_plan *plan);
int compile_tree(qpb_plan *plan);
int compile_warm(qpb_plan *plan, const std::string &kname, const std::function<std::string()> &gen_src, bool exact,
                 std::shared_ptr<std::vector<char>> **slot);
std::string wave_source_of(const qpb_plan *plan);   // wave or row form, as the plan chose
int set_error(int code, const char *msg);
// qpb_solve / qpb_solve_best / qpb_solve_warm in one: best != NULL fuses the
// argmin; sig != NULL receives every QP's last sigma (and, warm, supplies it);
// trace (warm only): KernelArgs::trace, QPB_TRACE_STRIDE doubles per QP
int solve_ex(qpb_plan *plan, long B, const double *P, const double *A, const double *G, const double *c,
             const double *h, const double *b, const qpb_settings *st, double *x, double *y, double *z, double *s,
             int *flag, int *iters, double *fval, double *stats, double *best, void *stream, double *sig, bool warm,
             double *trace = nullptr);
}  // namespace qpb

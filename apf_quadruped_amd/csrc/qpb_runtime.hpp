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
    bool wave_rowx = false;                     // row form: the wide kernel (qpb_rowx.hip, n <= 32)
    long wave_max_batch = 0;                    // auto: wave kernel for B <= this
    int kernel_pref = 0;                        // 0 auto, 1 lane only, 2 wave only, 3 tree, 4 band
    std::string wave_kname;
    std::shared_ptr<std::vector<char>> wave_code;
    // row form for large batches: the same kernel allocated for two waves per SIMD
    // (<= 256 registers), used from row_occ_batch QPs on (-1: never)
    std::string row2_kname;
    std::shared_ptr<std::vector<char>> row2_code;
    long row_occ_batch = -1;
    // the split form of the one-wave row kernel (QPB_R_SPLIT: two waves per four QPs),
    // used instead of it when row_split (QPB_ROW_SPLIT=1) for cold batched solves
    bool row_split = false;
    std::string rowsplit_kname;
    std::shared_ptr<std::vector<char>> rowsplit_code;
    // band kernel (one QP per wavefront, multi-stage patterns): cold solves only
    bool band_ok = false;
    std::string band_kname;
    std::shared_ptr<std::vector<char>> band_code;
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
    // variants compiled on first use, by name: "<name>_w" warm solve (qpb_solve_warm;
    // QPB_WARM = 1), "<name>_s" / "<name>_ws" persistent cold / warm (qpb::serve_ex)
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
int compile_rowsplit(qpb_plan *plan);
int compile_tree2(qpb_plan *plan);
int compile_band(qpb_plan *plan);
struct Pick { bool wave = false, band = false, tree = false; };   // neither: the lane kernel
Pick pick_kernel(const qpb_plan *plan, long B, bool warm);
bool band_auto();
bool rowx_auto();     // QPB_ROWX=0: the wave form instead of the wide row form
int compile_tree(qpb_plan *plan);
int compile_warm(qpb_plan *plan, const std::string &kname, const std::function<std::string()> &gen_src, bool exact,
                 std::shared_ptr<std::vector<char>> **slot);
// a variant of a plan's kernel: "<kname>_w" (warm), "_s" / "_ws" (persistent cold / warm)
int compile_variant(qpb_plan *plan, const std::string &kname, const std::function<std::string()> &gen_src, bool exact,
                    bool warm, bool serve, std::shared_ptr<std::vector<char>> **slot);
std::string wave_source_of(const qpb_plan *plan);   // wave or row form, as the plan chose
int set_error(int code, const char *msg);
// qpb_solve / qpb_solve_best / qpb_solve_warm in one: best != NULL fuses the
// argmin; sig != NULL receives every QP's last sigma (and, warm, supplies it);
// trace (warm only): KernelArgs::trace, QPB_TRACE_STRIDE doubles per QP
int solve_ex(qpb_plan *plan, long B, const double *P, const double *A, const double *G, const double *c,
             const double *h, const double *b, const qpb_settings *st, double *x, double *y, double *z, double *s,
             int *flag, int *iters, double *fval, double *stats, double *best, void *stream, double *sig, bool warm,
             double *trace = nullptr);

// A persistent solver for one QP at a time (the drop-in's per-tick QP_SETUP /
// QP_SOLVE): one wave of the plan's row or wave kernel, compiled with QPB_SERVE,
// stays resident and solves whenever the host posts a request in a mailbox in
// mapped pinned memory, so a solve costs no launch and no stream synchronisation.
// The kernel leaves by itself after `idle` without a request (and on a stop
// request); the host relaunches it when it finds it gone.  Its arguments (data
// pointers, settings) are fixed per launch: a call with different ones stops it
// and launches anew.
struct Server {
    std::string kname;                   // code object of the running launch
    KernelArgs args{};
    void *stream = nullptr;              // its own non-blocking stream
    unsigned long long *mb = nullptr;    // mailbox: [0] request, [16] answer, [32] its device ticks (host address)
    unsigned long long *mb_dev = nullptr;
    unsigned long long seq = 0;          // last request posted
    bool running = false;                // launched and not seen to end
    bool retiring = false;               // stop word posted by serve_retire_thread, launch not yet joined
    bool registered = false;             // listed for serve_retire_thread (this thread's servers)
    long long last_answer_ns = 0;        // steady-clock time of the last answer (one-request launches)
    long requests = 0, launches = 0, retires = 0;
    unsigned long long dev_ticks = 0;    // the last answer: 100 MHz ticks from request seen to answer
    Server() = default;
    Server(const Server &) = delete;
    Server &operator=(const Server &) = delete;
    ~Server();                           // stops the kernel, frees the mailbox and stream
};
constexpr int SERVE_NONE = 1;            // serve_ex: this plan's one-QP kernel has no persistent form
// The one predicate for "serve_ex answers this plan" (its one-QP kernel is the row or the
// wave form): serve_ex, qpb_plan_compile_serve and the drop-in's packed-slab choice all
// use it, so they cannot disagree (a packed slab read by a launched kernel would be wrong).
bool serve_eligible(const qpb_plan *plan);
// One QP (B = 1, the tiled slot of QP 0) through `srv`: returns once the results are
// in x .. trace.  SERVE_NONE when the plan's kernel for one QP is neither the row
// nor the wave form (the caller launches instead).
int serve_ex(qpb_plan *plan, Server *srv, const double *P, const double *A, const double *G, const double *c,
             const double *h, const double *b, const qpb_settings *st, double *x, double *y, double *z, double *s,
             int *flag, int *iters, double *fval, double *stats, double *sig, bool warm, double *trace,
             const double *win, const std::function<void()> &while_waiting = {});
// Stop the kernel (if running) and wait for it to leave; the mailbox stays.
int serve_stop(Server *srv);
// Post the stop word to every running server of the calling thread without
// waiting: their queued waves leave within microseconds, so a device-wide
// synchronisation that follows (hipDeviceSynchronize, a batched solve's caller)
// does not wait out the idle time.  The next serve_ex on a retired server joins the
// old launch first.  Called by the batched entry points (qpb_solve*, qpb_group_solve)
// and qpb_dropin_quiesce.
void serve_retire_thread();
}  // namespace qpb

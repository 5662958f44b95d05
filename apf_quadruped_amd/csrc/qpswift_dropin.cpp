// qpswift_dropin.cpp -- qpSWIFT's public API (include/qpSWIFT.h) on the gfx950
// kernel: QP_SETUP, QP_SETUP_dense, QP_SOLVE, QP_CLEANUP, QP_CLEANUP_dense.
//
// Mirrors reference dogbot_controller/src/qpSWIFT/qpSWIFT.c:
//   QP_SETUP          :60-234   (CSC inputs and c, h, b borrowed, caller sigma_d)
//   QP_SETUP_dense    :260-456  (dense -> CSC copies dropping exact zeros,
//                                Auxilary.c:1154-1273; sigma_d = 0)
//   QP_SOLVE          :473-644
//   QP_CLEANUP(_dense):661-839  (caller's Permut is never freed, AMD_RESULT -3)
// The pattern work of setup (transposes, KKT layout, ordering, symbolic LDL') is
// a cached qpb_plan; the value work (initial point, Mehrotra loop) runs on the
// GPU inside QP_SOLVE as a batch of one.  There is deliberately no host solver
// here: without a GPU, QP_SOLVE reports QP_FATAL.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/qpSWIFT.h"
#include "../../include/qpswift_hip.h"
#include "qpb_runtime.hpp"

namespace {

using clk = std::chrono::steady_clock;

double seconds_since(clk::time_point t0) {
    return std::chrono::duration<double>(clk::now() - t0).count();
}

struct PlanDeleter {
    void operator()(qpb_plan *p) const { qpb_plan_destroy(p); }
};
using PlanPtr = std::shared_ptr<qpb_plan>;

// Plan cache keyed by the exact sparsity pattern + ordering: the controller
// rebuilds its QP every tick with an unchanged pattern (main.cpp:1649), so after
// the first tick setup is a hash lookup instead of AMD + symbolic + JIT.
std::mutex g_cache_mu;
std::map<std::string, PlanPtr> g_cache;
constexpr size_t kCacheMax = 256;

void key_append(std::string &k, const long *v, long n) {
    if (n > 0 && v) k.append(reinterpret_cast<const char *>(v), sizeof(long) * (size_t)n);
    k.push_back('|');
}

// QP_SETUP / QP_SOLVE through the workspace's persistent solvers (qpb::serve_ex;
// zero-copy plans on the row or wave kernel).  QPSWIFT_HIP_SERVE=0: a launch and a
// stream synchronisation per call instead.
bool serve_enabled() {
    static const bool on = [] {
        const char *e = std::getenv("QPSWIFT_HIP_SERVE");
        return !(e && e[0] == '0');
    }();
    return on;
}

struct Priv {
    PlanPtr plan;
    std::string err;
    bool dense = false;
    // owned host storage (pointers in the public structs point here)
    std::vector<long> Pjc, Pir, Ajc, Air, Gjc, Gir;
    std::vector<double> Ppr, Apr, Gpr;
    std::vector<long> Atjc, Atir, Gtjc, Gtir;
    std::vector<double> Atpr, Gtpr;
    std::vector<long> Kjc, Kir;
    std::vector<double> Kpr;
    std::vector<long> perm, pinv, parent, lnzc, Lp, Li, Lti, Ltp, kflag, pattern, upattern;
    std::vector<double> kb, Y, Lx, D;
    std::vector<double> x, y, z, s, rx, ry, rz, delta, dx, dy, dz, dsv, ds, lambda, temp;
    smat Ps{}, As{}, Gs{}, Ats{}, Gts{}, Ks{};
    kkt K{};
    settings opt{};
    stats st{};
    // device buffers: borrowed from the solving thread's workspace (below) for
    // the duration of one QP_SOLVE -- the controller creates and destroys a QP
    // every tick, so nothing device-side is allocated per QP object
    int dev = -1;
    hipStream_t stream = nullptr;
    double *dmem = nullptr;   // tiled inputs/outputs + packed staging
    double *hmem = nullptr;   // pinned host staging: packed inputs, packed outputs
    double *zmem = nullptr, *zdev = nullptr;   // zero-copy slab (host / device address)
    long nP = 0, nA = 0, nG = 0, nin = 0, nout = 0;
    long oP = 0, oA = 0, oG = 0, oc = 0, oh = 0, ob = 0, ox = 0, oy = 0, oz = 0, os = 0, ost = 0, ofv = 0,
         oin = 0, oout = 0, otr = 0, owin = 0, ototal = 0;
    // kkt_initialize's point is in x, y, z, s (QP_SETUP ran it on the device):
    // QP_SOLVE then continues from the object's state (a warm solve), as the
    // reference's QP_SOLVE always does; otherwise its first QP_SOLVE is cold
    bool inited = false;
    const double *trace = nullptr;   // the last warm solve's trace (host copy, for verbose)
    qpb::Server *srv = nullptr;      // the workspace's persistent solvers (cold, warm)
    long tstride = 64;               // slab stride of QP 0's values: 64 tiled, 1 packed (persistent solver)
    bool mirror_pending = false;     // finish_mirror not run yet (QP_SETUP runs it while the device works)
    long *permut = nullptr;          // the caller's Permut (kkt.P points to it when given)
};

// Public struct first so that a QP* is also a Handle*.
struct Handle {
    QP qp;
    Priv *priv;
};

Handle *handle_of(QP *q) { return reinterpret_cast<Handle *>(q); }

// Auxilary.c:1154-1273: dense (column- or row-major) -> CSC, dropping exact zeros.
void dense_to_csc(long rows, long cols, const double *a, bool rowmajor, std::vector<long> &jc,
                  std::vector<long> &ir, std::vector<double> &pr) {
    jc.assign((size_t)cols + 1, 0);
    ir.clear();
    pr.clear();
    for (long j = 0; j < cols; j++) {
        for (long i = 0; i < rows; i++) {
            const double v = rowmajor ? a[i * cols + j] : a[j * rows + i];
            if (v != 0.0) {
                ir.push_back(i);
                pr.push_back(v);
            }
        }
        jc[(size_t)j + 1] = (long)ir.size();
    }
}

// Counting-sort transpose (Auxilary.c:901-951 computes the same result).
void csc_transpose(long rows, long cols, const long *jc, const long *ir, const double *pr, std::vector<long> &tjc,
                   std::vector<long> &tir, std::vector<double> &tpr) {
    const long nnz = jc[cols];
    tjc.assign((size_t)rows + 1, 0);
    tir.assign((size_t)nnz, 0);
    tpr.assign((size_t)nnz, 0.0);
    for (long k = 0; k < nnz; k++) tjc[(size_t)ir[k] + 1]++;
    for (long i = 0; i < rows; i++) tjc[(size_t)i + 1] += tjc[(size_t)i];
    std::vector<long> next(tjc.begin(), tjc.end() - 1);
    for (long j = 0; j < cols; j++)
        for (long k = jc[j]; k < jc[j + 1]; k++) {
            const long d = next[(size_t)ir[k]]++;
            tir[(size_t)d] = j;
            tpr[(size_t)d] = pr ? pr[k] : 0.0;
        }
}

void set_smat(smat &s, long rows, long cols, long *jc, long *ir, double *pr) {
    s.jc = jc;
    s.ir = ir;
    s.pr = pr;
    s.m = rows;
    s.n = cols;
    s.nnz = jc ? jc[cols] : 0;
}

double kkt_slot_value(const qpb::Slot &sl, const double *P, const double *A, const double *G, const double *s,
                      const double *z) {
    switch (sl.kind) {
        case qpb::Src::P: return P[sl.idx];
        case qpb::Src::A: return A[sl.idx];
        case qpb::Src::G: return G[sl.idx];
        case qpb::Src::NegOne: return -1.0;
        case qpb::Src::ZDiag: return (s && z) ? -s[sl.idx] / z[sl.idx] : -1.0;
    }
    return 0.0;
}

// QPSWIFT_HIP_ORDER=own: with Permut = NULL the plan takes its own KKT ordering (z and
// y rows first where the pattern allows: the wide row kernel for the controller's
// 30-variable QPs, DESIGN.md 4c') instead of the reference's AMD (qpSWIFT.c:424-440).
// Same QP, same algorithm, another elimination order: x agrees to rounding, not bit
// for bit, and an iteration count can differ where a stopping test is marginal.
// Exact mode (QPSWIFT_HIP_EXACT=1) promises the reference's bits, which need the
// reference's AMD order: the own order is then ignored, with one warning.
bool own_order(bool exact) {
    const char *e = std::getenv("QPSWIFT_HIP_ORDER");
    const bool own = e && std::strcmp(e, "own") == 0;
    if (own && exact) {
        static std::once_flag warned;
        std::call_once(warned, [] {
            std::fprintf(stderr, "qpswift-hip: QPSWIFT_HIP_ORDER=own ignored under QPSWIFT_HIP_EXACT=1 "
                                 "(exact mode keeps the reference's AMD order)\n");
        });
        return false;
    }
    return own;
}

PlanPtr get_plan(long n, long m, long p, const long *Pjc, const long *Pir, const long *Ajc, const long *Air,
                 const long *Gjc, const long *Gir, const long *perm, bool exact, std::string &err) {
    std::string key;
    const bool own = !perm && own_order(exact);
    const long hdr[6] = {n, m, p, exact ? 1L : 0L, perm ? 1L : 0L, own ? 1L : 0L};
    key_append(key, hdr, 6);
    key_append(key, Pjc, n + 1);
    key_append(key, Pir, Pjc[n]);
    if (p > 0) {
        key_append(key, Ajc, n + 1);
        key_append(key, Air, Ajc[n]);
    }
    key_append(key, Gjc, n + 1);
    key_append(key, Gir, Gjc[n]);
    if (perm) key_append(key, perm, n + m + p);
    {
        std::lock_guard<std::mutex> lk(g_cache_mu);
        auto it = g_cache.find(key);
        if (it != g_cache.end()) return it->second;
    }
    qpb_plan *raw = nullptr;
    int rc = qpb_plan_create(&raw, n, m, p, QPB_P_FULL | (own ? 0 : QPB_ORDER_AMD) | (exact ? QPB_EXACT : 0), Pjc, Pir, p > 0 ? Ajc : nullptr,
                             p > 0 ? Air : nullptr, Gjc, Gir, perm);
    if (rc) {
        err = qpb_last_error();
        return nullptr;
    }
    PlanPtr plan(raw, PlanDeleter());
    // compile only the kernel a batch of one runs (qpb::pick_kernel: the wave / row form
    // when the plan is eligible, the band or tree kernel for the plans that take them,
    // else the lane kernel -- round 5 compiled the lane kernel for band / tree plans too,
    // which takes minutes at N = 380).  With no GPU QP_SOLVE fails anyway (QP_FATAL), so
    // setup does not JIT at all.
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) rc = 0;
    else {
        const qpb::Pick pk = qpb::pick_kernel(raw, 1, false);
        rc = pk.wave ? qpb::compile_wave(raw) : pk.band ? qpb::compile_band(raw) : pk.tree ? qpb::compile_tree(raw)
                                                                                        : qpb::compile_plan(raw);
        // QP_SOLVE continues from the QP's state: the warm-solve variant
        if (!rc) rc = qpb_plan_compile_warm(raw, 1);
        // ... and the persistent forms the device solves go to (none: tree / lane)
        if (!rc && serve_enabled() && qpb_plan_compile_serve(raw) < 0) rc = -1;
    }
    if (rc != 0) {
        err = qpb_last_error();
        return nullptr;
    }
    std::lock_guard<std::mutex> lk(g_cache_mu);
    if (g_cache.size() >= kCacheMax) g_cache.clear();
    g_cache.emplace(key, plan);
    return plan;
}

// Everything of setup except the input conversion: transposes, plan, KKT
// mirror, work vectors, public pointers.
QP *finish_setup(Handle *hd, long *Permut) {
    QP &q = hd->qp;
    Priv &v = *hd->priv;
    const long n = q.n, m = q.m, p = q.p;

    q.options = &v.opt;
    q.stats = &v.st;
    v.opt.maxit = MAXIT;
    v.opt.reltol = RELTOL;
    v.opt.abstol = ABSTOL;
    v.opt.sigma = SIGMA;
    v.opt.verbose = VERBOSE;
    v.st.Flag = QP_FATAL;

    auto vec = [](std::vector<double> &b, long k) {
        b.assign((size_t)std::max(k, 1L), 0.0);
        return b.data();
    };
    q.x = vec(v.x, n);
    q.y = p > 0 ? vec(v.y, p) : nullptr;
    q.z = vec(v.z, m);
    q.s = vec(v.s, m);

    // default: fast arithmetic (the wave kernel where eligible: ~50 us per C1
    // tick instead of ~250 us); QPSWIFT_HIP_EXACT=1 selects the bit-faithful
    // lane kernel (bit-identical to qpSWIFT given the same permutation)
    const char *ex = getenv("QPSWIFT_HIP_EXACT");
    const bool exact = ex && *ex && *ex != '0';
    v.plan = get_plan(n, m, p, q.P->jc, q.P->ir, p > 0 ? q.A->jc : nullptr, p > 0 ? q.A->ir : nullptr, q.G->jc,
                      q.G->ir, Permut, exact, v.err);
    // the rest mirrors the reference's structs for callers that read them; the
    // device's initial point does not need it, so setup_init runs it while the
    // device computes (finish_mirror)
    v.permut = Permut;
    v.mirror_pending = true;
    return &q;
}

// The reference's QP struct contents that no device solve reads: G' and A', the work
// vectors, the KKT (values as assembled), its ordering and symbolic factor, and the
// LDL' workspace (qpSWIFT.c:60-456 fill them in QP_SETUP).
void finish_mirror(Priv &v, QP &q) {
    if (!v.mirror_pending) return;
    v.mirror_pending = false;
    const long n = q.n, m = q.m, p = q.p, N = n + m + p;
    long *Permut = v.permut;
    csc_transpose(m, n, q.G->jc, q.G->ir, q.G->pr, v.Gtjc, v.Gtir, v.Gtpr);
    set_smat(v.Gts, n, m, v.Gtjc.data(), v.Gtir.data(), v.Gtpr.data());
    q.Gt = &v.Gts;
    if (p > 0) {
        csc_transpose(p, n, q.A->jc, q.A->ir, q.A->pr, v.Atjc, v.Atir, v.Atpr);
        set_smat(v.Ats, n, p, v.Atjc.data(), v.Atir.data(), v.Atpr.data());
        q.At = &v.Ats;
    }
    auto vec = [](std::vector<double> &b, long k) {
        b.assign((size_t)std::max(k, 1L), 0.0);
        return b.data();
    };
    q.rx = vec(v.rx, n);
    q.ry = p > 0 ? vec(v.ry, p) : nullptr;
    q.rz = vec(v.rz, m);
    q.delta = vec(v.delta, N);
    q.delta_x = vec(v.dx, n);
    q.delta_y = p > 0 ? vec(v.dy, p) : nullptr;
    q.delta_z = vec(v.dz, m);
    q.delta_s = vec(v.dsv, m);
    q.ds = vec(v.ds, m);
    q.lambda = vec(v.lambda, m);
    q.temp = vec(v.temp, n);

    q.kkt = &v.K;
    v.st.AMD_RESULT = Permut ? -3 : 0;
    if (v.plan) {
        const qpb::Plan &pl = v.plan->pl;
        v.Kjc.assign(pl.K.jc.begin(), pl.K.jc.end());
        v.Kir.assign(pl.K.ir.begin(), pl.K.ir.end());
        v.Kpr.resize(pl.K_init.size());
        const double *Av = p > 0 ? q.A->pr : nullptr;
        for (size_t k = 0; k < pl.K_init.size(); k++)
            v.Kpr[k] = kkt_slot_value(pl.K_init[k], q.P->pr, Av, q.G->pr, nullptr, nullptr);
        set_smat(v.Ks, N, N, v.Kjc.data(), v.Kir.data(), v.Kpr.data());
        v.K.kktmatrix = &v.Ks;
        v.perm.assign(pl.perm.begin(), pl.perm.end());
        v.pinv.assign(pl.pinv.begin(), pl.pinv.end());
        v.parent.assign(pl.parent.begin(), pl.parent.end());
        v.Lp.assign(pl.Lp.begin(), pl.Lp.end());
        v.Li.assign(pl.Li.begin(), pl.Li.end());
        v.lnzc.assign((size_t)N, 0);
        for (long k = 0; k < N; k++) v.lnzc[(size_t)k] = pl.Lp[(size_t)k + 1] - pl.Lp[(size_t)k];
        v.K.P = Permut ? Permut : v.perm.data();
        v.K.Pinv = v.pinv.data();
        v.K.Parent = v.parent.data();
        v.K.Lp = v.Lp.data();
        v.K.Li = v.Li.data();
        v.K.Lnz = v.lnzc.data();
        const long lnz = std::max(pl.lnz, 1L);
        v.Lx.assign((size_t)lnz, 0.0);
        v.Lti.assign((size_t)lnz, 0);
        v.Ltp.assign((size_t)N + 1, 0);
        v.K.Lx = v.Lx.data();
        v.K.Lti = v.Lti.data();
        v.K.Ltp = v.Ltp.data();
    }
    v.kb.assign((size_t)N, 0.0);
    v.Y.assign((size_t)N, 0.0);
    v.D.assign((size_t)N, 0.0);
    v.kflag.assign((size_t)N, 0);
    v.pattern.assign((size_t)N, 0);
    v.upattern.assign((size_t)N, 0);
    v.K.b = v.kb.data();
    v.K.Y = v.Y.data();
    v.K.D = v.D.data();
    v.K.Flag = v.kflag.data();
    v.K.Pattern = v.pattern.data();
    v.K.UPattern = v.upattern.data();
}

// A few released QP objects' host storage per thread, reused by the next QP_SETUP:
// the controller builds and frees a QP every tick, and a fresh object's ~40 vectors
// reallocated and regrew every time (the mirror of the reference's QP struct).
// A reused Priv is a freshly constructed one that took over the old vectors'
// capacity -- every other field starts from its default.
constexpr size_t kPrivPool = 4;
// The pool owns what it holds: its destructor deletes the pooled objects when the
// thread exits (a controller on short-lived threads must not leak them).  A QP
// released after that (from another thread_local's destructor) is deleted outright.
struct PrivPool {
    std::vector<Priv *> v;
    PrivPool() = default;
    PrivPool(const PrivPool &) = delete;
    PrivPool &operator=(const PrivPool &) = delete;
    ~PrivPool();
};
thread_local PrivPool t_priv_pool;
thread_local bool t_priv_pool_gone = false;      // trivially destructible: readable at teardown
PrivPool::~PrivPool() {
    for (Priv *p : v) delete p;
    v.clear();
    t_priv_pool_gone = true;
}

void priv_put(Priv *v) {
    if (t_priv_pool_gone || t_priv_pool.v.size() >= kPrivPool) { delete v; return; }
    Priv fresh;
#define QPB_TAKE(f) fresh.f.swap(v->f); fresh.f.clear();
    QPB_TAKE(Pjc) QPB_TAKE(Pir) QPB_TAKE(Ajc) QPB_TAKE(Air) QPB_TAKE(Gjc) QPB_TAKE(Gir)
    QPB_TAKE(Ppr) QPB_TAKE(Apr) QPB_TAKE(Gpr) QPB_TAKE(Atjc) QPB_TAKE(Atir) QPB_TAKE(Gtjc) QPB_TAKE(Gtir)
    QPB_TAKE(Atpr) QPB_TAKE(Gtpr) QPB_TAKE(Kjc) QPB_TAKE(Kir) QPB_TAKE(Kpr)
    QPB_TAKE(perm) QPB_TAKE(pinv) QPB_TAKE(parent) QPB_TAKE(lnzc) QPB_TAKE(Lp) QPB_TAKE(Li) QPB_TAKE(Lti)
    QPB_TAKE(Ltp) QPB_TAKE(kflag) QPB_TAKE(pattern) QPB_TAKE(upattern) QPB_TAKE(kb) QPB_TAKE(Y) QPB_TAKE(Lx)
    QPB_TAKE(D) QPB_TAKE(x) QPB_TAKE(y) QPB_TAKE(z) QPB_TAKE(s) QPB_TAKE(rx) QPB_TAKE(ry) QPB_TAKE(rz)
    QPB_TAKE(delta) QPB_TAKE(dx) QPB_TAKE(dy) QPB_TAKE(dz) QPB_TAKE(dsv) QPB_TAKE(ds) QPB_TAKE(lambda)
    QPB_TAKE(temp)
#undef QPB_TAKE
    *v = std::move(fresh);
    t_priv_pool.v.push_back(v);
}

Priv *priv_get() {
    if (t_priv_pool_gone || t_priv_pool.v.empty()) return new (std::nothrow) Priv();
    Priv *v = t_priv_pool.v.back();
    t_priv_pool.v.pop_back();
    return v;
}

Handle *new_handle(long n, long m) {
    Handle *hd = static_cast<Handle *>(std::calloc(1, sizeof(Handle)));
    if (!hd) return nullptr;
    hd->priv = priv_get();
    if (!hd->priv) {
        std::free(hd);
        return nullptr;
    }
    hd->qp.n = n;
    hd->qp.m = m;
    return hd;
}

// Per-thread, per-device workspace: one stream, one device slab and one pinned
// staging slab, grown on demand and reused by every QP the thread solves.
struct Workspace {
    hipStream_t stream = nullptr;
    double *dmem = nullptr;
    double *hmem = nullptr;
    double *zmem = nullptr;    // zero-copy slab: fine-grained pinned host memory the kernel reads / writes
    double *zdev = nullptr;    //   its device-side address
    long dcap = 0, hcap = 0, zcap = 0;   // doubles
    // persistent solvers over the zero-copy slab: [0] QP_SETUP's initial point
    // (cold, maxit 0), [1] QP_SOLVE (warm) -- qpb::serve_ex
    qpb::Server srv[2];
    Workspace() = default;
    Workspace(const Workspace &) = delete;
    Workspace &operator=(const Workspace &) = delete;
    // released when the solving thread exits (a controller on pooled or
    // short-lived threads must not leak one stream + slabs per thread)
    ~Workspace() {
        for (auto &sv : srv) (void)qpb::serve_stop(&sv);   // before the slab they read goes
        if (stream) {
            (void)hipStreamSynchronize(stream);
            (void)hipStreamDestroy(stream);
        }
        if (dmem) (void)hipFree(dmem);
        if (hmem) (void)hipHostFree(hmem);
        if (zmem) (void)hipHostFree(zmem);
    }
};

// QP_SOLVE moves one QP's data either by zero copy (default for the fast kernels:
// the tiled slab lives in pinned, device-mapped host memory, so a solve is one
// kernel launch + one synchronisation; C1 per tick 51 -> 41 us) or staged
// (QPSWIFT_HIP_STAGED=1, and always for the exact lane kernel, which re-reads its
// inputs every iteration -- over the host link that costs more than the copies:
// H2D copy, scatter kernel, solve, gather kernel, D2H copy).
bool zero_copy_enabled() {
    static const bool z = [] {
        const char *e = std::getenv("QPSWIFT_HIP_STAGED");
        return !(e && e[0] == '1');
    }();
    return z;
}
thread_local std::map<int, Workspace> t_ws;


bool zero_copy(const Priv &v) { return zero_copy_enabled() && !v.plan->gen.exact; }


int ensure_device(Priv &v, const QP &q) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return qpb::set_error(QPB_EHIP, "QP_SOLVE: no HIP device available (the drop-in has no CPU path)");
    if (v.dev < 0 && hipGetDevice(&v.dev) != hipSuccess) return qpb::set_error(QPB_EHIP, "hipGetDevice failed");
    if (v.ototal == 0) {   // layout of this QP in the slab (tile of 64, QP in lane 0)
        // the persistent solver's variants read QP 0 packed (QPB_TSTR = 1): a zero-copy
        // slab it serves holds every vector contiguous -- 8 values per 64-byte line over
        // the host link instead of one; launched kernels read the tiled layout
        const char *wo = std::getenv("QPB_WAVE_OPTS");
        const bool packed = zero_copy(v) && serve_enabled() && qpb::serve_eligible(v.plan.get()) &&
                            !(wo && std::strstr(wo, "QPB_TSTR=64"));
        const long T = packed ? 1 : 64;
        v.tstride = T;
        v.nP = q.P->nnz;
        v.nA = q.p > 0 ? q.A->nnz : 0;
        v.nG = q.G->nnz;
        long o = 0;
        auto take = [&o](long k) { long r = o; o += std::max(k, 1L); return r; };
        v.oP = take(v.nP * T); v.oA = take(v.nA * T); v.oG = take(v.nG * T);
        v.oc = take(q.n * T); v.oh = take(q.m * T); v.ob = take(q.p * T);
        v.ox = take(q.n * T); v.oy = take(q.p * T); v.oz = take(q.m * T); v.os = take(q.m * T);
        v.ost = take(6 * T);
        v.nin = v.nP + v.nA + v.nG + q.n + q.m + q.p;
        v.nout = q.n + q.p + 2 * q.m + 6 + 1;   // x y z s stats fval
        v.oin = take(v.nin);
        v.oout = take(v.nout + 2);              // + flag, iters (two ints in one double slot), sigma
        v.otr = take(qpb::QPB_TRACE_STRIDE);   // timers + per-iteration statistics (warm solves)
        // the warm state the persistent solver continues from, on 128-B lines of its own
        // that only the host writes (KernelArgs::win)
        o = (o + 15) & ~15L;
        v.owin = take(((q.n + q.p + 2 * q.m + 2) + 15) & ~15L);
        v.ofv = v.oout + v.nout - 1;
        v.ototal = o;
    }
    Workspace &w = t_ws[v.dev];
    if (!w.stream && hipStreamCreateWithFlags(&w.stream, hipStreamNonBlocking) != hipSuccess) {
        w.stream = nullptr;
        return qpb::set_error(QPB_EHIP, "QP_SOLVE: stream creation failed");
    }
    if (!zero_copy(v) && w.dcap < v.ototal) {
        if (w.dmem) (void)hipFree(w.dmem);
        w.dcap = 0;
        if (hipMalloc((void **)&w.dmem, sizeof(double) * (size_t)v.ototal) != hipSuccess) {
            w.dmem = nullptr;
            return qpb::set_error(QPB_ENOMEM, "QP_SOLVE: device allocation failed");
        }
        w.dcap = v.ototal;
    }
    const long hneed = v.nin + v.nout + 2 + qpb::QPB_TRACE_STRIDE;
    if (!zero_copy(v) && w.hcap < hneed) {
        if (w.hmem) (void)hipHostFree(w.hmem);
        w.hcap = 0;
        if (hipHostMalloc((void **)&w.hmem, sizeof(double) * (size_t)hneed, hipHostMallocDefault) != hipSuccess) {
            w.hmem = nullptr;
            return qpb::set_error(QPB_ENOMEM, "QP_SOLVE: pinned host allocation failed");
        }
        w.hcap = hneed;
    }
    if (zero_copy(v) && w.zcap < v.ototal) {
        for (auto &sv : w.srv) (void)qpb::serve_stop(&sv);
        if (w.zmem) (void)hipHostFree(w.zmem);
        w.zcap = 0;
        w.zdev = nullptr;
        if (hipHostMalloc((void **)&w.zmem, sizeof(double) * (size_t)v.ototal, hipHostMallocCoherent) != hipSuccess) {
            w.zmem = nullptr;
            return qpb::set_error(QPB_ENOMEM, "QP_SOLVE: mapped pinned host allocation failed");
        }
        if (hipHostGetDevicePointer((void **)&w.zdev, w.zmem, 0) != hipSuccess) {
            (void)hipHostFree(w.zmem);
            w.zmem = nullptr;
            w.zdev = nullptr;
            return qpb::set_error(QPB_EHIP, "QP_SOLVE: mapped pinned host memory has no device address");
        }
        w.zcap = v.ototal;
    }
    v.dmem = w.dmem;
    v.hmem = w.hmem;
    v.zmem = w.zmem;
    v.zdev = w.zdev;
    v.stream = w.stream;
    v.srv = w.srv;
    return QPB_OK;
}

// The state a warm solve continues from / a solve leaves (the QP object's
// public fields), and the settings of this call.
struct CallState {
    bool warm;
    qpb_settings st;
};

CallState call_state(const Priv &v, const QP &q, long maxit) {
    CallState cs;
    cs.warm = v.inited;
    cs.st.maxit = maxit;
    cs.st.reltol = q.options->reltol;
    cs.st.abstol = q.options->abstol;
    cs.st.sigma_d = q.sigma_d;
    return cs;
}

// Results of one launch back into the QP object.  `setup_init`: the launch was
// QP_SETUP's kkt_initialize (maxit = 0): only x, y, z, s change.
// options->verbose > 0: the reference's messages (qpSWIFT.c:484-488, 506-509,
// 598-641), printed after the launch from the kernel's trace, in the same order
void print_verbose(const Priv &v, const QP &q, const double *tr, long it0) {
    const long ntop = tr ? (long)tr[2] : 0, nit = tr ? (long)tr[3] : 0;
    for (long i = 0; i < std::max(ntop, nit); i++) {
        const double *e = tr + 4 + 7 * i;
        if (i < ntop)
            printf("It: %ld || pcost : %e || rx:%e   ||  ry:%e ||  rz:%e || mu:%e\n", it0 + i, e[0], e[1], e[2], e[3],
                   e[4]);
        if (i < nit) printf("      || Primal Step Size : %f || Dual Step Size   : %f\n", e[5], e[6]);
    }
    const stats &st = v.st;
    if (st.Flag == QP_OPTIMAL) {
        printf("\nOptimal Solution Found\n");
        printf("Solve Time     : %f ms\n", (st.tsolve + st.tsetup) * 1000.0);
    } else if (st.Flag == QP_MAXIT) {
        printf("\nMaximum Iterations reached\n");
        printf("Solve Time     : %f ms\n", st.tsolve * 1000.0);
    }
    if (st.Flag == QP_OPTIMAL || st.Flag == QP_MAXIT) {
        printf("KKT_Solve Time : %f ms\n", st.kkt_time * 1000.0);
        printf("LDL Time       : %f ms\n", st.ldl_numeric * 1000.0);
        printf("Iterations     : %ld\n\n", st.IterationCount);
    }
    if (st.Flag == QP_FATAL) printf("\nUnknown Error Detected\n\n");
    if (st.Flag == QP_KKTFAIL) printf("\nLDL Factorization fail\n\n");
    (void)q;
    fflush(stdout);
}

// timers from the kernel's trace: kkt_time (this call's factor + solves,
// qpSWIFT.c:554-586, 611) and ldl_numeric (accumulated, Auxilary.c:476-484);
// s_memrealtime runs at 100 MHz
void take_timers(Priv &v, const double *tr) {
    if (!tr) return;
    v.st.kkt_time = tr[1] * 1e-8;
    v.st.ldl_numeric += tr[0] * 1e-8;
}

void take_results(Priv &v, QP &q, const double *x, const double *y, const double *z, const double *s,
                  const double *stv, double fval, const int *fl_it, double sigma, long maxit, bool setup_init) {
    const long n = q.n, m = q.m, p = q.p;
    std::memcpy(q.x, x, sizeof(double) * (size_t)n);
    if (p > 0) std::memcpy(q.y, y, sizeof(double) * (size_t)p);
    std::memcpy(q.z, z, sizeof(double) * (size_t)m);
    std::memcpy(q.s, s, sizeof(double) * (size_t)m);
    if (setup_init) return;
    const long before = v.st.IterationCount;
    v.st.Flag = fl_it[0];
    v.st.IterationCount = fl_it[1];
    q.options->sigma = sigma;
    // the loop body never ran (maxit <= 0): the reference touches no statistic;
    // no iteration ran: its step lengths stay as they were (qpSWIFT.c:506-596)
    if (maxit <= 0) return;
    v.st.fval = fval;
    v.st.n_rx = stv[0]; v.st.n_ry = stv[1]; v.st.n_rz = stv[2]; v.st.n_mu = stv[3];
    if (v.st.IterationCount != before) { v.st.alpha_p = stv[4]; v.st.alpha_d = stv[5]; }
}

// Zero-copy solve: inputs (and, warm, the QP's state) written straight into the
// tiled slot of QP 0 (stride 64) of the mapped pinned slab, one launch reads
// them over the host link and writes x, y, z, s, stats, flag, iterations, fval
// and sigma back into it.
int solve_zero_copy(Priv &v, QP &q, const CallState &cs, bool setup_init, const std::function<void()> &overlap) {
    const long n = q.n, m = q.m, p = q.p;
    double *h = v.zmem, *d = v.zdev;
    const long T = v.tstride;
    auto put = [h, T](long off, const double *src, long k) {
        for (long i = 0; i < k; i++) h[off + T * i] = src[i];
    };
    put(v.oP, q.P->pr, v.nP);
    if (p > 0) put(v.oA, q.A->pr, v.nA);
    put(v.oG, q.G->pr, v.nG);
    put(v.oc, q.c, n);
    put(v.oh, q.h, m);
    if (p > 0) put(v.ob, q.b, p);
    const long ofl = v.oout + v.nout;       // flag, iterations: two ints in one double slot
    const long osg = ofl + 1;               // sigma (options->sigma)
    if (cs.warm) {
        put(v.ox, q.x, n);
        if (p > 0) put(v.oy, q.y, p);
        put(v.oz, q.z, m);
        put(v.os, q.s, m);
        const int iv[2] = {(int)v.st.Flag, (int)v.st.IterationCount};
        std::memcpy(h + ofl, iv, sizeof(iv));
        h[osg] = q.options->sigma;
        // the same state, contiguous, for a resident wave (never read from the slots it writes)
        double *wi = h + v.owin;
        std::memcpy(wi, q.x, sizeof(double) * (size_t)n);
        if (p > 0) std::memcpy(wi + n, q.y, sizeof(double) * (size_t)p);
        std::memcpy(wi + n + p, q.z, sizeof(double) * (size_t)m);
        std::memcpy(wi + n + p + m, q.s, sizeof(double) * (size_t)m);
        std::memcpy(wi + n + p + 2 * m, iv, sizeof(iv));
        wi[n + p + 2 * m + 1] = q.options->sigma;
    }
    int *dfl = reinterpret_cast<int *>(d + ofl);
    // the persistent solver answers without a launch; plans whose one-QP kernel has
    // no persistent form (and QPSWIFT_HIP_SERVE=0) launch and synchronise
    int rc = qpb::SERVE_NONE;
    if (serve_enabled())
        rc = qpb::serve_ex(v.plan.get(), &v.srv[cs.warm ? 1 : 0], d + v.oP, p > 0 ? d + v.oA : nullptr, d + v.oG,
                           d + v.oc, d + v.oh, p > 0 ? d + v.ob : nullptr, &cs.st, d + v.ox, p > 0 ? d + v.oy : nullptr,
                           d + v.oz, d + v.os, dfl, dfl + 1, d + v.ofv, d + v.ost, d + osg, cs.warm, d + v.otr,
                           d + v.owin, overlap);
    if (rc == qpb::SERVE_NONE) {
        // a launched kernel reads the tiled slot (stride 64): a packed slab here would be
        // read wrongly without any error -- refuse instead (serve_eligible decides both)
        if (T != 64)
            return qpb::set_error(QPB_EHIP, "QP_SOLVE: packed slab but no persistent solver answered (internal)");
        if (overlap) overlap();       // (no persistent solver: nothing to overlap with)
        rc = qpb::solve_ex(v.plan.get(), 1, d + v.oP, p > 0 ? d + v.oA : nullptr, d + v.oG, d + v.oc, d + v.oh,
                           p > 0 ? d + v.ob : nullptr, &cs.st, d + v.ox, p > 0 ? d + v.oy : nullptr, d + v.oz,
                           d + v.os, dfl, dfl + 1, d + v.ofv, d + v.ost, nullptr, v.stream, d + osg, cs.warm,
                           d + v.otr);
        if (hipStreamSynchronize(v.stream) != hipSuccess && !rc)
            rc = qpb::set_error(QPB_EHIP, "QP_SOLVE: kernel failed");
    }
    if (rc) return rc;
    std::vector<double> tmp((size_t)(n + p + 2 * m + 6));
    double *tx = tmp.data(), *ty = tx + n, *tz = ty + p, *ts = tz + m, *tst = ts + m;
    auto get = [h, T](double *dst, long off, long k) {
        for (long i = 0; i < k; i++) dst[i] = h[off + T * i];
    };
    get(tx, v.ox, n);
    if (p > 0) get(ty, v.oy, p);
    get(tz, v.oz, m);
    get(ts, v.os, m);
    get(tst, v.ost, 6);
    int iv[2];
    std::memcpy(iv, h + ofl, sizeof(iv));
    static const bool recheck = getenv("QPB_SERVE_RECHECK") != nullptr;
    if (recheck) {
        // diagnostics: did any result land in the slab after the answer was seen?
        std::this_thread::sleep_for(std::chrono::microseconds(500));
        std::vector<double> t2(tmp.size());
        double *ux = t2.data(), *uy = ux + n, *uz = uy + p, *us = uz + m;
        get(ux, v.ox, n);
        if (p > 0) get(uy, v.oy, p);
        get(uz, v.oz, m);
        get(us, v.os, m);
        long nd = 0;
        for (long i = 0; i < n + p + 2 * m; i++) nd += std::memcmp(&tmp[(size_t)i], &t2[(size_t)i], sizeof(double)) != 0;
        if (nd) fprintf(stderr, "[recheck] %s: %ld of %ld results changed after the answer\n",
                        setup_init ? "setup" : (cs.warm ? "warm" : "cold"), nd, n + p + 2 * m);
    }
    take_results(v, q, tx, ty, tz, ts, tst, h[v.ofv], iv, h[osg], cs.st.maxit, setup_init);
    if (cs.warm) {
        take_timers(v, h + v.otr);
        v.trace = h + v.otr;
    }
    return QPB_OK;
}

// host mirror of the KKT after the solve: z-block diagonal as the last
// updatekktmatrix left it (Auxilary.c:205-233); mu from the last residuals
void mirror_kkt(Priv &v, QP &q) {
    q.mu = v.st.n_mu;
    const qpb::Plan &pl = v.plan->pl;
    const double *Av = q.p > 0 ? q.A->pr : nullptr;
    for (size_t k = 0; k < pl.K_loop.size() && k < v.Kpr.size(); k++)
        if (pl.K_loop[k].kind == qpb::Src::ZDiag && v.st.IterationCount > 0)
            v.Kpr[k] = kkt_slot_value(pl.K_loop[k], q.P->pr, Av, q.G->pr, q.s, q.z);
}

// Staged solve (QPSWIFT_HIP_STAGED=1, and always for the exact lane kernel,
// which re-reads its inputs every iteration -- over the host link that costs more
// than the copies).  The pinned host slab mirrors the device region [oin, oout +
// nout + 2): packed inputs | packed x y z s stats fval | flag, iterations | sigma,
// so ONE host-to-device copy carries the inputs and (warm) the QP's state, a
// scatter kernel spreads them to the tiled slots, the solve runs, a gather kernel
// packs the results and ONE device-to-host copy brings them back.
int solve_staged(Priv &v, QP &q, const CallState &cs, bool setup_init, const std::function<void()> &overlap) {
    if (overlap) overlap();
    const long n = q.n, m = q.m, p = q.p;
    double *hin = v.hmem, *hout = v.hmem + v.nin;
    double *w = hin;
    auto put = [&w](const double *src, long k) {
        if (k > 0) std::memcpy(w, src, sizeof(double) * (size_t)k);
        w += k;
    };
    put(q.P->pr, v.nP);
    if (p > 0) put(q.A->pr, v.nA);
    put(q.G->pr, v.nG);
    put(q.c, n);
    put(q.h, m);
    if (p > 0) put(q.b, p);
    long up = v.nin;                         // doubles to upload
    if (cs.warm) {                           // the QP's state into the packed output region
        w = hout;
        put(q.x, n);
        if (p > 0) put(q.y, p);
        put(q.z, m);
        put(q.s, m);
        const int iv[2] = {(int)v.st.Flag, (int)v.st.IterationCount};
        std::memcpy(hout + v.nout, iv, sizeof(iv));
        hout[v.nout + 1] = q.options->sigma;
        up = v.nin + v.nout + 2;
    }
    double *d = v.dmem;
    hipError_t e = hipMemcpyAsync(d + v.oin, hin, sizeof(double) * (size_t)up, hipMemcpyHostToDevice, v.stream);
    int rc = e == hipSuccess ? QPB_OK : qpb::set_error(QPB_EHIP, "QP_SOLVE: upload failed");
    qpb::CopySegs sc{};
    long po = v.oin;
    auto scatter = [&](long dst, long k) {
        if (k <= 0) return;
        if (sc.nseg >= qpb::CopySegs::kMax) { sc.nseg = qpb::CopySegs::kMax + 1; return; }   // refused below
        sc.seg[sc.nseg++] = {d + po, d + dst, k, 1, 64};
        po += k;
    };
    scatter(v.oP, v.nP);
    scatter(v.oA, v.nA);
    scatter(v.oG, v.nG);
    scatter(v.oc, n);
    scatter(v.oh, m);
    scatter(v.ob, p);
    if (cs.warm) {
        po = v.oout;
        scatter(v.ox, n);
        scatter(v.oy, p);
        scatter(v.oz, m);
        scatter(v.os, m);
    }
    if (!rc) rc = qpb::strided_copy(sc, v.stream);
    int *fl = reinterpret_cast<int *>(d + v.oout + v.nout);
    double *sg = d + v.oout + v.nout + 1;
    if (!rc)
        rc = qpb::solve_ex(v.plan.get(), 1, d + v.oP, p > 0 ? d + v.oA : nullptr, d + v.oG, d + v.oc, d + v.oh,
                           p > 0 ? d + v.ob : nullptr, &cs.st, d + v.ox, p > 0 ? d + v.oy : nullptr, d + v.oz,
                           d + v.os, fl, fl + 1, d + v.ofv, d + v.ost, nullptr, v.stream, sg, cs.warm, d + v.otr);
    qpb::CopySegs gc{};
    long qo = v.oout;
    auto gather = [&](long src, long k, long ss) {
        if (k <= 0) return;
        if (gc.nseg >= qpb::CopySegs::kMax) { gc.nseg = qpb::CopySegs::kMax + 1; return; }   // refused below
        gc.seg[gc.nseg++] = {d + src, d + qo, k, ss, 1};
        qo += k;
    };
    gather(v.ox, n, 64);
    gather(v.oy, p, 64);
    gather(v.oz, m, 64);
    gather(v.os, m, 64);
    gather(v.ost, 6, 64);
    if (!rc) rc = qpb::strided_copy(gc, v.stream);
    if (!rc && hipMemcpyAsync(hout, d + v.oout, sizeof(double) * (size_t)(v.nout + 2), hipMemcpyDeviceToHost,
                              v.stream) != hipSuccess)
        rc = qpb::set_error(QPB_EHIP, "QP_SOLVE: download failed");
    double *htr = hout + v.nout + 2;        // the trace: header + the entries maxit can fill
    const long ntr = 4 + 7 * std::min<long>(std::max<long>(cs.st.maxit, 0), qpb::QPB_TRACE_MAX);
    if (!rc && cs.warm && hipMemcpyAsync(htr, d + v.otr, sizeof(double) * (size_t)ntr, hipMemcpyDeviceToHost,
                                         v.stream) != hipSuccess)
        rc = qpb::set_error(QPB_EHIP, "QP_SOLVE: trace download failed");
    if (hipStreamSynchronize(v.stream) != hipSuccess && !rc) rc = qpb::set_error(QPB_EHIP, "QP_SOLVE: kernel failed");
    if (rc) return rc;
    const double *r = hout;
    int iv[2];
    std::memcpy(iv, hout + v.nout, sizeof(iv));
    take_results(v, q, r, r + n, r + n + p, r + n + p + m, r + n + p + 2 * m, hout[v.nout - 1], iv, hout[v.nout + 1],
                 cs.st.maxit, setup_init);
    if (cs.warm) {
        take_timers(v, htr);
        v.trace = htr;
    }
    return QPB_OK;
}

// One launch for this QP: QP_SETUP's kkt_initialize (setup_init: maxit = 0,
// cold) or a QP_SOLVE (warm once the initial point is in the object).
int solve_on_device(Priv &v, QP &q, bool setup_init, const std::function<void()> &overlap = {}) {
    int rc = ensure_device(v, q);
    if (rc) return rc;
    int cur = -1;
    (void)hipGetDevice(&cur);
    if (cur != v.dev) (void)hipSetDevice(v.dev);
    CallState cs = call_state(v, q, setup_init ? 0 : q.options->maxit);
    if (setup_init) cs.warm = false;
    rc = zero_copy(v) ? solve_zero_copy(v, q, cs, setup_init, overlap) : solve_staged(v, q, cs, setup_init, overlap);
    if (cur != v.dev && cur >= 0) (void)hipSetDevice(cur);
    if (rc) return rc;
    if (setup_init) v.inited = true;
    else {
        v.inited = true;            // the object now holds an iterate to continue from
        mirror_kkt(v, q);
    }
    return QPB_OK;
}

// QP_SETUP's kkt_initialize (qpSWIFT.c:447): the initial point in x, y, z, s
// when setup returns, computed on the device (maxit = 0 launch).  Skipped without
// a GPU or with QPSWIFT_HIP_SETUP_INIT=0 (the first QP_SOLVE is then a cold solve,
// one launch per tick instead of two; x, y, z, s stay zero until it).
QP *setup_init(QP *q, clk::time_point t0) {
    if (!q) return q;
    Priv &v = *handle_of(q)->priv;
    const char *e = std::getenv("QPSWIFT_HIP_SETUP_INIT");
    int ndev = 0;
    if (v.plan && !(e && e[0] == '0') && hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0) {
        // the reference's struct mirror is filled while the device computes the point
        if (solve_on_device(v, *q, true, [&v, q] { finish_mirror(v, *q); }) != QPB_OK) v.err = qpb_last_error();
    }
    finish_mirror(v, *q);    // (no device init, or it failed before posting)
    v.st.tsetup = seconds_since(t0);
    return q;
}

void release(QP *q) {
    if (!q) return;
    Handle *hd = handle_of(q);
    priv_put(hd->priv);   // device buffers belong to the thread workspace, not the QP
    std::free(hd);
}

}  // namespace

extern "C" {

QP *QP_SETUP(qp_int n, qp_int m, qp_int p, qp_int *Pjc, qp_int *Pir, qp_real *Ppr, qp_int *Ajc, qp_int *Air,
             qp_real *Apr, qp_int *Gjc, qp_int *Gir, qp_real *Gpr, qp_real *c, qp_real *h, qp_real *b,
             qp_real sigma_d, qp_int *Permut) {
    const auto t0 = clk::now();
    Handle *hd = new_handle(n, m);
    if (!hd) return nullptr;
    QP &q = hd->qp;
    Priv &v = *hd->priv;
    // qpSWIFT.c:91-104: the equality block exists only with all of A and b
    if (Apr && Ajc && Air && b && p != 0) {
        q.p = p;
        set_smat(v.As, p, n, Ajc, Air, Apr);
        q.A = &v.As;
        q.b = b;
    }
    set_smat(v.Ps, n, n, Pjc, Pir, Ppr);
    set_smat(v.Gs, m, n, Gjc, Gir, Gpr);
    q.P = &v.Ps;
    q.G = &v.Gs;
    q.c = c;
    q.h = h;
    q.sigma_d = sigma_d;
    return setup_init(finish_setup(hd, Permut), t0);
}

QP *QP_SETUP_dense(qp_int n, qp_int m, qp_int p, qp_real *Ppr, qp_real *Apr, qp_real *Gpr, qp_real *c,
                   qp_real *h, qp_real *b, qp_int *Permut, int ordering) {
    const auto t0 = clk::now();
    Handle *hd = new_handle(n, m);
    if (!hd) return nullptr;
    QP &q = hd->qp;
    Priv &v = *hd->priv;
    v.dense = true;
    const bool rowmajor = ordering != COLUMN_MAJOR_ORDERING;   // qpSWIFT.c:296-303
    if (Apr && b && p != 0) {
        q.p = p;
        dense_to_csc(p, n, Apr, rowmajor, v.Ajc, v.Air, v.Apr);
        set_smat(v.As, p, n, v.Ajc.data(), v.Air.data(), v.Apr.data());
        q.A = &v.As;
        q.b = b;
    }
    dense_to_csc(n, n, Ppr, rowmajor, v.Pjc, v.Pir, v.Ppr);
    dense_to_csc(m, n, Gpr, rowmajor, v.Gjc, v.Gir, v.Gpr);
    set_smat(v.Ps, n, n, v.Pjc.data(), v.Pir.data(), v.Ppr.data());
    set_smat(v.Gs, m, n, v.Gjc.data(), v.Gir.data(), v.Gpr.data());
    q.P = &v.Ps;
    q.G = &v.Gs;
    q.c = c;
    q.h = h;
    q.sigma_d = 0.0;   // qpSWIFT.c:334
    return setup_init(finish_setup(hd, Permut), t0);
}

qp_int QP_SOLVE(QP *myQP) {
    if (!myQP) return QP_FATAL;
    const auto t0 = clk::now();
    Priv &v = *handle_of(myQP)->priv;
    const bool verbose = myQP->options && myQP->options->verbose > 0;
    if (verbose) {                                  // qpSWIFT.c:484-488
        printf("****qpSWIFT : Sparse Quadratic Programming Solver****\n\n");
        printf("================Data Statistics======================\n");
    }
    const long it0 = v.st.IterationCount;
    v.trace = nullptr;
    int rc;
    if (!v.plan) {
        rc = qpb::set_error(QPB_ECOMPILE, ("QP_SOLVE: no kernel for this QP: " + v.err).c_str());
    } else {
        rc = solve_on_device(v, *myQP, false);
    }
    if (rc) v.st.Flag = QP_FATAL;
    v.st.tsolve = seconds_since(t0);
    if (verbose) print_verbose(v, *myQP, v.trace, it0);
    return v.st.Flag;
}

void QP_CLEANUP(QP *myQP) { release(myQP); }
void QP_CLEANUP_dense(QP *myQP) { release(myQP); }

int qpb_dropin_serve_stats(long out[4]) {
    if (!out) return qpb::set_error(QPB_EINVAL, "NULL argument");
    out[0] = out[1] = out[2] = out[3] = 0;
    for (auto &kv : t_ws)
        for (int k = 0; k < 2; k++) {
            const qpb::Server &sv = kv.second.srv[k];
            out[0] += sv.requests;
            out[1] += sv.launches;
            if (sv.dev_ticks) out[2 + k] = (long)sv.dev_ticks * 10;
        }
    return QPB_OK;
}

}  // extern "C"

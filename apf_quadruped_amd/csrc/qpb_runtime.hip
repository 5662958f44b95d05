// qpb_runtime.hip -- C ABI of the batched solver: plans, the code-object cache
// (hiprtc JIT for gfx950 + on-disk cache), launches, and the argmin reduction.
#include <dlfcn.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <spawn.h>
#include <sys/wait.h>
#include <hip/hiprtc.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "../../include/qpswift_hip.h"
#include "qpb_codegen.hpp"
#include "qpb_plan.hpp"
#include "qpb_hazard.hpp"
#include "qpb_runtime.hpp"
#include "qpb_tree.hpp"
#include "qpb_wave.hpp"

extern char **environ;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

std::mutex g_mu;
// kernel name -> code object bytes (compiled or read from disk)
std::map<std::string, std::shared_ptr<std::vector<char>>> g_code;
// (device, kernel name) -> loaded function
std::map<std::pair<int, std::string>, std::pair<hipModule_t, hipFunction_t>> g_funcs;

std::string cache_dir() {
    const char *env = getenv("QPB_KCACHE");
    if (env && *env) return env;
    Dl_info info;
    if (dladdr((void *)&cache_dir, &info) && info.dli_fname) {
        std::string p(info.dli_fname);
        size_t s = p.rfind('/');
        if (s != std::string::npos) return p.substr(0, s) + "/kcache";
    }
    return "kcache";
}

bool read_file(const std::string &path, std::vector<char> &out) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    out.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
    return !out.empty();
}

void write_file(const std::string &path, const std::vector<char> &data) {
    std::string tmp = path + ".tmp" + std::to_string((long)getpid());
    {
        std::ofstream f(tmp, std::ios::binary);
        if (!f) return;
        f.write(data.data(), (std::streamsize)data.size());
    }
    rename(tmp.c_str(), path.c_str());
}

// Lowest fval among optimal QPs, ties -> lowest index.  Two stages: every
// block reduces a contiguous chunk to one (fval, index) pair, then one block
// reduces the pairs.  "better(a, b)": a is optimal and (lower fval, or equal
// fval and lower index).
__device__ __forceinline__ bool qpb_better(double va, long ia, double vb, long ib) {
    return ia >= 0 && (ib < 0 || va < vb || (va == vb && ia < ib));
}

__device__ __forceinline__ void qpb_block_argmin(double &bv, long &bi) {
    __shared__ double sv[1024 / 64];
    __shared__ long si[1024 / 64];
    for (int off = 32; off > 0; off >>= 1) {
        double ov = __shfl_xor(bv, off, 64);
        long oi = __shfl_xor(bi, off, 64);
        if (qpb_better(ov, oi, bv, bi)) { bv = ov; bi = oi; }
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { sv[w] = bv; si[w] = bi; }
    __syncthreads();
    if (threadIdx.x == 0)
        for (int k = 1; k < (int)(blockDim.x >> 6); k++)
            if (qpb_better(sv[k], si[k], bv, bi)) { bv = sv[k]; bi = si[k]; }
}

__global__ void __launch_bounds__(256) qpb_argmin_partial(long B, long chunk, const double *__restrict__ fval,
                                                          const int *__restrict__ flag, double *__restrict__ pv,
                                                          long *__restrict__ pi) {
    const long lo = (long)blockIdx.x * chunk, hi = lo + chunk < B ? lo + chunk : B;
    double bv = INFINITY;
    long bi = -1;
    for (long q = lo + threadIdx.x; q < hi; q += blockDim.x)
        if (flag[q] == 0 && qpb_better(fval[q], q, bv, bi)) { bv = fval[q]; bi = q; }
    qpb_block_argmin(bv, bi);
    if (threadIdx.x == 0) { pv[blockIdx.x] = bv; pi[blockIdx.x] = bi; }
}

__global__ void __launch_bounds__(1024) qpb_argmin_final(long nb, const double *__restrict__ pv,
                                                         const long *__restrict__ pi, double *__restrict__ out) {
    double bv = INFINITY;
    long bi = -1;
    for (long k = threadIdx.x; k < nb; k += blockDim.x)
        if (qpb_better(pv[k], pi[k], bv, bi)) { bv = pv[k]; bi = pi[k]; }
    qpb_block_argmin(bv, bi);
    if (threadIdx.x == 0) { out[0] = bv; out[1] = (double)bi; }
}

__global__ void __launch_bounds__(1024) qpb_argmin_single(long B, const double *__restrict__ fval,
                                                          const int *__restrict__ flag, double *__restrict__ out) {
    double bv = INFINITY;
    long bi = -1;
    for (long q = threadIdx.x; q < B; q += blockDim.x)
        if (flag[q] == 0 && qpb_better(fval[q], q, bv, bi)) { bv = fval[q]; bi = q; }
    qpb_block_argmin(bv, bi);
    if (threadIdx.x == 0) { out[0] = bv; out[1] = (double)bi; }
}

// The winner's payload for the multi-GPU gather: {fval, index,
// x*[0..n)} -- x of QP `index` read from the tiled outputs, NaN when the batch
// has no optimal QP (index -1).  One wavefront; stream-ordered after the solve.
__global__ void __launch_bounds__(64) qpb_winner_k(const double *__restrict__ best, const double *__restrict__ x,
                                                   long n, long B, double *__restrict__ out) {
    const double fv = best[0];
    const long q = (long)best[1];
    const bool ok = q >= 0 && q < B;
    if (threadIdx.x == 0) { out[0] = fv; out[1] = best[1]; }
    for (long j = threadIdx.x; j < n; j += 64)
        out[2 + j] = ok ? x[(q >> 6) * n * 64 + j * 64 + (q & 63)] : __builtin_nan("");
}

// Strided segment copies dst[i * ds] = src[i * ss]; blockIdx.y selects the
// segment.  Used by the single-QP drop-in to move packed host-order vectors in
// and out of the tiled SoA layout with one H2D and one D2H transfer.
__global__ void __launch_bounds__(256) qpb_strided_copy(qpb::CopySegs t) {
    const qpb::CopySeg sg = t.seg[blockIdx.y];
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < sg.n; i += (long)gridDim.x * blockDim.x)
        sg.dst[i * sg.ds] = sg.src[i * sg.ss];
}

}  // namespace

qpb_plan::~qpb_plan() {
    for (auto &kv : ctl_dev) {
        int cur = 0;
        if (hipGetDevice(&cur) == hipSuccess && hipSetDevice(kv.first) == hipSuccess) {
            (void)hipFree(kv.second);
            (void)hipSetDevice(cur);
        }
    }
    for (auto *m : {&tree_dev, &tree2_dev})
        for (auto &kv : *m) {
            int cur = 0;
            if (hipGetDevice(&cur) == hipSuccess && hipSetDevice(kv.first) == hipSuccess) {
                (void)hipFree(kv.second);
                (void)hipSetDevice(cur);
            }
        }
}

namespace qpb {

// ---- the kernel compiler ------------------------------------------------------
// Generated kernels are compiled for gfx950 by ONE pinned compiler: ROCm's clang
// (ROCM_PATH or /opt/rocm, lib/llvm/bin/clang++; QPB_CLANG overrides), run as a
// child process.  In-process hiprtc would use whichever libamd_comgr the process
// loaded first -- torch ships its own ROCm 7.0 comgr, a C++ controller gets
// /opt/rocm's -- so the same source could become different code objects in a test
// and in the product.  hiprtc stays as the fallback when no clang is installed.
// The code-object cache file name carries the compiler's identity and options:
// <kernel name>.<hash(compiler version, options)>.hsaco.

struct Compiler {
    std::string clang;   // path, empty -> hiprtc
    std::string ident;   // version line(s) of the compiler actually used
};

// run argv, stdout+stderr into *out; returns the exit status (-1: not started)
static int run_child(const std::vector<std::string> &argv, std::string *out) {
    char tmpl[] = "/tmp/qpb_logXXXXXX";
    std::string dir = getenv("TMPDIR") && *getenv("TMPDIR") ? getenv("TMPDIR") : "/tmp";
    std::string logp = dir + "/qpb_logXXXXXX";
    std::vector<char> lp(logp.begin(), logp.end());
    lp.push_back(0);
    int fd = mkstemp(lp.data());
    if (fd < 0) { fd = mkstemp(tmpl); if (fd < 0) return -1; lp.assign(tmpl, tmpl + sizeof(tmpl)); }
    posix_spawn_file_actions_t fa;
    posix_spawn_file_actions_init(&fa);
    posix_spawn_file_actions_adddup2(&fa, fd, 1);
    posix_spawn_file_actions_adddup2(&fa, fd, 2);
    posix_spawn_file_actions_addopen(&fa, 0, "/dev/null", O_RDONLY, 0);
    std::vector<char *> av;
    for (auto &a : argv) av.push_back(const_cast<char *>(a.c_str()));
    av.push_back(nullptr);
    pid_t pid = 0;
    int rc = posix_spawn(&pid, av[0], &fa, nullptr, av.data(), environ);
    posix_spawn_file_actions_destroy(&fa);
    int status = -1;
    if (rc == 0) {
        while (waitpid(pid, &status, 0) < 0 && errno == EINTR) {}
        status = WIFEXITED(status) ? WEXITSTATUS(status) : 128 + (WIFSIGNALED(status) ? WTERMSIG(status) : 0);
    }
    close(fd);
    if (out) {
        std::vector<char> buf;
        read_file(lp.data(), buf);
        out->assign(buf.begin(), buf.end());
    }
    unlink(lp.data());
    return rc == 0 ? status : -1;
}

static const Compiler &compiler() {
    static Compiler c = [] {
        Compiler r;
        std::string path;
        if (const char *e = getenv("QPB_CLANG")) path = e;
        else {
            const char *rp = getenv("ROCM_PATH");
            path = std::string(rp && *rp ? rp : "/opt/rocm") + "/lib/llvm/bin/clang++";
        }
        std::string ver;
        if (path != "hiprtc" && access(path.c_str(), X_OK) == 0 && run_child({path, "--version"}, &ver) == 0) {
            r.clang = path;
            r.ident = ver.substr(0, ver.find("\nInstalledDir"));
        } else {
            int maj = 0, min = 0;
            hiprtcVersion(&maj, &min);
            r.ident = "hiprtc " + std::to_string(maj) + "." + std::to_string(min);
            // the comgr hiprtc resolved in THIS process (torch's or ROCm's)
            using getv_t = void (*)(size_t *, size_t *);
            if (auto gv = (getv_t)dlsym(RTLD_DEFAULT, "amd_comgr_get_version")) {
                size_t a = 0, b = 0;
                gv(&a, &b);
                r.ident += " comgr " + std::to_string(a) + "." + std::to_string(b);
            }
            Dl_info di;
            if (auto sym = dlsym(RTLD_DEFAULT, "amd_comgr_get_version"))
                if (dladdr(sym, &di) && di.dli_fname) r.ident += std::string(" ") + di.dli_fname;
        }
        return r;
    }();
    return c;
}

static std::vector<std::string> compile_options(bool exact) {
    // The default LLVM pipeline.  Round 2 shipped -amdgpu-enable-pre-ra-optimizations=0
    // against a wrong-iterate bug of the leaves-first trot wave kernel that an
    // -opt-bisect-limit search tied to that pass.  With today's kernel
    // sources the pass is harmless: every GPU test passes with it on, and the
    // round-2 source still fails with it on today (profiles/r03_diag72.log).
    // QPB_PRERA_OFF=1 brings the workaround back (part of the cache key).
    std::vector<std::string> o = {"--offload-arch=gfx950", "-O3", "-std=c++17"};
    if (getenv("QPB_PRERA_OFF")) {
        o.push_back("-mllvm");
        o.push_back("-amdgpu-enable-pre-ra-optimizations=0");
    }
    if (exact) o.push_back("-ffp-contract=off");
    // experiments only (diagnostics): extra compiler options, e.g. "-O1"; part of
    // the cache key.  A process keeps one code object per kernel name, so run
    // each variant in its own process.
    if (const char *e = getenv("QPB_CLANG_FLAGS")) {
        std::istringstream in(e);
        std::string t;
        while (in >> t) o.push_back(t);
    }
    return o;
}

// Every kernel is compiled through assembly: clang -S, then qpb_hazard's join_fixup
// moves lane-masked instructions the register allocator left ahead of an EXEC restore
// to just after it (the wide row kernel's aperture violation), and
// asm_fixup pads every DPP instruction of an inline-asm region with the wait states its
// operands' producers require (qpb_hazard.cpp); then the text is assembled and linked
// into the code object.
static int compile_with_clang(const std::string &clang, const std::string &kname, const std::string &src,
                              bool exact, std::vector<char> &code, std::string *fixup_report = nullptr) {
    std::string dir = getenv("TMPDIR") && *getenv("TMPDIR") ? getenv("TMPDIR") : "/tmp";
    const std::string base = dir + "/qpb_" + kname + "_" + std::to_string((long)getpid()) + "_" +
                             std::to_string((unsigned long)std::hash<std::thread::id>()(std::this_thread::get_id()));
    const std::string sp = base + ".hip", op = base + ".co", ap = base + ".s", obp = base + ".o";
    {
        std::ofstream f(sp, std::ios::binary);
        if (!f) return fail(QPB_ECOMPILE, "cannot write " + sp);
        f << src;
    }
    // QPB_NO_ASM_FIXUP=1: experiments only (no assembly pass at all); part of the cache key
    const bool via_asm = !getenv("QPB_NO_ASM_FIXUP");
    const std::string bindir = clang.substr(0, clang.rfind('/'));
    std::vector<std::string> argv = {clang, "-x", "hip", "--cuda-device-only", "--no-gpu-bundle-output",
                                     "-I" + clang.substr(0, clang.rfind("/lib/llvm/bin/")) + "/include",
                                     "-include", "hip/hip_runtime.h"};
    for (auto &o : compile_options(exact)) argv.push_back(o);
    if (via_asm) argv.push_back("-S");
    argv.push_back("-o");
    argv.push_back(via_asm ? ap : op);
    argv.push_back(sp);
    std::string log;
    int st = run_child(argv, &log);
    unlink(sp.c_str());
    if (st == 0 && via_asm) {
        std::vector<char> txt;
        if (!read_file(ap, txt)) st = -1;
        else {
            std::string as(txt.begin(), txt.end());
            std::string rep, jrep;
            const int jr = join_fixup(as, &jrep);
            asm_fixup(as, &rep);
            if (fixup_report) *fixup_report = jrep + "; " + rep;
            if (jr < 0) {
                unlink(ap.c_str());
                return fail(QPB_ECOMPILE, "kernel " + kname + ": " + jrep);
            }
            write_file(ap, std::vector<char>(as.begin(), as.end()));
            st = run_child({bindir + "/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa", "-mcpu=gfx950", "-c",
                            ap, "-o", obp}, &log);
            if (st == 0) st = run_child({bindir + "/ld.lld", "-shared", obp, "-o", op}, &log);
        }
        unlink(ap.c_str());
        unlink(obp.c_str());
    }
    if (st != 0 || !read_file(op, code)) {
        unlink(op.c_str());
        return fail(QPB_ECOMPILE, "clang (" + clang + ") exit " + std::to_string(st) + ": " + log.substr(0, 4000));
    }
    unlink(op.c_str());
    return QPB_OK;
}

static int compile_with_hiprtc(const std::string &kname, const std::string &src, bool exact, std::vector<char> &code) {
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, src.c_str(), (kname + ".hip").c_str(), 0, nullptr, nullptr) != HIPRTC_SUCCESS)
        return fail(QPB_ECOMPILE, "hiprtcCreateProgram failed");
    const auto opt = compile_options(exact);
    std::vector<const char *> opts;
    for (auto &o : opt) opts.push_back(o.c_str());
    hiprtcResult rc = hiprtcCompileProgram(prog, (int)opts.size(), opts.data());
    if (rc != HIPRTC_SUCCESS) {
        size_t ls = 0;
        hiprtcGetProgramLogSize(prog, &ls);
        std::string log(ls, '\0');
        if (ls) hiprtcGetProgramLog(prog, &log[0]);
        hiprtcDestroyProgram(&prog);
        return fail(QPB_ECOMPILE, "hiprtc: " + log.substr(0, 4000));
    }
    size_t cs = 0;
    hiprtcGetCodeSize(prog, &cs);
    code.resize(cs);
    hiprtcGetCode(prog, code.data());
    hiprtcDestroyProgram(&prog);
    return QPB_OK;
}

std::string compiler_ident() { return compiler().ident; }

// ---- DPP hazard audit of a compiled code object ----------------------------
// llvm-objdump the code object and check every DPP instruction on every path into
// it (qpb_hazard.cpp: 2 wait states after a VALU write of any VGPR it reads, 5
// after a VALU write of EXEC).  Returns 1 clean, 0 hazard found (report says
// where), -1 could not audit.
int dpp_audit(const std::vector<char> &code, std::string *report) {
    const Compiler &cc = compiler();
    std::string objdump;
    if (!cc.clang.empty()) objdump = cc.clang.substr(0, cc.clang.rfind('/')) + "/llvm-objdump";
    else {
        const char *rp = getenv("ROCM_PATH");
        objdump = std::string(rp && *rp ? rp : "/opt/rocm") + "/lib/llvm/bin/llvm-objdump";
    }
    if (access(objdump.c_str(), X_OK) != 0) { *report = "no llvm-objdump"; return -1; }
    std::string dir = getenv("TMPDIR") && *getenv("TMPDIR") ? getenv("TMPDIR") : "/tmp";
    const std::string path = dir + "/qpb_audit_" + std::to_string((long)getpid()) + "_" +
                             std::to_string((unsigned long)std::hash<std::thread::id>()(std::this_thread::get_id())) + ".co";
    write_file(path, code);
    std::string dis;
    const int st = run_child({objdump, "-d", "--mcpu=gfx950", path}, &dis);
    unlink(path.c_str());
    if (st != 0) { *report = "llvm-objdump failed"; return -1; }
    return audit_disassembly(dis, report);
}


// Compile or fetch from the memory / disk cache (keyed by compiler identity).
int compile_kernel(const std::string &kname, const std::function<std::string()> &gen_src, bool exact,
                   std::shared_ptr<std::vector<char>> *out) {
    if (*out) return QPB_OK;
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_code.find(kname);
    if (it != g_code.end()) { *out = it->second; return QPB_OK; }
    const Compiler &cc = compiler();
    std::string id = cc.ident;
    for (auto &o : compile_options(exact)) id += " " + o;
    id += getenv("QPB_NO_ASM_FIXUP") ? " no-dpp-fixup" : " dpp-wait-states-v2 join-fixup-v1";   // qpb_hazard.cpp's rules
    char tag[17];
    snprintf(tag, sizeof tag, "%016llx", (unsigned long long)fnv1a(id));
    const std::string dir = cache_dir();
    const std::string path = dir + "/" + kname + "." + tag + ".hsaco";
    auto code = std::make_shared<std::vector<char>>();
    // a cached object must define the kernel it is filed under (its symbol table holds the
    // name): one that does not is discarded and rebuilt
    auto defines = [&kname](const std::vector<char> &obj) {
        return std::search(obj.begin(), obj.end(), kname.begin(), kname.end()) != obj.end();
    };
    if (!getenv("QPB_NO_DISK_CACHE") && read_file(path, *code) && defines(*code)) {
        g_code[kname] = code;
        *out = code;
        return QPB_OK;
    }
    std::string src = gen_src();
    // the name is a hash of the source the plan was made with; a source generated under
    // other knobs (QPB_WAVE_OPTS changed since the plan was made) defines another kernel
    // and must not be filed under this name
    if (src.find(kname) == std::string::npos)
        return fail(QPB_ECOMPILE, "kernel " + kname + ": the source generated now defines another kernel "
                                  "(QPB_WAVE_OPTS changed since the plan was made?)");
    std::string fix;
    int rc = cc.clang.empty() ? compile_with_hiprtc(kname, src, exact, *code)
                              : compile_with_clang(cc.clang, kname, src, exact, *code, &fix);
    if (rc) return rc;
    // every code object is audited (qpb_hazard.cpp): DPP wait states, trans forwarding,
    // VALU SGPR -> VMEM, and lane-masked code ahead of an EXEC restore at a join
    std::string audit;
    const int ok = dpp_audit(*code, &audit);
    if (!fix.empty()) audit = fix + "; audit: " + audit;
    auto join_bad = [](const std::string &a) {
        return a.find("lane-partial join") != std::string::npos && a.find(" 0 lane-partial join(s)") == std::string::npos;
    };
    if (ok != 1 && src.find("v_fmac_f64_dpp") != std::string::npos && !join_bad(audit)) {
        // DPP from inline asm: on a hazard (or no way to check) rebuild with wait
        // states inside every DPP asm (QPB_DPP_NOP = 2), hazard-free by construction
        src = "#define QPB_DPP_NOP 2\n" + src;
        rc = cc.clang.empty() ? compile_with_hiprtc(kname, src, exact, *code)
                              : compile_with_clang(cc.clang, kname, src, exact, *code, &fix);
        if (rc) return rc;
        audit += " -> rebuilt with QPB_DPP_NOP=2";
    } else if (ok != 1 && join_bad(audit)) {
        // a lane-partial join the assembly pass could not repair (or no assembly pass:
        // hiprtc): the code object would read stale registers in some lanes -- refuse it
        return fail(QPB_ECOMPILE, "kernel " + kname + " failed the audit: " + audit);
    }
    mkdir(dir.c_str(), 0755);
    write_file(path, *code);
    write_file(path + ".audit", std::vector<char>(audit.begin(), audit.end()));
    g_code[kname] = code;
    *out = code;
    return QPB_OK;
}

int compile_plan(qpb_plan *plan) {
    return compile_kernel(plan->kname, [plan] { return generate_kernel(plan->pl, plan->gen); }, plan->gen.exact,
                          &plan->code);
}

std::string wave_source_of(const qpb_plan *plan) {
    return plan->wave_rowx ? generate_rowx_kernel(plan->pl, nullptr)
           : plan->wave_qpw == 4 ? generate_row_kernel(plan->pl, nullptr)
                                 : generate_wave_kernel(plan->pl, plan->wave_wg, nullptr);
}

int compile_wave(qpb_plan *plan) {
    if (!plan->wave_ok) return fail(QPB_EINVAL, "plan is not eligible for the wave kernel");
    return compile_kernel(plan->wave_kname, [plan] { return wave_source_of(plan); }, false, &plan->wave_code);
}

int compile_rowsplit(qpb_plan *plan) {
    if (!plan->row_split) return fail(QPB_EINVAL, "plan has no split row kernel");
    return compile_kernel(plan->rowsplit_kname, [plan] { return generate_row_kernel(plan->pl, nullptr, 1, true); },
                          false, &plan->rowsplit_code);
}

int compile_row2(qpb_plan *plan) {
    if (plan->row_occ_batch < 0) return fail(QPB_EINVAL, "plan has no two-wave row kernel");
    return compile_kernel(plan->row2_kname, [plan] { return generate_row_kernel(plan->pl, nullptr, 2); }, false,
                          &plan->row2_code);
}

// the tree kernel's plan tables on the current device (uploaded on first use;
// a regular hipMalloc buffer, so they are cached in L2 like any input)
int tree_tables_on_device(qpb_plan *plan, const void **out, bool second) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return fail(QPB_EHIP, "hipGetDevice failed (no GPU?)");
    std::map<int, void *> &cache = second ? plan->tree2_dev : plan->tree_dev;
    const std::vector<char> &tab = second ? plan->tree2_tables : plan->tree_tables;
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = cache.find(dev);
    if (it != cache.end()) { *out = it->second; return QPB_OK; }
    void *p = nullptr;
    const size_t n = std::max<size_t>(tab.size(), 8);
    if (hipMalloc(&p, n) != hipSuccess) return fail(QPB_ENOMEM, "tree tables: hipMalloc failed");
    if (hipMemcpy(p, tab.data(), tab.size(), hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(p);
        return fail(QPB_EHIP, "tree tables: upload failed");
    }
    cache[dev] = p;
    *out = p;
    return QPB_OK;
}

// per-(device, stream) partials + arrival counter of the fused argmin (the counter
// is zeroed once here and re-armed by every launch's last wave; launches on one
// stream are ordered, launches on different streams use different scratch)
int argmin_scratch(void *stream, long nw, unsigned long long **part, unsigned **ctr) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return fail(QPB_EHIP, "hipGetDevice failed (no GPU?)");
    struct Scratch { void *p = nullptr; long cap = 0; };
    static std::map<std::pair<int, void *>, Scratch> pool;
    std::lock_guard<std::mutex> lk(g_mu);
    Scratch &sc = pool[{dev, stream}];
    if (sc.cap < nw) {
        if (sc.p) {
            (void)hipStreamSynchronize((hipStream_t)stream);
            (void)hipFree(sc.p);
        }
        const long cap = std::max(nw, 4096L);
        if (hipMalloc(&sc.p, 256 + (size_t)cap * 16) != hipSuccess) { sc = Scratch(); return fail(QPB_ENOMEM, "argmin scratch"); }
        if (hipMemset(sc.p, 0, 256) != hipSuccess) return fail(QPB_EHIP, "argmin scratch: memset failed");
        sc.cap = cap;
    }
    *ctr = (unsigned *)sc.p;
    *part = (unsigned long long *)((char *)sc.p + 256);
    return QPB_OK;
}

int compile_tree(qpb_plan *plan) {
    if (!plan->tree_ok) return fail(QPB_EINVAL, "plan is not eligible for the tree kernel");
    return compile_kernel(plan->tree_kname, [plan] { return generate_tree_kernel(plan->pl, plan->tree_wg, nullptr); },
                          false, &plan->tree_code);
}

bool rowx_auto() {
    static const bool on = [] { const char *e = getenv("QPB_ROWX"); return !(e && atoi(e) == 0); }();
    return on;
}

bool band_auto() {
    static const bool on = [] { const char *e = getenv("QPB_BAND"); return !(e && atoi(e) == 0); }();
    return on;
}

// the kernel a solve of B QPs runs: wave (row) form, band, tree, else the lane kernel
Pick pick_kernel(const qpb_plan *plan, long B, bool warm) {
    Pick k;
    const int pref = plan->kernel_pref;
    k.wave = plan->wave_ok && (pref == 2 || (pref == 0 && (plan->wave_max_batch < 0 || B <= plan->wave_max_batch)));
    // cold and warm solves alike (the band kernel's QPB_WARM variant, round 6)
    k.band = !k.wave && plan->band_ok && (pref == 4 || (pref == 0 && plan->large_tree && band_auto()));
    // QPB_KERNEL_BAND on a plan the band kernel cannot take: the tree kernel whenever it can
    // run the plan (such solves fell to the lane kernel for N <= 64)
    k.tree = !k.wave && !k.band && (pref == 3 || (pref == 4 && plan->tree_ok) || (pref == 0 && plan->large_tree));
    return k;
}

int compile_band(qpb_plan *plan) {
    if (!plan->band_ok) return fail(QPB_EINVAL, "plan is not eligible for the band kernel");
    return compile_kernel(plan->band_kname, [plan] { return generate_band_kernel(plan->pl, nullptr); }, false,
                          &plan->band_code);
}

int compile_tree2(qpb_plan *plan) {
    if (plan->tree_occ_batch < 0) return fail(QPB_EINVAL, "plan has no large-batch tree kernel");
    return compile_kernel(plan->tree2_kname, [plan] { return generate_tree_kernel(plan->pl, plan->tree2_wg, nullptr); },
                          false, &plan->tree2_code);
}

// The warm-solve variant of a plan's kernel: its source with QPB_WARM = 1 under
// the name <kname>_w (a separate code object, so the cold kernels -- the batched
// hot path -- keep their register allocation).
static std::mutex g_warm_mu;

// Device side of qpb::serve_ex, prepended to a QPB_SERVE variant's source.  The
// mailbox lives in fine-grained (coherent) pinned host memory: the request word is
// read with system-scope loads (no cache holds it), the answer is written after a
// system-scope release, which makes the solve's results visible to the host first.
// The wave polls with a short sleep between reads and leaves after `idle` ticks of
// the 100 MHz s_memrealtime clock without a new request, or on the stop value, so
// every launch ends on its own.
static const char *kServePrelude = R"QPBS(
struct qpb_mailbox;
#define QPB_SERVE_STOP (~0ull)
static __device__ __forceinline__ unsigned long long qpb_uniform64(unsigned long long v) {
    const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)v);
    const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(v >> 32));
    return ((unsigned long long)hi << 32) | lo;
}
// idle: ticks without a request before leaving; life: ticks since the launch
// (t_launch) after which the wave leaves at its next idle moment, so that work
// queued behind it on a shared hardware queue (more streams than queues) waits
// at most that long
static __device__ bool qpb_serve_wait(qpb_mailbox *mb, unsigned long long *last, unsigned long long idle,
                                      unsigned long long life, unsigned long long t_launch,
                                      unsigned long long *t_seen) {
    unsigned long long *req = (unsigned long long *)mb;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        const unsigned long long r = qpb_uniform64(__hip_atomic_load(req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
        if (r == QPB_SERVE_STOP) return false;
        if (r != *last) {
            *last = r;
            *t_seen = __builtin_amdgcn_s_memrealtime();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            // the fence's L1 invalidate completes asynchronously: wait for it before the
            // body's first load, or lines this CU read for the previous request (the
            // zero-copy slab, re-read every request) can be served stale
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            return true;
        }
        const unsigned long long now = __builtin_amdgcn_s_memrealtime();
        if (now - t0 > idle || (*t_seen != 0 && now - t_launch > life)) return false;   // life: after a first request
        __builtin_amdgcn_s_sleep(4);
    }
}
// the answer: [16] the request's number, [32] the ticks from seeing it to here
static __device__ void qpb_serve_done(qpb_mailbox *mb, unsigned long long r, unsigned long long t_seen) {
    unsigned long long *ack = (unsigned long long *)mb + 16, *dt = (unsigned long long *)mb + 32;
    if ((threadIdx.x & 63) == 0) *dt = __builtin_amdgcn_s_memrealtime() - t_seen;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    if ((threadIdx.x & 63) == 0) __hip_atomic_store(ack, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
)QPBS";

// a variant's name: `<kname>_w` (warm), `_s<tag>` (persistent cold) or `_ws<tag>`
// (persistent warm); the persistent forms carry a hash of the prelude they are
// built with, so a changed prelude never reuses a cached code object
static std::string variant_name(const std::string &kname, bool warm, bool serve) {
    static const std::string tag = [] {
        char t[9];
        snprintf(t, sizeof t, "%08x", (unsigned)(fnv1a(kServePrelude) & 0xffffffffu));
        return std::string(t);
    }();
    return kname + (warm ? (serve ? "_ws" : "_w") : "_s") + (serve ? tag : std::string());
}

// a variant of a plan's kernel -- its source with QPB_WARM / QPB_SERVE set, under
// variant_name()
int compile_variant(qpb_plan *plan, const std::string &kname, const std::function<std::string()> &gen_src,
                           bool exact, bool warm, bool serve, std::shared_ptr<std::vector<char>> **slot) {
    const std::string vname = variant_name(kname, warm, serve);
    {
        std::lock_guard<std::mutex> lk(g_warm_mu);
        *slot = &plan->warm_code[vname];     // std::map nodes are stable
    }
    return compile_kernel(vname, [&] {
        std::string src = gen_src();
        for (size_t pos = 0; (pos = src.find(kname, pos)) != std::string::npos; pos += vname.size())
            src.replace(pos, kname.size(), vname);
        return std::string(warm ? "#define QPB_WARM 1\n" : "") + (serve ? "#define QPB_SERVE 1\n" : "") +
               (serve ? kServePrelude : "") + src;
    }, exact, *slot);
}

int compile_warm(qpb_plan *plan, const std::string &kname, const std::function<std::string()> &gen_src, bool exact,
                 std::shared_ptr<std::vector<char>> **slot) {
    return compile_variant(plan, kname, gen_src, exact, true, false, slot);
}

int load_function(const std::string &kname, const std::shared_ptr<std::vector<char>> &code, hipFunction_t *fn) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return fail(QPB_EHIP, "hipGetDevice failed (no GPU?)");
    std::lock_guard<std::mutex> lk(g_mu);
    auto key = std::make_pair(dev, kname);
    auto it = g_funcs.find(key);
    if (it != g_funcs.end()) { *fn = it->second.second; return QPB_OK; }
    hipModule_t mod;
    hipError_t e = hipModuleLoadData(&mod, code->data());
    if (e != hipSuccess) {
        (void)hipGetLastError();     // not left behind for a later launch's hipGetLastError to report
        return fail(QPB_EHIP, std::string("hipModuleLoadData: ") + hipGetErrorString(e));
    }
    hipFunction_t f;
    e = hipModuleGetFunction(&f, mod, kname.c_str());
    if (e != hipSuccess) {
        (void)hipGetLastError();
        (void)hipModuleUnload(mod);
        return fail(QPB_EHIP, std::string("hipModuleGetFunction(") + kname + "): " + hipGetErrorString(e));
    }
    g_funcs[key] = {mod, f};
    *fn = f;
    return QPB_OK;
}

int set_error(int code, const char *msg) { return fail(code, msg); }

int strided_copy(const CopySegs &t, void *stream) {
    if (t.nseg <= 0) return QPB_OK;
    if (t.nseg > CopySegs::kMax) return fail(QPB_EINVAL, "strided copy: too many segments");
    long mx = 1;
    for (int i = 0; i < t.nseg; i++) mx = std::max(mx, t.seg[i].n);
    const unsigned gx = (unsigned)std::min<long>(64, (mx + 255) / 256);
    (void)hipGetLastError();   // a stale error of an earlier API call is not this launch's
    hipLaunchKernelGGL(qpb_strided_copy, dim3(gx, (unsigned)t.nseg), dim3(256), 0, (hipStream_t)stream, t);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(QPB_EHIP, std::string("strided copy: ") + hipGetErrorString(e));
    return QPB_OK;
}

}  // namespace qpb

extern "C" {

const char *qpb_last_error(void) { return g_err.c_str(); }
const char *qpb_version(void) { return "qpswift-hip 0.2 (gfx950)"; }

int qpb_audit_dpp(const void *code, long size, char *report, long cap) {
    if (!code || size <= 0) return fail(QPB_EINVAL, "empty code object");
    std::vector<char> c((const char *)code, (const char *)code + size);
    std::string rep;
    const int r = qpb::dpp_audit(c, &rep);
    if (report && cap > 0) {
        const long k = std::min<long>(cap - 1, (long)rep.size());
        std::memcpy(report, rep.data(), (size_t)k);
        report[k] = 0;
    }
    return r;
}

long qpb_join_fixup(char *text, long cap, char *report, long rcap) {
    if (!text || cap <= 0) return fail(QPB_EINVAL, "no text");
    std::string s(text), rep;
    const int r = qpb::join_fixup(s, &rep);
    if (report && rcap > 0) {
        const long k = std::min<long>(rcap - 1, (long)rep.size());
        std::memcpy(report, rep.data(), (size_t)k);
        report[k] = 0;
    }
    if ((long)s.size() + 1 > cap) return fail(QPB_EINVAL, "repaired text does not fit");
    std::memcpy(text, s.c_str(), s.size() + 1);
    return r;
}

const char *qpb_compiler(void) {
    static std::string id = qpb::compiler_ident();
    return id.c_str();
}

void qpb_default_settings(qpb_settings *st) {
    st->maxit = 100;
    st->reltol = 1e-6;
    st->abstol = 1e-6;
    st->sigma_d = 0.0;
}

int qpb_plan_create(qpb_plan **out, long n, long m, long p, int flags,
                    const long *Pjc, const long *Pir, const long *Ajc, const long *Air,
                    const long *Gjc, const long *Gir, const long *perm) {
    if (!out) return fail(QPB_EINVAL, "plan out-pointer is NULL");
    *out = nullptr;
    std::unique_ptr<qpb_plan> plan(new (std::nothrow) qpb_plan());
    if (!plan) return fail(QPB_ENOMEM, "out of host memory");
    std::string err;
    const int order = (flags & QPB_ORDER_LEAVES) ? qpb::ORDER_LEAVES : (flags & QPB_ORDER_MINDEG) ? qpb::ORDER_MINDEG
                    : (flags & QPB_ORDER_AMD) ? qpb::ORDER_AMD : qpb::ORDER_OWN;
    int rc = qpb::build_plan(plan->pl, n, m, p, (flags & QPB_P_UPPER) ? qpb::P_UPPER : qpb::P_FULL,
                             Pjc, Pir, Ajc, Air, Gjc, Gir, perm, &err, order);
    if (rc) return fail(rc, err);
    plan->gen = qpb::choose_options(plan->pl, (flags & QPB_EXACT) != 0);
    // experiment overrides (kernel name encodes them, so caches stay consistent)
    if (const char *e = getenv("QPB_WG")) plan->gen.wg = atoi(e);
    if (const char *e = getenv("QPB_LDS")) plan->gen.lds_mode = atoi(e);
    if (const char *e = getenv("QPB_PARKZ")) plan->gen.park_z = atoi(e);
    plan->kname = qpb::kernel_name_of(qpb::generate_kernel(plan->pl, plan->gen));
    // wave-cooperative kernel: fast mode only (its elimination order differs
    // from the reference's), for plans whose KKT has the z/y-leaf structure
    std::string why;
    plan->wave_ok = !plan->gen.exact && qpb::wave_eligible(plan->pl, &why);
    plan->kernel_pref = (flags & QPB_KERNEL_BAND) ? 4 : (flags & QPB_KERNEL_TREE) ? 3 : (flags & QPB_KERNEL_WAVE) ? 2
                      : (flags & QPB_KERNEL_LANE) ? 1 : 0;
    if (plan->kernel_pref == 2 && !plan->wave_ok)
        return fail(QPB_EINVAL, "QPB_KERNEL_WAVE: " + (plan->gen.exact ? std::string("exact plans use the lane kernel") : why));
    // tree kernel (one QP per workgroup, level-scheduled sparse LDL'): any
    // fast-mode plan whose per-QP state fits the LDS; auto dispatch uses it for
    // KKT systems too large for one QP per lane (N > 64)
    std::string why_tree;
    plan->tree_ok = !plan->gen.exact && qpb::tree_eligible(plan->pl, &why_tree);
    plan->large_tree = plan->tree_ok && plan->pl.N > 64;
    if (plan->kernel_pref == 3 && !plan->tree_ok)
        return fail(QPB_EINVAL, "QPB_KERNEL_TREE: " + (plan->gen.exact ? std::string("exact plans use the lane kernel") : why_tree));
    if (plan->tree_ok) {
        plan->tree_wg = qpb::tree_wg_for(plan->pl);
        qpb::generate_tree_kernel(plan->pl, plan->tree_wg, &plan->tree_kname, nullptr, &plan->tree_tables);
        // 256-thread plans (N > 160): beyond two QPs per CU (512 QPs) a 192-thread
        // form, whose registers (<= 168: three waves per SIMD) and LDS allow four
        // (MPC 1 024 QPs: 3.04 -> 1.65 ms; 128 threads 1.70; at 512 and below the
        // 256-thread form's shorter step chain wins)
        if (plan->tree_wg == 256 && !getenv("QPB_TREE_WG")) {
            plan->tree_occ_batch = 512;
            if (const char *e = getenv("QPB_TREE_OCC_BATCH")) plan->tree_occ_batch = atol(e);
            if (plan->tree_occ_batch >= 0) {
                plan->tree2_wg = 192;
                if (const char *e = getenv("QPB_TREE2_WG")) plan->tree2_wg = atoi(e) == 128 ? 128 : 192;
                qpb::generate_tree_kernel(plan->pl, plan->tree2_wg, &plan->tree2_kname, nullptr, &plan->tree2_tables);
            }
        }
    }
    // band kernel (multi-stage patterns in leaves-first order, cold solves): auto
    // dispatch takes it where the tree kernel would run (QPB_BAND=0: the tree kernel)
    std::string why_band;
    plan->band_ok = !plan->gen.exact && qpb::band_eligible(plan->pl, &why_band);
    if (plan->kernel_pref == 4 && !plan->band_ok)
        return fail(QPB_EINVAL, "QPB_KERNEL_BAND: " + (plan->gen.exact ? std::string("exact plans use the lane kernel") : why_band));
    if (plan->band_ok) qpb::generate_band_kernel(plan->pl, &plan->band_kname);
    plan->wave_max_batch = 4096;   // measured crossover vs the lane kernel
    if (plan->wave_ok) {
        // row form (four QPs per wavefront, all exchanges DPP) where the plan fits
        // a 16-lane row; QPB_KERNEL_NOROW or QPB_ROW=0 keep one QP per wavefront
        const char *er = getenv("QPB_ROW");
        if (!(flags & QPB_KERNEL_NOROW) && !(er && atoi(er) == 0) && qpb::row_eligible(plan->pl)) {
            plan->wave_qpw = 4;
            plan->wave_wg = 64;
            plan->wave_max_batch = -1;   // the row form beats the lane kernel at every batch size
            qpb::generate_row_kernel(plan->pl, &plan->wave_kname);
            // beyond one wave per SIMD (4 QPs x 1 024 SIMDs) the two-wave allocation:
            // 2^20 C1 QPs 5.79 -> 3.98 ms; below it the one-wave kernel's latency wins
            // (1 024 QPs 32.7 vs 34.6 us: the two-wave form spills 11 registers)
            plan->row_occ_batch = 4096;
            if (const char *e = getenv("QPB_ROW_OCC_BATCH")) plan->row_occ_batch = atol(e);
            if (plan->row_occ_batch >= 0) qpb::generate_row_kernel(plan->pl, &plan->row2_kname, 2);
            if (const char *e = getenv("QPB_ROW_SPLIT")) plan->row_split = atoi(e) > 0;
            if (plan->row_split) qpb::generate_row_kernel(plan->pl, &plan->rowsplit_kname, 1, true);
        } else if (!(flags & QPB_KERNEL_NOROW) && !(er && atoi(er) == 0) && qpb::rowx_auto() &&
                   qpb::rowx_eligible(plan->pl, nullptr)) {
            // the wide row form (two x rows per lane) for plans up to 32 variables -- the
            // controller's 30-variable QPs in leaves-first order (QPB_ROWX=0: the wave form)
            plan->wave_qpw = 4;
            plan->wave_wg = 64;
            plan->wave_rowx = true;
            plan->wave_max_batch = -1;
            qpb::generate_rowx_kernel(plan->pl, &plan->wave_kname);
        } else {
            plan->wave_wg = qpb::wave_wg_for(plan->pl);
            qpb::generate_wave_kernel(plan->pl, plan->wave_wg, &plan->wave_kname);
        }
    }
    // for a large KKT system the alternative is the tree kernel.  On 30/68/18 the
    // wave kernel, with its leaf-row G'diag(w)G on the matrix cores (QPB_W_MFMA),
    // wins at every batch size: 1 024 QPs 0.95 vs 1.26 ms, 8 192 6.4 vs 7.0 ms
    // (before MFMA the tree kernel won beyond 512)
    if (plan->wave_ok && plan->large_tree) plan->wave_max_batch = -1;
    if (const char *e = getenv("QPB_WAVE_MAX")) plan->wave_max_batch = atol(e);
    *out = plan.release();
    return QPB_OK;
}

void qpb_plan_destroy(qpb_plan *plan) { delete plan; }

long qpb_plan_tree_tables(const qpb_plan *plan, void *buf, long cap) {
    if (!plan) return fail(QPB_EINVAL, "NULL plan");
    if (!plan->tree_ok) return fail(QPB_EINVAL, "plan is not eligible for the tree kernel");
    const long n = (long)plan->tree_tables.size();
    if (buf && cap > 0) std::memcpy(buf, plan->tree_tables.data(), (size_t)std::min(cap, n));
    return n;
}

int qpb_plan_get_info(const qpb_plan *plan, qpb_plan_info *info) {
    if (!plan || !info) return fail(QPB_EINVAL, "NULL argument");
    const qpb::Plan &pl = plan->pl;
    info->n = pl.n; info->m = pl.m; info->p = pl.p; info->N = pl.N;
    info->nnzP = pl.Pin.nnz(); info->nnzA = pl.p ? pl.A.nnz() : 0; info->nnzG = pl.G.nnz();
    info->nnzK = pl.K.nnz(); info->lnz = pl.lnz;
    info->fac_updates = pl.fac_updates; info->fac_divs = pl.fac_divs;
    info->ordering = pl.ordering_kind; info->exact = plan->gen.exact ? 1 : 0;
    info->hash = pl.hash;
    info->wave_ok = plan->wave_ok ? 1 : 0;
    info->wave_max_batch = (plan->kernel_pref == 1 || plan->kernel_pref == 3 || plan->kernel_pref == 4) ? 0 : plan->kernel_pref == 2 ? -1 : plan->wave_max_batch;
    info->wave_qpw = plan->wave_qpw;
    info->tree_ok = plan->tree_ok ? 1 : 0;
    info->large_kernel = qpb::pick_kernel(plan, 1L << 20, false).band ? 4
                       : plan->kernel_pref == 3 ? 3 : plan->kernel_pref == 2 ? 2 : plan->kernel_pref == 1 ? 1
                       : plan->large_tree ? 3 : 1;
    return QPB_OK;
}

int qpb_amd_order(long n, const long *Ap, const long *Ai, long *perm) {
    int rc = qpb::amd_order(n, Ap, Ai, perm);
    if (rc < 0) return fail(QPB_EINVAL, "qpb_amd_order: invalid pattern");
    return rc;
}

int qpb_plan_get_perm(const qpb_plan *plan, long *perm) {
    if (!plan || !perm) return fail(QPB_EINVAL, "NULL argument");
    std::memcpy(perm, plan->pl.perm.data(), sizeof(long) * plan->pl.N);
    return QPB_OK;
}

long qpb_plan_source(const qpb_plan *plan, char *buf, long cap) {
    if (!plan) return fail(QPB_EINVAL, "NULL plan");
    std::string s = qpb::generate_kernel(plan->pl, plan->gen);
    if (buf && cap > 0) {
        long k = std::min<long>(cap - 1, (long)s.size());
        std::memcpy(buf, s.data(), k);
        buf[k] = 0;
    }
    return (long)s.size();
}

long qpb_plan_tree_source(const qpb_plan *plan, char *buf, long cap) {
    if (!plan) return fail(QPB_EINVAL, "NULL plan");
    if (!plan->tree_ok) return fail(QPB_EINVAL, "plan is not eligible for the tree kernel");
    std::string s = qpb::generate_tree_kernel(plan->pl, plan->tree_wg, nullptr);
    if (buf && cap > 0) {
        long k = std::min<long>(cap - 1, (long)s.size());
        std::memcpy(buf, s.data(), k);
        buf[k] = 0;
    }
    return (long)s.size();
}

long qpb_plan_wave_source(const qpb_plan *plan, char *buf, long cap) {
    if (!plan) return fail(QPB_EINVAL, "NULL plan");
    if (!plan->wave_ok) return fail(QPB_EINVAL, "plan is not eligible for the wave kernel");
    std::string s = qpb::wave_source_of(plan);
    if (buf && cap > 0) {
        long k = std::min<long>(cap - 1, (long)s.size());
        std::memcpy(buf, s.data(), k);
        buf[k] = 0;
    }
    return (long)s.size();
}

long qpb_plan_kernel_name(const qpb_plan *plan, long B, char *buf, long cap) {
    if (!plan) return fail(QPB_EINVAL, "NULL plan");
    const qpb::Pick pk = qpb::pick_kernel(plan, B, false);
    const bool wave = pk.wave, tree = pk.tree;
    const std::string &s = pk.band ? plan->band_kname : wave ? (plan->row_occ_batch >= 0 && B > plan->row_occ_batch ? plan->row2_kname
                                   : plan->row_split ? plan->rowsplit_kname : plan->wave_kname)
                         : tree ? (plan->tree_occ_batch >= 0 && B > plan->tree_occ_batch ? plan->tree2_kname : plan->tree_kname)
                                : plan->kname;
    if (buf && cap > 0) {
        long k = std::min<long>(cap - 1, (long)s.size());
        std::memcpy(buf, s.data(), k);
        buf[k] = 0;
    }
    return (long)s.size();
}

int qpb_plan_compile_warm(qpb_plan *plan, long B) {
    if (!plan) return fail(QPB_EINVAL, "NULL plan");
    if (B < 1) B = 1;
    const qpb::Pick pk = qpb::pick_kernel(plan, B, true);
    const bool wave = pk.wave, tree = pk.tree, band = pk.band;
    const bool row2 = wave && plan->row_occ_batch >= 0 && B > plan->row_occ_batch;
    const bool tree2 = tree && plan->tree_occ_batch >= 0 && B > plan->tree_occ_batch;
    const std::string &kn = band ? plan->band_kname : row2 ? plan->row2_kname : wave ? plan->wave_kname
                          : tree2 ? plan->tree2_kname : tree ? plan->tree_kname : plan->kname;
    std::function<std::string()> gen =
        band ? std::function<std::string()>([plan] { return qpb::generate_band_kernel(plan->pl, nullptr); })
        : row2 ? std::function<std::string()>([plan] { return qpb::generate_row_kernel(plan->pl, nullptr, 2); })
        : wave ? std::function<std::string()>([plan] { return qpb::wave_source_of(plan); })
        : tree2 ? std::function<std::string()>([plan] { return qpb::generate_tree_kernel(plan->pl, plan->tree2_wg, nullptr); })
        : tree ? std::function<std::string()>([plan] { return qpb::generate_tree_kernel(plan->pl, plan->tree_wg, nullptr); })
               : std::function<std::string()>([plan] { return qpb::generate_kernel(plan->pl, plan->gen); });
    std::shared_ptr<std::vector<char>> *slot = nullptr;
    return qpb::compile_warm(plan, kn, gen, !wave && !tree && !band && plan->gen.exact, &slot);
}

int qpb_plan_compile_serve(qpb_plan *plan) {
    if (!plan) return fail(QPB_EINVAL, "NULL plan");
    if (!qpb::serve_eligible(plan)) return qpb::SERVE_NONE;
    std::shared_ptr<std::vector<char>> *slot = nullptr;
    auto gen = [plan] { return qpb::wave_source_of(plan); };
    int rc = qpb::compile_variant(plan, plan->wave_kname, gen, false, false, true, &slot);
    if (!rc) rc = qpb::compile_variant(plan, plan->wave_kname, gen, false, true, true, &slot);
    return rc;
}

int qpb_plan_compile(qpb_plan *plan) {
    if (!plan) return fail(QPB_EINVAL, "NULL plan");
    const int k = plan->kernel_pref;
    int rc = QPB_OK;
    if (k == 1 || (k == 0 && !plan->large_tree)) rc = qpb::compile_plan(plan);
    if (!rc && plan->wave_ok && (k == 0 || k == 2)) rc = qpb::compile_wave(plan);
    if (!rc && plan->wave_ok && (k == 0 || k == 2) && plan->row_occ_batch >= 0) rc = qpb::compile_row2(plan);
    if (!rc && plan->wave_ok && (k == 0 || k == 2) && plan->row_split) rc = qpb::compile_rowsplit(plan);
    if (!rc && plan->tree_ok && (k == 3 || (k == 0 && plan->large_tree))) rc = qpb::compile_tree(plan);
    if (!rc && plan->tree_ok && (k == 3 || (k == 0 && plan->large_tree)) && plan->tree_occ_batch >= 0)
        rc = qpb::compile_tree2(plan);
    if (!rc && plan->band_ok && (k == 4 || (k == 0 && plan->large_tree && qpb::band_auto()))) rc = qpb::compile_band(plan);
    return rc;
}

}  // extern "C"

int qpb::solve_ex(qpb_plan *plan, long B, const double *P, const double *A, const double *G,
                      const double *c, const double *h, const double *b, const qpb_settings *st,
                      double *x, double *y, double *z, double *s, int *flag, int *iters, double *fval,
                      double *stats, double *best, void *stream, double *sig, bool warm, double *trace) {
    if (warm && !sig) return fail(QPB_EINVAL, "a warm solve needs sigma");
    if (!plan) return fail(QPB_EINVAL, "NULL plan");
    if (B < 0) return fail(QPB_EINVAL, "need B >= 0");
    if (B == 0) return QPB_OK;
    const qpb::Plan &pl = plan->pl;
    if (!P || !G || !c || !h || !x || !z || !s || !flag || !iters || !fval)
        return fail(QPB_EINVAL, "NULL data pointer");
    if (pl.p > 0 && (!A || !b || !y)) return fail(QPB_EINVAL, "p > 0 needs A, b and y");
    // kernel choice: the wave kernel (one QP per wavefront) has the lower latency
    // and wins while the batch does not fill the GPU with lane-kernel waves
    // beyond it: the lane kernel (one QP per lane) for small KKT systems, the tree
    // kernel (one QP per workgroup) for large ones
    const qpb::Pick pk = qpb::pick_kernel(plan, B, warm);
    const bool wave = pk.wave, tree = pk.tree, band = pk.band;
    hipFunction_t fn;
    const bool row2 = wave && plan->row_occ_batch >= 0 && B > plan->row_occ_batch;
    const bool tree2 = tree && plan->tree_occ_batch >= 0 && B > plan->tree_occ_batch;
    const bool split = wave && !row2 && !warm && plan->row_split;      // cold batched solves only
    int rc;
    if (!warm) {
        rc = band ? qpb::compile_band(plan) : split ? qpb::compile_rowsplit(plan) : row2 ? qpb::compile_row2(plan)
           : wave ? qpb::compile_wave(plan) : tree2 ? qpb::compile_tree2(plan) : tree ? qpb::compile_tree(plan)
           : qpb::compile_plan(plan);
        if (!rc) rc = band ? qpb::load_function(plan->band_kname, plan->band_code, &fn)
                    : split ? qpb::load_function(plan->rowsplit_kname, plan->rowsplit_code, &fn)
                    : row2 ? qpb::load_function(plan->row2_kname, plan->row2_code, &fn)
                    : wave ? qpb::load_function(plan->wave_kname, plan->wave_code, &fn)
                    : tree2 ? qpb::load_function(plan->tree2_kname, plan->tree2_code, &fn)
                    : tree ? qpb::load_function(plan->tree_kname, plan->tree_code, &fn)
                           : qpb::load_function(plan->kname, plan->code, &fn);
    } else {
        if (wave && !plan->wave_ok) return fail(QPB_EINVAL, "plan is not eligible for the wave kernel");
        if (tree && !plan->tree_ok) return fail(QPB_EINVAL, "plan is not eligible for the tree kernel");
        const std::string &kn = band ? plan->band_kname : row2 ? plan->row2_kname : wave ? plan->wave_kname
                              : tree2 ? plan->tree2_kname : tree ? plan->tree_kname : plan->kname;
        std::function<std::string()> gen =
            band ? std::function<std::string()>([plan] { return qpb::generate_band_kernel(plan->pl, nullptr); })
            : row2 ? std::function<std::string()>([plan] { return qpb::generate_row_kernel(plan->pl, nullptr, 2); })
            : wave ? std::function<std::string()>([plan] { return qpb::wave_source_of(plan); })
            : tree2 ? std::function<std::string()>([plan] { return qpb::generate_tree_kernel(plan->pl, plan->tree2_wg, nullptr); })
            : tree ? std::function<std::string()>([plan] { return qpb::generate_tree_kernel(plan->pl, plan->tree_wg, nullptr); })
                   : std::function<std::string()>([plan] { return qpb::generate_kernel(plan->pl, plan->gen); });
        std::shared_ptr<std::vector<char>> *slot = nullptr;
        rc = qpb::compile_warm(plan, kn, gen, !wave && !tree && !band && plan->gen.exact, &slot);
        if (!rc) rc = qpb::load_function(kn + "_w", *slot, &fn);
    }
    if (rc) return rc;
    qpb_settings def;
    qpb_default_settings(&def);
    if (!st) st = &def;
    qpb::KernelArgs a;
    a.P = P; a.A = A; a.G = G; a.c = c; a.h = h; a.b = b;
    a.x = x; a.y = y; a.z = z; a.s = s;
    a.flag = flag; a.iters = iters; a.fval = fval; a.stats = stats;
    a.B = B;
    a.tol = st->reltol / std::sqrt(3.0);
    a.abstol = st->abstol;
    a.sigma_d = st->sigma_d;
    a.maxit = st->maxit;
    a.sig = sig;
    a.warm = warm ? 1 : 0;
    a.trace = warm ? trace : nullptr;      // only the warm variants trace
    if (tree && (rc = qpb::tree_tables_on_device(plan, &a.tab, tree2))) return rc;
    // qpb_solve_best on the row kernel: the argmin runs inside the solve launch
    // (its last wave reduces the per-wave partials), saving the separate launch
    // and the gap between two dependent launches; up to 4 096 waves
    bool fused = false;
    void *params[] = {&a};
    const unsigned wg = (unsigned)(band ? 64 : split ? 128 : wave ? plan->wave_wg : tree2 ? plan->tree2_wg
                                   : tree ? plan->tree_wg : plan->gen.wg);
    const long per_block = band ? 1 : split ? 4 : wave ? (wg / 64) * plan->wave_qpw : tree ? 1 : wg;    // QPs per workgroup
    unsigned grid = (unsigned)((B + per_block - 1) / per_block);
    if (wave || tree || band) grid = (grid + 7) & ~7u;      // XCD-aware block order (qpb_xcd_block)
    if (best && wave && plan->wave_qpw == 4 && !getenv("QPB_NO_FUSED_ARGMIN")) {
        const long nw = (long)grid * (wg / 64);
        if (nw <= 4096) {
            if ((rc = qpb::argmin_scratch(stream, nw, &a.part, &a.ctr))) return rc;
            a.best = best;
            fused = true;
        }
    }
    hipError_t e = hipModuleLaunchKernel(fn, grid, 1, 1, wg, 1, 1, 0, (hipStream_t)stream, params, nullptr);
    if (e != hipSuccess) return fail(QPB_EHIP, std::string("launch: ") + hipGetErrorString(e));
    // an in-kernel "last wave reduces" argmin was measured slower than this
    // separate single-block launch (agent-coherent stores + counter tail), DESIGN.md
    if (best && !fused) return qpb_argmin(B, fval, flag, best, stream);
    return QPB_OK;
}

// ---- persistent one-QP solver (qpb::Server) ---------------------------------
namespace {
constexpr unsigned long long kStop = ~0ull;
unsigned long long ms_ticks(const char *env, double dflt) {     // s_memrealtime ticks (100 MHz)
    const char *e = getenv(env);
    const double ms = e ? atof(e) : dflt;
    return (unsigned long long)(std::max(0.1, std::min(ms, 10000.0)) * 1e5);
}
unsigned long long serve_idle_ticks() {
    static const unsigned long long t = ms_ticks("QPSWIFT_HIP_SERVE_IDLE_MS", 20.0);
    return t;
}
// 0 (the default): a launch answers ONE request and leaves, and the host launches the
// next wave as soon as it has the answer, so the next call still finds a wave waiting.
// A wave that answers request after request (QPSWIFT_HIP_SERVE_LIFE_MS > 0, then also
// its lifetime) was measured to go wrong in some kernel builds -- the AMD-ordered trot
// kernel's resident setup wave returned wrong initial points from its second or third
// request on, depending on the loop's code layout -- so it is a
// diagnostic mode only.
// It is refused unless QPB_SERVE_DIAG=1 is set as well, so the knob alone can never
// put wrong answers into a controller.
unsigned long long serve_life_ticks() {
    static const unsigned long long t = [] {
        const char *e = getenv("QPSWIFT_HIP_SERVE_LIFE_MS");
        if (!(e && atof(e) > 0.0)) return 0ull;
        const char *d = getenv("QPB_SERVE_DIAG");
        if (!(d && d[0] == '1')) {
            fprintf(stderr, "qpswift-hip: QPSWIFT_HIP_SERVE_LIFE_MS ignored: multi-request persistent waves are a "
                            "diagnostics mode (set QPB_SERVE_DIAG=1 as well); one request per wave\n");
            return 0ull;
        }
        return ms_ticks("QPSWIFT_HIP_SERVE_LIFE_MS", 10.0);
    }();
    return t;
}
// the calling thread's servers, for serve_retire_thread (a server belongs to the
// workspace of the thread that solves through it).  A plain pointer, not a vector:
// thread_local objects are destroyed in reverse order of construction, and the
// drop-in's workspaces (which own Servers) are constructed before this list is first
// used -- so at thread exit ~Server runs after a thread_local vector would already be
// gone.  A trivially destructible pointer stays readable through the whole teardown;
// the list itself is freed by the last ~Server that empties it.
thread_local std::vector<qpb::Server *> *t_servers = nullptr;
unsigned long long mb_load(const unsigned long long *p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }
void mb_store(unsigned long long *p, unsigned long long v) { __atomic_store_n(p, v, __ATOMIC_RELEASE); }
}  // namespace

bool qpb::serve_eligible(const qpb_plan *plan) {
    return plan && plan->wave_ok &&
           (plan->kernel_pref == 2 || (plan->kernel_pref == 0 && (plan->wave_max_batch < 0 || 1 <= plan->wave_max_batch)));
}

// A retired server's wave saw the stop word (or will, the moment it starts): wait for
// it to leave and re-arm the mailbox before the next launch.
static int serve_settle(qpb::Server *srv) {
    if (!srv->retiring) return QPB_OK;
    srv->retiring = false;
    const hipError_t e = hipStreamSynchronize((hipStream_t)srv->stream);
    mb_store(srv->mb, srv->seq);
    return e == hipSuccess ? QPB_OK : fail(QPB_EHIP, std::string("persistent solver: ") + hipGetErrorString(e));
}

void qpb::serve_retire_thread() {
    if (!t_servers) return;
    for (Server *srv : *t_servers) {
        if (!srv->running) continue;
        mb_store(srv->mb, kStop);        // the queued wave leaves at its next poll (~0.1 us)
        srv->running = false;
        srv->retiring = true;
        srv->retires++;
    }
}

int qpb::serve_stop(Server *srv) {
    if (srv && srv->retiring) return serve_settle(srv);
    if (!srv || !srv->running) return QPB_OK;
    mb_store(srv->mb, kStop);
    const hipError_t e = hipStreamSynchronize((hipStream_t)srv->stream);
    srv->running = false;
    srv->kname.clear();
    mb_store(srv->mb, srv->seq);             // the next launch starts from `seq` again
    return e == hipSuccess ? QPB_OK : fail(QPB_EHIP, std::string("persistent solver: ") + hipGetErrorString(e));
}

qpb::Server::~Server() {
    (void)serve_stop(this);
    if (registered && t_servers) {
        auto &v = *t_servers;
        for (size_t i = 0; i < v.size(); i++)
            if (v[i] == this) { v.erase(v.begin() + (long)i); break; }
        if (v.empty()) { delete t_servers; t_servers = nullptr; }
    }
    if (stream) (void)hipStreamDestroy((hipStream_t)stream);
    if (mb) (void)hipHostFree(mb);
}

int qpb::serve_ex(qpb_plan *plan, Server *srv, const double *P, const double *A, const double *G, const double *c,
                  const double *h, const double *b, const qpb_settings *st, double *x, double *y, double *z,
                  double *s, int *flag, int *iters, double *fval, double *stats, double *sig, bool warm,
                  double *trace, const double *win, const std::function<void()> &while_waiting) {
    if (!plan || !srv) return fail(QPB_EINVAL, "NULL plan or server");
    if (warm && (!sig || !win)) return fail(QPB_EINVAL, "a warm solve needs sigma and the state block");
    const qpb::Plan &pl = plan->pl;
    if (!P || !G || !c || !h || !x || !z || !s || !flag || !iters || !fval) return fail(QPB_EINVAL, "NULL data pointer");
    if (pl.p > 0 && (!A || !b || !y)) return fail(QPB_EINVAL, "p > 0 needs A, b and y");
    // the kernel solve_ex would launch for one QP must be the row or the wave form
    if (!serve_eligible(plan)) return SERVE_NONE;
    std::shared_ptr<std::vector<char>> *slot = nullptr;
    int rc = compile_variant(plan, plan->wave_kname, [plan] { return qpb::wave_source_of(plan); }, false, warm, true,
                             &slot);
    const std::string kn = variant_name(plan->wave_kname, warm, true);
    hipFunction_t fn;
    if (!rc) rc = load_function(kn, *slot, &fn);
    if (rc) return rc;
    qpb_settings def;
    qpb_default_settings(&def);
    if (!st) st = &def;
    KernelArgs a;
    std::memset((void *)&a, 0, sizeof a);    // compared bytewise below
    a.P = P; a.A = A; a.G = G; a.c = c; a.h = h; a.b = b;
    a.x = x; a.y = y; a.z = z; a.s = s;
    a.flag = flag; a.iters = iters; a.fval = fval; a.stats = stats;
    a.B = 1;
    a.tol = st->reltol / std::sqrt(3.0);
    a.abstol = st->abstol;
    a.sigma_d = st->sigma_d;
    a.maxit = st->maxit;
    a.sig = sig;
    a.warm = warm ? 1 : 0;
    a.trace = warm ? trace : nullptr;
    a.win = warm ? win : nullptr;
    if (!srv->mb) {
        void *m = nullptr;
        if (hipHostMalloc(&m, 512, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess)
            return fail(QPB_ENOMEM, "persistent solver: mailbox allocation failed");
        std::memset(m, 0, 512);
        void *md = nullptr;
        if (hipHostGetDevicePointer(&md, m, 0) != hipSuccess) {
            (void)hipHostFree(m);
            return fail(QPB_EHIP, "persistent solver: mailbox has no device address");
        }
        srv->mb = (unsigned long long *)m;
        srv->mb_dev = (unsigned long long *)md;
        srv->seq = 0;
    }
    if (!srv->stream) {
        hipStream_t sm;
        if (hipStreamCreateWithFlags(&sm, hipStreamNonBlocking) != hipSuccess)
            return fail(QPB_EHIP, "persistent solver: stream creation failed");
        srv->stream = sm;
    }
    hipStream_t sm = (hipStream_t)srv->stream;
    if (!srv->registered) {
        if (!t_servers) t_servers = new std::vector<Server *>();
        t_servers->push_back(srv);
        srv->registered = true;
    }
    if ((rc = serve_settle(srv))) return rc;
    // a running kernel with other arguments or code: stop it first
    if (srv->running && (srv->kname != kn || std::memcmp(&srv->args, &a, sizeof a) != 0) && (rc = serve_stop(srv)))
        return rc;
    unsigned long long *req = srv->mb, *ack = srv->mb + 16;
    // (diagnostics: QPB_SERVE_DIAG_ONLY=cold|warm keeps the other kind one-shot)
    const char *only = getenv("QPB_SERVE_DIAG_ONLY");
    const unsigned long long life_k =
        (only && *only && std::strcmp(only, warm ? "warm" : "cold") != 0) ? 0ull : serve_life_ticks();
    auto launch = [&](unsigned long long last) {
        unsigned long long idle = serve_idle_ticks(), life = life_k;
        void *mbd = srv->mb_dev;
        void *params[] = {&a, &mbd, &last, &idle, &life};
        const hipError_t e = hipModuleLaunchKernel(fn, 1, 1, 1, 64, 1, 1, 0, sm, params, nullptr);
        if (e != hipSuccess) return fail(QPB_EHIP, std::string("persistent solver launch: ") + hipGetErrorString(e));
        srv->running = true;
        srv->kname = kn;
        srv->args = a;
        srv->launches++;
        return QPB_OK;
    };
    // a kernel that left on its own (idle) is relaunched before the request
    if (srv->running && life_k != 0) {
        const hipError_t q = hipStreamQuery(sm);
        if (q == hipSuccess) srv->running = false;
        else if (q != hipErrorNotReady) {
            srv->running = false;
            return fail(QPB_EHIP, std::string("persistent solver: ") + hipGetErrorString(q));
        }
    }
    // One request per launch (the default): each call posts its request to the wave
    // launched for it and, while that wave solves, launches the next call's wave
    // behind it on the stream (the launch's host cost overlaps the solve).  A queued
    // wave waits up to the idle time; a call that comes later than half of it stops
    // whatever may still be waiting and launches afresh, so a request is never posted
    // to a wave that may already have left (its idle clock starts after the previous
    // answer the host saw, within microseconds).
    const bool oneshot = life_k == 0;
    const long long now_ns = std::chrono::duration_cast<std::chrono::nanoseconds>(
                                 std::chrono::steady_clock::now().time_since_epoch()).count();
    if (oneshot && srv->running && (double)(now_ns - srv->last_answer_ns) > 0.5e1 * (double)serve_idle_ticks() &&
        (rc = serve_stop(srv)))
        return rc;
    if (!srv->running && (rc = launch(srv->seq))) return rc;
    const unsigned long long r = ++srv->seq;
    // (diagnostics: QPB_SERVE_PREDELAY_US holds the request back after the inputs were written)
    static const long predelay = getenv("QPB_SERVE_PREDELAY_US") ? atol(getenv("QPB_SERVE_PREDELAY_US")) : 0;
    if (predelay > 0) std::this_thread::sleep_for(std::chrono::microseconds(predelay));
    mb_store(req, r);
    srv->requests++;
    if (oneshot && (rc = launch(r))) return rc;
    // host work that does not need the answer (the drop-in's struct mirror) runs while
    // the wave solves
    if (while_waiting) while_waiting();
    auto answered = [&]() {
        srv->dev_ticks = srv->mb[32];
        if (getenv("QPB_SERVE_DEBUG"))
            fprintf(stderr, "[serve] %s request %llu exec %016llx\n", kn.c_str(), r, srv->mb[40]);
        srv->last_answer_ns = std::chrono::duration_cast<std::chrono::nanoseconds>(
                                  std::chrono::steady_clock::now().time_since_epoch()).count();
        return (int)QPB_OK;
    };
    // wait for the answer; every ~20 us make sure the kernel is still there (it
    // may have left idle just before the request arrived: then launch again, the
    // new launch finds the request pending)
    const auto t0 = std::chrono::steady_clock::now();
    auto tq = t0;
    for (unsigned k = 1;; k++) {
        if (mb_load(ack) == r) return answered();
        __builtin_ia32_pause();
        if ((k & 63) != 0) continue;
        const auto now = std::chrono::steady_clock::now();
        // (one-request launches: only a fault or a stop ends the queued wave early, so
        // the stream is looked at rarely -- a query costs the spinning host ~1-2 us)
        if (now - tq < std::chrono::microseconds(oneshot ? 200 : 20)) continue;
        tq = now;
        const hipError_t q = hipStreamQuery(sm);
        if (q == hipErrorNotReady) {
            if (now - t0 > std::chrono::seconds(60)) {
                (void)serve_stop(srv);
                return fail(QPB_EHIP, "persistent solver: no answer within 60 s");
            }
            continue;
        }
        srv->running = false;
        if (q != hipSuccess) return fail(QPB_EHIP, std::string("persistent solver: ") + hipGetErrorString(q));
        if (mb_load(ack) == r) return answered();
        // the wave had left: a fresh one answers r (it starts with last = r - 1) and,
        // one request per launch, the next call's wave is queued behind it as usual
        if ((rc = launch(r - 1))) return rc;
        if (oneshot && (rc = launch(r))) return rc;
    }
}

extern "C" {

/* Retire the calling thread's queued persistent drop-in waves (qpb::serve_retire_thread):
 * they leave within microseconds instead of polling for the idle time, so a device-wide
 * synchronisation the caller is about to do cannot wait on them.  The batched solves
 * call it themselves; the next QP_SOLVE relaunches. */
int qpb_dropin_quiesce(void) {
    qpb::serve_retire_thread();
    return QPB_OK;
}

int qpb_serve_config(double *idle_ms, double *life_ms) {
    if (idle_ms) *idle_ms = (double)serve_idle_ticks() * 1e-5;    // 100 MHz ticks -> ms
    if (life_ms) *life_ms = (double)serve_life_ticks() * 1e-5;
    return QPB_OK;
}

int qpb_solve(qpb_plan *plan, long B, const double *P, const double *A, const double *G,
              const double *c, const double *h, const double *b, const qpb_settings *st,
              double *x, double *y, double *z, double *s, int *flag, int *iters, double *fval,
              double *stats, void *stream) {
    qpb::serve_retire_thread();      // no queued drop-in wave of this thread outlives the caller's sync
    return qpb::solve_ex(plan, B, P, A, G, c, h, b, st, x, y, z, s, flag, iters, fval, stats, nullptr, stream,
                         nullptr, false, nullptr);
}

int qpb_solve_best(qpb_plan *plan, long B, const double *P, const double *A, const double *G,
                   const double *c, const double *h, const double *b, const qpb_settings *st,
                   double *x, double *y, double *z, double *s, int *flag, int *iters, double *fval,
                   double *stats, double *best, void *stream) {
    qpb::serve_retire_thread();      // no queued drop-in wave of this thread outlives the caller's sync
    if (!best) return fail(QPB_EINVAL, "qpb_solve_best: best is NULL");
    return qpb::solve_ex(plan, B, P, A, G, c, h, b, st, x, y, z, s, flag, iters, fval, stats, best, stream,
                         nullptr, false, nullptr);
}

int qpb_solve_warm(qpb_plan *plan, long B, const double *P, const double *A, const double *G,
                   const double *c, const double *h, const double *b, const qpb_settings *st,
                   double *x, double *y, double *z, double *s, int *flag, int *iters, double *fval,
                   double *stats, double *sigma, void *stream) {
    qpb::serve_retire_thread();      // no queued drop-in wave of this thread outlives the caller's sync
    if (!sigma) return fail(QPB_EINVAL, "qpb_solve_warm: sigma is NULL");
    return qpb::solve_ex(plan, B, P, A, G, c, h, b, st, x, y, z, s, flag, iters, fval, stats, nullptr, stream, sigma,
                         true, nullptr);
}

/* ---- plan groups: one launch for a mixed-pattern batch (qpb_group_*) ---- */

struct qpb_group {
    std::vector<long> p;                         // per member: equality count (A, b, y needed when > 0)
    std::string kname, src;
    std::shared_ptr<std::vector<char>> code;
};

namespace {
struct GroupArgs {                               // = qpb_group_args of the generated kernel
    qpb::KernelArgs m[qpb::QPB_GROUP_MAX];
    long bend[qpb::QPB_GROUP_MAX];
    long qoff[qpb::QPB_GROUP_MAX];
};
}  // namespace

int qpb_group_create(qpb_group **out, qpb_plan *const *plans, int nplans) {
    if (!out) return fail(QPB_EINVAL, "NULL output");
    *out = nullptr;
    if (!plans || nplans < 1 || nplans > qpb::QPB_GROUP_MAX)
        return fail(QPB_EINVAL, "a group holds 1.." + std::to_string(qpb::QPB_GROUP_MAX) + " plans");
    std::vector<const qpb::Plan *> pls;
    auto g = std::make_unique<qpb_group>();
    for (int i = 0; i < nplans; i++) {
        const qpb_plan *pl = plans[i];
        if (!pl) return fail(QPB_EINVAL, "NULL plan in group");
        if (!pl->wave_ok || pl->wave_qpw != 4 || pl->wave_rowx || pl->gen.exact)
            return fail(QPB_EINVAL, "plan " + std::to_string(i) +
                                        " has no row-form kernel (groups need n, p <= 16, m <= 32, z/y rows leaves, fast mode)");
        pls.push_back(&pl->pl);
        g->p.push_back(pl->pl.p);
    }
    g->src = qpb::generate_row_group_kernel(pls, &g->kname);
    *out = g.release();
    return QPB_OK;
}

void qpb_group_destroy(qpb_group *g) { delete g; }

long qpb_group_source(const qpb_group *g, char *buf, long cap) {
    if (!g) return fail(QPB_EINVAL, "NULL group");
    if (buf && cap > 0) {
        long k = std::min<long>(cap - 1, (long)g->src.size());
        std::memcpy(buf, g->src.data(), k);
        buf[k] = 0;
    }
    return (long)g->src.size();
}

int qpb_group_compile(qpb_group *g) {
    if (!g) return fail(QPB_EINVAL, "NULL group");
    return qpb::compile_kernel(g->kname, [g] { return g->src; }, false, &g->code);
}

int qpb_group_solve(qpb_group *g, const qpb_io *io, const qpb_settings *st, double *best, void *stream) {
    qpb::serve_retire_thread();
    if (!g || !io) return fail(QPB_EINVAL, "NULL group or io");
    const int nm = (int)g->p.size();
    qpb_settings def;
    qpb_default_settings(&def);
    if (!st) st = &def;
    GroupArgs ga;
    std::memset(&ga, 0, sizeof ga);
    long blocks = 0, qs = 0;
    for (int i = 0; i < nm; i++) {
        const qpb_io &b = io[i];
        if (b.B < 0) return fail(QPB_EINVAL, "need B >= 0");
        if (b.B > 0) {
            if (!b.P || !b.G || !b.c || !b.h || !b.x || !b.z || !b.s || !b.flag || !b.iters || !b.fval)
                return fail(QPB_EINVAL, "NULL data pointer (member " + std::to_string(i) + ")");
            if (g->p[i] > 0 && (!b.A || !b.b || !b.y))
                return fail(QPB_EINVAL, "p > 0 needs A, b and y (member " + std::to_string(i) + ")");
        }
        qpb::KernelArgs &a = ga.m[i];
        a.P = b.P; a.A = b.A; a.G = b.G; a.c = b.c; a.h = b.h; a.b = b.b;
        a.x = b.x; a.y = b.y; a.z = b.z; a.s = b.s;
        a.flag = b.flag; a.iters = b.iters; a.fval = b.fval; a.stats = b.stats;
        a.B = b.B;
        a.tol = st->reltol / std::sqrt(3.0);
        a.abstol = st->abstol;
        a.sigma_d = st->sigma_d;
        a.maxit = st->maxit;
        ga.qoff[i] = qs;
        qs += b.B;
        blocks += (b.B + 3) / 4;                 // row form: 4 QPs per one-wave block
        ga.bend[i] = blocks;
    }
    if (blocks == 0) {
        if (best) {   // empty batch: {+inf, -1}, as qpb_argmin
            const double none[2] = {INFINITY, -1.0};
            if (hipMemcpyAsync(best, none, sizeof none, hipMemcpyHostToDevice, (hipStream_t)stream) != hipSuccess)
                return fail(QPB_EHIP, "group: best copy failed");
        }
        return QPB_OK;
    }
    const unsigned grid = (unsigned)((blocks + 7) & ~7L);    // XCD-aware block order (qpb_xcd_block)
    if (best) {
        unsigned long long *part;
        unsigned *ctr;
        int rc = qpb::argmin_scratch(stream, grid, &part, &ctr);
        if (rc) return rc;
        for (int i = 0; i < nm; i++) { ga.m[i].best = best; ga.m[i].part = part; ga.m[i].ctr = ctr; }
    }
    int rc = qpb_group_compile(g);
    hipFunction_t fn;
    if (!rc) rc = qpb::load_function(g->kname, g->code, &fn);
    if (rc) return rc;
    void *params[] = {&ga};
    hipError_t e = hipModuleLaunchKernel(fn, grid, 1, 1, 64, 1, 1, 0, (hipStream_t)stream, params, nullptr);
    if (e != hipSuccess) return fail(QPB_EHIP, std::string("group launch: ") + hipGetErrorString(e));
    return QPB_OK;
}

int qpb_winner(const double *best, const double *x, long n, long B, double *out, void *stream) {
    if (!best || !x || !out || n < 0 || B < 0) return fail(QPB_EINVAL, "bad winner arguments");
    (void)hipGetLastError();   // a stale error of an earlier API call is not this launch's
    hipLaunchKernelGGL(qpb_winner_k, dim3(1), dim3(64), 0, (hipStream_t)stream, best, x, n, B, out);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(QPB_EHIP, std::string("winner: ") + hipGetErrorString(e));
    return QPB_OK;
}

int qpb_argmin(long B, const double *fval, const int *flag, double *out2, void *stream) {
    if (B < 0 || !out2 || (B > 0 && (!fval || !flag))) return fail(QPB_EINVAL, "bad argmin arguments");
    // partials live in the per-(device, stream) scratch of the fused argmin:
    // launches on one stream are ordered, launches on different streams never
    // share partials
    const long nb = std::max(1L, std::min(1024L, (B + 4095) / 4096));
    const long chunk = (B + nb - 1) / nb;
    unsigned long long *part = nullptr;
    unsigned *ctr = nullptr;
    if (int rc = qpb::argmin_scratch(stream, nb, &part, &ctr)) return rc;
    double *pv = (double *)part;
    long *pi = (long *)((char *)part + nb * 8);
    (void)hipGetLastError();   // a stale error of an earlier API call is not these launches'
    if (nb == 1) {   // one block covers the batch: a single launch writes the result
        hipLaunchKernelGGL(qpb_argmin_single, dim3(1), dim3(1024), 0, (hipStream_t)stream, B, fval, flag, out2);
    } else {
        hipLaunchKernelGGL(qpb_argmin_partial, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, B, chunk, fval,
                           flag, pv, pi);
        hipLaunchKernelGGL(qpb_argmin_final, dim3(1), dim3(1024), 0, (hipStream_t)stream, nb, pv, pi, out2);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(QPB_EHIP, std::string("argmin: ") + hipGetErrorString(e));
    return QPB_OK;
}

}  // extern "C"

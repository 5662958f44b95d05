// qpb_codegen.cpp -- emit the batched IPM kernel for one plan.
//
// One QP per lane.  The whole qpSWIFT solve (kkt_initialize + QP_SOLVE loop) is
// emitted as straight-line code over named scalars: every CSC / elimination-tree
// index is resolved at generation time, so the device code has no index arrays,
// no indirect loads and no data-dependent branches besides the per-lane iteration
// loop and the step-length selects.  Device layout is "tiled SoA": QPs are grouped
// in tiles of 64 (one wavefront); array X with nv values per QP stores value j of
// QP q at X[(q/64)*nv*64 + j*64 + q%64], so every wave reads and writes whole
// contiguous 512-byte rows and every offset is a compile-time constant.
//
// Reference anchors for the emitted phases (dogbot_controller/src/qpSWIFT/):
//   init point            Auxilary.c:992-1089
//   residuals, objective  Auxilary.c:745-786, 1133-1141
//   exit test             qpSWIFT.c:519-534
//   predictor/corrector   qpSWIFT.c:537-595, Auxilary.c:205-295, 315-393, 471-564, 879-892
//   LDL numeric / solves  ldl.c:253-326, 495-597
#include "qpb_codegen.hpp"

#include <sstream>
#include <vector>

namespace qpb {

namespace {

struct Gen {
    const Plan &pl;
    const GenOptions &opt;
    std::ostringstream o;
    int indent = 1;

    // Inputs are (re)loaded lazily per phase: each phase gets an opaque copy of
    // the lane offset so the compiler can neither hoist the loads out of the IPM
    // loop nor keep them live across phases (keeps register pressure to one
    // phase's working set).
    int phase = 0;
    std::vector<std::vector<std::string>> scopes{{}};

    Gen(const Plan &p, const GenOptions &g) : pl(p), opt(g) {}

    void ln(const std::string &s) {
        for (int i = 0; i < indent; i++) o << "  ";
        o << s << '\n';
    }
    void open(const std::string &s) { ln(s); indent++; scopes.push_back({}); }
    void close(const std::string &s = "}") { scopes.pop_back(); indent--; ln(s); }
    void begin_phase() {
        phase++;
        ln("int lo" + S(phase) + " = lane; asm volatile(\"\" : \"+v\"(lo" + S(phase) + "));");
    }
    // name of input value arr[j] for the current phase; emits its load on first use
    std::string in(const char *arr, long j) {
        std::string name = std::string(arr) + S(j) + "_" + S(phase);
        for (auto &sc : scopes)
            for (auto &nm : sc)
                if (nm == name) return name;
        ln("const double " + name + " = t" + arr + "[" + S(j * 64) + " + lo" + S(phase) + "];");
        scopes.back().push_back(name);
        return name;
    }
    static std::string S(long v) { return std::to_string(v); }
    static std::string V(const char *base, long i) { return std::string(base) + std::to_string(i); }

    // a - b*c  (exact: separate multiply and subtract; fast: fused)
    std::string msub(const std::string &a, const std::string &b, const std::string &c) const {
        if (opt.exact) return a + " - " + b + " * " + c;
        return "__builtin_fma(-(" + b + "), " + c + ", " + a + ")";
    }
    // a + b*c
    std::string madd(const std::string &a, const std::string &b, const std::string &c) const {
        if (opt.exact) return a + " + " + b + " * " + c;
        return "__builtin_fma(" + b + ", " + c + ", " + a + ")";
    }

    std::string slot(const Slot &s) {
        switch (s.kind) {
            case Src::P: return in("P", s.idx);
            case Src::A: return in("A", s.idx);
            case Src::G: return in("G", s.idx);
            case Src::NegOne: return "(-1.0)";
            case Src::ZDiag: return V("kd", s.idx);
        }
        return "0.0";
    }

    // LDL_numeric (ldl.c:253-326) with the given KKT value map.
    void factor(const std::vector<Slot> &map) {
        const long N = pl.N;
        std::vector<char> yset(N, 0);
        bool dk_ready = false;
        long k = 0;
        auto yname = [&](long i) { return V("Y", i); };
        auto yval = [&](long i) { return yset[i] ? yname(i) : std::string("0.0"); };
        auto ensure_dk = [&]() {
            if (!dk_ready) { ln("double Dk = " + yval(k) + ";"); dk_ready = true; }
        };
        for (const FacStep &st : pl.fac) {
            switch (st.op) {
                case FacOp::RowBegin:
                    k = st.a;
                    std::fill(yset.begin(), yset.end(), 0);
                    dk_ready = false;
                    open("{ // LDL row " + S(k));
                    break;
                case FacOp::Scatter: {
                    std::string v = slot(map[st.b]);
                    if (yset[st.a]) ln(yname(st.a) + " = " + yname(st.a) + " + " + v + ";");
                    else { ln("double " + yname(st.a) + " = " + v + ";"); yset[st.a] = 1; }
                    break;
                }
                case FacOp::Update: {
                    ensure_dk();
                    std::string yi = yval(st.c), L = V("L", st.b);
                    if (yset[st.a]) ln(yname(st.a) + " = " + msub(yname(st.a), L, yi) + ";");
                    else { ln("double " + yname(st.a) + " = -(" + L + " * " + yi + ");"); yset[st.a] = 1; }
                    break;
                }
                case FacOp::NewL: {
                    ensure_dk();
                    std::string yi = yval(st.a), L = V("L", st.b);
                    if (opt.exact) ln(L + " = " + yi + " / " + V("D", st.a) + ";");
                    else ln(L + " = " + yi + " * " + V("rD", st.a) + ";");
                    ln("Dk = " + msub("Dk", L, yi) + ";");
                    break;
                }
                case FacOp::RowEnd: {
                    ensure_dk();
                    // ldl.c:319-320
                    if (opt.exact)
                        ln("{ const double sg = Dk <= 0.0 ? -1.0 : 1.0; " + V("D", k) +
                           " = (sg * Dk <= 1e-14) ? sg * 1e-7 : Dk; }");
                    else
                        ln("{ const double sg = Dk <= 0.0 ? -1.0 : 1.0; " + V("rD", k) +
                           " = qpb_rcp((sg * Dk <= 1e-14) ? sg * 1e-7 : Dk); }");
                    close();
                    break;
                }
            }
        }
    }

    // LDL_perm / lsolve / dsolve / ltsolve / permt (ldl.c:495-597).
    template <class In, class Out>
    void solve(In rhs, Out out) {
        const long N = pl.N;
        open("{ // KKT solve");
        for (long j = 0; j < N; j++) ln("double X" + S(j) + " = " + rhs(pl.perm[j]) + ";");
        for (long j = 0; j < N; j++)
            for (long e = pl.Lp[j]; e < pl.Lp[j + 1]; e++) {
                std::string t = V("X", pl.Li[e]);
                ln(t + " = " + msub(t, V("L", e), V("X", j)) + ";");
            }
        for (long j = 0; j < N; j++) {
            if (opt.exact) ln(V("X", j) + " = " + V("X", j) + " / " + V("D", j) + ";");
            else ln(V("X", j) + " = " + V("X", j) + " * " + V("rD", j) + ";");
        }
        for (long j = N - 1; j >= 0; j--)
            for (long e = pl.Lp[j]; e < pl.Lp[j + 1]; e++) {
                std::string t = V("X", j);
                ln(t + " = " + msub(t, V("L", e), V("X", pl.Li[e])) + ";");
            }
        for (long j = 0; j < N; j++) {
            std::string dst = out(pl.perm[j]);
            if (!dst.empty()) ln(dst + " = " + V("X", j) + ";");
        }
        close();
    }

    // y(rows) = 0 - M x  in column order (Auxilary.c:839-860, start = 1).
    // Emits declarations "double <dst>r" for every row.
    void spmv_neg(const Pattern &M, const std::vector<long> *src, const char *val, const char *xv, const char *dst) {
        std::vector<char> set(M.rows, 0);
        for (long i = 0; i < M.cols; i++)
            for (long k = M.jc[i]; k < M.jc[i + 1]; k++) {
                long r = M.ir[k];
                std::string a = in(val, src ? (*src)[k] : k), x = V(xv, i), d = V(dst, r);
                if (set[r]) ln(d + " = " + msub(d, x, a) + ";");
                else { ln("double " + d + " = -(" + x + " * " + a + ");"); set[r] = 1; }
            }
        for (long r = 0; r < M.rows; r++)
            if (!set[r]) ln("double " + V(dst, r) + " = 0.0;");
    }

    // acc = sum a_i*b_i, sequential from 0 (Auxilary.c:451-462)
    void dot(const std::string &acc, long cnt, const char *a, const char *b) {
        if (cnt == 0) { ln("double " + acc + " = 0.0;"); return; }
        ln("double " + acc + " = " + V(a, 0) + " * " + V(b, 0) + ";");
        for (long i = 1; i < cnt; i++) ln(acc + " = " + madd(acc, V(a, i), V(b, i)) + ";");
    }

    void decl_vec(const char *base, long cnt, const char *init = nullptr) {
        for (long i0 = 0; i0 < cnt; i0 += 8) {
            std::string s = "double ";
            for (long i = i0; i < cnt && i < i0 + 8; i++) {
                if (i > i0) s += ", ";
                s += V(base, i);
                if (init) s += std::string(" = ") + init;
            }
            ln(s + ";");
        }
    }

    // findsteplength (Auxilary.c:359-393) into variables ap, ad.
    void step_length() {
        const long m = pl.m;
        if (opt.exact) {
            ln("ap = 1e10; ad = 1e10;");
            open("{ bool hp = false, hd = false;");
            for (long i = 0; i < m; i++) {
                ln("{ const double r = (-" + V("s", i) + ") / " + V("dsl", i) + "; const bool t = (" + V("dsl", i) +
                   " < 0.0) && (r < ap); ap = t ? r : ap; hp = hp || t; }");
                ln("{ const double r = (-" + V("z", i) + ") / " + V("dz", i) + "; const bool t = (" + V("dz", i) +
                   " < 0.0) && (r < ad); ad = t ? r : ad; hd = hd || t; }");
            }
            ln("if (!hp) ap = 1.0;");
            ln("if (!hd) ad = 1.0;");
            close();
        } else {
            // min over {i: d_i < 0} of s_i / (-d_i), tracked as a fraction (num/den,
            // den > 0) with cross-multiplied compares; one division at the end.
            open("{ double pn = 1e10, pd = 1.0, dn = 1e10, dd = 1.0; bool hp = false, hd = false;");
            for (long i = 0; i < m; i++) {
                ln("{ const double nd = -" + V("dsl", i) + "; const bool t = (nd > 0.0) && (" + V("s", i) +
                   " * pd < pn * nd); pn = t ? " + V("s", i) + " : pn; pd = t ? nd : pd; hp = hp || t; }");
                ln("{ const double nd = -" + V("dz", i) + "; const bool t = (nd > 0.0) && (" + V("z", i) +
                   " * dd < dn * nd); dn = t ? " + V("z", i) + " : dn; dd = t ? nd : dd; hd = hd || t; }");
            }
            ln("ap = hp ? pn / pd : 1.0;");
            ln("ad = hd ? dn / dd : 1.0;");
            close();
        }
    }

    std::string div(const std::string &a, const std::string &zidx_base, long i) const {
        // a / z_i (exact) or a * (1/z_i) (fast)
        if (opt.exact) return "(" + a + ") / " + V(zidx_base.c_str(), i);
        return "(" + a + ") * " + V("rz_", i);
    }

    std::string build() {
        const long n = pl.n, m = pl.m, p = pl.p, N = pl.N;
        const std::string kname = kernel_name(pl, opt);
        o << "// generated by qpb_codegen for plan " << std::hex << pl.hash << std::dec
          << ": n=" << n << " m=" << m << " p=" << p << " N=" << N << " nnz(L)=" << pl.lnz
          << (opt.exact ? " [exact]" : " [fast]") << "\n";
        o << "#pragma clang fp contract(" << (opt.exact ? "off" : "fast") << ")\n";
        o << "struct qpb_args {\n"
             "  const double *P, *A, *G, *c, *h, *b;\n"
             "  double *x, *y, *z, *s;\n"
             "  int *flag, *iters;\n"
             "  double *fval;\n"
             "  double *stats;\n"
             "  long B;\n"
             "  double tol, abstol, sigma_d;\n"
             "  long maxit;\n"
             "};\n";
        o << "static __device__ __forceinline__ double qpb_rcp(double v) {\n"
             "  double r = __builtin_amdgcn_rcp(v);\n"
             "  double e = __builtin_fma(-v, r, 1.0); r = __builtin_fma(r, e, r);\n"
             "  e = __builtin_fma(-v, r, 1.0); return __builtin_fma(r, e, r);\n"
             "}\n";
        o << "extern \"C\" __global__ void __launch_bounds__(" << opt.wg << ", " << opt.waves_per_eu << ") "
          << kname << "(qpb_args a) {\n";
        ln("const long q = (long)blockIdx.x * " + S(opt.wg) + " + threadIdx.x;");
        ln("if (q >= a.B) return;");
        ln("const long tile = (long)blockIdx.x * " + S(opt.wg / 64) +
           " + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);");
        ln("const int lane = threadIdx.x & 63;");
        auto tbase = [&](const char *arr, long nv) {
            ln(std::string("const double *__restrict__ t") + arr + " = a." + arr + " + tile * " + S(nv * 64) + ";");
        };
        tbase("P", pl.Pin.nnz());
        if (p) tbase("A", pl.A.nnz());
        tbase("G", pl.G.nnz());
        tbase("c", n);
        tbase("h", m);
        if (p) tbase("b", p);
        // inputs
        decl_vec("L", pl.lnz);
        if (opt.exact) decl_vec("D", N);
        else decl_vec("rD", N);
        decl_vec("x", n);
        decl_vec("y", p);
        decl_vec("s", m);
        decl_vec("z", m);

        // ---- kkt_initialize (Auxilary.c:992-1089)
        ln("// setup: factor the KKT holding -I, solve for rhs [-c; b; h]");
        begin_phase();
        factor(pl.K_init);
        solve([&](long t) -> std::string {
                  if (t < n) return "(-" + in("c", t) + ")";
                  if (t < n + p) return in("b", t - n);
                  return in("h", t - n - p);
              },
              [&](long t) -> std::string {
                  if (t < n) return V("x", t);
                  if (t < n + p) return V("y", t - n);
                  return "";
              });
        open("{");
        spmv_neg(pl.G, nullptr, "G", "x", "zi");
        for (long i = 0; i < m; i++) ln(V("zi", i) + " = " + V("zi", i) + " + " + in("h", i) + ";");
        ln("double lo = zi0, hi = zi0;");
        for (long i = 1; i < m; i++) {
            ln("if (" + V("zi", i) + " < lo) lo = " + V("zi", i) + ";");
            ln("if (" + V("zi", i) + " > hi) hi = " + V("zi", i) + ";");
        }
        ln("const double sh = -lo;");
        for (long i = 0; i < m; i++) ln(V("s", i) + " = sh < 0 ? " + V("zi", i) + " : " + V("zi", i) + " + (1 + sh);");
        for (long i = 0; i < m; i++) ln(V("z", i) + " = hi < 0 ? -" + V("zi", i) + " : -" + V("zi", i) + " + (1 + hi);");
        close();

        // ---- QP_SOLVE loop (qpSWIFT.c:502-602)
        ln("long it = 0; int flag = 3;");
        ln("double fval = 0.0, st_rx = 0.0, st_ry = 0.0, st_rz = 0.0, st_mu = 0.0, ap = 0.0, ad = 0.0;");
        ln("double sigma = 100.0;");
        open("for (;;) {");
        ln("if (it >= a.maxit) { flag = 2; break; }");
        begin_phase();
        // residuals
        spmv_neg(pl.Pf, &pl.Pf_src, "P", "x", "t");
        dot("f1", n, "t", "x");
        for (long j = 0; j < n; j++) in("c", j);
        ln("double f2 = " + V("c", 0) + "_" + S(phase) + " * x0;");
        for (long j = 1; j < n; j++) ln("f2 = " + madd("f2", V("c", j) + "_" + S(phase), V("x", j)) + ";");
        ln("fval = -0.5 * f1 + f2;");
        for (long j = 0; j < n; j++) ln("double " + V("rx", j) + " = " + V("t", j) + ";");
        for (long j = 0; j < n; j++)
            for (long k = pl.G.jc[j]; k < pl.G.jc[j + 1]; k++)
                ln(V("rx", j) + " = " + msub(V("rx", j), in("G", k), V("z", pl.G.ir[k])) + ";");
        if (p)
            for (long j = 0; j < n; j++)
                for (long k = pl.A.jc[j]; k < pl.A.jc[j + 1]; k++)
                    ln(V("rx", j) + " = " + msub(V("rx", j), in("A", k), V("y", pl.A.ir[k])) + ";");
        for (long j = 0; j < n; j++) ln(V("rx", j) + " = " + V("rx", j) + " - " + in("c", j) + ";");
        dot("nrx2", n, "rx", "rx");
        ln("st_rx = __builtin_sqrt(nrx2);");
        if (p) {
            spmv_neg(pl.A, nullptr, "A", "x", "ry");
            for (long i = 0; i < p; i++) ln(V("ry", i) + " = " + V("ry", i) + " + " + in("b", i) + ";");
            dot("nry2", p, "ry", "ry");
            ln("st_ry = __builtin_sqrt(nry2);");
        }
        spmv_neg(pl.G, nullptr, "G", "x", "rz");
        for (long i = 0; i < m; i++) ln(V("rz", i) + " = " + V("rz", i) + " + (" + in("h", i) + " - " + V("s", i) + ");");
        dot("nrz2", m, "rz", "rz");
        ln("st_rz = __builtin_sqrt(nrz2);");
        dot("sz", m, "s", "z");
        ln("st_mu = sz / " + S(m) + ".0;");
        ln(std::string("if (st_rx < a.tol && st_rz < a.tol") + (p ? " && st_ry < a.tol" : "") +
           " && st_mu < a.abstol) { flag = 0; break; }");
        // lambda, mu (qpSWIFT.c:537-538)
        for (long i = 0; i < m; i++) ln("const double " + V("lam", i) + " = __builtin_sqrt(" + V("s", i) + " * " + V("z", i) + ");");
        dot("mu2", m, "lam", "lam");
        ln("const double mu = mu2 / " + S(m) + ".0;");
        ln("const bool pc = sigma > a.sigma_d;");
        if (!opt.exact)
            for (long i = 0; i < m; i++) ln("const double " + V("rz_", i) + " = qpb_rcp(" + V("z", i) + ");");
        // updatekktmatrix: -s/z on the z diagonal (Auxilary.c:211-215)
        for (long i = 0; i < m; i++) {
            if (opt.exact) ln("const double " + V("kd", i) + " = (-" + V("s", i) + ") / " + V("z", i) + ";");
            else ln("const double " + V("kd", i) + " = -" + V("s", i) + " * " + V("rz_", i) + ";");
        }
        // form_ds: predictor (pure Newton) or pure centering (qpSWIFT.c:542, 574-575)
        decl_vec("ds", m);
        ln("if (!pc) sigma = a.sigma_d;");
        for (long i = 0; i < m; i++)
            ln(V("ds", i) + " = pc ? (-" + V("lam", i) + ") * " + V("lam", i) + " : -(" + V("lam", i) + " * " +
               V("lam", i) + ") + (sigma * mu);");
        begin_phase();
        factor(pl.K_loop);
        decl_vec("dx", n);
        decl_vec("dy", p);
        decl_vec("dz", m);
        decl_vec("dsl", m);
        auto rhs = [&](long t) -> std::string {
            if (t < n) return V("rx", t);
            if (t < n + p) return V("ry", t - n);
            long i = t - n - p;
            if (opt.exact) return "(" + V("rz", i) + " - (" + V("ds", i) + " / " + V("z", i) + "))";
            return "__builtin_fma(-" + V("ds", i) + ", " + V("rz_", i) + ", " + V("rz", i) + ")";
        };
        auto dsl_from_dz = [&]() {
            for (long i = 0; i < m; i++) {
                std::string num = V("ds", i) + " - (" + V("s", i) + " * " + V("dz", i) + ")";
                if (opt.exact) ln(V("dsl", i) + " = (" + num + ") / " + V("z", i) + ";");
                else ln(V("dsl", i) + " = __builtin_fma(-" + V("s", i) + ", " + V("dz", i) + ", " + V("ds", i) +
                        ") * " + V("rz_", i) + ";");
            }
        };
        // predictor solve, step, rho, sigma, corrector ds (kktsolve_1, qpSWIFT.c:552-569)
        open("if (pc) {");
        solve(rhs, [&](long t) -> std::string {
            if (t < n + p) return "";
            return V("dz", t - n - p);
        });
        dsl_from_dz();
        step_length();
        ln("double rho_n = 0.0;");
        for (long i = 0; i < m; i++)
            ln("rho_n = rho_n + (" + V("s", i) + " + (ap * " + V("dsl", i) + ")) * (" + V("z", i) + " + (ad * " + V("dz", i) + "));");
        ln("const double rho = rho_n / sz;");
        ln("const double r1 = 1 > rho ? rho : 1;");
        ln("const double cube = r1 * r1 * r1;");
        ln("sigma = a.sigma_d < cube ? cube : a.sigma_d;");
        for (long i = 0; i < m; i++)
            ln(V("ds", i) + " = -(" + V("lam", i) + " * " + V("lam", i) + ") - (" + V("dsl", i) + " * " + V("dz", i) +
               ") + (sigma * mu);");
        close();
        // corrector / centering solve (kktsolve_2, Auxilary.c:524-564)
        solve(rhs, [&](long t) -> std::string {
            if (t < n) return V("dx", t);
            if (t < n + p) return V("dy", t - n);
            return V("dz", t - n - p);
        });
        dsl_from_dz();
        step_length();
        ln("ap = 0.99 * ap > 1.0 ? 1.0 : 0.99 * ap;");
        ln("ad = 0.99 * ad > 1.0 ? 1.0 : 0.99 * ad;");
        for (long i = 0; i < n; i++) ln(V("x", i) + " = " + madd(V("x", i), V("dx", i), "ap") + ";");
        for (long i = 0; i < p; i++) ln(V("y", i) + " = " + madd(V("y", i), V("dy", i), "ad") + ";");
        for (long i = 0; i < m; i++) ln(V("s", i) + " = " + madd(V("s", i), V("dsl", i), "ap") + ";");
        for (long i = 0; i < m; i++) ln(V("z", i) + " = " + madd(V("z", i), V("dz", i), "ad") + ";");
        ln("it++;");
        close();
        // outputs
        auto store = [&](const char *arr, long nv, const char *base) {
            ln(std::string("{ double *__restrict__ o = a.") + arr + " + tile * " + S(nv * 64) + " + lane;");
            for (long i = 0; i < nv; i++) ln("  o[" + S(i * 64) + "] = " + V(base, i) + ";");
            ln("}");
        };
        store("x", n, "x");
        if (p) store("y", p, "y");
        store("z", m, "z");
        store("s", m, "s");
        ln("a.flag[q] = flag; a.iters[q] = (int)it; a.fval[q] = fval;");
        ln("if (a.stats) { double *o = a.stats + tile * 384 + lane; o[0] = st_rx; o[64] = st_ry; o[128] = st_rz;"
           " o[192] = st_mu; o[256] = ap; o[320] = ad; }");
        o << "}\n";
        return o.str();
    }
};

}  // namespace

std::string kernel_name(const Plan &pl, const GenOptions &opt) {
    char buf[96];
    snprintf(buf, sizeof buf, "qpb_ipm_%016llx_%s_w%d", (unsigned long long)pl.hash, opt.exact ? "x" : "f", opt.wg);
    return buf;
}

std::string generate_kernel(const Plan &pl, const GenOptions &opt) {
    Gen g(pl, opt);
    return g.build();
}

}  // namespace qpb

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

#include <map>
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
    // Fast mode: "leaf" columns of L (no entries in their row, e.g. the z and y
    // pivots eliminated before any x) satisfy L(k,j) = K(j,k) / D(j) exactly; their
    // L entries are never stored -- every use is rewritten in terms of the KKT input
    // value and 1/D(j).  leaf_slot[e] = KKT slot holding K(j,k) for L entry e.
    std::vector<char> leaf;
    std::vector<long> leaf_slot;
    // Fast mode: A and G values live in LDS (each lane owns one private column, so
    // no barriers are needed); lds_base[arr] = first LDS row of that array.
    bool use_lds = false;
    long lds_rows = 0, lds_A = -1, lds_G = -1, lds_P = -1, lds_c = -1, lds_h = -1, lds_b = -1;

    Gen(const Plan &p, const GenOptions &g) : pl(p), opt(g) {
        const long N = pl.N;
        leaf.assign(N, !opt.exact);
        if (!opt.exact) {
            for (long e = 0; e < pl.lnz; e++) leaf[pl.Li[e]] = 0;     // row Li[e] has an entry
            leaf_slot.assign(pl.lnz, -1);
            std::vector<long> scat(N, -1);
            for (const FacStep &st : pl.fac) {
                if (st.op == FacOp::RowBegin) std::fill(scat.begin(), scat.end(), -1);
                else if (st.op == FacOp::Scatter) scat[st.a] = st.b;
                else if (st.op == FacOp::NewL && leaf[st.a]) leaf_slot[st.b] = scat[st.a];
            }
            for (long e = 0; e < pl.lnz; e++) {
                long j = -1;
                for (long c = 0; c < N; c++) if (e >= pl.Lp[c] && e < pl.Lp[c + 1]) { j = c; break; }
                if (leaf[j] && leaf_slot[e] < 0) leaf[j] = 0;          // not a pure scatter: keep L
            }
        }
        const long nA = pl.p ? pl.A.nnz() : 0, nG = pl.G.nnz(), nP = pl.Pin.nnz();
        if (opt.lds_mode >= 1) {
            lds_A = 0; lds_G = nA; lds_rows = nA + nG;
            if (opt.lds_mode == 2 || opt.lds_mode == 4) { lds_P = lds_rows; lds_rows += nP; }
            if (opt.lds_mode == 4) {      // every input on chip
                lds_c = lds_rows; lds_rows += pl.n;
                lds_h = lds_rows; lds_rows += pl.m;
                if (pl.p) { lds_b = lds_rows; lds_rows += pl.p; }
            }
            if (opt.lds_mode == 3 || opt.lds_mode == 4) {      // park the loop vectors too
                const long n = pl.n, p = pl.p, m = pl.m;
                park["x"] = lds_rows; lds_rows += n;
                if (p) { park["y"] = lds_rows; lds_rows += p; }
                park["rx"] = lds_rows; lds_rows += n;
                if (p) { park["ry"] = lds_rows; lds_rows += p; }
                park["rz"] = lds_rows; lds_rows += m;
                if ((lds_rows + m) * opt.wg * 8 <= 160 * 1024) { park["s"] = lds_rows; lds_rows += m; }
                if (opt.lds_mode == 4 && opt.park_z && (lds_rows + 2 * m) * opt.wg * 8 <= 160 * 1024) {
                    park["z"] = lds_rows; lds_rows += m;
                    park["rzi"] = lds_rows; lds_rows += m;
                }
            }
            use_lds = lds_rows > 0 && lds_rows * opt.wg * 8 <= 160 * 1024;
            if (!use_lds) { lds_A = lds_G = lds_P = lds_c = lds_h = lds_b = -1; park.clear(); }
        }
    }
    long col_of(long e) const {
        long lo = 0, hi = pl.N;
        while (hi - lo > 1) { long mid = (lo + hi) / 2; if (pl.Lp[mid] <= e) lo = mid; else hi = mid; }
        return lo;
    }

    void ln(const std::string &s) {
        for (int i = 0; i < indent; i++) o << "  ";
        o << s << '\n';
    }
    // Two independent "phases": gph for global-memory inputs, lph for LDS rows.
    // A new phase gives fresh opaque lane offsets, i.e. forces re-loads.
    int gph = 0, lph = 0, gctr = 0, lctr = 0;
    std::vector<std::pair<int, int>> phase_stack;
    void open(const std::string &s) { ln(s); indent++; scopes.push_back({}); phase_stack.push_back({gph, lph}); }
    void close(const std::string &s = "}") {
        scopes.pop_back(); indent--; ln(s);
        // phases begun inside the block die with it; names stay unique via the counters
        gph = phase_stack.back().first; lph = phase_stack.back().second; phase_stack.pop_back();
    }
    void begin_phase(bool global = true, bool lds = true) {
        if (global) {
            gph = ++gctr;
            ln("int lo" + S(gph) + " = lane; asm volatile(\"\" : \"+v\"(lo" + S(gph) + "));");
        }
        if (lds && use_lds) {
            lph = ++lctr;
            // one opaque base per 64 KiB window of the LDS image, so every access
            // is base + 16-bit immediate (no per-access address arithmetic)
            for (long w = 0; w * win_rows() < lds_rows; w++)
                ln("int lt" + S(lph) + "_" + S(w) + " = threadIdx.x + " + S(w * win_rows() * opt.wg) +
                   "; asm volatile(\"\" : \"+v\"(lt" + S(lph) + "_" + S(w) + "));");
        }
    }
    long win_rows() const { return 65536 / (8 * opt.wg); }
    bool cached(const std::string &name) const {
        for (auto &sc : scopes)
            for (auto &nm : sc)
                if (nm == name) return true;
        return false;
    }
    void uncache(const std::string &prefix) {
        for (auto &sc : scopes)
            for (auto it = sc.begin(); it != sc.end();)
                it = (it->compare(0, prefix.size(), prefix) == 0) ? sc.erase(it) : it + 1;
    }
    std::string lds_at(long row) const {
        const long w = row / win_rows();
        return "qpb_lds[" + S((row - w * win_rows()) * opt.wg) + " + lt" + S(lph) + "_" + S(w) + "]";
    }
    std::string lds_st(long row) const { return "qpb_lds[" + S(row * opt.wg) + " + threadIdx.x]"; }
    // name of input value arr[j] for the current phase; emits its load on first use
    std::string in(const char *arr, long j) {
        long base = (arr[1] != 0) ? -1 : arr[0] == 'A' ? lds_A : arr[0] == 'G' ? lds_G : arr[0] == 'P' ? lds_P
                  : arr[0] == 'c' ? lds_c : arr[0] == 'h' ? lds_h : arr[0] == 'b' ? lds_b : -1;
        const bool lds = use_lds && base >= 0;
        std::string name = std::string(arr) + S(j) + (lds ? "_l" + S(lph) : "_g" + S(gph));
        if (cached(name)) return name;
        if (lds) ln("const double " + name + " = " + lds_at(base + j) + ";");
        else ln("const double " + name + " = t" + arr + "[" + S(j * 64) + " + lo" + S(gph) + "];");
        scopes.back().push_back(name);
        return name;
    }
    // Loop vectors (x, y, rx, ry, rz) may be "parked" in LDS rows (fast mode):
    // rd() reads element i, wr() writes it.
    std::map<std::string, long> park;
    std::string rd(const std::string &v, long i) {
        auto it = park.find(v);
        if (it == park.end()) return V(v.c_str(), i);
        std::string name = "pk_" + v + S(i) + "_l" + S(lph);
        if (cached(name)) return name;
        ln("const double " + name + " = " + lds_at(it->second + i) + ";");
        scopes.back().push_back(name);
        return name;
    }
    void wr(const std::string &v, long i, const std::string &expr) {
        auto it = park.find(v);
        if (it == park.end()) { ln(V(v.c_str(), i) + " = " + expr + ";"); return; }
        ln(lds_st(it->second + i) + " = " + expr + ";");
        uncache("pk_" + v + S(i) + "_");
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
        auto update = [&](long r, const std::string &lv, const std::string &yi) {
            if (yset[r]) ln(yname(r) + " = " + msub(yname(r), lv, yi) + ";");
            else { ln("double " + yname(r) + " = -(" + lv + " * " + yi + ");"); yset[r] = 1; }
        };
        std::vector<const FacStep *> pend;     // buffered updates of a leaf column
        bool dk_zero = false;                  // D(k) structurally 0 (no diag, no updates)
        for (const FacStep &st : pl.fac) {
            switch (st.op) {
                case FacOp::RowBegin:
                    k = st.a;
                    std::fill(yset.begin(), yset.end(), 0);
                    dk_ready = false;
                    dk_zero = true;
                    open("{ // LDL row " + S(k));
                    break;
                case FacOp::Scatter: {
                    if (st.a == k) dk_zero = false;
                    std::string v = slot(map[st.b]);
                    if (yset[st.a]) ln(yname(st.a) + " = " + yname(st.a) + " + " + v + ";");
                    else { ln("double " + yname(st.a) + " = " + v + ";"); yset[st.a] = 1; }
                    break;
                }
                case FacOp::Update: {
                    ensure_dk();
                    if (leaf[st.c]) { pend.push_back(&st); break; }
                    update(st.a, V("L", st.b), yval(st.c));
                    break;
                }
                case FacOp::NewL: {
                    ensure_dk();
                    dk_zero = false;
                    std::string yi = yval(st.a);
                    if (opt.exact) {
                        std::string L = V("L", st.b);
                        ln(L + " = " + yi + " / " + V("D", st.a) + ";");
                        ln("Dk = " + msub("Dk", L, yi) + ";");
                    } else if (leaf[st.a]) {
                        // l = L(k,i) = K(i,k)/D(i); Y[r] -= L(r,i)*K(i,k) == K(i,r)*l
                        std::string l = "l" + S(st.b);
                        ln("const double " + l + " = " + yi + " * " + V("rD", st.a) + ";");
                        for (const FacStep *u : pend) update(u->a, slot(map[leaf_slot[u->b]]), l);
                        pend.clear();
                        ln("Dk = " + msub("Dk", l, yi) + ";");
                    } else {
                        std::string L = V("L", st.b);
                        ln(L + " = " + yi + " * " + V("rD", st.a) + ";");
                        ln("Dk = " + msub("Dk", L, yi) + ";");
                    }
                    break;
                }
                case FacOp::RowEnd: {
                    ensure_dk();
                    // ldl.c:319-320
                    if (opt.exact)
                        ln("{ const double sg = Dk <= 0.0 ? -1.0 : 1.0; " + V("D", k) +
                           " = (sg * Dk <= 1e-14) ? sg * 1e-7 : Dk; }");
                    else if (dk_zero) {
                        // D = 0 exactly -> always regularised to -1e-7 (ldl.c:319-320)
                        char buf[64];
                        snprintf(buf, sizeof buf, "%.17g", 1.0 / -1e-7);
                        ln(V("rD", k) + " = " + buf + "; (void)Dk;");
                    } else
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
    void solve(const std::vector<Slot> &map, In rhs, Out out) {
        const long N = pl.N;
        open("{ // KKT solve");
        begin_phase(false, true);   // fresh LDS offsets: no load merging across solves
        for (long j = 0; j < N; j++) ln("double X" + S(j) + " = " + rhs(pl.perm[j]) + ";");
        if (!opt.exact) begin_phase();
        for (long j = 0; j < N; j++) {
            if (pl.Lp[j] == pl.Lp[j + 1]) continue;
            if (!opt.exact && leaf[j]) {
                ln("{ const double t = " + V("rD", j) + " * " + V("X", j) + ";");
                for (long e = pl.Lp[j]; e < pl.Lp[j + 1]; e++) {
                    std::string t = V("X", pl.Li[e]);
                    ln("  " + t + " = " + msub(t, slot(map[leaf_slot[e]]), "t") + ";");
                }
                ln("}");
                continue;
            }
            for (long e = pl.Lp[j]; e < pl.Lp[j + 1]; e++) {
                std::string t = V("X", pl.Li[e]);
                ln(t + " = " + msub(t, V("L", e), V("X", j)) + ";");
            }
        }
        for (long j = 0; j < N; j++) {
            if (opt.exact) ln(V("X", j) + " = " + V("X", j) + " / " + V("D", j) + ";");
            else ln(V("X", j) + " = " + V("X", j) + " * " + V("rD", j) + ";");
        }
        if (!opt.exact) begin_phase();
        for (long j = N - 1; j >= 0; j--) {
            if (pl.Lp[j] == pl.Lp[j + 1]) continue;
            std::string t = V("X", j);
            if (!opt.exact && leaf[j]) {
                std::string acc;
                for (long e = pl.Lp[j]; e < pl.Lp[j + 1]; e++) {
                    std::string term = slot(map[leaf_slot[e]]);
                    acc = acc.empty() ? term + " * " + V("X", pl.Li[e]) : madd(acc, term, V("X", pl.Li[e]));
                }
                ln(t + " = " + msub(t, V("rD", j), "(" + acc + ")") + ";");
                continue;
            }
            for (long e = pl.Lp[j]; e < pl.Lp[j + 1]; e++)
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
                std::string a = in(val, src ? (*src)[k] : k), x = rd(xv, i), d = V(dst, r);
                if (set[r]) ln(d + " = " + msub(d, x, a) + ";");
                else { ln("double " + d + " = -(" + x + " * " + a + ");"); set[r] = 1; }
            }
        for (long r = 0; r < M.rows; r++)
            if (!set[r]) ln("double " + V(dst, r) + " = 0.0;");
    }

    // acc = sum a_i*b_i, sequential from 0 (Auxilary.c:451-462)
    // regs = true: the operands are the register copies (e.g. residuals just
    // computed, before they are parked)
    void dot(const std::string &acc, long cnt, const char *a, const char *b, bool regs = false) {
        auto get = [&](const char *v, long i) { return regs ? V(v, i) : rd(v, i); };
        if (cnt == 0) { ln("double " + acc + " = 0.0;"); return; }
        ln("double " + acc + " = " + get(a, 0) + " * " + get(b, 0) + ";");
        for (long i = 1; i < cnt; i++) ln(acc + " = " + madd(acc, get(a, i), get(b, i)) + ";");
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
        begin_phase(false, true);
        if (opt.exact) {
            ln("ap = 1e10; ad = 1e10;");
            open("{ bool hp = false, hd = false;");
            for (long i = 0; i < m; i++) {
                ln("{ const double r = (-" + rd("s", i) + ") / " + V("dsl", i) + "; const bool t = (" + V("dsl", i) +
                   " < 0.0) && (r < ap); ap = t ? r : ap; hp = hp || t; }");
                ln("{ const double r = (-" + rd("z", i) + ") / " + V("dz", i) + "; const bool t = (" + V("dz", i) +
                   " < 0.0) && (r < ad); ad = t ? r : ad; hd = hd || t; }");
            }
            ln("if (!hp) ap = 1.0;");
            ln("if (!hd) ad = 1.0;");
            close();
        } else {
            // alpha = min over {i: d_i < 0} of v_i/(-d_i)  ==  1 / max_i(-d_i / v_i)
            // (v = s or z > 0); the reference keeps alpha = 1 when no ratio is below
            // its 1e10 start value (Auxilary.c:362-391) -> beta threshold 1e-10.
            // v_rcp_f64 alone suffices: the step is damped by 0.99 afterwards.
            open("{ double bp = 0.0, bd = 0.0;");
            for (long i = 0; i < m; i++) {
                ln("bp = __builtin_fmax(bp, -" + V("dsl", i) + " * __builtin_amdgcn_rcp(" + rd("s", i) + "));");
                ln("bd = __builtin_fmax(bd, -" + V("dz", i) + " * " + rd("rzi", i) + ");");
            }
            ln("ap = bp > 1e-10 ? __builtin_amdgcn_rcp(bp) : 1.0;");
            ln("ad = bd > 1e-10 ? __builtin_amdgcn_rcp(bd) : 1.0;");
            close();
        }
    }


    std::string build() {
        const long n = pl.n, m = pl.m, p = pl.p, N = pl.N;
        const std::string kname = "QPB_KERNEL_NAME";
        o << "// generated by qpb_codegen for plan " << std::hex << pl.hash << std::dec
          << ": n=" << n << " m=" << m << " p=" << p << " N=" << N << " nnz(L)=" << pl.lnz
          << (opt.exact ? " [exact]" : " [fast]") << "\n";
        o << "#pragma clang fp contract(" << (opt.exact ? "off" : "fast") << ")\n";
        o << "#ifndef QPB_WARM\n#define QPB_WARM 0   // 1: the warm-solve variant (qpb_solve_warm)\n#endif\n";
        o << "struct qpb_args {\n"
             "  const double *P, *A, *G, *c, *h, *b;\n"
             "  double *x, *y, *z, *s;\n"
             "  int *flag, *iters;\n"
             "  double *fval;\n"
             "  double *stats;\n"
             "  long B;\n"
             "  double tol, abstol, sigma_d;\n"
             "  long maxit;\n"
             "  const void *tab; double *best; unsigned long long *part; unsigned *ctr;\n"
             "  double *sig;   // per-QP sigma: in (warm) / out (NULL: not tracked)\n"
             "  long warm;     // 1: continue from x, y, z, s, iters, flag, sig (no kkt_initialize)\n"
             "  double *trace; // warm variant: per-QP timers + per-iteration statistics (or NULL)\n"
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
        {
            std::vector<long> keep;
            for (long e = 0; e < pl.lnz; e++)
                if (opt.exact || !leaf[col_of(e)]) keep.push_back(e);
            for (size_t i0 = 0; i0 < keep.size(); i0 += 8) {
                std::string d = "double ";
                for (size_t i = i0; i < keep.size() && i < i0 + 8; i++) d += (i > i0 ? ", " : "") + V("L", keep[i]);
                ln(d + ";");
            }
        }
        if (use_lds) {
            ln("__shared__ double qpb_lds[" + S(lds_rows * opt.wg) + "];");
            ln("{ // stage this lane's matrix values in its private LDS column");
            for (long j = 0; lds_A >= 0 && j < (pl.p ? pl.A.nnz() : 0); j++)
                ln("  qpb_lds[" + S((lds_A + j) * opt.wg) + " + threadIdx.x] = tA[" + S(j * 64) + " + lane];");
            for (long j = 0; lds_G >= 0 && j < pl.G.nnz(); j++)
                ln("  qpb_lds[" + S((lds_G + j) * opt.wg) + " + threadIdx.x] = tG[" + S(j * 64) + " + lane];");
            for (long j = 0; lds_P >= 0 && j < pl.Pin.nnz(); j++)
                ln("  qpb_lds[" + S((lds_P + j) * opt.wg) + " + threadIdx.x] = tP[" + S(j * 64) + " + lane];");
            for (long j = 0; lds_c >= 0 && j < n; j++)
                ln("  qpb_lds[" + S((lds_c + j) * opt.wg) + " + threadIdx.x] = tc[" + S(j * 64) + " + lane];");
            for (long j = 0; lds_h >= 0 && j < m; j++)
                ln("  qpb_lds[" + S((lds_h + j) * opt.wg) + " + threadIdx.x] = th[" + S(j * 64) + " + lane];");
            for (long j = 0; lds_b >= 0 && j < p; j++)
                ln("  qpb_lds[" + S((lds_b + j) * opt.wg) + " + threadIdx.x] = tb[" + S(j * 64) + " + lane];");
            ln("}");
        }
        if (opt.exact) decl_vec("D", N);
        else decl_vec("rD", N);
        if (!park.count("x")) decl_vec("x", n);
        if (!park.count("y")) decl_vec("y", p);
        if (!park.count("s")) decl_vec("s", m);
        if (!park.count("z")) decl_vec("z", m);

        // ---- kkt_initialize (Auxilary.c:992-1089); a warm solve (QP_SOLVE called
        // again, qpSWIFT.c:502-596) instead continues from the output arrays
        ln("long it0 = 0; int flag0 = 3; double sigma = 100.0;");
        open("if (QPB_WARM) {   // the warm-solve variant (qpb_solve_warm)");
        begin_phase(false, false);
        auto warm_load = [&](const char *arr, long nv) {
            for (long i = 0; i < nv; i++)
                wr(arr, i, std::string("a.") + arr + "[tile * " + S(nv * 64) + " + " + S(i * 64) + " + lane]");
        };
        warm_load("x", n);
        warm_load("y", p);
        warm_load("s", m);
        warm_load("z", m);
        ln("it0 = a.iters[q]; flag0 = a.flag[q]; sigma = a.sig[q];");
        close();
        open("else {");
        ln("// setup: factor the KKT holding -I, solve for rhs [-c; b; h]");
        begin_phase();
        factor(pl.K_init);
        decl_vec("x0_", n);
        decl_vec("y0_", p);
        solve(pl.K_init, [&](long t) -> std::string {
                  if (t < n) return "(-" + in("c", t) + ")";
                  if (t < n + p) return in("b", t - n);
                  return in("h", t - n - p);
              },
              [&](long t) -> std::string {
                  if (t < n) return V("x0_", t);
                  if (t < n + p) return V("y0_", t - n);
                  return "";
              });
        for (long i = 0; i < n; i++) wr("x", i, V("x0_", i));
        for (long i = 0; i < p; i++) wr("y", i, V("y0_", i));
        open("{");
        spmv_neg(pl.G, nullptr, "G", "x", "zi");
        for (long i = 0; i < m; i++) ln(V("zi", i) + " = " + V("zi", i) + " + " + in("h", i) + ";");
        ln("double lo = zi0, hi = zi0;");
        for (long i = 1; i < m; i++) {
            ln("if (" + V("zi", i) + " < lo) lo = " + V("zi", i) + ";");
            ln("if (" + V("zi", i) + " > hi) hi = " + V("zi", i) + ";");
        }
        ln("const double sh = -lo;");
        for (long i = 0; i < m; i++) wr("s", i, "sh < 0 ? " + V("zi", i) + " : " + V("zi", i) + " + (1 + sh)");
        for (long i = 0; i < m; i++) wr("z", i, "hi < 0 ? -" + V("zi", i) + " : -" + V("zi", i) + " + (1 + hi)");
        close();
        close();   // else (cold)

        // ---- QP_SOLVE loop (qpSWIFT.c:502-602); QP_MAXIT only when IterationCount
        // == maxit (qpSWIFT.c:598-601), IterationCount = it0 + it
        ln("long it = 0; int flag = flag0;");
        ln("double fval = 0.0, st_rx = 0.0, st_ry = 0.0, st_rz = 0.0, st_mu = 0.0, ap = 0.0, ad = 0.0;");
        // the drop-in's timers and verbose trace (KernelArgs::trace): warm variant only
        ln("double *const trc = (QPB_WARM && a.trace) ? a.trace + q * " + S(QPB_TRACE_STRIDE) + " : nullptr;");
        ln("long t_fac = 0, t_kkt = 0, n_top = 0, n_it = 0, tk0 = 0;");
        open("for (;;) {");
        ln("if (it >= a.maxit) { flag = it0 + it == a.maxit ? 2 : flag0; break; }");
        begin_phase();
        // residuals (Auxilary.c:745-786) and objective (Auxilary.c:1133-1141)
        if (opt.exact) {
            spmv_neg(pl.Pf, &pl.Pf_src, "P", "x", "t");
            ln("double f1 = t0 * " + rd("x", 0) + ";");
            for (long j = 1; j < n; j++) ln("f1 = " + madd("f1", V("t", j), rd("x", j)) + ";");
            ln("double f2 = " + in("c", 0) + " * " + rd("x", 0) + ";");
            for (long j = 1; j < n; j++) ln("f2 = " + madd("f2", in("c", j), rd("x", j)) + ";");
            ln("fval = -0.5 * f1 + f2;");
            for (long j = 0; j < n; j++) ln("double " + V("rx", j) + " = " + V("t", j) + ";");
            for (long j = 0; j < n; j++)
                for (long k = pl.G.jc[j]; k < pl.G.jc[j + 1]; k++)
                    ln(V("rx", j) + " = " + msub(V("rx", j), in("G", k), rd("z", pl.G.ir[k])) + ";");
            if (p)
                for (long j = 0; j < n; j++)
                    for (long k = pl.A.jc[j]; k < pl.A.jc[j + 1]; k++)
                        ln(V("rx", j) + " = " + msub(V("rx", j), in("A", k), rd("y", pl.A.ir[k])) + ";");
            for (long j = 0; j < n; j++) ln(V("rx", j) + " = " + V("rx", j) + " - " + in("c", j) + ";");
            dot("nrx2", n, "rx", "rx", true);
            ln("st_rx = __builtin_sqrt(nrx2);");
            if (park.count("rx")) for (long j = 0; j < n; j++) wr("rx", j, V("rx", j));
            if (p) {
                spmv_neg(pl.A, nullptr, "A", "x", "ry");
                for (long i = 0; i < p; i++) ln(V("ry", i) + " = " + V("ry", i) + " + " + in("b", i) + ";");
                dot("nry2", p, "ry", "ry", true);
                ln("st_ry = __builtin_sqrt(nry2);");
                if (park.count("ry")) for (long i = 0; i < p; i++) wr("ry", i, V("ry", i));
            }
            spmv_neg(pl.G, nullptr, "G", "x", "rz");
            for (long i = 0; i < m; i++) ln(V("rz", i) + " = " + V("rz", i) + " + (" + in("h", i) + " - " + rd("s", i) + ");");
            dot("nrz2", m, "rz", "rz", true);
            ln("st_rz = __builtin_sqrt(nrz2);");
            if (park.count("rz")) for (long i = 0; i < m; i++) wr("rz", i, V("rz", i));

        } else {
            // Fast: one pass over every stored value, each used for both of its
            // products while in a register (P upper-symmetric, A and G for their
            // product and transposed product) -- same sums, another order.
            for (long j = 0; j < n; j++) ln("double " + V("t", j) + " = 0.0;");
            for (long j = 0; j < n; j++) ln("double " + V("rx", j) + " = 0.0;");
            for (long i = 0; i < p; i++) ln("double " + V("ry", i) + " = " + in("b", i) + ";");
            for (long i = 0; i < m; i++) ln("double " + V("rz", i) + " = " + in("h", i) + " - " + rd("s", i) + ";");
            if (pl.pmode == P_UPPER) {
                for (long c = 0; c < n; c++)
                    for (long k = pl.Pin.jc[c]; k < pl.Pin.jc[c + 1]; k++) {
                        long r = pl.Pin.ir[k];
                        std::string v = in("P", k);
                        ln(V("t", r) + " = " + msub(V("t", r), v, rd("x", c)) + ";");
                        if (r != c) ln(V("t", c) + " = " + msub(V("t", c), v, rd("x", r)) + ";");
                    }
            } else {
                for (long c = 0; c < n; c++)
                    for (long k = pl.Pf.jc[c]; k < pl.Pf.jc[c + 1]; k++)
                        ln(V("t", pl.Pf.ir[k]) + " = " + msub(V("t", pl.Pf.ir[k]), in("P", pl.Pf_src[k]), rd("x", c)) + ";");
            }
            for (long j = 0; j < n; j++)
                for (long k = pl.G.jc[j]; k < pl.G.jc[j + 1]; k++) {
                    std::string v = in("G", k);
                    long r = pl.G.ir[k];
                    ln(V("rx", j) + " = " + msub(V("rx", j), v, rd("z", r)) + ";");
                    ln(V("rz", r) + " = " + msub(V("rz", r), v, rd("x", j)) + ";");
                }
            if (p)
                for (long j = 0; j < n; j++)
                    for (long k = pl.A.jc[j]; k < pl.A.jc[j + 1]; k++) {
                        std::string v = in("A", k);
                        long r = pl.A.ir[k];
                        ln(V("rx", j) + " = " + msub(V("rx", j), v, rd("y", r)) + ";");
                        ln(V("ry", r) + " = " + msub(V("ry", r), v, rd("x", j)) + ";");
                    }
            ln("double f1 = t0 * " + rd("x", 0) + ";");
            for (long j = 1; j < n; j++) ln("f1 = " + madd("f1", V("t", j), rd("x", j)) + ";");
            ln("double f2 = " + in("c", 0) + " * " + rd("x", 0) + ";");
            for (long j = 1; j < n; j++) ln("f2 = " + madd("f2", in("c", j), rd("x", j)) + ";");
            ln("fval = -0.5 * f1 + f2;");
            for (long j = 0; j < n; j++) ln(V("rx", j) + " = " + V("rx", j) + " + " + V("t", j) + " - " + in("c", j) + ";");
            dot("nrx2", n, "rx", "rx", true);
            ln("st_rx = __builtin_sqrt(nrx2);");
            if (park.count("rx")) for (long j = 0; j < n; j++) wr("rx", j, V("rx", j));
            if (p) {
                dot("nry2", p, "ry", "ry", true);
                ln("st_ry = __builtin_sqrt(nry2);");
                if (park.count("ry")) for (long i = 0; i < p; i++) wr("ry", i, V("ry", i));
            }
            dot("nrz2", m, "rz", "rz", true);
            ln("st_rz = __builtin_sqrt(nrz2);");
            if (park.count("rz")) for (long i = 0; i < m; i++) wr("rz", i, V("rz", i));
        }
        dot("sz", m, "s", "z");
        ln("st_mu = sz / " + S(m) + ".0;");
        ln("if (trc && it < " + S(QPB_TRACE_MAX) + ") { double *e = trc + 4 + 7 * it; e[0] = fval; e[1] = st_rx; "
           "e[2] = st_ry; e[3] = st_rz; e[4] = st_mu; n_top = it + 1; }");
        ln(std::string("if (st_rx < a.tol && st_rz < a.tol") + (p ? " && st_ry < a.tol" : "") +
           " && st_mu < a.abstol) { flag = it0 + it == a.maxit ? 2 : 0; break; }");
        // lambda, mu (qpSWIFT.c:537-538)
        // lambda = sqrt(s.*z) (Auxilary.c:638-646) only ever enters squared, so the
        // fast kernel uses lambda^2 = s.*z directly (no sqrt).
        if (opt.exact) {
            for (long i = 0; i < m; i++) ln("const double " + V("lam", i) + " = __builtin_sqrt(" + rd("s", i) + " * " + rd("z", i) + ");");
            dot("mu2", m, "lam", "lam");
            ln("const double mu = mu2 / " + S(m) + ".0;");
        } else {
            ln("const double mu = st_mu;");
        }
        auto lam2 = [&](long i) {
            return opt.exact ? "(" + V("lam", i) + " * " + V("lam", i) + ")" : "(" + rd("s", i) + " * " + rd("z", i) + ")";
        };
        ln("const bool pc = sigma > a.sigma_d;");
        if (!opt.exact)
            for (long i = 0; i < m; i++) {
                if (park.count("rzi")) wr("rzi", i, "qpb_rcp(" + rd("z", i) + ")");
                else ln("const double " + V("rzi", i) + " = qpb_rcp(" + rd("z", i) + ");");
            }

        // updatekktmatrix: -s/z on the z diagonal (Auxilary.c:211-215)
        for (long i = 0; i < m; i++) {
            if (opt.exact) ln("const double " + V("kd", i) + " = (-" + rd("s", i) + ") / " + rd("z", i) + ";");
            else ln("const double " + V("kd", i) + " = -" + rd("s", i) + " * " + rd("rzi", i) + ";");
        }
        begin_phase();
        ln("if (trc) tk0 = (long)__builtin_amdgcn_s_memrealtime();");
        factor(pl.K_loop);
        ln("if (trc) { const long d_ = (long)__builtin_amdgcn_s_memrealtime() - tk0; t_fac += d_; t_kkt += d_; }");
        // form_ds: predictor (pure Newton) or pure centering (qpSWIFT.c:542, 574-575);
        // ds does not enter the factorisation, so it is formed after it.
        //
        // Fast kernel algebra (same Newton systems, fewer live values): with
        // ds = -s.*z + cc the rhs z-part is rz - ds/z = rz + s - cc/z and
        // dsl = (ds - s.*dz)/z = -s + (cc - s.*dz)/z, where cc = 0 for the
        // predictor, cc = sigma*mu - dsl.*dz for the corrector and sigma_d*mu for
        // the pure centering step; so ds itself is never materialised.
        ln("if (!pc) sigma = a.sigma_d;");
        if (opt.exact) {
            begin_phase(false, true);
            decl_vec("ds", m);
            for (long i = 0; i < m; i++)
                ln(V("ds", i) + " = pc ? (-" + V("lam", i) + ") * " + V("lam", i) + " : -" + lam2(i) + " + (sigma * mu);");
        } else {
            decl_vec("cc", m);
        }
        decl_vec("dx", n);
        decl_vec("dy", p);
        decl_vec("dz", m);
        decl_vec("dsl", m);
        // rhs z-part; pred = true only for the predictor solve (cc == 0)
        auto rhs_with = [&](bool pred) {
            return [&, pred](long t) -> std::string {
                if (t < n) return rd("rx", t);
                if (t < n + p) return rd("ry", t - n);
                long i = t - n - p;
                if (opt.exact) return "(" + rd("rz", i) + " - (" + V("ds", i) + " / " + rd("z", i) + "))";
                if (pred) return "(" + rd("rz", i) + " + " + rd("s", i) + ")";
                return "__builtin_fma(-" + V("cc", i) + ", " + rd("rzi", i) + ", " + rd("rz", i) + " + " + rd("s", i) + ")";
            };
        };
        auto dsl_from_dz = [&](bool pred) {
            begin_phase(false, true);
            for (long i = 0; i < m; i++) {
                if (opt.exact) {
                    std::string num = V("ds", i) + " - (" + rd("s", i) + " * " + V("dz", i) + ")";
                    ln(V("dsl", i) + " = (" + num + ") / " + rd("z", i) + ";");
                } else if (pred) {
                    ln(V("dsl", i) + " = -" + rd("s", i) + " * __builtin_fma(" + V("dz", i) + ", " + rd("rzi", i) + ", 1.0);");
                } else {
                    ln(V("dsl", i) + " = __builtin_fma(__builtin_fma(-" + rd("s", i) + ", " + V("dz", i) + ", " + V("cc", i) +
                       "), " + rd("rzi", i) + ", -" + rd("s", i) + ");");
                }
            }
        };
        // predictor solve, step, rho, sigma, corrector ds (kktsolve_1, qpSWIFT.c:552-569)
        if (!opt.exact)
            for (long i = 0; i < m; i++) ln(V("cc", i) + " = sigma * mu;");   // centering (!pc) default
        open("if (pc) {");
        ln("if (trc) tk0 = (long)__builtin_amdgcn_s_memrealtime();");
        solve(pl.K_loop, rhs_with(true), [&](long t) -> std::string {
            if (t < n + p) return "";
            return V("dz", t - n - p);
        });
        ln("if (trc) t_kkt += (long)__builtin_amdgcn_s_memrealtime() - tk0;");
        dsl_from_dz(true);
        step_length();
        begin_phase(false, true);
        ln("double rho_n = 0.0;");
        for (long i = 0; i < m; i++)
            ln("rho_n = rho_n + (" + rd("s", i) + " + (ap * " + V("dsl", i) + ")) * (" + rd("z", i) + " + (ad * " + V("dz", i) + "));");
        ln("const double rho = rho_n / sz;");
        ln("const double r1 = 1 > rho ? rho : 1;");
        ln("const double cube = r1 * r1 * r1;");
        ln("sigma = a.sigma_d < cube ? cube : a.sigma_d;");
        for (long i = 0; i < m; i++) {
            if (opt.exact)
                ln(V("ds", i) + " = -" + lam2(i) + " - (" + V("dsl", i) + " * " + V("dz", i) + ") + (sigma * mu);");
            else
                ln(V("cc", i) + " = __builtin_fma(-" + V("dsl", i) + ", " + V("dz", i) + ", sigma * mu);");
        }
        close();
        // corrector / centering solve (kktsolve_2, Auxilary.c:524-564)
        ln("if (trc) tk0 = (long)__builtin_amdgcn_s_memrealtime();");
        solve(pl.K_loop, rhs_with(false), [&](long t) -> std::string {
            if (t < n) return V("dx", t);
            if (t < n + p) return V("dy", t - n);
            return V("dz", t - n - p);
        });
        ln("if (trc) t_kkt += (long)__builtin_amdgcn_s_memrealtime() - tk0;");
        dsl_from_dz(false);
        step_length();
        begin_phase(false, true);
        ln("ap = 0.99 * ap > 1.0 ? 1.0 : 0.99 * ap;");
        ln("ad = 0.99 * ad > 1.0 ? 1.0 : 0.99 * ad;");
        ln("if (trc && it < " + S(QPB_TRACE_MAX) + ") { trc[4 + 7 * it + 5] = ap; trc[4 + 7 * it + 6] = ad; n_it = it + 1; }");
        for (long i = 0; i < n; i++) wr("x", i, madd(rd("x", i), V("dx", i), "ap"));
        for (long i = 0; i < p; i++) wr("y", i, madd(rd("y", i), V("dy", i), "ad"));
        for (long i = 0; i < m; i++) wr("s", i, madd(rd("s", i), V("dsl", i), "ap"));
        for (long i = 0; i < m; i++) wr("z", i, madd(rd("z", i), V("dz", i), "ad"));
        ln("it++;");
        close();
        // outputs
        begin_phase(false, true);
        auto store = [&](const char *arr, long nv, const char *base) {
            ln(std::string("double *__restrict__ o_") + arr + " = a." + arr + " + tile * " + S(nv * 64) + " + lane;");
            for (long i = 0; i < nv; i++) ln("o_" + std::string(arr) + "[" + S(i * 64) + "] = " + rd(base, i) + ";");
        };
        store("x", n, "x");
        if (p) store("y", p, "y");
        store("z", m, "z");
        store("s", m, "s");
        ln("a.flag[q] = flag; a.iters[q] = (int)(it0 + it); a.fval[q] = fval;");
        ln("if (QPB_WARM || a.sig) a.sig[q] = sigma;   // cold: options->sigma for the drop-in");
        ln("if (trc) { trc[0] = (double)t_fac; trc[1] = (double)t_kkt; trc[2] = (double)n_top; trc[3] = (double)n_it; }");
        ln("if (a.stats) { double *o = a.stats + tile * 384 + lane; o[0] = st_rx; o[64] = st_ry; o[128] = st_rz;"
           " o[192] = st_mu; o[256] = ap; o[320] = ad; }");
        o << "}\n";
        return o.str();
    }
};

}  // namespace

std::string kernel_name(const Plan &pl, const GenOptions &opt) {
    char buf[96];
    snprintf(buf, sizeof buf, "qpb_ipm_%016llx_%s_w%d_l%d", (unsigned long long)pl.hash, opt.exact ? "x" : "f",
             opt.wg, opt.lds_mode);
    return buf;
}

GenOptions choose_options(const Plan &pl, bool exact) {
    // Measured on MI355X (profiles/): what costs is VMEM latency of
    // spills and reloads, so keep the matrix values (P, A, G) on chip and then
    // maximise waves per CU; all inputs + loop vectors on chip (mode 4) wins only
    // at equal wave count.  LDS is 160 KiB per CU.
    GenOptions o;
    o.exact = exact;
    o.waves_per_eu = 1;
    const long nA = pl.p ? pl.A.nnz() : 0, nG = pl.G.nnz(), nP = pl.Pin.nnz();
    const long mats = nP + nA + nG;
    const long all = mats + pl.n + pl.m + pl.p + (2 * pl.n + 2 * pl.p + 2 * pl.m);   // mode 4 rows (no z park)
    const long cap = 160 * 1024 / 8;            // doubles of LDS per CU
    struct Cand { int wg, mode; long rows; };
    const Cand cands[] = {{256, 4, all}, {256, 2, mats}, {128, 4, all}, {128, 2, mats},
                          {256, 1, nA + nG}, {64, 4, all}, {128, 1, nA + nG}};
    o.wg = 256;
    o.lds_mode = 0;
    o.park_z = 0;
    for (const Cand &c : cands)
        if (c.rows > 0 && c.rows * c.wg <= cap) { o.wg = c.wg; o.lds_mode = c.mode; break; }
    return o;
}

std::string generate_kernel(const Plan &pl, const GenOptions &opt) {
    Gen g(pl, opt);
    std::string src = g.build();
    // The kernel (and code-object cache) name carries a hash of the generated
    // source, so any change of the generator yields a new name.
    const uint64_t h = fnv1a(src);
    char suffix[32];
    snprintf(suffix, sizeof suffix, "_%08llx", (unsigned long long)(h & 0xffffffffull));
    const std::string name = kernel_name(pl, opt) + suffix;
    for (size_t pos; (pos = src.find("QPB_KERNEL_NAME")) != std::string::npos;) src.replace(pos, 15, name);
    return src;
}

std::string kernel_name_of(const std::string &src) {
    size_t a = src.find("qpb_ipm_");
    size_t b = src.find('(', a);
    return src.substr(a, b - a);
}

}  // namespace qpb

// qpb_wave.cpp -- plan -> source of the wave-cooperative kernel (qpb_wave.hip).
//
// The kernel body is a fixed template; what is plan-specific is prepended as
// macros and constant tables: sizes, where every CSC value of P, A, G lands in
// the per-QP dense LDS copies, and the structural pattern of G (which G'WG
// updates exist).  See qpb_wave.hip for the algorithm.
#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <sstream>
#include <string>

#include "qpb_plan.hpp"
#include "qpb_wave.hpp"

namespace qpb {

namespace {
const char *kWaveTemplate =
#include "qpb_wave_src.inc"
    ;
const char *kRowTemplate =
#include "qpb_row_src.inc"
    ;
const char *kBandTemplate =
#include "qpb_band_src.inc"
    ;
const char *kRowxTemplate =
#include "qpb_rowx_src.inc"
    ;

template <class F>
void table(std::ostringstream &o, const char *decl, long cnt, F f) {
    o << decl << "[" << (cnt > 0 ? cnt : 1) << "] = {";
    if (cnt <= 0) o << "0";
    for (long k = 0; k < cnt; k++) o << (k ? "," : "") << f(k);
    o << "};\n";
}
}  // namespace

WaveLayout wave_layout(const Plan &pl) {
    const long n = pl.n, m = pl.m, p = pl.p;
    WaveLayout L;
    L.zleaf.assign(m, 1);
    L.yleaf.assign(p, 1);
    // a z or y row is a leaf when every neighbour (an x row) comes later in the
    // permutation: its row of L is empty and D = its diagonal (ldl.c:300)
    for (long j = 0; j < n; j++) {
        for (long k = pl.G.jc[j]; k < pl.G.jc[j + 1]; k++)
            if (pl.pinv[n + p + pl.G.ir[k]] > pl.pinv[j]) L.zleaf[pl.G.ir[k]] = 0;
        if (p)
            for (long k = pl.A.jc[j]; k < pl.A.jc[j + 1]; k++)
                if (pl.pinv[n + pl.A.ir[k]] > pl.pinv[j]) L.yleaf[pl.A.ir[k]] = 0;
    }
    for (long pos = 0; pos < pl.N; pos++) {
        const long k = pl.perm[pos];
        const bool leaf = (k >= n + p) ? L.zleaf[k - n - p] : (k >= n ? L.yleaf[k - n] : false);
        if (!leaf) L.dense.push_back(k);
    }
    return L;
}

// odd leading dimensions of the staged P, A, G (qpb_wave.hip QPB_W_PAD, off by
// default; QPB_WAVE_OPTS="QPB_W_PAD=1" turns them on on both sides)
static bool wave_pad() {
    const char *e = getenv("QPB_WAVE_OPTS");
    return e && strstr(e, "QPB_W_PAD=1");
}

// per-wave LDS doubles (qpb_wave.hip LDS_WAVE): dense P, A, G, the L transpose
// and the vector exchange area; ldg = the staged G's leading dimension
static long wave_lds_doubles(const Plan &pl, long nd, long ldg) {
    // T: packed strictly-lower -L, or the MFMA tiles / broadcast buffers (TSZ in qpb_wave.hip)
    const long nt = (pl.n + 15) / 16;
    const bool mfma = pl.G.nnz() > 48 && pl.n <= 64;
    long t = std::max(nd * (nd - 1) / 2, mfma ? 256 * nt * nt : 0L);
    if (nd > 16) t = std::max(t, 128L);
    if (nd > 16 && nd <= 32) t = std::max(t, nd * nd);          // two rows per lane (QPB_W_DUP) scratch
    const char *opts = getenv("QPB_WAVE_OPTS");
    if (nd > 32 && opts && strstr(opts, "QPB_W_BLK=1"))
        t = std::max(t, 128L + 2 * 48 * 17 + 16);               // blocked LDL' scratch (QPB_W_BLK)
    t = ((t + 1) & ~1L) + 2;
    // staged P, A, G with odd leading dimensions (LDP, LDY, LDZ)
    const long pad = wave_pad() ? 1 : 0;
    const long stage = pl.n * (pl.n | pad) + (pl.p ? pl.n * (pl.p | pad) : 0) + pl.n * ldg;
    return stage + t + 2 * pl.N + pl.m + pl.n + 8;
}

// workgroup size and QPs per CU for a footprint of `doubles` per QP
static int wg_for_doubles(long doubles, int *qps_per_cu) {
    const long bytes = doubles * 8;
    // as many QPs per CU as the 160 KiB allow (whole workgroups), ties -> larger
    // workgroups; except where the LDS holds a CU to at most 16 QPs: there the smallest
    // size that reaches the same count, since a workgroup's LDS is freed only when its
    // slowest QP finishes and one-wave workgroups refill the CU QP by QP (8 192
    // AMD-ordered 30/68/18 QPs 2.33 -> 2.24 ms against four-wave workgroups,
    // profiles/r04_wave_wg_ab.log; 1 024 QPs unchanged)
    int best = 0, best_qps = 0;
    for (int waves = 4; waves >= 1; waves--) {
        const long per_cu = (160L * 1024) / (bytes * waves);
        if (per_cu * waves > best_qps) { best_qps = (int)(per_cu * waves); best = waves; }
    }
    for (int waves = 1; waves < best && best_qps <= 16; waves++) {
        const long per_cu = (160L * 1024) / (bytes * waves);
        if (per_cu * waves == best_qps) { best = waves; break; }
    }
    if (qps_per_cu) *qps_per_cu = best_qps;
    return 64 * best;
}

// The staged G's leading dimension.  Its columns are read lane-strided (G(r, i) by the
// lane of x_i: the residual's G'z, the solve's leaf elimination, the MFMA operands); a
// stride of m doubles with m = 0 mod 4 puts those reads on 8 of the 64 LDS banks.  Padded
// to 2 mod 4 (16-byte column alignment kept) the lanes spread over 16 bank pairs -- when
// that costs no QP per CU (QPB_W_PADZ=0 turns it off; QPB_W_PAD=1, odd, overrides).
static long wave_ldz(const Plan &pl, long nd) {
    if (wave_pad()) return pl.m | 1;
    const char *e = getenv("QPB_WAVE_OPTS");
    if (e && strstr(e, "QPB_W_PADZ=0")) return pl.m;
    const long padded = pl.m + ((2 - pl.m % 4) + 4) % 4;
    if (padded == pl.m) return pl.m;
    int q0 = 0, q1 = 0;
    wg_for_doubles(wave_lds_doubles(pl, nd, pl.m), &q0);
    wg_for_doubles(wave_lds_doubles(pl, nd, padded), &q1);
    return q1 >= q0 ? padded : pl.m;
}

int wave_wg_for(const Plan &pl) {
    const long nd = (long)wave_layout(pl).dense.size();
    const long doubles = wave_lds_doubles(pl, nd, wave_ldz(pl, nd));
    const int wg = wg_for_doubles(doubles, nullptr);
    // QPB_WAVE_OPTS="QPB_W_WG=64|128|192|256": a smaller workgroup with the same QPs per CU
    // (a workgroup's LDS is freed only when its slowest QP finishes)
    if (const char *e = getenv("QPB_WAVE_OPTS"))
        if (const char *k = strstr(e, "QPB_W_WG=")) {
            const int w = atoi(k + 9);
            if (w >= 64 && w <= wg && w % 64 == 0) return w;
        }
    return wg;
}

bool wave_eligible(const Plan &pl, std::string *why) {
    auto no = [&](const char *m) { if (why) *why = m; return false; };
    if (pl.n < 1 || pl.n > 64 || pl.m < 1 || pl.m > 256 || pl.p > 64)
        return no("need 1 <= n <= 64, 1 <= m <= 256, p <= 64");
    const long nd = (long)wave_layout(pl).dense.size();
    if (nd > 64) return no("more than 64 non-leaf KKT rows (the dense block is one row per lane)");
    if (wave_wg_for(pl) == 0) return no("dense per-QP copies exceed the LDS of a CU");
    // every G row must be non-empty: only then does each z column of the KKT
    // carry its own diagonal slot (Auxilary.c:126-131), which the leaf
    // elimination assumes.
    std::vector<int> rowcnt(pl.m, 0);
    for (long k = 0; k < pl.G.nnz(); k++) rowcnt[pl.G.ir[k]]++;
    for (long r = 0; r < pl.m; r++)
        if (!rowcnt[r]) return no("a row of G is empty");
    if (why) why->clear();
    return true;
}

// sizes, experiment knobs and the CSC -> dense LDS scatter tables shared by
// the wave and the row kernels; gcol_out receives the column of every G entry
// ldp / lda / ldg: leading dimensions of the staged dense P, A, G (the wave
// kernel pads them odd, qpb_wave.hip LDP / LDY / LDZ; the row kernel's are n, p, m)
static void common_header(std::ostringstream &o, const Plan &pl, int wg, const char *kind,
                          std::vector<long> *gcol_out, long ldp, long lda, long ldg) {
    const long n = pl.n, m = pl.m, p = pl.p;
    o << "// generated by qpb_wave for plan " << std::hex << pl.hash << std::dec << ": n=" << n << " m=" << m
      << " p=" << p << " [" << kind << ", fast]\n";
    o << "#define QPB_NX " << n << "\n#define QPB_NZ " << m << "\n#define QPB_NY " << p << "\n";
    o << "#define QPB_WG " << wg << "\n";
    // experiment knobs (the #ifndef blocks at the top of qpb_wave.hip / qpb_row.hip),
    // e.g. QPB_WAVE_OPTS="QPB_W_GG=0 QPB_W_SPLIT=2"; they change the source, hence the name
    if (const char *e = getenv("QPB_WAVE_OPTS")) {
        std::istringstream in(e);
        std::string kv;
        while (in >> kv) {
            const size_t eq = kv.find('=');
            // QPB_R_SPLIT changes the launch shape: selected per plan by QPB_ROW_SPLIT, never here
            if (eq != std::string::npos && kv.substr(0, eq) != "QPB_R_SPLIT")
                o << "#define " << kv.substr(0, eq) << " " << kv.substr(eq + 1) << "\n";
        }
    }
    const long nP = pl.Pin.nnz(), nA = p ? pl.A.nnz() : 0, nG = pl.G.nnz();
    o << "#define QPB_NNZP " << nP << "\n#define QPB_NNZA " << nA << "\n#define QPB_NNZG " << nG << "\n";
    std::vector<long> pcol(nP), acol(nA), gcol(nG);
    for (long j = 0; j < n; j++) {
        for (long k = pl.Pin.jc[j]; k < pl.Pin.jc[j + 1]; k++) pcol[k] = j;
        if (nA)
            for (long k = pl.A.jc[j]; k < pl.A.jc[j + 1]; k++) acol[k] = j;
        for (long k = pl.G.jc[j]; k < pl.G.jc[j + 1]; k++) gcol[k] = j;
    }
    table(o, "static __device__ const int qpb_scP", nP, [&](long k) { return pcol[k] * ldp + pl.Pin.ir[k]; });
    table(o, "static __device__ const int qpb_scP2", nP, [&](long k) {
        const long i = pl.Pin.ir[k], j = pcol[k];
        return (pl.pmode == P_UPPER && i != j) ? i * ldp + j : -1L;
    });
    table(o, "static __device__ const int qpb_scA", nA, [&](long k) { return acol[k] * lda + pl.A.ir[k]; });
    table(o, "static __device__ const int qpb_scG", nG, [&](long k) { return gcol[k] * ldg + pl.G.ir[k]; });
    if (gcol_out) *gcol_out = gcol;
}

static std::string named(const std::string &body, const char *prefix, const Plan &pl, int wg) {
    const uint64_t h = fnv1a(body);
    char name[96];
    snprintf(name, sizeof name, "%s_%016llx_w%d_%08llx", prefix, (unsigned long long)pl.hash, wg,
             (unsigned long long)(h & 0xffffffffull));
    return name;
}

bool row_eligible(const Plan &pl) {
    if (pl.n > 16 || pl.p > 16 || pl.m > 32 || !wave_eligible(pl, nullptr)) return false;
    const WaveLayout L = wave_layout(pl);
    if ((long)L.dense.size() != pl.n) return false;
    for (long d = 0; d < pl.n; d++)
        if (L.dense[d] != d) return false;
    return true;
}

// Gathered sparse products of the row kernel (qpb_row.hip QPB_R_GATHER).  A product
// with G or A done by DPP broadcasts costs one instruction per column (or row) in the
// union of the pattern -- G's 20 x 12 with 36 non-zeros takes 20 broadcasts for G'z
// and 12 for G x, each useful in the 2-3 lanes whose coefficient is non-zero.  Done as
// gathers, lane c reads exactly the vector entries its own row / column needs from the
// row's LDS vector area (one ds_read_b64 each, lane-dependent slot) and issues one FMA
// per term: the count is the longest list, not the union.  Per lane c (tables [16][len],
// padded with the zero slot):
//   XT: x row c's G'- then A'-column terms: G rows r with G(r,c) != 0 (first XG entries;
//       z slot r), then A rows l with A(l,c) != 0 (y slot 32 + l);
//   ZX0 / ZX1: z row c / 16 + c's G-row terms (x slot 48 + j);  AX: y row c's A-row terms.
// Each term: its slot and the index of its coefficient in the staged dense matrices
// (Ls: P at 0, A at n*n, G at n*n + max(p,1)*n, column-major), -1 for padding.
// qpb_xtpos[r][j]: where G row r sits in lane j's XT list (the G'WG update's source).
static void row_gather_tables(std::ostringstream &o, const Plan &pl, const std::vector<std::vector<int>> &gnz) {
    const long n = pl.n, m = pl.m, p = pl.p;
    const long off_a = n * n, off_g = off_a + std::max(p, 1L) * n;
    std::vector<std::vector<int>> anz(std::max(p, 1L), std::vector<int>(n, 0));
    for (long j = 0; j < n && p > 0; j++)
        for (long k = pl.A.jc[j]; k < pl.A.jc[j + 1]; k++) anz[pl.A.ir[k]][j] = 1;
    const int kZero = 64;
    typedef std::vector<std::pair<int, int>> Terms;
    std::vector<Terms> xg(16), xa(16), zx0(16), zx1(16), ax(16);
    for (long c = 0; c < 16; c++) {
        if (c < n) {
            for (long r = 0; r < m; r++)
                if (gnz[r][c]) xg[c].push_back({(int)r, (int)(off_g + c * m + r)});
            for (long l = 0; l < p; l++)
                if (anz[l][c]) xa[c].push_back({(int)(32 + l), (int)(off_a + c * p + l)});
        }
        for (long j = 0; j < n; j++) {
            if (c < m && gnz[c][j]) zx0[c].push_back({(int)(48 + j), (int)(off_g + j * m + c)});
            if (16 + c < m && gnz[16 + c][j]) zx1[c].push_back({(int)(48 + j), (int)(off_g + j * m + 16 + c)});
            if (c < p && anz[c][j]) ax[c].push_back({(int)(48 + j), (int)(off_a + j * p + c)});
        }
    }
    auto len = [](const std::vector<Terms> &t) {
        size_t k = 0;
        for (auto &v : t) k = std::max(k, v.size());
        return (long)k;
    };
    const long XG = len(xg), XA = len(xa);
    std::vector<Terms> xt(16);
    for (int c = 0; c < 16; c++) {
        xt[c] = xg[c];
        xt[c].resize((size_t)XG, {kZero, -1});
        xt[c].insert(xt[c].end(), xa[c].begin(), xa[c].end());
    }
    auto emit = [&](const char *nm, std::vector<Terms> t, long L) {
        o << "#define QPB_" << nm << "_LEN " << L << "\n";
        const long Lp = std::max(L, 1L);
        for (int which = 0; which < 2; which++) {
            o << "static __device__ const int qpb_" << (which ? "src_" : "slot_") << nm << "[16][" << Lp << "] = {";
            for (int c = 0; c < 16; c++) {
                t[c].resize((size_t)Lp, {kZero, -1});
                o << (c ? "," : "") << "{";
                for (long k = 0; k < Lp; k++) o << (k ? "," : "") << (which ? t[c][k].second : t[c][k].first);
                o << "}";
            }
            o << "};\n";
        }
    };
    o << "#define QPB_XG_LEN " << XG << "\n";
    emit("XT", xt, XG + XA);
    emit("ZX0", zx0, len(zx0));
    emit("ZX1", zx1, len(zx1));
    emit("AX", ax, len(ax));
    o << "static constexpr int qpb_xtpos[" << m << "][" << n << "] = {";
    for (long r = 0; r < m; r++) {
        o << (r ? "," : "") << "{";
        for (long j = 0; j < n; j++) {
            int pos = -1;
            for (size_t k = 0; k < xg[j].size(); k++)
                if (xg[j][k].first == r) pos = (int)k;
            o << (j ? "," : "") << pos;
        }
        o << "}";
    }
    o << "};\n";
    // unions of the DPP forms (what the gathers replace), for the generator's choice
    long ucol = 0;
    for (long j = 0; j < n; j++) {
        int any = 0;
        for (long l = 0; l < p; l++) any |= anz[l][j];
        ucol += any;
    }
    o << "#define QPB_AX_UNION " << ucol << "\n";
}

// plan-specific prefix of the row kernel (sizes, scatter tables, G pattern)
static std::string row_prefix(const Plan &pl) {
    const long n = pl.n, m = pl.m;
    const int wg = 64;
    std::ostringstream o;
    std::vector<long> gcol;
    common_header(o, pl, wg, "row-cooperative", &gcol, n, pl.p ? pl.p : 1, m);
    std::vector<std::vector<int>> gnz(m, std::vector<int>(n, 0));
    for (long k = 0; k < pl.G.nnz(); k++) gnz[pl.G.ir[k]][gcol[k]] = 1;
    o << "static constexpr bool qpb_Gnz[" << m << "][" << n << "] = {";
    for (long r = 0; r < m; r++) {
        o << (r ? "," : "") << "{";
        for (long j = 0; j < n; j++) o << (j ? "," : "") << gnz[r][j];
        o << "}";
    }
    o << "};\n";
    // columns touched by the z rows 16.. (second z register)
    o << "static constexpr bool qpb_ghmask[" << n << "] = {";
    for (long j = 0; j < n; j++) {
        int any = 0;
        for (long r = 16; r < m; r++) any |= gnz[r][j];
        o << (j ? "," : "") << any;
    }
    o << "};\n";
    row_gather_tables(o, pl, gnz);
    return o.str();
}

// split: the two-wave form of the one-wave kernel (QPB_R_SPLIT, 128-thread workgroups,
// one four-QP group per workgroup: wave 0 factors while wave 1 forms the residuals)
std::string generate_row_kernel(const Plan &pl, std::string *name_out, int wpe, bool split) {
    std::string prefix = row_prefix(pl);
    if (split) {
        const std::string wg = "#define QPB_WG 64\n";
        prefix.replace(prefix.find(wg), wg.size(), "#define QPB_WG 128\n#define QPB_R_SPLIT 1\n");
    }
    const std::string body = (wpe > 1 ? "#define QPB_R_WPE " + std::to_string(wpe) + "\n" : std::string()) +
                             prefix + kRowTemplate;
    const std::string name = named(body, split ? "qpb_rowsplit" : "qpb_row", pl, split ? 128 : 64);
    if (name_out) *name_out = name;
    return "#define QPB_KERNEL_NAME " + name + "\n" + body;
}

// One launch for several row-form plans (a mixed-pattern batch, e.g. the gait
// phases of configs[2]): the template's plan-independent helpers once, then each
// member's prefix + body inside namespace qpb_g<i> (its macros undefined after
// it), and a kernel that maps the logical block to its member.  Every member's
// body is the single-plan kernel's, so results are bit-identical to per-plan
// launches; the fused argmin counts all waves of the grid and reports indices
// into the concatenation of the members' batches.
std::string generate_row_group_kernel(const std::vector<const Plan *> &pls, std::string *name_out) {
    std::ostringstream o;
    o << "#define QPB_GROUP 1\n#define QPB_ROW_COMMON_ONLY 1\n" << kRowTemplate << "\n#undef QPB_ROW_COMMON_ONLY\n";
    static const char *undef[] = {"QPB_NX", "QPB_NZ", "QPB_NY", "QPB_WG", "QPB_NNZP", "QPB_NNZA", "QPB_NNZG",
                                  "NX", "NZ", "NY", "NY1", "WPB", "ZH", "EVEN", "OFF_A", "OFF_G", "OFF_T",
                                  "OFF_PR", "OFF_H0", "LDS_ROW", "STG_END", "LOOP_END", "OFF_VEC",
                                  "QPB_XG_LEN", "QPB_XT_LEN", "QPB_ZX0_LEN", "QPB_ZX1_LEN", "QPB_AX_LEN",
                                  "QPB_AX_UNION", "QPB_R_GATHER_A"};
    for (size_t i = 0; i < pls.size(); i++) {
        o << "namespace qpb_g" << i << " {\n" << row_prefix(*pls[i]) << kRowTemplate
          << "\nstatic constexpr long qpb_lds_doubles = 4 * LDS_ROW;\n}  // namespace qpb_g" << i << "\n";
        for (const char *u : undef) o << "#undef " << u << "\n";
    }
    o << "struct qpb_group_args {\n    qpb_args m[" << QPB_GROUP_MAX << "];\n    long bend[" << QPB_GROUP_MAX
      << "];\n    long qoff[" << QPB_GROUP_MAX << "];\n};\n";
    const std::string src = o.str();
    // LDS of the group kernel: the largest member's (members run in disjoint blocks)
    std::ostringstream k;
    k << "template <long A, long B> struct qpb_cmax { static constexpr long value = A > B ? A : B; };\n";
    k << "static constexpr long qpb_glds = ";
    for (size_t i = 0; i + 1 < pls.size(); i++) k << "qpb_cmax<qpb_g" << i << "::qpb_lds_doubles, ";
    k << "qpb_g" << pls.size() - 1 << "::qpb_lds_doubles";
    for (size_t i = 0; i + 1 < pls.size(); i++) k << ">::value";
    k << ";\n";
    k << "extern \"C\" __global__ void __launch_bounds__(64, 1) QPB_KERNEL_NAME(qpb_group_args g) {\n"
      << "    __shared__ __attribute__((aligned(16))) double qpb_lds[qpb_glds];\n"
      << "    const long lb = qpb_xcd_block();\n";
    for (size_t i = 0; i < pls.size(); i++)
        k << "    if (lb < g.bend[" << i << "]) { qpb_g" << i << "::qpb_row_body(g.m[" << i << "], lb"
          << (i ? " - g.bend[" + std::to_string(i - 1) + "]" : std::string()) << ", g.qoff[" << i
          << "], qpb_lds); return; }\n";
    k << "    if (g.m[0].best) qpb_argmin_arrive(g.m[0], __builtin_huge_val(), -1);   // grid padding\n}\n";
    const std::string body = src + k.str();
    const uint64_t h = fnv1a(body);
    char name[96];
    snprintf(name, sizeof name, "qpb_rowgroup%zu_%016llx", pls.size(), (unsigned long long)h);
    if (name_out) *name_out = name;
    return std::string("#define QPB_KERNEL_NAME ") + name + "\n" + body;
}

std::string generate_wave_kernel(const Plan &pl, int wg, std::string *name_out) {
    const long n = pl.n, m = pl.m, p = pl.p;
    std::ostringstream o;
    std::vector<long> gcol;
    const long pad = wave_pad() ? 1 : 0;
    // elimination layout: leaves first, the rest as a dense block in perm order
    const WaveLayout L = wave_layout(pl);
    const long nd = (long)L.dense.size();
    const long ldz = wave_ldz(pl, nd);
    common_header(o, pl, wg, "wave-cooperative", &gcol, pl.n | pad, (pl.p ? pl.p : 1) | pad, ldz);
    o << "#define QPB_LDZ " << ldz << "\n";
    const long nG = pl.G.nnz();
    std::vector<int> dkind(nd), didx(nd), xpos(n, -1);
    for (long d = 0; d < nd; d++) {
        const long k = L.dense[d];
        dkind[d] = k < n ? 0 : (k < n + p ? 1 : 2);
        didx[d] = (int)(k < n ? k : (k < n + p ? k - n : k - n - p));
        if (k < n) xpos[k] = (int)d;
    }
    o << "#define QPB_ND " << nd << "\n";
    // the common case: every z and y row is a leaf and the x rows come in natural
    // order, so dense row d IS x_d (the kernel then skips the re-distribution)
    bool xid = nd == n;
    for (long d = 0; xid && d < nd; d++) xid = L.dense[d] == d;
    o << "#define QPB_XID " << (xid ? 1 : 0) << "\n";
    auto carr = [&](const char *decl, const std::vector<int> &v) {
        o << "static constexpr int " << decl << "[" << (v.empty() ? 1 : v.size()) << "] = {";
        if (v.empty()) o << "0";
        for (size_t k = 0; k < v.size(); k++) o << (k ? "," : "") << v[k];
        o << "};\n";
        o << "static __device__ const int " << decl << "_d[" << (v.empty() ? 1 : v.size()) << "] = {";
        if (v.empty()) o << "0";
        for (size_t k = 0; k < v.size(); k++) o << (k ? "," : "") << v[k];
        o << "};\n";
    };
    // structure of the dense block's L: the plan's symbolic factor restricted to the
    // dense rows (moving the leaves first leaves it unchanged -- every leaf's neighbours
    // come after it in both orders).  qpb_lnz[j][k] = L(j, k) may be nonzero (j > k):
    // the factor skips the updates whose broadcast H(j, k) is a structural zero.
    {
        std::vector<long> dpos(pl.N, -1);
        for (long d = 0; d < nd; d++) dpos[pl.pinv[L.dense[d]]] = d;
        std::vector<std::vector<int>> lnz(nd, std::vector<int>(nd, 0));
        for (long c = 0; c < pl.N; c++) {
            const long kd = dpos[c];
            if (kd < 0) continue;
            for (long q = pl.Lp[c]; q < pl.Lp[c + 1]; q++) {
                const long jd = dpos[pl.Li[q]];
                if (jd > kd) lnz[jd][kd] = 1;
            }
        }
        o << "static constexpr bool qpb_lnz[" << std::max<long>(nd, 1) << "][" << std::max<long>(nd, 1) << "] = {";
        for (long j = 0; j < nd; j++) {
            o << (j ? "," : "") << "{";
            for (long k = 0; k < nd; k++) o << (k ? "," : "") << lnz[j][k];
            o << "}";
        }
        if (nd == 0) o << "{0}";
        o << "};\n";
    }
    carr("qpb_dkind", dkind);
    carr("qpb_didx", didx);
    carr("qpb_xpos", xpos);
    carr("qpb_zleaf", L.zleaf);
    carr("qpb_yleaf", L.yleaf);
    // structural G(r, j) of LEAF z rows: their G'diag(w)G updates of the x block
    std::vector<std::vector<int>> gnz(m, std::vector<int>(n, 0));
    for (long k = 0; k < nG; k++)
        if (L.zleaf[pl.G.ir[k]]) gnz[pl.G.ir[k]][gcol[k]] = 1;
    // leaf z rows grouped by their column pattern (e.g. the 24 torque-limit rows
    // of the controller QP share one): a runtime loop over a group's rows with
    // the pattern's columns unrolled keeps the G'diag(w)G update compact
    std::vector<std::vector<int>> gpat;
    std::vector<std::vector<int>> grows;
    for (long r = 0; r < m; r++) {
        if (!L.zleaf[r]) continue;
        std::vector<int> cols;
        for (long j = 0; j < n; j++)
            if (gnz[r][j]) cols.push_back((int)j);
        size_t g = 0;
        while (g < gpat.size() && gpat[g] != cols) g++;
        if (g == gpat.size()) { gpat.push_back(cols); grows.emplace_back(); }
        grows[g].push_back((int)r);
    }
    size_t maxc = 1;
    for (auto &c : gpat) maxc = std::max(maxc, c.size());
    o << "#define QPB_NGRP " << gpat.size() << "\n";
    o << "static constexpr int qpb_gncol[" << std::max<size_t>(gpat.size(), 1) << "] = {";
    for (size_t g = 0; g < gpat.size(); g++) o << (g ? "," : "") << gpat[g].size();
    if (gpat.empty()) o << "0";
    o << "};\nstatic constexpr int qpb_gcol[" << std::max<size_t>(gpat.size(), 1) << "][" << maxc << "] = {";
    for (size_t g = 0; g < gpat.size(); g++) {
        o << (g ? "," : "") << "{";
        for (size_t c = 0; c < maxc; c++) o << (c ? "," : "") << (c < gpat[g].size() ? gpat[g][c] : 0);
        o << "}";
    }
    if (gpat.empty()) o << "{0}";
    o << "};\nstatic constexpr int qpb_goff[" << gpat.size() + 1 << "] = {0";
    size_t acc = 0;
    std::vector<int> allrows;
    for (size_t g = 0; g < gpat.size(); g++) {
        acc += grows[g].size();
        o << "," << acc;
        allrows.insert(allrows.end(), grows[g].begin(), grows[g].end());
    }
    o << "};\nstatic __device__ const int qpb_grow[" << std::max<size_t>(allrows.size(), 1) << "] = {";
    for (size_t k = 0; k < allrows.size(); k++) o << (k ? "," : "") << allrows[k];
    if (allrows.empty()) o << "0";
    o << "};\n";
    o << "static constexpr bool qpb_Gnz[" << m << "][" << n << "] = {";
    for (long r = 0; r < m; r++) {
        o << (r ? "," : "") << "{";
        for (long j = 0; j < n; j++) o << (j ? "," : "") << gnz[r][j];
        o << "}";
    }
    o << "};\n";
    const std::string body = o.str() + kWaveTemplate;
    const std::string name = named(body, "qpb_wave", pl, wg);
    if (name_out) *name_out = name;
    return "#define QPB_KERNEL_NAME " + name + "\n" + body;
}

}  // namespace qpb

namespace qpb {

// LDS layout of the band kernel (qpb_band.hip), doubles per QP: packed stage blocks
// (P_k upper triangle, strictly lower -L_k, G_k on the union of the stages' G patterns)
struct BandLayout {
    long PP, LP, GS, O_P, O_L, O_RD, O_Y, O_G, O_AR, O_AL, O_DUMP, O_STATIC_END;
    long V_X, V_DX, V_Y, V_RY, V_Z, V_S, V_RZ, V_DZ, LDS_QP;
};

// (row, column) pairs of the stage-relative G pattern, union over the stages, row-major
static std::vector<std::pair<long, long>> band_gunion(const Plan &pl) {
    const long nb = pl.band_nb, mz = pl.band_mz;
    std::vector<std::pair<long, long>> u;
    for (long j = 0; j < pl.n; j++)
        for (long k = pl.G.jc[j]; k < pl.G.jc[j + 1]; k++) u.push_back({pl.G.ir[k] % mz, j % nb});
    std::sort(u.begin(), u.end());
    u.erase(std::unique(u.begin(), u.end()), u.end());
    return u;
}

static BandLayout band_layout(const Plan &pl) {
    const long nb = pl.band_nb, ns = pl.band_ns, mz = pl.band_mz, my = pl.band_my;
    const long nx = nb * ns, nz = mz * ns, ny = my * ns, ny1 = ny > 0 ? ny : 1;
    BandLayout L;
    L.PP = nb * (nb + 1) / 2;
    L.LP = nb * (nb - 1) / 2;
    L.GS = (long)band_gunion(pl).size() + 1;          // + a zero slot
    L.O_P = 0;
    L.O_L = L.O_P + ns * L.PP;
    L.O_RD = L.O_L + ns * L.LP;
    L.O_Y = L.O_RD + ns * nb;                         // stages 1 .. ns - 1
    L.O_G = L.O_Y + (ns - 1) * my * nb;
    L.O_AR = L.O_G + ns * L.GS;
    L.O_AL = L.O_AR + ns * my * nb;                   // stages 1 .. ns - 1
    L.O_STATIC_END = (L.O_AL + (ns - 1) * my * nb + 1) & ~1L;   // even: 16-byte zero-fill stores
    L.V_X = L.O_STATIC_END;
    L.V_DX = L.V_X + nx;
    L.V_Y = L.V_DX + nx;
    L.V_RY = L.V_Y + ny1;
    L.V_Z = L.V_RY + ny1;
    L.V_S = L.V_Z + nz;
    L.V_RZ = L.V_S + nz;
    L.V_DZ = L.V_RZ + nz;
    L.LDS_QP = L.V_DZ + nz;
    // masked stores of the factor go to one slot per lane inside dz (dead while the
    // factor runs), or after everything when dz is shorter than a wavefront
    if (nz >= 64) {
        L.O_DUMP = L.V_DZ;
    } else {
        L.O_DUMP = L.LDS_QP;
        L.LDS_QP += 64;
    }
    return L;
}

long band_lds_bytes(const Plan &pl) { return pl.band_nb > 0 ? band_layout(pl).LDS_QP * 8 : 0; }

bool band_eligible(const Plan &pl, std::string *why) {
    auto no = [&](const char *m) { if (why) *why = m; return false; };
    if (pl.band_nb <= 0) return no("not a multi-stage pattern (band_shape)");
    // the kernel eliminates z rows, y rows, then x in natural order: the plan's
    // permutation must be exactly that (ORDER_LEAVES), or results would follow a
    // different factorisation than the plan's oracle
    const long n = pl.n, m = pl.m, p = pl.p;
    for (long k = 0; k < m; k++)
        if (pl.perm[k] != n + p + k) return no("permutation is not leaves-first");
    for (long k = 0; k < p; k++)
        if (pl.perm[m + k] != n + k) return no("permutation is not leaves-first");
    for (long k = 0; k < n; k++)
        if (pl.perm[m + p + k] != k) return no("permutation is not leaves-first");
    if (band_lds_bytes(pl) > 160L * 1024) return no("per-QP state exceeds the LDS of a CU");
    if (why) why->clear();
    return true;
}

std::string generate_band_kernel(const Plan &pl, std::string *name_out) {
    const long nb = pl.band_nb, ns = pl.band_ns, mz = pl.band_mz, my = pl.band_my;
    const BandLayout L = band_layout(pl);
    std::ostringstream o;
    o << "#define QPB_ROW_COMMON_ONLY 1\n" << kRowTemplate << "\n#undef QPB_ROW_COMMON_ONLY\n";
    o << "// generated by qpb_wave for plan " << std::hex << pl.hash << std::dec << ": n=" << pl.n << " m=" << pl.m
      << " p=" << pl.p << " [band: " << ns << " stages of " << nb << "/" << mz << "/" << my << ", fast]\n";
    if (const char *e = getenv("QPB_WAVE_OPTS")) {
        std::istringstream in(e);
        std::string kv;
        while (in >> kv) {
            const size_t eq = kv.find('=');
            if (eq != std::string::npos) o << "#define " << kv.substr(0, eq) << " " << kv.substr(eq + 1) << "\n";
        }
    }
    o << "#define QPB_BNB " << nb << "\n#define QPB_BNS " << ns << "\n#define QPB_BMZ " << mz << "\n#define QPB_BMY " << my
      << "\n";
    const long nP = pl.Pin.nnz(), nA = pl.p ? pl.A.nnz() : 0, nG = pl.G.nnz();
    o << "#define QPB_NNZP " << nP << "\n#define QPB_NNZA " << nA << "\n#define QPB_NNZG " << nG << "\n";
    const char *names[] = {"PP", "LP", "GS", "O_P", "O_L", "O_RD", "O_Y", "O_G", "O_AR", "O_AL", "O_DUMP",
                           "O_STATIC_END", "V_X", "V_DX", "V_Y", "V_RY", "V_Z", "V_S", "V_RZ", "V_DZ", "LDS_QP"};
    const long vals[] = {L.PP, L.LP, L.GS, L.O_P, L.O_L, L.O_RD, L.O_Y, L.O_G, L.O_AR, L.O_AL, L.O_DUMP,
                         L.O_STATIC_END, L.V_X, L.V_DX, L.V_Y, L.V_RY, L.V_Z, L.V_S, L.V_RZ, L.V_DZ, L.LDS_QP};
    for (size_t i = 0; i < sizeof vals / sizeof vals[0]; i++) o << "#define " << names[i] << " " << vals[i] << "\n";
    // CSC value -> LDS slot of the stage blocks
    std::vector<long> pcol(nP), acol(nA), gcol(nG);
    for (long j = 0; j < pl.n; j++) {
        for (long k = pl.Pin.jc[j]; k < pl.Pin.jc[j + 1]; k++) pcol[k] = j;
        if (nA)
            for (long k = pl.A.jc[j]; k < pl.A.jc[j + 1]; k++) acol[k] = j;
        for (long k = pl.G.jc[j]; k < pl.G.jc[j + 1]; k++) gcol[k] = j;
    }
    // P_k packed upper: (i, j), i <= j, at j (j + 1) / 2 + i (both triangles of a full P
    // land on the same slot)
    auto pslot = [&](long i, long j) {
        const long a = std::min(i % nb, j % nb), b = std::max(i % nb, j % nb);
        return L.O_P + (j / nb) * L.PP + b * (b + 1) / 2 + a;
    };
    table(o, "static __device__ const int qpb_bsP", nP, [&](long k) { return pslot(pl.Pin.ir[k], pcol[k]); });
    // G_k on the union pattern; per-lane position tables (the zero slot GS - 1 where the
    // union has no entry): column c's rows (x lanes), row r's columns (z lanes)
    const std::vector<std::pair<long, long>> gu = band_gunion(pl);
    auto gpos = [&](long r, long j) {
        auto it = std::lower_bound(gu.begin(), gu.end(), std::make_pair(r, j));
        return (it != gu.end() && *it == std::make_pair(r, j)) ? (long)(it - gu.begin()) : L.GS - 1;
    };
    o << "static __device__ const unsigned short qpb_bgc[16][" << mz << "] = {";
    for (long cc = 0; cc < 16; cc++) {
        o << (cc ? "," : "") << "{";
        for (long r = 0; r < mz; r++) o << (r ? "," : "") << (cc < nb ? gpos(r, cc) : L.GS - 1);
        o << "}";
    }
    o << "};\nstatic __device__ const unsigned short qpb_bgr[64][" << nb << "] = {";
    for (long r = 0; r < 64; r++) {
        o << (r ? "," : "") << "{";
        for (long j = 0; j < nb; j++) o << (j ? "," : "") << (r < mz ? gpos(r, j) : L.GS - 1);
        o << "}";
    }
    o << "};\n";
    std::vector<unsigned> gm(mz, 0), arm(my > 0 ? my : 1, 0), alm(my > 0 ? my : 1, 0);
    table(o, "static __device__ const int qpb_bsG", nG, [&](long k) {
        const long r = pl.G.ir[k], j = gcol[k];
        gm[r % mz] |= 1u << (j % nb);
        return L.O_G + (r / mz) * L.GS + gpos(r % mz, j % nb);
    });
    table(o, "static __device__ const int qpb_bsA", nA, [&](long k) {
        const long l = pl.A.ir[k], j = acol[k], st = l / my;
        const bool right = j / nb == st;
        (right ? arm : alm)[l % my] |= 1u << (j % nb);
        return (right ? L.O_AR + st * my * nb : L.O_AL + (st - 1) * my * nb) + (l % my) * nb + (j % nb);
    });
    auto masks = [&](const char *nm, const std::vector<unsigned> &v) {
        unsigned u = 0;
        o << "static constexpr unsigned " << nm << "m[" << v.size() << "] = {";
        for (size_t i = 0; i < v.size(); i++) { o << (i ? "," : "") << v[i] << "u"; u |= v[i]; }
        o << "};\nstatic constexpr unsigned " << nm << "u = " << u << "u;\n";
    };
    masks("qpb_bG", gm);
    masks("qpb_bAR", arm);
    masks("qpb_bAL", alm);
    const std::string body = o.str() + kBandTemplate;
    const std::string name = named(body, "qpb_band", pl, 64);
    if (name_out) *name_out = name;
    return "#define QPB_KERNEL_NAME " + name + "\n" + body;
}

// ---- wide row form (qpb_rowx.hip): one 16-lane row per QP, up to 32 variables

// leading dimensions of the row's dense copies: 2 mod 4 doubles, so that the 16 lanes
// of a row reading a column (stride ld) hit distinct bank pairs
static long rowx_ld(long v) { return v + ((2 - v % 4) + 4) % 4; }

RowxLayout rowx_layout(const Plan &pl) {
    RowxLayout L;
    const long n = pl.n;
    L.LDG = rowx_ld(pl.m);
    L.LDA = rowx_ld(std::max(pl.p, 1L));
    L.LDP = rowx_ld(n);
    L.OFF_G = 0;
    L.OFF_A = L.OFF_G + n * L.LDG;
    L.OFF_P = L.OFF_A + (pl.p ? n * L.LDA : 0);
    L.STG_END = (L.OFF_P + n * L.LDP + 1) & ~1L;
    // H0 and -L by rows padded to the end of their x slot's column range (row e: 16 (e / 16)
    // + 16 entries, stride 17 / 33 so the 16 lanes' row stores spread over the banks), the
    // entries beyond the diagonal zero (-L: from the diagonal on): the factor starts from
    // rows whose upper part is zero, the backward solves read -L's columns without masks
    const long rows = n <= 16 ? 17 * n : 17 * 16 + 33 * (n - 16);
    L.OFF_H0 = L.STG_END;
    L.OFF_L = L.OFF_H0 + rows;
    L.O_DUMP = L.OFF_L + rows;
    // LDS_QP = 17 mod 32 doubles: the two QPs of a 32-lane half (rows 0 / 1, 2 / 3: the
    // bank-conflict groups of ds_read_b64) then sit 34 banks apart -- 2 mod 4 keeps their
    // column reads (lane strides LDG, LDA: multiples of 4 banks) on disjoint banks, 32 mod
    // 64 their row reads (consecutive lanes)
    L.LDS_QP = L.O_DUMP + 16;
    const char *e = getenv("QPB_WAVE_OPTS");
    if (e && strstr(e, "QPB_X_EVEN=1"))
        L.LDS_QP = (L.LDS_QP + 1) & ~1L;                 // (A/B: an even stride)
    else
        L.LDS_QP += ((17 - L.LDS_QP % 32) + 32) % 32;
    return L;
}

bool rowx_eligible(const Plan &pl, std::string *why) {
    auto no = [&](const char *m) { if (why) *why = m; return false; };
    if (pl.n > 32 || pl.p > 32 || pl.m > 128) return no("need n, p <= 32, m <= 128");
    if (!wave_eligible(pl, why)) return false;
    const WaveLayout L = wave_layout(pl);
    if ((long)L.dense.size() != pl.n) return no("a z or y row is not a leaf of the plan's ordering");
    for (long d = 0; d < pl.n; d++)
        if (L.dense[d] != d) return no("the x block is not in natural order (leaves-first ordering needed)");
    if (4 * rowx_layout(pl).LDS_QP * 8 > 160L * 1024) return no("four QPs' dense copies exceed the LDS of a CU");
    // (round 5 kept upper-triangle P with off-diagonals in rows < 16 off this kernel after
    // a memory-aperture violation at 17 / 20 / 6; the cause was a register-allocator copy
    // placed ahead of an EXEC restore, now repaired in every kernel -- DESIGN.md §3)
    if (why) why->clear();
    return true;
}

std::string generate_rowx_kernel(const Plan &pl, std::string *name_out) {
    const long n = pl.n, m = pl.m, p = pl.p;
    const RowxLayout L = rowx_layout(pl);
    std::ostringstream o;
    o << "#define QPB_ROW_COMMON_ONLY 1\n" << kRowTemplate << "\n#undef QPB_ROW_COMMON_ONLY\n";
    std::vector<long> gcol;
    common_header(o, pl, 64, "row-cooperative, two x rows per lane", &gcol, L.LDP, L.LDA, L.LDG);
    const char *names[] = {"LDG", "LDA", "LDP", "OFF_G", "OFF_A", "OFF_P", "STG_END", "OFF_H0", "OFF_L", "O_DUMP",
                           "LDS_QP"};
    const long vals[] = {L.LDG, L.LDA, L.LDP, L.OFF_G, L.OFF_A, L.OFF_P, L.STG_END, L.OFF_H0, L.OFF_L, L.O_DUMP,
                         L.LDS_QP};
    for (size_t i = 0; i < sizeof vals / sizeof vals[0]; i++) o << "#define " << names[i] << " " << vals[i] << "\n";
    auto bools = [&](const char *nm, long rows, long cols, const std::vector<std::vector<int>> &v) {
        o << "static constexpr bool " << nm << "[" << std::max(rows, 1L) << "][" << cols << "] = {";
        for (long r = 0; r < std::max(rows, 1L); r++) {
            o << (r ? "," : "") << "{";
            for (long j = 0; j < cols; j++) o << (j ? "," : "") << (r < rows ? v[r][j] : 0);
            o << "}";
        }
        o << "};\n";
    };
    std::vector<std::vector<int>> gnz(m, std::vector<int>(n, 0)), anz(std::max(p, 1L), std::vector<int>(n, 0)),
        pnz(n, std::vector<int>(n, 0)), lnz(n, std::vector<int>(n, 0));
    for (long k = 0; k < pl.G.nnz(); k++) gnz[pl.G.ir[k]][gcol[k]] = 1;
    for (long j = 0; j < n; j++) {
        if (p)
            for (long k = pl.A.jc[j]; k < pl.A.jc[j + 1]; k++) anz[pl.A.ir[k]][j] = 1;
        for (long k = pl.Pin.jc[j]; k < pl.Pin.jc[j + 1]; k++) pnz[pl.Pin.ir[k]][j] = pnz[j][pl.Pin.ir[k]] = 1;
    }
    // L(j, k), j > k, of the x block: the plan's symbolic factor (x rows in natural order
    // after the leaves, so KKT position p_x + j is x_j)
    for (long cpos = 0; cpos < pl.N; cpos++) {
        const long kx = pl.perm[cpos];
        if (kx >= n) continue;
        for (long q = pl.Lp[cpos]; q < pl.Lp[cpos + 1]; q++) {
            const long jx = pl.perm[pl.Li[q]];
            if (jx < n && jx > kx) lnz[jx][kx] = 1;
        }
    }
    bools("qpb_Gnz", m, n, gnz);
    bools("qpb_Anz", p, n, anz);
    bools("qpb_Pnz", n, n, pnz);
    bools("qpb_lnz", n, n, lnz);
    const std::string body = o.str() + kRowxTemplate;
    const std::string name = named(body, "qpb_rowx", pl, 64);
    if (name_out) *name_out = name;
    return "#define QPB_KERNEL_NAME " + name + "\n" + body;
}

}  // namespace qpb

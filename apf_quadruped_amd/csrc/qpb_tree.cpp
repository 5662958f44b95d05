// qpb_tree.cpp -- plan -> source of the tree kernel (qpb_tree.hip).
//
// The tree kernel solves one QP per workgroup for ANY plan (no leaf/dense-block
// structure assumed, e.g. the MPC-horizon QP of BASELINE configs[3], N = 380):
// every sparse operation of the IPM is a "gather program" -- a list of tasks,
// each task one output value accumulated over a list of terms, grouped into the
// levels of a dependency order.  Tasks of one level are independent; a level is
// split into steps of at most QPB_WG lanes with 2^g lanes per task (the terms of
// a task are dealt round-robin to its lanes and summed with a lane butterfly),
// and a workgroup barrier closes each level.  This file turns the plan's KKT,
// permutation and elimination tree into five such programs:
//
//   fac  left-looking LDL' of P K P' over the elimination-tree levels
//        (level = height above the leaves): task (i, j) of column j computes
//        K(i,j) - sum_k LD(i,k) LD(j,k) / D(k) over the k with L(j,k), L(i,k) != 0;
//        the factor is stored unscaled, LD = L D, next to 1/D (reference:
//        LDL_numeric, ldl.c:253-326, with its pivot regularisation ldl.c:273-274,
//        319-320; same factor, different summation order)
//   fwd  w = D^-1 L^-1 b, one task per row over the same levels (LDL_lsolve +
//        LDL_dsolve, ldl.c:495-532)
//   bwd  x = w - D^-1 LD' x, levels in reverse (LDL_ltsolve, ldl.c:539-557)
//   mv   the residual products [P A' G'; A; G] [x; y; z] (computeresiduals,
//        Auxilary.c:745-786), one task per KKT row
//   obj  P x for the objective (obj_value, Auxilary.c:1133-1141)
// plus the KKT assembly tables (Auxilary.c:71-181 and updatekktmatrix
// Auxilary.c:205-233, including its "last slot of the z column" rule).
#include "qpb_tree.hpp"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <numeric>
#include <sstream>

namespace qpb {

namespace {
const char *kTreeTemplate =
#include "qpb_tree_src.inc"
    ;

// descriptor fields: LDS byte offsets (element index * 8) from the region base,
// 16 bits each -- fac terms [a | b | k] in a u64, all other programs [a | j] in a u32
constexpr int FB = 16;
constexpr long FMAX = ((1L << FB) - 1) / 8;   // largest element index a field can address

uint64_t pk(uint64_t a, uint64_t b, uint64_t c = 0) { return (a * 8) | ((b * 8) << FB) | ((c * 8) << (2 * FB)); }

// rounds of a step, padded to the widths the kernel sums without branches
long round_bucket(long R) { return R <= 1 ? 1 : R <= 2 ? 2 : R <= 4 ? 4 : R <= 8 ? 8 : R; }

struct Task {
    int32_t out;
    std::vector<uint64_t> con;
};

constexpr int32_t STEP_BARRIER = 1 << 16, STEP_PANEL = 1 << 17;

struct Prog {
    // 4 ints per step: desc offset, task offset, ntask << 4 | log2 G, R | flags.  A panel
    // step (STEP_PANEL, no gather lanes) holds a panel-list index and a count instead.
    std::vector<int32_t> steps;
    std::vector<int32_t> hdr;     // one output code per task
    std::vector<uint64_t> desc;   // [R][ntask * G] per step
    std::vector<std::vector<int32_t>> panels;   // supernode ids of every panel step
    long nsteps() const { return (long)steps.size() / 4; }
    void panel_step(const std::vector<int32_t> &ids) {
        if (ids.empty()) return;
        steps.insert(steps.end(), {(int32_t)panels.size(), (int32_t)ids.size(), 0, 1 | STEP_BARRIER | STEP_PANEL});
        panels.push_back(ids);
    }
};

// A relaxed supernode: columns j0 .. j0+w-1 with parent(j) = j+1 and nested
// structure (colcount(j) = colcount(j+1) + 1).  Its panel has R = colcount(j0) + 1
// rows (the supernode's own w and the rows below), one per lane of a wavefront.
struct Snode {
    long j0, w, R;
};

// One level's tasks -> steps.  Tasks are sorted by term count; a level is cut into
// at most two groups (heavy prefix, light suffix), each with its own lanes-per-task
// exponent g, minimising a rough latency model: per step, one round per term a lane
// sums (kRound), log2 G butterfly stages and a fixed step cost.  (One g for a whole
// level pads every light task to the heaviest one's rounds: MPC's factor levels had
// 1 504 real terms in 5 106 slots.)  The steps of a level need no barrier between
// them; the level's last step carries it.
void pack_level(std::vector<Task> &tasks, int wg, uint64_t dummy, Prog &P) {
    if (tasks.empty()) return;
    // weight of one round (a term per lane: its descriptor load and LDS reads)
    // against the fixed cost of a step (30); measured on MPC: 3 -> 10 is -7 % per QP
    static const double kRound = [] {
        const char *e = getenv("QPB_TREE_RW");
        return e ? atof(e) : 10.0;
    }();
    static const bool kSplit = !getenv("QPB_TREE_NOSPLIT");
    std::stable_sort(tasks.begin(), tasks.end(),
                     [](const Task &a, const Task &b) { return a.con.size() > b.con.size(); });
    const size_t n = tasks.size();
    auto group_cost = [&](size_t b, size_t e, int g) {
        const long G = 1L << g, per = wg >> g;
        double cost = 0;
        for (size_t s = b; s < e; s += per) {
            const long R = round_bucket(((long)tasks[s].con.size() + G - 1) / G);
            // rounds past the 8 prefetched ones add a memory latency per 24 (qpb_run)
            cost += kRound * R + 3.0 * g + 30.0 + (R > 8 ? 12.0 * (double)((R - 8 + 23) / 24) : 0.0);
        }
        return cost;
    };
    auto best_g = [&](size_t b, size_t e, double *c) {
        int bg = 0;
        double bc = 1e300;
        for (int g = 0; (1 << g) <= std::min(64, wg); g++) {
            const double cost = group_cost(b, e, g);
            if (cost < bc - 1e-9) { bc = cost; bg = g; }
        }
        *c = bc;
        return bg;
    };
    double best;
    int g1 = best_g(0, n, &best), g2 = 0;
    size_t split = n;
    if (kSplit)
        for (size_t s = 1; s < n; s++) {
            if (tasks[s].con.size() == tasks[s - 1].con.size()) continue;   // cut where the count changes
            double c1, c2;
            const int a1 = best_g(0, s, &c1), a2 = best_g(s, n, &c2);
            if (c1 + c2 < best - 1e-9) { best = c1 + c2; g1 = a1; g2 = a2; split = s; }
        }
    auto emit = [&](size_t b, size_t e_end, int g, bool last_group) {
        const long G = 1L << g, per = wg >> g;
        for (size_t s = b; s < e_end; s += per) {
            const size_t e = std::min(e_end, s + (size_t)per);
            const long nt = (long)(e - s), act = nt * G;
            const long R = round_bucket(((long)tasks[s].con.size() + G - 1) / G);
            const long doff = (long)P.desc.size(), toff = (long)P.hdr.size();
            P.desc.resize(P.desc.size() + (size_t)(R * act), dummy);
            for (size_t t = s; t < e; t++) {
                P.hdr.push_back(tasks[t].out);
                const long lt = (long)(t - s);
                for (size_t ci = 0; ci < tasks[t].con.size(); ci++) {
                    const long r = (long)ci / G, sub = (long)ci % G;
                    P.desc[doff + r * act + lt * G + sub] = tasks[t].con[ci];
                }
            }
            const bool last = last_group && e == e_end;
            P.steps.insert(P.steps.end(), {(int32_t)doff, (int32_t)toff, (int32_t)((nt << 4) | g),
                                           (int32_t)(R | (last ? STEP_BARRIER : 0))});
        }
    };
    emit(0, split, g1, split == n);
    if (split < n) emit(split, n, g2, true);
}

// Plan-wide tables of the tree kernel, one device buffer: every program's
// descriptors (u64) first, then the int tables (permutation, assembly sources,
// program steps and output codes).  The source receives their offsets.
struct Blob {
    std::vector<uint64_t> d;     // fac descriptors
    std::vector<uint32_t> d32;   // fwd / bwd / mv / obj descriptors
    std::vector<int32_t> i;
    std::ostringstream macros;
    int wg = 64;
    void ints(const char *name, const std::vector<int32_t> &v) {
        while (i.size() % 4) i.push_back(0);       // 16-byte aligned: the kernel reads step records as int4
        macros << "#define QPB_I_" << name << " " << i.size() << "\n";
        i.insert(i.end(), v.begin(), v.end());
    }
    // lanes past a step's active count and rounds past its count read (and
    // ignore) entries beyond the program's end: wg entries of padding keep
    // those reads inside the buffer
    std::vector<int32_t> snrec;   // TI offset of every supernode record [j0, w, R, Lp[j0] .. Lp[j0+w-1]]
    std::vector<std::vector<int32_t>> list_off;   // per program: TI offset of each panel list
    // the panel lists of a program, right after the records: the kernel stages
    // TI[0, QPB_PANEL_INTS) -- records and lists -- in LDS once
    void lists(const Prog &P) {
        list_off.emplace_back();
        for (auto &ids : P.panels) {
            list_off.back().push_back((int32_t)i.size());
            for (int32_t id : ids) i.push_back(snrec[id]);
        }
    }
    int nprog = 0;
    void prog(const char *name, const Prog &P0, bool wide) {
        Prog P = P0;
        const std::vector<int32_t> &lo = list_off[nprog++];
        for (long st = 0; st < P.nsteps(); st++) {
            int32_t *m = &P.steps[4 * st];
            if (m[3] & STEP_PANEL) m[0] = lo[m[0]];
        }
        macros << "#define QPB_" << name << "_NSTEPS " << P.nsteps() << "\n";
        if (wide) {
            macros << "#define QPB_D_" << name << " " << d.size() << "\n";
            d.insert(d.end(), P.desc.begin(), P.desc.end());
            d.insert(d.end(), (size_t)wg, 0ull);
        } else {
            macros << "#define QPB_D_" << name << " " << d32.size() << "\n";
            for (uint64_t v : P.desc) d32.push_back((uint32_t)v);
            d32.insert(d32.end(), (size_t)wg, 0u);
        }
        ints((std::string(name) + "_steps").c_str(), P.steps);
        std::vector<int32_t> h = P.hdr;
        h.insert(h.end(), (size_t)wg, 0);
        ints((std::string(name) + "_hdr").c_str(), h);
    }
};

long lds_doubles(const Plan &pl) {
    const long n = pl.n, m = pl.m, p = pl.p, N = pl.N;
    const long npag = pl.Pin.nnz() + (p ? pl.A.nnz() : 0) + pl.G.nnz();
    // qpb_tree.hip LDS layout: LD+1, rD, V, S, R, W, RED (+ the supernode records and
    // panel lists, <= 3 N + 16 ints); P / A / G, c | b | h and the step tables stay in
    // global memory, the z-row work vectors in registers
    (void)npag; (void)n; (void)p;
    return (pl.lnz + 1) + 4 * N + m + 64 + (3 * N + 16) / 2 + (10 * N + 16) / 2;   // + step tables
}

// position of row i in column k of L (Li ascends within a column), -1 if absent
long lpos(const Plan &pl, long i, long k) {
    auto b = pl.Li.begin() + pl.Lp[k], e = pl.Li.begin() + pl.Lp[k + 1];
    auto it = std::lower_bound(b, e, i);
    return (it != e && *it == i) ? (long)(it - pl.Li.begin()) : -1;
}
}  // namespace

int tree_wg_for(const Plan &pl) {
    if (const char *e = getenv("QPB_TREE_WG")) {
        const int w = atoi(e);
        if (w == 64 || w == 128 || w == 192 || w == 256 || w == 512) return w;
    }
    return pl.N <= 64 ? 64 : pl.N <= 160 ? 128 : 256;
}

bool tree_eligible(const Plan &pl, std::string *why) {
    auto no = [&](const char *m) { if (why) *why = m; return false; };
    const long npag = pl.Pin.nnz() + (pl.p ? pl.A.nnz() : 0) + pl.G.nnz();
    if (pl.lnz + 1 > FMAX || pl.N > FMAX || npag + 1 > FMAX)
        return no("factor, KKT or value count beyond the 16-bit LDS offsets of the descriptors (8191)");
    if (lds_doubles(pl) * 8 > 160 * 1024) return no("per-QP state exceeds the 160 KiB LDS of a CU");
    if (why) why->clear();
    return true;
}

std::string generate_tree_kernel(const Plan &pl, int wg, std::string *name_out, TreeStats *stats,
                                 std::vector<char> *tables) {
    const long n = pl.n, m = pl.m, p = pl.p, N = pl.N, lnz = pl.lnz;
    const long nP = pl.Pin.nnz(), nA = p ? pl.A.nnz() : 0, nG = pl.G.nnz(), npag = nP + nA + nG;
    std::ostringstream o;
    o << "// generated by qpb_tree for plan " << std::hex << pl.hash << std::dec << ": n=" << n << " m=" << m
      << " p=" << p << " N=" << N << " Lnz=" << lnz << " [tree, fast]\n";
    o << "#define QPB_NX " << n << "\n#define QPB_NZ " << m << "\n#define QPB_NY " << p << "\n#define QPB_N " << N
      << "\n#define QPB_LNZ " << lnz << "\n#define QPB_NNZP " << nP << "\n#define QPB_NNZA " << nA
      << "\n#define QPB_NNZG " << nG << "\n#define QPB_WG " << wg << "\n";
    // four 192-thread workgroups per CU are three waves per SIMD: <= 168 registers
    // and 4 prefetched descriptor rounds, not 8: 58 -> 14 spilled registers, MPC 10 x
    // 1 024 QPs 1.72 -> 1.48 ms, HBM 183 -> 51 MB per launch (profiles/r03_tree_pf.log)
    if (wg == 192) o << "#define QPB_T_WPE 3\n#define QPB_T_PF 4\n";
    if (const char *e = getenv("QPB_TREE_OPTS")) {     // experiment knobs (#ifndef blocks of qpb_tree.hip)
        std::istringstream in(e);
        std::string kv;
        while (in >> kv) {
            const size_t eq = kv.find('=');
            if (eq != std::string::npos) o << "#define " << kv.substr(0, eq) << " " << kv.substr(eq + 1) << "\n";
        }
    }

    // supernodes and node levels.  A node is a supernode or a single column; its
    // level is its height above the leaves of the node tree (parent > child).
    std::vector<long> cc(N);
    for (long k = 0; k < N; k++) cc[k] = pl.Lp[k + 1] - pl.Lp[k];
    std::vector<Snode> sns;
    std::vector<long> sn_of(N, -1);
    const bool panels = !getenv("QPB_TREE_NOPANEL");
    // widest panel: 12 columns; wider supernodes split into 12-column panels.
    // Measured on 30/68/18 (one 36-wide supernode): 24 -> 1.38 ms per 1 024 QPs, 48 ->
    // 2.21 ms (VGPRs 209 vs 264); on MPC 12 (with QPB_T_XR 8) keeps the kernel at 72 KB
    // of code and 223 registers (24: 139 KB, 256 + AGPRs -> one wave per SIMD):
    // 1 024 QPs 1.77 ms (24 wide: 3.06 ms)
    long maxw = 12;
    if (const char *e = getenv("QPB_TREE_MAXW")) maxw = std::max(2L, std::min(48L, atol(e)));
    for (long j = 0; j < N;) {
        long e = j;
        if (panels && cc[j] + 1 <= 64)
            while (e + 1 < N && pl.parent[e] == e + 1 && cc[e] == cc[e + 1] + 1 && e + 2 - j <= maxw) e++;
        if (e > j) {
            for (long c = j; c <= e; c++) sn_of[c] = (long)sns.size();
            sns.push_back({j, e - j + 1, cc[j] + 1});
        }
        j = e + 1;
    }
    auto key = [&](long j) { return sn_of[j] >= 0 ? N + sn_of[j] : j; };
    std::vector<long> nlev(N + sns.size(), 0);
    for (long k = 0; k < N; k++) {
        const long par = pl.parent[k];
        if (par >= 0 && key(par) != key(k)) nlev[key(par)] = std::max(nlev[key(par)], nlev[key(k)] + 1);
    }
    std::vector<long> level(N);
    long H = 0;
    for (long j = 0; j < N; j++) { level[j] = nlev[key(j)]; H = std::max(H, level[j] + 1); }
    std::vector<std::vector<int32_t>> lvl_sn(H);
    for (size_t t = 0; t < sns.size(); t++) lvl_sn[level[sns[t].j0]].push_back((int32_t)t);
    auto j0_of = [&](long j) { return sn_of[j] >= 0 ? sns[sn_of[j]].j0 : j; };   // external terms: k < j0
    // row structures of L: rs[i] = (k, position of L(i,k)), k ascending
    std::vector<std::vector<std::pair<long, long>>> rs(N);
    for (long k = 0; k < N; k++)
        for (long e = pl.Lp[k]; e < pl.Lp[k + 1]; e++) rs[pl.Li[e]].push_back({k, e});

    // fac: single columns complete here (diagonal -> 1/D); supernode columns get
    // their external updates only (diagonal kept raw), then the level's panel step
    Prog fac, fwd, bwd, mv, obj;
    long fac_contrib = 0;
    {
        std::vector<std::vector<Task>> lv(H);
        for (long j = 0; j < N; j++) {
            const bool sn = sn_of[j] >= 0;
            const long lim = j0_of(j);
            Task d{(int32_t)(sn ? -1 - N - j : -1 - j), {}};
            for (auto &kp : rs[j])
                if (kp.first < lim) d.con.push_back(pk(kp.second, kp.second, kp.first));
            fac_contrib += (long)d.con.size();
            if (!sn || !d.con.empty()) lv[level[j]].push_back(std::move(d));
            for (long e = pl.Lp[j]; e < pl.Lp[j + 1]; e++) {
                const long i = pl.Li[e];
                Task t{(int32_t)e, {}};
                size_t a = 0, b = 0;
                const auto &ri = rs[i], &rj = rs[j];
                while (a < ri.size() && b < rj.size() && ri[a].first < lim && rj[b].first < lim) {
                    if (ri[a].first < rj[b].first) a++;
                    else if (ri[a].first > rj[b].first) b++;
                    else { t.con.push_back(pk(ri[a].second, rj[b].second, ri[a].first)); a++; b++; }
                }
                fac_contrib += (long)t.con.size();
                if (!t.con.empty()) lv[level[j]].push_back(std::move(t));   // else LD(i,j) = K(i,j) as assembled
            }
        }
        for (long h = 0; h < H; h++) {
            pack_level(lv[h], wg, pk(lnz, lnz, 0), fac);
            fac.panel_step(lvl_sn[h]);
        }
    }
    // fwd / bwd
    {
        std::vector<std::vector<Task>> lf(H), lb(H);
        for (long i = 0; i < N; i++) {
            const bool sn = sn_of[i] >= 0;
            const long lim = j0_of(i);
            Task t{(int32_t)(sn ? -1 - i : i), {}};          // supernode rows: raw external sum
            for (auto &kp : rs[i])
                if (kp.first < lim) t.con.push_back(pk(kp.second, kp.first));
            if (!sn || !t.con.empty()) lf[level[i]].push_back(std::move(t));
            const long rowlim = sn ? sns[sn_of[i]].j0 + sns[sn_of[i]].w : 0;   // bwd: rows below the supernode
            Task u{(int32_t)i, {}};
            for (long e = pl.Lp[i]; e < pl.Lp[i + 1]; e++)
                if (pl.Li[e] >= rowlim) u.con.push_back(pk(e, pl.Li[e]));
            if (!u.con.empty()) lb[level[i]].push_back(std::move(u));
        }
        for (long h = 0; h < H; h++) {
            pack_level(lf[h], wg, pk(lnz, 0), fwd);
            fwd.panel_step(lvl_sn[h]);
        }
        for (long h = H - 1; h >= 0; h--) {
            pack_level(lb[h], wg, pk(lnz, 0), bwd);
            bwd.panel_step(lvl_sn[h]);
        }
    }
    // mv / obj (natural KKT rows; K is symmetric in pattern and, before the z
    // diagonal update, in value: column r lists row r)
    auto pag = [&](const Slot &s) -> long {
        return s.kind == Src::P ? s.idx : s.kind == Src::A ? nP + s.idx : s.kind == Src::G ? nP + nA + s.idx : -1;
    };
    {
        std::vector<Task> lm, lo;
        for (long r = 0; r < N; r++) {
            Task t{(int32_t)r, {}}, u{(int32_t)r, {}};
            for (long s = pl.K.jc[r]; s < pl.K.jc[r + 1]; s++) {
                const Slot &sl = pl.K_init[s];
                const long v = pag(sl);
                if (v < 0) continue;
                t.con.push_back(pk(v, pl.K.ir[s]));
                if (sl.kind == Src::P) u.con.push_back(pk(v, pl.K.ir[s]));
            }
            lm.push_back(std::move(t));
            if (r < n) lo.push_back(std::move(u));
        }
        pack_level(lm, wg, pk(npag, 0), mv);
        pack_level(lo, wg, pk(npag, 0), obj);
    }
    // KKT assembly into the factor layout: column c = perm[a] of the KKT gives
    // entry (a, b = pinv[row]) of P K P' for b <= a only (ldl.c:287-288)
    std::vector<int32_t> asrc_i(lnz + N, -1), asrc_l(lnz + N, -1);
    auto code = [&](const Slot &s) -> int32_t {
        if (s.kind == Src::NegOne) return -2;
        if (s.kind == Src::ZDiag) return -3 - s.idx;
        return (int32_t)pag(s);
    };
    for (long c = 0; c < N; c++) {
        const long a = pl.pinv[c];
        for (long s = pl.K.jc[c]; s < pl.K.jc[c + 1]; s++) {
            const long b = pl.pinv[pl.K.ir[s]];
            if (b > a) continue;
            const long tgt = b == a ? lnz + a : lpos(pl, a, b);
            if (tgt < 0) continue;   // cannot happen: the symbolic factor holds every KKT entry
            asrc_i[tgt] = code(pl.K_init[s]);
            asrc_l[tgt] = code(pl.K_loop[s]);
        }
    }
    Blob bl;
    bl.wg = wg;
    {
        std::vector<long> widths;
        for (auto &sn : sns) {
            bl.snrec.push_back((int32_t)bl.i.size());
            bl.i.insert(bl.i.end(), {(int32_t)sn.j0, (int32_t)sn.w, (int32_t)sn.R});
            for (long c = 0; c < sn.w; c++) bl.i.push_back((int32_t)pl.Lp[sn.j0 + c]);
            if (std::find(widths.begin(), widths.end(), sn.w) == widths.end()) widths.push_back(sn.w);
        }
        std::sort(widths.begin(), widths.end());
        o << "#define QPB_NSNODE " << sns.size() << "\n#define QPB_PANEL_WIDTHS(X)";
        for (long w : widths) o << " X(" << w << ")";
        o << "\n";
    }
    for (const Prog *P : {&fac, &fwd, &bwd, &mv, &obj}) bl.lists(*P);
    o << "#define QPB_PANEL_INTS " << bl.i.size() << "\n";
    bl.prog("fac", fac, true);
    bl.prog("fwd", fwd, false);
    bl.prog("bwd", bwd, false);
    bl.prog("mv", mv, false);
    bl.prog("obj", obj, false);
    bl.ints("pinv", std::vector<int32_t>(pl.pinv.begin(), pl.pinv.end()));
    bl.ints("asrc_i", asrc_i);
    bl.ints("asrc_l", asrc_l);
    if (bl.d32.size() % 2) bl.d32.push_back(0u);   // keep the int tables 8-byte aligned
    o << bl.macros.str() << "#define QPB_NDESC " << bl.d.size() << "\n#define QPB_NDESC32 " << bl.d32.size() << "\n";
    // the tables' content is part of the kernel's identity (code-object cache key)
    {
        std::string raw((const char *)bl.d.data(), bl.d.size() * 8);
        raw.append((const char *)bl.d32.data(), bl.d32.size() * 4);
        raw.append((const char *)bl.i.data(), bl.i.size() * 4);
        char hx[40];
        snprintf(hx, sizeof hx, "%016llx", (unsigned long long)fnv1a(raw));
        o << "// tables " << hx << "\n";
    }
    if (tables) {
        const size_t n8 = bl.d.size() * 8, n4 = bl.d32.size() * 4, ni = bl.i.size() * 4;
        tables->assign(n8 + n4 + ni + 64, 0);
        std::memcpy(tables->data(), bl.d.data(), n8);
        std::memcpy(tables->data() + n8, bl.d32.data(), n4);
        std::memcpy(tables->data() + n8 + n4, bl.i.data(), ni);
    }
    if (stats) {
        stats->levels = H;
        stats->supernodes = (long)sns.size();
        stats->fac_steps = fac.nsteps(); stats->fwd_steps = fwd.nsteps();
        stats->bwd_steps = bwd.nsteps(); stats->mv_steps = mv.nsteps();
        stats->fac_contrib = fac_contrib;
        stats->desc_words = (long)(fac.desc.size() + fwd.desc.size() + bwd.desc.size() + mv.desc.size() + obj.desc.size());
        stats->lds_bytes = lds_doubles(pl) * 8;
    }
    const std::string body = o.str() + kTreeTemplate;
    const uint64_t h = fnv1a(body);
    char name[96];
    snprintf(name, sizeof name, "qpb_tree_%016llx_w%d_%08llx", (unsigned long long)pl.hash, wg,
             (unsigned long long)(h & 0xffffffffull));
    if (name_out) *name_out = name;
    return std::string("#define QPB_KERNEL_NAME ") + name + "\n" + body;
}

}  // namespace qpb

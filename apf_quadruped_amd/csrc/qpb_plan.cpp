// qpb_plan.cpp -- pattern-only analysis of a qpSWIFT QP (see qpb_plan.hpp).
#include "qpb_plan.hpp"

#include <algorithm>
#include <cstring>
#include <sstream>

namespace qpb {

uint64_t fnv1a(const std::string &s) {
    uint64_t h = 1469598103934665603ull;
    for (unsigned char ch : s) { h ^= ch; h *= 1099511628211ull; }
    return h;
}

static bool check_csc(long rows, long cols, const long *jc, const long *ir, std::string *err, const char *name) {
    if (cols > 0 && !jc) { if (err) *err = std::string(name) + ": null column pointer"; return false; }
    if (cols == 0) return true;
    if (jc[0] != 0) { if (err) *err = std::string(name) + ": jc[0] != 0"; return false; }
    for (long j = 0; j < cols; j++)
        if (jc[j + 1] < jc[j]) { if (err) *err = std::string(name) + ": jc not monotone"; return false; }
    if (jc[cols] > 0 && !ir) { if (err) *err = std::string(name) + ": null row index"; return false; }
    for (long k = 0; k < jc[cols]; k++)
        if (ir[k] < 0 || ir[k] >= rows) { if (err) *err = std::string(name) + ": row index out of range"; return false; }
    return true;
}

static Pattern make_pattern(long rows, long cols, const long *jc, const long *ir) {
    Pattern P;
    P.rows = rows; P.cols = cols;
    P.jc.assign(jc, jc + cols + 1);
    P.ir.assign(ir, ir + jc[cols]);
    return P;
}

// Counting-sort transpose with source indices (Auxilary.c:901-951 order).
static void transpose_src(const Pattern &a, Pattern &t, std::vector<long> &src) {
    t.rows = a.cols; t.cols = a.rows;
    t.jc.assign(a.rows + 1, 0);
    t.ir.assign(a.nnz(), 0);
    src.assign(a.nnz(), 0);
    std::vector<long> fill(a.rows, 0);
    for (long k = 0; k < a.nnz(); k++) fill[a.ir[k]]++;
    for (long r = 0; r < a.rows; r++) t.jc[r + 1] = t.jc[r] + fill[r];
    std::fill(fill.begin(), fill.end(), 0);
    for (long j = 0; j < a.cols; j++)
        for (long k = a.jc[j]; k < a.jc[j + 1]; k++) {
            long dst = t.jc[a.ir[k]] + fill[a.ir[k]]++;
            t.ir[dst] = j;
            src[dst] = k;
        }
}

std::vector<long> min_degree_order(const Pattern &sym) {
    const long N = sym.cols;
    const long W = (N + 63) / 64;
    std::vector<uint64_t> adj((size_t)N * W, 0), alive(W, 0);
    auto row = [&](long i) { return &adj[(size_t)i * W]; };
    for (long j = 0; j < N; j++)
        for (long k = sym.jc[j]; k < sym.jc[j + 1]; k++) {
            long i = sym.ir[k];
            if (i == j) continue;
            row(i)[j >> 6] |= 1ull << (j & 63);
            row(j)[i >> 6] |= 1ull << (i & 63);
        }
    for (long i = 0; i < N; i++) alive[i >> 6] |= 1ull << (i & 63);
    std::vector<long> order;
    order.reserve(N);
    std::vector<uint64_t> nb(W);
    for (long step = 0; step < N; step++) {
        long best = -1, bestdeg = 0;
        for (long i = 0; i < N; i++) {
            if (!(alive[i >> 6] >> (i & 63) & 1)) continue;
            long d = 0;
            const uint64_t *r = row(i);
            for (long w = 0; w < W; w++) d += __builtin_popcountll(r[w] & alive[w]);
            if (best < 0 || d < bestdeg) { best = i; bestdeg = d; }
        }
        order.push_back(best);
        alive[best >> 6] &= ~(1ull << (best & 63));
        const uint64_t *rb = row(best);
        for (long w = 0; w < W; w++) nb[w] = rb[w] & alive[w];
        for (long w = 0; w < W; w++) {
            uint64_t bits = nb[w];
            while (bits) {
                long a = w * 64 + __builtin_ctzll(bits);
                bits &= bits - 1;
                uint64_t *ra = row(a);
                for (long u = 0; u < W; u++) ra[u] |= nb[u];
                ra[a >> 6] &= ~(1ull << (a & 63));
            }
        }
    }
    return order;
}

void band_shape(Plan &pl) {
    pl.band_nb = pl.band_ns = pl.band_mz = pl.band_my = 0;
    const long n = pl.n, m = pl.m, p = pl.p;
    std::vector<long> gcnt(m, 0);
    for (long k = 0; k < pl.G.nnz(); k++) gcnt[pl.G.ir[k]]++;
    for (long r = 0; r < m; r++)
        if (!gcnt[r]) return;
    for (long nb = 1; nb <= 16; nb++) {
        if (n % nb) continue;
        const long ns = n / nb;
        if (ns < 2 || m % ns || p % ns) continue;
        const long mz = m / ns, my = p / ns;
        if (mz > 64 || my > 16) continue;
        bool ok = true;
        for (long j = 0; j < n && ok; j++) {
            const long sj = j / nb;
            for (long k = pl.Pf.jc[j]; k < pl.Pf.jc[j + 1] && ok; k++) ok = pl.Pf.ir[k] / nb == sj;
            for (long k = pl.G.jc[j]; k < pl.G.jc[j + 1] && ok; k++) ok = pl.G.ir[k] / mz == sj;
            if (p > 0)
                for (long k = pl.A.jc[j]; k < pl.A.jc[j + 1] && ok; k++) {
                    const long sl = pl.A.ir[k] / my;
                    ok = sl == sj || sl == sj + 1;
                }
        }
        if (!ok) continue;
        pl.band_nb = (int)nb; pl.band_ns = (int)ns; pl.band_mz = (int)mz; pl.band_my = (int)my;
        return;
    }
}

int build_plan(Plan &pl, long n, long m, long p, int pmode,
               const long *Pjc, const long *Pir,
               const long *Ajc, const long *Air,
               const long *Gjc, const long *Gir,
               const long *perm, std::string *err, int order) {
    if (n <= 0 || m <= 0 || p < 0) { if (err) *err = "need n > 0, m > 0, p >= 0"; return E_INVAL; }
    if (!check_csc(n, n, Pjc, Pir, err, "P") || !check_csc(m, n, Gjc, Gir, err, "G")) return E_INVAL;
    if (p > 0 && !check_csc(p, n, Ajc, Air, err, "A")) return E_INVAL;
    pl = Plan();
    pl.n = n; pl.m = m; pl.p = p; pl.N = n + m + p; pl.pmode = pmode;
    pl.Pin = make_pattern(n, n, Pjc, Pir);
    pl.G = make_pattern(m, n, Gjc, Gir);
    if (p > 0) pl.A = make_pattern(p, n, Ajc, Air);
    else { pl.A.rows = 0; pl.A.cols = n; pl.A.jc.assign(n + 1, 0); }

    // Full P pattern with value sources.
    if (pmode == P_FULL) {
        pl.Pf = pl.Pin;
        pl.Pf_src.resize(pl.Pf.nnz());
        for (long k = 0; k < pl.Pf.nnz(); k++) pl.Pf_src[k] = k;
    } else {
        // Upper storage: column c holds rows r <= c (ascending).  Column c of the
        // full matrix = upper column c, then rows r > c taken from upper column r.
        for (long c = 0; c < n; c++)
            for (long k = Pjc[c]; k < Pjc[c + 1]; k++) {
                if (Pir[k] > c) { if (err) *err = "P upper: entry below the diagonal"; return E_INVAL; }
                if (k > Pjc[c] && Pir[k] <= Pir[k - 1]) { if (err) *err = "P upper: rows must ascend"; return E_INVAL; }
            }
        std::vector<std::vector<std::pair<long, long>>> lower(n);   // col c -> (row r > c, src)
        for (long r = 0; r < n; r++)
            for (long k = Pjc[r]; k < Pjc[r + 1]; k++)
                if (Pir[k] < r) lower[Pir[k]].push_back({r, k});
        pl.Pf.rows = pl.Pf.cols = n;
        pl.Pf.jc.assign(n + 1, 0);
        for (long c = 0; c < n; c++) {
            for (long k = Pjc[c]; k < Pjc[c + 1]; k++) { pl.Pf.ir.push_back(Pir[k]); pl.Pf_src.push_back(k); }
            for (auto &e : lower[c]) { pl.Pf.ir.push_back(e.first); pl.Pf_src.push_back(e.second); }
            pl.Pf.jc[c + 1] = (long)pl.Pf.ir.size();
        }
    }
    if (p > 0) transpose_src(pl.A, pl.At, pl.At_src);
    band_shape(pl);
    transpose_src(pl.G, pl.Gt, pl.Gt_src);

    // KKT assembly with sources, Auxilary.c:71-181.
    const long N = pl.N;
    Pattern &K = pl.K;
    K.rows = K.cols = N;
    K.jc.assign(N + 1, 0);
    auto push = [&](long row, Src s, long idx) {
        K.ir.push_back(row);
        pl.K_init.push_back(Slot{(int32_t)row, s, (int32_t)idx});
    };
    for (long i = 0; i < n; i++) {
        for (long k = pl.Pf.jc[i]; k < pl.Pf.jc[i + 1]; k++) push(pl.Pf.ir[k], Src::P, pl.Pf_src[k]);
        if (p > 0)
            for (long k = pl.A.jc[i]; k < pl.A.jc[i + 1]; k++) push(n + pl.A.ir[k], Src::A, k);
        for (long k = pl.G.jc[i]; k < pl.G.jc[i + 1]; k++) push(n + p + pl.G.ir[k], Src::G, k);
        K.jc[i + 1] = (long)K.ir.size();
    }
    for (long i = 0; i < p; i++) {
        for (long k = pl.At.jc[i]; k < pl.At.jc[i + 1]; k++) push(pl.At.ir[k], Src::A, pl.At_src[k]);
        K.jc[n + i + 1] = (long)K.ir.size();
    }
    for (long i = 0; i < m; i++) {
        long b0 = pl.Gt.jc[i], b1 = pl.Gt.jc[i + 1];
        for (long k = b0; k < b1; k++) push(pl.Gt.ir[k], Src::G, pl.Gt_src[k]);
        if (b1 > b0) push(n + p + i, Src::NegOne, 0);
        K.jc[n + p + i + 1] = (long)K.ir.size();
    }
    // updatekktmatrix (Auxilary.c:211-215) writes -s/z into the LAST slot of every
    // z column -- for an empty column that is the previous column's last slot.
    pl.K_loop = pl.K_init;
    for (long i = 0; i < m; i++) {
        long slot = K.jc[n + p + i + 1] - 1;
        if (slot < 0) { if (err) *err = "KKT has no slot for the z diagonal"; return E_SHAPE; }
        pl.K_loop[slot].kind = Src::ZDiag;
        pl.K_loop[slot].idx = (int32_t)i;
    }

    // Ordering.
    if (perm) {
        std::vector<char> seen(N, 0);
        for (long i = 0; i < N; i++) {
            if (perm[i] < 0 || perm[i] >= N || seen[perm[i]]) { if (err) *err = "perm is not a permutation"; return E_INVAL; }
            seen[perm[i]] = 1;
        }
        pl.perm.assign(perm, perm + N);
        pl.ordering_kind = 0;
    } else {
        // own ordering: leaves first wherever the x block fits the wave kernel's
        // dense block (one row per lane): the row kernel for the contact-force
        // shapes, a 30-row dense block instead of AMD's 45-51 for the controller
        // shapes; minimum degree beyond (MPC horizon: the tree kernel)
        // own ordering: leaves first wherever the x block fits the wave kernel's
        // dense block, and for multi-stage patterns (the band kernel eliminates the
        // z / y leaves, then the block-tridiagonal x block stage by stage)
        if (order == ORDER_OWN)
            order = ((n <= 64 && p <= 64 && m <= 256) || pl.band_nb > 0) ? ORDER_LEAVES : ORDER_MINDEG;
        if (order == ORDER_LEAVES) {
            // z rows, y rows, then x in natural order.  Every z / y row is then a
            // leaf (its neighbours are x rows, all later) and the x block is dense --
            // the elimination of the row kernel (qpb_row.hip); on C1 the fill equals
            // AMD's (Lnz 138).
            for (long i = n + p; i < N; i++) pl.perm.push_back(i);
            for (long i = n; i < n + p; i++) pl.perm.push_back(i);
            for (long i = 0; i < n; i++) pl.perm.push_back(i);
        } else if (order == ORDER_MINDEG) {
            pl.perm = min_degree_order(K);
        } else if (order == ORDER_AMD) {
            // qpSWIFT.c:424-440: AMD with default controls; identity if it fails
            pl.perm.assign(N, 0);
            if (amd_order(N, K.jc.data(), K.ir.data(), pl.perm.data()) < 0)
                for (long i = 0; i < N; i++) pl.perm[i] = i;
        } else {
            if (err) *err = "unknown ordering";
            return E_INVAL;
        }
        pl.ordering_kind = order;
    }
    pl.pinv.assign(N, 0);
    for (long k = 0; k < N; k++) pl.pinv[pl.perm[k]] = k;

    // LDL_symbolic, ldl.c:187-240.
    std::vector<long> lnz(N, 0), flag(N, 0);
    pl.parent.assign(N, -1);
    for (long k = 0; k < N; k++) {
        long col = pl.perm[k];
        pl.parent[k] = -1; flag[k] = k; lnz[k] = 0;
        for (long t = K.jc[col]; t < K.jc[col + 1]; t++) {
            long i = pl.pinv[K.ir[t]];
            if (i >= k) continue;
            for (; flag[i] != k; i = pl.parent[i]) {
                if (pl.parent[i] == -1) pl.parent[i] = k;
                lnz[i]++;
                flag[i] = k;
            }
        }
    }
    pl.Lp.assign(N + 1, 0);
    for (long k = 0; k < N; k++) pl.Lp[k + 1] = pl.Lp[k] + lnz[k];
    pl.lnz = pl.Lp[N];

    // Symbolic execution of LDL_numeric (ldl.c:276-322): record every value
    // operation in order; the index logic is exactly the reference's.
    pl.Li.assign(pl.lnz, 0);
    std::vector<long> cnt(N, 0), pattern(N, 0);
    std::fill(flag.begin(), flag.end(), -1);
    pl.fac.clear();
    for (long k = 0; k < N; k++) {
        pl.fac.push_back({FacOp::RowBegin, (int32_t)k, 0, 0});
        long top = N;
        flag[k] = k;
        cnt[k] = 0;
        long col = pl.perm[k];
        for (long t = K.jc[col]; t < K.jc[col + 1]; t++) {
            long i = pl.pinv[K.ir[t]];
            if (i > k) continue;
            pl.fac.push_back({FacOp::Scatter, (int32_t)i, (int32_t)t, 0});
            long len = 0;
            for (; flag[i] != k; i = pl.parent[i]) { pattern[len++] = i; flag[i] = k; }
            while (len > 0) pattern[--top] = pattern[--len];
        }
        for (; top < N; top++) {
            long i = pattern[top];
            long end = pl.Lp[i] + cnt[i];
            for (long e = pl.Lp[i]; e < end; e++) {
                pl.fac.push_back({FacOp::Update, (int32_t)pl.Li[e], (int32_t)e, (int32_t)i});
                pl.fac_updates++;
            }
            pl.fac.push_back({FacOp::NewL, (int32_t)i, (int32_t)end, 0});
            pl.fac_divs++;
            pl.Li[end] = k;
            cnt[i]++;
        }
        pl.fac.push_back({FacOp::RowEnd, (int32_t)k, 0, 0});
    }

    std::ostringstream key;
    key << "qpb1|" << n << ',' << m << ',' << p << ',' << pmode << "|P";
    for (long v : pl.Pin.jc) key << ',' << v;
    key << ';';
    for (long v : pl.Pin.ir) key << ',' << v;
    key << "|A";
    for (long v : pl.A.jc) key << ',' << v;
    key << ';';
    for (long v : pl.A.ir) key << ',' << v;
    key << "|G";
    for (long v : pl.G.jc) key << ',' << v;
    key << ';';
    for (long v : pl.G.ir) key << ',' << v;
    key << "|perm";
    for (long v : pl.perm) key << ',' << v;
    pl.key = key.str();
    pl.hash = fnv1a(pl.key);
    return E_OK;
}

}  // namespace qpb

// qpb_amd.cpp -- approximate-minimum-degree ordering of the KKT pattern.
//
// qpSWIFT orders its KKT matrix with SuiteSparse AMD (amd_l_order, called at
// src/qpSWIFT/qpSWIFT.c:424-440 with amd_l_defaults: dense = 10, aggressive
// absorption on, include/qpSWIFT/amd.h:339-348) whenever the caller passes
// Permut = NULL -- which every dogbot_controller call site does
// (src/client/main.cpp:1649, 2005, 2408, 2695, 3232).  The ordering decides which
// pivots the dynamic regularisation of LDL_numeric touches (ldl.c:273-274,
// 319-320), so reproducing the reference's solutions to 1e-6 at the controller's
// tolerance 1e-2 needs the reference's permutation, bit for bit.
//
// This file restates the published algorithm (Amestoy, Davis & Duff, "An
// approximate minimum degree ordering algorithm", SIAM J. Matrix Anal. Appl.
// 17(4), 1996, and "Algorithm 837: AMD", ACM TOMS 30(3), 2004) as a small state
// machine.  To land on the same permutation it keeps every choice the vendored
// code makes where the algorithm leaves freedom:
//   * the quotient graph lives in one integer workspace of length
//     1.2 |A+A'| + n with in-place compaction when it runs full (amd_order.c:
//     150-157, amd_2.c:870-938); list order after compaction is preserved;
//   * degree lists are LIFO (new entries at the head), the pivot is the head of
//     the lowest non-empty list (amd_2.c:719-735);
//   * approximate degrees with aggressive element absorption (amd_2.c:1034-1284);
//   * supervariables are found through hash buckets keyed by (sum of the list)
//     mod n that share the Head array with the degree lists (amd_2.c:1254-1437);
//   * rows of initial degree > max(16, 10 sqrt n) are "dense" and ordered last,
//     empty rows are eliminated first (amd_2.c:596-692);
//   * the assembly tree is post-ordered depth first with each node's largest
//     child last (amd_postorder.c:15-206, amd_post_tree.c:15-120), and absorbed
//     variables are placed just before their element (amd_2.c:1778-1841).
// Nothing here is on the device: it runs once per sparsity pattern, host side.
#include <cmath>
#include <climits>
#include <vector>

#include "qpb_plan.hpp"

namespace qpb {
namespace {

constexpr long NIL = -1;                      // "empty" marker
inline long tag(long i) { return -i - 2; }    // involution mapping ids >= 0 to <= -2

// Visit the off-diagonal pairs {i, j} of A + A' once each, in the order the
// reference builds A + A' (amd_aat.c:59-141 counts in this order, amd_1.c:86-165
// fills in it): column k's strictly-upper entries, each followed by the pending
// lower-only entries of that entry's column, then whatever lower entries remain.
template <class F>
void for_each_aat_pair(long n, const long *ap, const long *ai, std::vector<long> &cursor, F pair) {
    for (long k = 0; k < n; k++) {
        long p = ap[k];
        while (p < ap[k + 1]) {
            long j = ai[p];
            if (j > k) break;                    // first entry below the diagonal
            p++;
            if (j == k) break;                   // the diagonal is ignored
            pair(j, k);                          // A(j,k), j < k
            long q = cursor[j];
            while (q < ap[j + 1]) {              // column j's lower part up to row k
                long i = ai[q];
                if (i > k) break;
                q++;
                if (i == k) break;               // A(k,j) mirrors A(j,k): already paired
                pair(i, j);                      // A(i,j) has no upper mirror
            }
            cursor[j] = q;
        }
        cursor[k] = p;
    }
    for (long j = 0; j < n; j++)
        for (long q = cursor[j]; q < ap[j + 1]; q++) pair(ai[q], j);
}

class AmdState {
public:
    AmdState(long n, long nzaat)
        : n_(n), pe_(n), len_(n, 0), nv_(n), next_(n), last_(n), head_(n), elen_(n), deg_(n), w_(n),
          iw_(nzaat + nzaat / 5 + n) {}

    // Quotient graph = the pattern of A + A' (no diagonal), one list per row.
    void load(const long *ap, const long *ai) {
        std::vector<long> cursor(n_, 0), fill(n_);
        for_each_aat_pair(n_, ap, ai, cursor, [&](long a, long b) { len_[a]++; len_[b]++; });
        pfree_ = 0;
        for (long j = 0; j < n_; j++) { pe_[j] = fill[j] = pfree_; pfree_ += len_[j]; }
        std::fill(cursor.begin(), cursor.end(), 0);
        for_each_aat_pair(n_, ap, ai, cursor, [&](long a, long b) {
            iw_[fill[a]++] = b;
            iw_[fill[b]++] = a;
        });
    }

    void order(double dense_ratio, bool aggressive, long *perm) {
        init(dense_ratio);
        while (eliminated_ < n_) {
            long me = take_min_degree();
            eliminate(me, aggressive);
        }
        postorder_and_permute(perm);
    }

private:
    long n_;
    std::vector<long> pe_, len_, nv_, next_, last_, head_, elen_, deg_, w_, iw_;
    long pfree_ = 0, wflg_ = 0, mindeg_ = 0, eliminated_ = 0, lemax_ = 0, dense_ = 0;

    long wbig() const { return LONG_MAX - n_; }
    void reset_marks_if_needed() {               // amd_2.c:22-35
        if (wflg_ < 2 || wflg_ >= wbig()) {
            for (long x = 0; x < n_; x++)
                if (w_[x] != 0) w_[x] = 1;
            wflg_ = 2;
        }
    }

    void unlink_degree(long i) {
        long prev = last_[i], nxt = next_[i];
        if (nxt != NIL) last_[nxt] = prev;
        if (prev != NIL) next_[prev] = nxt;
        else head_[deg_[i]] = nxt;
    }
    void push_degree(long i, long d) {
        long first = head_[d];
        if (first != NIL) last_[first] = i;
        next_[i] = first;
        head_[d] = i;
    }

    void init(double dense_ratio) {
        long d = dense_ratio < 0 ? n_ - 2 : (long)(dense_ratio * std::sqrt((double)n_));
        dense_ = std::min(n_, std::max(16L, d));
        for (long i = 0; i < n_; i++) {
            last_[i] = head_[i] = next_[i] = NIL;
            nv_[i] = 1;
            w_[i] = 1;
            elen_[i] = 0;
            deg_[i] = len_[i];
        }
        wflg_ = 0;
        reset_marks_if_needed();
        for (long i = 0; i < n_; i++) {
            long di = deg_[i];
            if (di == 0) {                       // isolated row: an element at once
                elen_[i] = tag(1);
                eliminated_++;
                pe_[i] = NIL;
                w_[i] = 0;
            } else if (di > dense_) {            // dense row: ordered last, no parent
                nv_[i] = 0;
                elen_[i] = NIL;
                eliminated_++;
                pe_[i] = NIL;
            } else {
                push_degree(i, di);
            }
        }
    }

    long take_min_degree() {
        long d = mindeg_, me = NIL;
        for (; d < n_; d++)
            if ((me = head_[d]) != NIL) break;
        mindeg_ = d;
        long nxt = next_[me];
        if (nxt != NIL) last_[nxt] = NIL;
        head_[d] = nxt;
        return me;
    }

    // Compact iw_ while the new element is being built in its tail (amd_2.c:870-938):
    // every live object keeps its relative order; the partial element moves last.
    // `me_pos` / `e_pos` are the scan positions in me's list and in the object
    // being scanned, rewritten to their new places.
    void compact(long me, long e, long &me_pos, long me_consumed, long &e_pos, long e_left, long &pme1) {
        pe_[me] = me_pos;
        len_[me] -= me_consumed;
        if (len_[me] == 0) pe_[me] = NIL;
        pe_[e] = e_pos;
        len_[e] = e_left;
        if (len_[e] == 0) pe_[e] = NIL;
        for (long j = 0; j < n_; j++) {          // mark each object's first slot
            long pos = pe_[j];
            if (pos >= 0) { pe_[j] = iw_[pos]; iw_[pos] = tag(j); }
        }
        long src = 0, dst = 0;
        while (src <= pme1 - 1) {
            long j = tag(iw_[src++]);
            if (j < 0) continue;
            iw_[dst] = pe_[j];
            pe_[j] = dst++;
            for (long t = 0; t + 2 <= len_[j]; t++) iw_[dst++] = iw_[src++];
        }
        long moved = dst;
        for (src = pme1; src <= pfree_ - 1; src++) iw_[dst++] = iw_[src];
        pme1 = moved;
        pfree_ = dst;
        e_pos = pe_[e];
        me_pos = pe_[me];
    }

    void eliminate(long me, bool aggressive) {
        const long elenme = elen_[me];
        long nvpiv = nv_[me];
        eliminated_ += nvpiv;
        nv_[me] = -nvpiv;                        // negative nv = "in the new element"
        long degme = 0, pme1, pme2;

        // ---- new element Lme = the principal variables reachable from me ----
        if (elenme == 0) {                       // no adjacent elements: build in place
            pme1 = pe_[me];
            pme2 = pme1 - 1;
            for (long q = pme1; q <= pme1 + len_[me] - 1; q++) {
                long i = iw_[q];
                long nvi = nv_[i];
                if (nvi <= 0) continue;
                degme += nvi;
                nv_[i] = -nvi;
                iw_[++pme2] = i;
                unlink_degree(i);
            }
        } else {                                 // union of elements + variables, at pfree
            long pos = pe_[me];
            pme1 = pfree_;
            const long own_vars = len_[me] - elenme;
            for (long round = 1; round <= elenme + 1; round++) {
                long e, scan, count;
                if (round > elenme) { e = me; scan = pos; count = own_vars; }
                else { e = iw_[pos++]; scan = pe_[e]; count = len_[e]; }
                for (long t = 1; t <= count; t++) {
                    long i = iw_[scan++];
                    long nvi = nv_[i];
                    if (nvi <= 0) continue;
                    if (pfree_ >= (long)iw_.size())
                        compact(me, e, pos, round, scan, count - t, pme1);
                    degme += nvi;
                    nv_[i] = -nvi;
                    iw_[pfree_++] = i;
                    unlink_degree(i);
                }
                if (e != me) { pe_[e] = tag(me); w_[e] = 0; }   // e absorbed into me
            }
            pme2 = pfree_ - 1;
        }
        deg_[me] = degme;
        pe_[me] = pme1;
        len_[me] = pme2 - pme1 + 1;
        elen_[me] = tag(nvpiv + degme);
        reset_marks_if_needed();

        // ---- scan 1: w(e) - wflg = |Le \ Lme| for every element e next to Lme ----
        for (long q = pme1; q <= pme2; q++) {
            long i = iw_[q];
            long eln = elen_[i];
            if (eln <= 0) continue;
            long nvi = -nv_[i];
            long base = wflg_ - nvi;
            for (long r = pe_[i]; r <= pe_[i] + eln - 1; r++) {
                long e = iw_[r];
                long we = w_[e];
                if (we >= wflg_) we -= nvi;
                else if (we != 0) we = deg_[e] + base;
                w_[e] = we;
            }
        }

        // ---- scan 2: approximate degrees, absorption, mass elimination, hashing ----
        for (long q = pme1; q <= pme2; q++) {
            long i = iw_[q];
            long p1 = pe_[i], p2 = p1 + elen_[i] - 1, out = p1;
            unsigned long hash = 0;
            long d = 0;
            for (long r = p1; r <= p2; r++) {
                long e = iw_[r];
                long we = w_[e];
                if (we == 0) continue;           // already absorbed
                long ext = we - wflg_;
                if (!aggressive || ext > 0) {
                    d += ext;
                    iw_[out++] = e;
                    hash += (unsigned long)e;
                } else {                         // Le inside Lme: absorb e (aggressive)
                    pe_[e] = tag(me);
                    w_[e] = 0;
                }
            }
            elen_[i] = out - p1 + 1;             // + me, inserted below
            long vars_begin = out, end = p1 + len_[i];
            for (long r = p2 + 1; r < end; r++) {
                long j = iw_[r];
                long nvj = nv_[j];
                if (nvj <= 0) continue;
                d += nvj;
                iw_[out++] = j;
                hash += (unsigned long)j;
            }
            if (elen_[i] == 1 && vars_begin == out) {   // only me left: mass elimination
                pe_[i] = tag(me);
                long nvi = -nv_[i];
                degme -= nvi;
                nvpiv += nvi;
                eliminated_ += nvi;
                nv_[i] = 0;
                elen_[i] = NIL;
                continue;
            }
            deg_[i] = std::min(deg_[i], d);
            iw_[out] = iw_[vars_begin];          // first variable -> end
            iw_[vars_begin] = iw_[p1];           // first element -> end of elements
            iw_[p1] = me;                        // me first
            len_[i] = out - p1 + 1;
            long bucket = (long)(hash % (unsigned long)n_);
            long h = head_[bucket];              // buckets share Head with degree lists
            if (h <= NIL) { next_[i] = tag(h); head_[bucket] = tag(i); }
            else { next_[i] = last_[h]; last_[h] = i; }
            last_[i] = bucket;
        }
        deg_[me] = degme;
        lemax_ = std::max(lemax_, degme);
        wflg_ += lemax_;
        reset_marks_if_needed();

        // ---- supervariable detection within each touched hash bucket ----
        for (long q = pme1; q <= pme2; q++) {
            long i = iw_[q];
            if (nv_[i] >= 0) continue;
            long bucket = last_[i];
            long h = head_[bucket], cur;
            if (h == NIL) cur = NIL;
            else if (h < NIL) { cur = tag(h); head_[bucket] = NIL; }
            else { cur = last_[h]; last_[h] = NIL; }
            while (cur != NIL && next_[cur] != NIL) {
                long ln = len_[cur], eln = elen_[cur];
                for (long r = pe_[cur] + 1; r <= pe_[cur] + ln - 1; r++) w_[iw_[r]] = wflg_;
                long prev = cur, j = next_[cur];
                while (j != NIL) {
                    bool same = len_[j] == ln && elen_[j] == eln;
                    for (long r = pe_[j] + 1; same && r <= pe_[j] + ln - 1; r++)
                        if (w_[iw_[r]] != wflg_) same = false;
                    if (same) {                  // j indistinguishable from cur: merge
                        pe_[j] = tag(cur);
                        nv_[cur] += nv_[j];
                        nv_[j] = 0;
                        elen_[j] = NIL;
                        j = next_[j];
                        next_[prev] = j;
                    } else {
                        prev = j;
                        j = next_[j];
                    }
                }
                wflg_++;
                cur = next_[cur];
            }
        }

        // ---- back into the degree lists; drop non-principal variables from Lme ----
        long kept = pme1;
        const long nleft = n_ - eliminated_;
        for (long q = pme1; q <= pme2; q++) {
            long i = iw_[q];
            long nvi = -nv_[i];
            if (nvi <= 0) continue;
            nv_[i] = nvi;
            long d = std::min(deg_[i] + degme - nvi, nleft - nvi);
            push_degree(i, d);
            last_[i] = NIL;
            mindeg_ = std::min(mindeg_, d);
            deg_[i] = d;
            iw_[kept++] = i;
        }
        nv_[me] = nvpiv;
        len_[me] = kept - pme1;
        if (len_[me] == 0) { pe_[me] = NIL; w_[me] = 0; }   // a root of the assembly tree
        if (elenme != 0) pfree_ = kept;
    }

    void postorder_and_permute(long *perm) {
        for (long i = 0; i < n_; i++) { pe_[i] = tag(pe_[i]); elen_[i] = tag(elen_[i]); }
        // every absorbed variable points straight at the element that absorbed it
        for (long i = 0; i < n_; i++) {
            if (nv_[i] != 0 || pe_[i] == NIL) continue;
            long e = pe_[i];
            while (nv_[e] == 0) e = pe_[e];
            for (long j = i; nv_[j] == 0;) { long up = pe_[j]; pe_[j] = e; j = up; }
        }
        // children lists of the elements, ascending id, largest front moved last
        std::vector<long> child(n_, NIL), sibling(n_, NIL), rank(n_, NIL), stack(n_);
        for (long j = n_ - 1; j >= 0; j--)
            if (nv_[j] > 0 && pe_[j] != NIL) { sibling[j] = child[pe_[j]]; child[pe_[j]] = j; }
        for (long i = 0; i < n_; i++) {
            if (nv_[i] <= 0 || child[i] == NIL) continue;
            long prev = NIL, big = NIL, bigprev = NIL, bigsize = NIL;
            for (long f = child[i]; f != NIL; f = sibling[f]) {
                if (elen_[f] >= bigsize) { bigsize = elen_[f]; bigprev = prev; big = f; }
                prev = f;
            }
            long after = sibling[big];
            if (after == NIL) continue;
            if (bigprev == NIL) child[i] = after;
            else sibling[bigprev] = after;
            sibling[big] = NIL;
            sibling[prev] = big;
        }
        long k = 0;
        for (long root = 0; root < n_; root++) {
            if (pe_[root] != NIL || nv_[root] <= 0) continue;
            long top = 0;
            stack[0] = root;
            while (top >= 0) {                   // explicit-stack DFS, children in list order
                long i = stack[top];
                if (child[i] != NIL) {
                    long cnt = 0;
                    for (long f = child[i]; f != NIL; f = sibling[f]) cnt++;
                    top += cnt;
                    long h = top;
                    for (long f = child[i]; f != NIL; f = sibling[f]) stack[h--] = f;
                    child[i] = NIL;
                } else {
                    top--;
                    rank[i] = k++;
                }
            }
        }
        // element ranks -> first pivot position of each element
        std::vector<long> by_rank(n_, NIL), pos(n_, NIL);
        for (long e = 0; e < n_; e++)
            if (rank[e] != NIL) by_rank[rank[e]] = e;
        long next_pos = 0;
        for (long r = 0; r < n_; r++) {
            long e = by_rank[r];
            if (e == NIL) break;
            pos[e] = next_pos;
            next_pos += nv_[e];
        }
        for (long i = 0; i < n_; i++) {          // absorbed variables just before their element
            if (nv_[i] != 0) continue;
            long e = pe_[i];
            if (e != NIL) pos[i] = pos[e]++;
            else pos[i] = next_pos++;            // dense rows go last
        }
        for (long i = 0; i < n_; i++) perm[pos[i]] = i;
    }
};

}  // namespace

int amd_order(long n, const long *ap, const long *ai, long *perm, double dense_ratio, bool aggressive) {
    // input validation and the sorted / jumbled split (amd_valid.c:38-92, amd_order.c:52-135)
    if (!ap || !ai || !perm || n < 0) return AMD_STATUS_INVALID;
    if (n == 0) return AMD_STATUS_OK;
    if (ap[0] != 0 || ap[n] < 0) return AMD_STATUS_INVALID;
    int status = AMD_STATUS_OK;
    for (long j = 0; j < n; j++) {
        if (ap[j] > ap[j + 1]) return AMD_STATUS_INVALID;
        long prev = NIL;
        for (long q = ap[j]; q < ap[j + 1]; q++) {
            if (ai[q] < 0 || ai[q] >= n) return AMD_STATUS_INVALID;
            if (ai[q] <= prev) status = AMD_STATUS_JUMBLED;
            prev = ai[q];
        }
    }
    std::vector<long> rp, ri;
    if (status == AMD_STATUS_JUMBLED) {
        // order the transposed pattern with rows sorted and duplicates dropped
        // (amd_preprocess.c:56-109): A + A' is unchanged, the build order follows R
        std::vector<long> cnt(n, 0), seen(n, NIL);
        for (long j = 0; j < n; j++)
            for (long q = ap[j]; q < ap[j + 1]; q++)
                if (seen[ai[q]] != j) { cnt[ai[q]]++; seen[ai[q]] = j; }
        rp.assign(n + 1, 0);
        for (long i = 0; i < n; i++) rp[i + 1] = rp[i] + cnt[i];
        ri.assign(std::max(rp[n], 1L), 0);
        std::vector<long> fill(rp.begin(), rp.end() - 1);
        std::fill(seen.begin(), seen.end(), NIL);
        for (long j = 0; j < n; j++)
            for (long q = ap[j]; q < ap[j + 1]; q++)
                if (seen[ai[q]] != j) { ri[fill[ai[q]]++] = j; seen[ai[q]] = j; }
        ap = rp.data();
        ai = ri.data();
    }
    long nzaat = 0;
    {
        std::vector<long> cursor(n, 0);
        for_each_aat_pair(n, ap, ai, cursor, [&](long, long) { nzaat += 2; });
    }
    AmdState st(n, nzaat);
    st.load(ap, ai);
    st.order(dense_ratio, aggressive, perm);
    return status;
}

}  // namespace qpb

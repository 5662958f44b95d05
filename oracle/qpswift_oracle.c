/*
 * qpswift_oracle.c -- TEST INFRASTRUCTURE ONLY: the CPU checker for the HIP path.
 *
 * From-scratch restatement of the reference qpSWIFT primal-dual interior-point
 * solve as called by dogbot_controller (QP_SETUP_dense -> QP_SOLVE).  Every
 * floating-point operation is issued in the same order and association as the
 * reference so that results are bit-identical (tests/test_oracle.py pins this
 * against golden vectors made by the reference build in oracle/_ref).
 * Build with -ffp-contract=off (oracle/Makefile) so no FMA is formed.
 *
 * Reference anchors (paths under dogbot_controller/):
 *   dense -> CSC           src/qpSWIFT/Auxilary.c:1154-1206, 1219-1273
 *   transpose              src/qpSWIFT/Auxilary.c:901-951
 *   KKT assembly           src/qpSWIFT/Auxilary.c:71-181
 *   LDL symbolic/numeric   src/qpSWIFT/ldl.c:187-240, 253-326
 *   LDL solves             src/qpSWIFT/ldl.c:495-597
 *   initial point          src/qpSWIFT/Auxilary.c:992-1089
 *   residuals / SpMV       src/qpSWIFT/Auxilary.c:745-860
 *   IPM loop               src/qpSWIFT/qpSWIFT.c:473-644
 * The AMD ordering (amd_*.c) is not restated: the permutation is an input.
 */
#include "qpswift_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    long rows, cols, nnz;
    long *jc, *ir;
    double *v;
} csc_t;

static void *xcalloc(size_t n, size_t sz) { return calloc(n ? n : 1, sz); }

static void csc_free(csc_t *a) {
    free(a->jc); free(a->ir); free(a->v);
    memset(a, 0, sizeof(*a));
}

/* Auxilary.c:1154 / :1219 -- exact zeros are dropped, so the pattern is
 * value-dependent; rows ascend inside every column for both input orders. */
static void dense_to_csc(long rows, long cols, const double *d, int row_major, csc_t *out) {
    long cnt = 0, i, j;
    out->rows = rows; out->cols = cols;
    out->jc = xcalloc((size_t)cols + 1, sizeof(long));
    for (j = 0; j < cols; j++) {
        for (i = 0; i < rows; i++) {
            double e = row_major ? d[i * cols + j] : d[j * rows + i];
            if (e != 0.0) cnt++;
        }
        out->jc[j + 1] = cnt;
    }
    out->nnz = cnt;
    out->ir = xcalloc((size_t)cnt, sizeof(long));
    out->v = xcalloc((size_t)cnt, sizeof(double));
    cnt = 0;
    for (j = 0; j < cols; j++)
        for (i = 0; i < rows; i++) {
            double e = row_major ? d[i * cols + j] : d[j * rows + i];
            if (e != 0.0) { out->ir[cnt] = i; out->v[cnt] = e; cnt++; }
        }
}

static void csc_copy(long rows, long cols, const long *jc, const long *ir, const double *v, csc_t *out) {
    long nnz = jc[cols];
    out->rows = rows; out->cols = cols; out->nnz = nnz;
    out->jc = xcalloc((size_t)cols + 1, sizeof(long));
    out->ir = xcalloc((size_t)nnz, sizeof(long));
    out->v = xcalloc((size_t)nnz, sizeof(double));
    memcpy(out->jc, jc, sizeof(long) * (size_t)(cols + 1));
    memcpy(out->ir, ir, sizeof(long) * (size_t)nnz);
    memcpy(out->v, v, sizeof(double) * (size_t)nnz);
}

/* Auxilary.c:901-951: counting-sort transpose. */
static void csc_transpose(const csc_t *a, csc_t *t) {
    long r, k, j;
    long *fill = xcalloc((size_t)a->rows, sizeof(long));
    t->rows = a->cols; t->cols = a->rows; t->nnz = a->nnz;
    t->jc = xcalloc((size_t)a->rows + 1, sizeof(long));
    t->ir = xcalloc((size_t)a->nnz, sizeof(long));
    t->v = xcalloc((size_t)a->nnz, sizeof(double));
    for (k = 0; k < a->nnz; k++) fill[a->ir[k]]++;
    for (r = 0; r < a->rows; r++) t->jc[r + 1] = t->jc[r] + fill[r];
    memset(fill, 0, sizeof(long) * (size_t)a->rows);
    for (j = 0; j < a->cols; j++)
        for (k = a->jc[j]; k < a->jc[j + 1]; k++) {
            long dst = t->jc[a->ir[k]] + fill[a->ir[k]]++;
            t->ir[dst] = j;
            t->v[dst] = a->v[k];
        }
    free(fill);
}

/* Solver context: one QP. */
typedef struct {
    long n, m, p, N;
    csc_t P, A, G, At, Gt, K;     /* K = full symmetric KKT (Auxilary.c:71) */
    const double *c, *h, *b;
    double sigma_d, sigma;
    /* LDL workspace (ldl.c) */
    long *perm, *pinv, *parent, *lnz, *flag, *pattern, *Lp, *Li;
    double *Lx, *D, *Y;
    long nreg;
    /* iterates & temporaries (Auxilary.h:106-151) */
    double *x, *y, *z, *s, *rx, *ry, *rz, *dx, *dy, *dz, *dsl, *ds, *lam, *tmp, *rhs, *sol;
    double n_rx, n_ry, n_rz, n_mu, mu, rho, alpha_p, alpha_d, fval;
} ctx_t;

/* Auxilary.c:71-181: [P A' G'; A 0 0; G 0 -I]; the -1 is appended only when the
 * G' column is non-empty (Auxilary.c:126-131). */
static void build_kkt(ctx_t *q) {
    long n = q->n, p = q->p, m = q->m, i, k, nz = 0;
    csc_t *K = &q->K;
    long cap = q->P.nnz + 2 * q->G.nnz + m + (p ? 2 * q->A.nnz : 0);
    K->rows = K->cols = q->N;
    K->jc = xcalloc((size_t)q->N + 1, sizeof(long));
    K->ir = xcalloc((size_t)cap, sizeof(long));
    K->v = xcalloc((size_t)cap, sizeof(double));
    for (i = 0; i < n; i++) {
        for (k = q->P.jc[i]; k < q->P.jc[i + 1]; k++) { K->ir[nz] = q->P.ir[k]; K->v[nz++] = q->P.v[k]; }
        if (p)
            for (k = q->A.jc[i]; k < q->A.jc[i + 1]; k++) { K->ir[nz] = n + q->A.ir[k]; K->v[nz++] = q->A.v[k]; }
        for (k = q->G.jc[i]; k < q->G.jc[i + 1]; k++) { K->ir[nz] = n + p + q->G.ir[k]; K->v[nz++] = q->G.v[k]; }
        K->jc[i + 1] = nz;
    }
    for (i = 0; i < p; i++) {
        for (k = q->At.jc[i]; k < q->At.jc[i + 1]; k++) { K->ir[nz] = q->At.ir[k]; K->v[nz++] = q->At.v[k]; }
        K->jc[n + i + 1] = nz;
    }
    for (i = 0; i < m; i++) {
        long b0 = q->Gt.jc[i], b1 = q->Gt.jc[i + 1];
        for (k = b0; k < b1; k++) { K->ir[nz] = q->Gt.ir[k]; K->v[nz++] = q->Gt.v[k]; }
        if (b1 > b0) { K->ir[nz] = n + p + i; K->v[nz++] = -1.0; }
        K->jc[n + p + i + 1] = nz;
    }
    K->nnz = nz;
}

/* ldl.c:187-240: elimination tree and column counts of L for P K P'. */
static void ldl_symbolic(ctx_t *q) {
    long N = q->N, k, t;
    for (k = 0; k < N; k++) q->pinv[q->perm[k]] = k;
    for (k = 0; k < N; k++) {
        long col = q->perm[k];
        q->parent[k] = -1; q->flag[k] = k; q->lnz[k] = 0;
        for (t = q->K.jc[col]; t < q->K.jc[col + 1]; t++) {
            long i = q->pinv[q->K.ir[t]];
            if (i >= k) continue;
            while (q->flag[i] != k) {
                if (q->parent[i] == -1) q->parent[i] = k;
                q->lnz[i]++;
                q->flag[i] = k;
                i = q->parent[i];
            }
        }
    }
    q->Lp[0] = 0;
    for (k = 0; k < N; k++) q->Lp[k + 1] = q->Lp[k] + q->lnz[k];
}

/* ldl.c:253-326: up-looking row-by-row LDL' with the dynamic regularisation
 * D <- sign(D)*1e-7 when sign(D)*D <= 1e-14 (ldl.c:273-274, 319-320). */
static void ldl_numeric(ctx_t *q) {
    const double reg_delta = 1e-7, reg_eps = 1e-14;
    long N = q->N, k, t;
    double *Y = q->Y, *D = q->D;
    q->nreg = 0;
    for (k = 0; k < N; k++) {
        long col = q->perm[k], top = N;
        Y[k] = 0.0;
        q->flag[k] = k;
        q->lnz[k] = 0;
        for (t = q->K.jc[col]; t < q->K.jc[col + 1]; t++) {
            long i = q->pinv[q->K.ir[t]], len = 0;
            if (i > k) continue;
            Y[i] += q->K.v[t];
            while (q->flag[i] != k) {      /* walk the etree, collect pattern */
                q->pattern[len++] = i;
                q->flag[i] = k;
                i = q->parent[i];
            }
            while (len > 0) q->pattern[--top] = q->pattern[--len];
        }
        D[k] = Y[k];
        Y[k] = 0.0;
        for (; top < N; top++) {
            long i = q->pattern[top], e, end;
            double yi = Y[i], lki;
            Y[i] = 0.0;
            end = q->Lp[i] + q->lnz[i];
            for (e = q->Lp[i]; e < end; e++) Y[q->Li[e]] -= q->Lx[e] * yi;
            lki = yi / D[i];
            D[k] -= lki * yi;
            q->Li[end] = k;
            q->Lx[end] = lki;
            q->lnz[i]++;
        }
        {
            double sgn = D[k] <= 0 ? -1.0 : 1.0;
            if (sgn * D[k] <= reg_eps) { D[k] = sgn * reg_delta; q->nreg++; }
        }
    }
}

/* ldl.c:564-597 (+495-557): rhs <- (P' L^-T D^-1 L^-1 P) rhs, in place. */
static void ldl_solve_inplace(ctx_t *q, double *rhs) {
    long N = q->N, j, e;
    double *X = q->sol;
    for (j = 0; j < N; j++) X[j] = rhs[q->perm[j]];
    for (j = 0; j < N; j++)
        for (e = q->Lp[j]; e < q->Lp[j + 1]; e++) X[q->Li[e]] -= q->Lx[e] * X[j];
    for (j = 0; j < N; j++) X[j] /= q->D[j];
    for (j = N - 1; j >= 0; j--)
        for (e = q->Lp[j]; e < q->Lp[j + 1]; e++) X[j] -= q->Lx[e] * X[q->Li[e]];
    for (j = 0; j < N; j++) rhs[q->perm[j]] = X[j];
}

/* y = 0 - M x, column order (Auxilary.c:839-860 with start=1). */
static void spmv_neg(const csc_t *M, const double *x, double *y) {
    long i, k;
    for (i = 0; i < M->rows; i++) y[i] = 0;
    for (i = 0; i < M->cols; i++)
        for (k = M->jc[i]; k < M->jc[i + 1]; k++) y[M->ir[k]] -= x[i] * M->v[k];
}

/* y -= M' x (Auxilary.c:802-823 with start=0). */
static void spmtv_sub(const csc_t *M, const double *x, double *y) {
    long j, k;
    for (j = 0; j < M->cols; j++)
        for (k = M->jc[j]; k < M->jc[j + 1]; k++) y[j] -= M->v[k] * x[M->ir[k]];
}

static double dot(const double *a, const double *b, long n) {
    double acc = 0; long i;
    for (i = 0; i < n; i++) acc += a[i] * b[i];
    return acc;
}

static double nrm2(const double *a, long n) { return sqrt(dot(a, a, n)); }

/* Auxilary.c:745-786 */
static void residuals(ctx_t *q) {
    long i;
    spmv_neg(&q->P, q->x, q->rx);
    spmtv_sub(&q->G, q->z, q->rx);
    if (q->p) spmtv_sub(&q->A, q->y, q->rx);
    for (i = 0; i < q->n; i++) q->rx[i] += q->c[i] * -1.0;
    q->n_rx = nrm2(q->rx, q->n);
    if (q->p) {
        spmv_neg(&q->A, q->x, q->ry);
        for (i = 0; i < q->p; i++) q->ry[i] += q->b[i] * 1.0;
        q->n_ry = nrm2(q->ry, q->p);
    }
    spmv_neg(&q->G, q->x, q->rz);
    for (i = 0; i < q->m; i++) q->rz[i] += q->h[i] - q->s[i];
    q->n_rz = nrm2(q->rz, q->m);
    q->n_mu = dot(q->s, q->z, q->m) / q->m;
}

/* Auxilary.c:1133-1141 */
static double objective(ctx_t *q) {
    spmv_neg(&q->P, q->x, q->tmp);
    return -0.5 * dot(q->tmp, q->x, q->n) + dot(q->c, q->x, q->n);
}

/* Auxilary.c:359-393 */
static void step_length(ctx_t *q) {
    long i; int hit_p = 0, hit_d = 0;
    q->alpha_p = 1e10; q->alpha_d = 1e10;
    for (i = 0; i < q->m; i++) {
        if (q->dsl[i] < 0 && (-q->s[i] / q->dsl[i]) < q->alpha_p) { q->alpha_p = -(q->s[i] / q->dsl[i]); hit_p = 1; }
        if (q->dz[i] < 0 && (-q->z[i] / q->dz[i]) < q->alpha_d) { q->alpha_d = -(q->z[i] / q->dz[i]); hit_d = 1; }
    }
    if (!hit_p) q->alpha_p = 1;
    if (!hit_d) q->alpha_d = 1;
}

/* Auxilary.c:274-295: b = [rx; ry; rz - ds/z] */
static void build_rhs(ctx_t *q) {
    long i, n = q->n, p = q->p;
    for (i = 0; i < n; i++) q->rhs[i] = q->rx[i];
    for (i = 0; i < p; i++) q->rhs[n + i] = q->ry[i];
    for (i = 0; i < q->m; i++) q->rhs[n + p + i] = q->rz[i] - (q->ds[i] / q->z[i]);
}

/* Auxilary.c:205-216 (indicator 0): last entry of every z column <- -s/z. */
static void update_kkt_diag(ctx_t *q) {
    long i, base = q->n + q->p;
    for (i = 0; i < q->m; i++) q->K.v[q->K.jc[base + i + 1] - 1] = -q->s[i] / q->z[i];
}

/* Auxilary.c:471-564: extract deltas from the solved rhs. */
static void extract_deltas(ctx_t *q, int all) {
    long i, n = q->n, p = q->p;
    if (all) {
        for (i = 0; i < n; i++) q->dx[i] = q->rhs[i];
        for (i = 0; i < p; i++) q->dy[i] = q->rhs[n + i];
    }
    for (i = 0; i < q->m; i++) q->dz[i] = q->rhs[n + p + i];
    for (i = 0; i < q->m; i++) q->dsl[i] = (q->ds[i] - (q->s[i] * q->dz[i])) / q->z[i];
}

static int ctx_alloc(ctx_t *q) {
    long N = q->N, n = q->n, m = q->m, p = q->p;
    q->perm = xcalloc((size_t)N, sizeof(long)); q->pinv = xcalloc((size_t)N, sizeof(long));
    q->parent = xcalloc((size_t)N, sizeof(long)); q->lnz = xcalloc((size_t)N, sizeof(long));
    q->flag = xcalloc((size_t)N, sizeof(long)); q->pattern = xcalloc((size_t)N, sizeof(long));
    q->Lp = xcalloc((size_t)N + 1, sizeof(long));
    q->D = xcalloc((size_t)N, sizeof(double)); q->Y = xcalloc((size_t)N, sizeof(double));
    q->rhs = xcalloc((size_t)N, sizeof(double)); q->sol = xcalloc((size_t)N, sizeof(double));
    q->x = xcalloc((size_t)n, sizeof(double)); q->y = xcalloc((size_t)p, sizeof(double));
    q->z = xcalloc((size_t)m, sizeof(double)); q->s = xcalloc((size_t)m, sizeof(double));
    q->rx = xcalloc((size_t)n, sizeof(double)); q->ry = xcalloc((size_t)p, sizeof(double));
    q->rz = xcalloc((size_t)m, sizeof(double));
    q->dx = xcalloc((size_t)n, sizeof(double)); q->dy = xcalloc((size_t)p, sizeof(double));
    q->dz = xcalloc((size_t)m, sizeof(double)); q->dsl = xcalloc((size_t)m, sizeof(double));
    q->ds = xcalloc((size_t)m, sizeof(double)); q->lam = xcalloc((size_t)m, sizeof(double));
    q->tmp = xcalloc((size_t)n, sizeof(double));
    return 0;
}

static void ctx_free(ctx_t *q) {
    csc_free(&q->P); csc_free(&q->A); csc_free(&q->G); csc_free(&q->At); csc_free(&q->Gt); csc_free(&q->K);
    free(q->perm); free(q->pinv); free(q->parent); free(q->lnz); free(q->flag); free(q->pattern);
    free(q->Lp); free(q->Li); free(q->Lx); free(q->D); free(q->Y); free(q->rhs); free(q->sol);
    free(q->x); free(q->y); free(q->z); free(q->s); free(q->rx); free(q->ry); free(q->rz);
    free(q->dx); free(q->dy); free(q->dz); free(q->dsl); free(q->ds); free(q->lam); free(q->tmp);
}

/* Shared tail of both setups (qpSWIFT.c:176-233 / :398-455) and QP_SOLVE
 * (qpSWIFT.c:473-644). */
static long setup_and_solve(ctx_t *q, const long *perm, double reltol, double abstol, long maxit,
                            double *x, double *y, double *z, double *s, oracle_result *res) {
    long i, n = q->n, m = q->m, p = q->p, iters = 0;
    long flag = 3;                         /* stats->Flag = QP_FATAL (qpSWIFT.c:80) */
    double *zint;
    q->N = n + m + p;
    ctx_alloc(q);
    zint = xcalloc((size_t)m, sizeof(double));
    if (p) csc_transpose(&q->A, &q->At);
    csc_transpose(&q->G, &q->Gt);
    build_kkt(q);
    for (i = 0; i < q->N; i++) q->perm[i] = perm ? perm[i] : i;
    q->sigma = 100.0;                      /* SIGMA, GlobalOptions.h:49 */

    /* kkt_initialize (Auxilary.c:992-1089): one solve of the KKT holding the -I
     * block, rhs [-c; b; h] -> x0, y0; then s0, z0 from r = h - G x0. */
    ldl_symbolic(q);
    q->Li = xcalloc((size_t)q->Lp[q->N] + 1, sizeof(long));
    q->Lx = xcalloc((size_t)q->Lp[q->N] + 1, sizeof(double));
    for (i = 0; i < n; i++) q->rhs[i] = -q->c[i];
    for (i = 0; i < p; i++) q->rhs[n + i] = q->b[i];
    for (i = 0; i < m; i++) q->rhs[n + p + i] = q->h[i];
    ldl_numeric(q);
    ldl_solve_inplace(q, q->rhs);
    for (i = 0; i < n; i++) q->x[i] = q->rhs[i];
    for (i = 0; i < p; i++) q->y[i] = q->rhs[n + i];
    spmv_neg(&q->G, q->x, zint);
    for (i = 0; i < m; i++) zint[i] += q->h[i] * 1.0;
    {
        double lo = zint[0], hi = zint[0], shift;
        for (i = 1; i < m; i++) { if (zint[i] < lo) lo = zint[i]; if (zint[i] > hi) hi = zint[i]; }
        shift = -lo;
        for (i = 0; i < m; i++) q->s[i] = shift < 0 ? zint[i] : zint[i] + (1 + shift);
        for (i = 0; i < m; i++) q->z[i] = hi < 0 ? -zint[i] : -zint[i] + (1 + hi);
    }
    free(zint);
    q->alpha_p = q->alpha_d = 0.0;

    /* QP_SOLVE main loop, qpSWIFT.c:502-602 */
    for (long it = 0; it < maxit; it++) {
        const double tol = reltol / sqrt(3.0);
        int pc;
        residuals(q);
        q->fval = objective(q);
        if (q->n_rx < tol && q->n_rz < tol && (!p || q->n_ry < tol) && q->n_mu < abstol) {
            flag = 0;
            break;
        }
        for (i = 0; i < m; i++) q->lam[i] = sqrt(q->s[i] * q->z[i]);
        q->mu = dot(q->lam, q->lam, m) / m;
        pc = q->sigma > q->sigma_d;
        if (pc) {
            /* predictor: ds = -lambda.^2 (Auxilary.c:319-326) */
            for (i = 0; i < m; i++) q->ds[i] = -q->lam[i] * q->lam[i];
            update_kkt_diag(q);
            build_rhs(q);
            ldl_numeric(q);                 /* kktsolve_1, Auxilary.c:471-515 */
            ldl_solve_inplace(q, q->rhs);
            extract_deltas(q, 0);
            step_length(q);
            {   /* formrho, Auxilary.c:879-892; sigma rule qpSWIFT.c:567 */
                double acc = 0.0, r1, cube;
                for (i = 0; i < m; i++) acc += (q->s[i] + (q->alpha_p * q->dsl[i])) * (q->z[i] + (q->alpha_d * q->dz[i]));
                q->rho = acc / dot(q->s, q->z, m);
                r1 = 1 > q->rho ? q->rho : 1;
                cube = r1 * r1 * r1;
                q->sigma = q->sigma_d < cube ? cube : q->sigma_d;
            }
            for (i = 0; i < m; i++)
                q->ds[i] = -(q->lam[i] * q->lam[i]) - (q->dsl[i] * q->dz[i]) + (q->sigma * q->mu);
            build_rhs(q);
        } else {
            /* pure centering branch with refactorisation (qpSWIFT.c:572-579,
             * Auxilary.c:530-533) */
            q->sigma = q->sigma_d;
            for (i = 0; i < m; i++) q->ds[i] = -(q->lam[i] * q->lam[i]) + (q->sigma * q->mu);
            update_kkt_diag(q);
            build_rhs(q);
            ldl_numeric(q);
        }
        ldl_solve_inplace(q, q->rhs);     /* kktsolve_2, Auxilary.c:524-564 */
        extract_deltas(q, 1);
        step_length(q);
        q->alpha_p = 0.99 * q->alpha_p > 1.0 ? 1.0 : 0.99 * q->alpha_p;
        q->alpha_d = 0.99 * q->alpha_d > 1.0 ? 1.0 : 0.99 * q->alpha_d;
        for (i = 0; i < n; i++) q->x[i] += q->dx[i] * q->alpha_p;
        for (i = 0; i < p; i++) q->y[i] += q->dy[i] * q->alpha_d;
        for (i = 0; i < m; i++) q->s[i] += q->dsl[i] * q->alpha_p;
        for (i = 0; i < m; i++) q->z[i] += q->dz[i] * q->alpha_d;
        iters++;
    }
    if (iters == maxit) flag = 2;           /* qpSWIFT.c:604-607 */

    if (x) memcpy(x, q->x, sizeof(double) * (size_t)n);
    if (y && p) memcpy(y, q->y, sizeof(double) * (size_t)p);
    if (z) memcpy(z, q->z, sizeof(double) * (size_t)m);
    if (s) memcpy(s, q->s, sizeof(double) * (size_t)m);
    if (res) {
        res->flag = flag; res->iters = iters; res->fval = q->fval;
        res->n_rx = q->n_rx; res->n_ry = q->n_ry; res->n_rz = q->n_rz; res->n_mu = q->n_mu;
        res->alpha_p = q->alpha_p; res->alpha_d = q->alpha_d;
        res->n_regularised = q->nreg; res->lnz = q->Lp[q->N];
    }
    ctx_free(q);
    return flag;
}

int oracle_solve_csc(long n, long m, long p,
                     const long *Pjc, const long *Pir, const double *Ppr,
                     const long *Ajc, const long *Air, const double *Apr,
                     const long *Gjc, const long *Gir, const double *Gpr,
                     const double *c, const double *h, const double *b,
                     double sigma_d, const long *perm,
                     double reltol, double abstol, long maxit,
                     double *x, double *y, double *z, double *s,
                     oracle_result *res) {
    ctx_t q;
    memset(&q, 0, sizeof(q));
    q.n = n; q.m = m;
    q.p = (Apr && Ajc && Air && b && p != 0) ? p : 0;      /* qpSWIFT.c:91 */
    csc_copy(n, n, Pjc, Pir, Ppr, &q.P);
    if (q.p) csc_copy(q.p, n, Ajc, Air, Apr, &q.A);
    csc_copy(m, n, Gjc, Gir, Gpr, &q.G);
    q.c = c; q.h = h; q.b = b; q.sigma_d = sigma_d;
    return (int)setup_and_solve(&q, perm, reltol, abstol, maxit, x, y, z, s, res);
}

int oracle_solve_dense(long n, long m, long p,
                       const double *P, const double *A, const double *G,
                       const double *c, const double *h, const double *b,
                       const long *perm, int ordering,
                       double reltol, double abstol, long maxit,
                       double *x, double *y, double *z, double *s,
                       oracle_result *res) {
    ctx_t q;
    int rm = (ordering != 30);            /* COLUMN_MAJOR_ORDERING = 30 */
    memset(&q, 0, sizeof(q));
    q.n = n; q.m = m;
    q.p = (A && b && p != 0) ? p : 0;      /* qpSWIFT.c:292 */
    if (q.p) dense_to_csc(q.p, n, A, rm, &q.A);
    dense_to_csc(n, n, P, rm, &q.P);
    dense_to_csc(m, n, G, rm, &q.G);
    q.c = c; q.h = h; q.b = b; q.sigma_d = 0.0;                /* qpSWIFT.c:334 */
    return (int)setup_and_solve(&q, perm, reltol, abstol, maxit, x, y, z, s, res);
}

typedef struct {
    long lo, hi, n, m, p, maxit;
    const double *P, *A, *G, *c, *h, *b;
    const long *perm;
    double reltol, abstol;
    double *x; long *flags, *iters;
} batch_job_t;

static void *batch_worker(void *arg) {
    batch_job_t *j = (batch_job_t *)arg;
    for (long q = j->lo; q < j->hi; q++) {
        oracle_result r;
        oracle_solve_dense(j->n, j->m, j->p, j->P + q * j->n * j->n,
                           j->A ? j->A + q * j->p * j->n : NULL, j->G + q * j->m * j->n,
                           j->c + q * j->n, j->h + q * j->m, j->b ? j->b + q * j->p : NULL,
                           j->perm, 30, j->reltol, j->abstol, j->maxit,
                           j->x ? j->x + q * j->n : NULL, NULL, NULL, NULL, &r);
        if (j->flags) j->flags[q] = r.flag;
        if (j->iters) j->iters[q] = r.iters;
    }
    return NULL;
}

int oracle_solve_dense_batch(long B, long n, long m, long p,
                             const double *P, const double *A, const double *G,
                             const double *c, const double *h, const double *b,
                             const long *perm, double reltol, double abstol,
                             long maxit, double *x, long *flags, long *iters,
                             int threads) {
    pthread_t tid[256];
    batch_job_t jobs[256];
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    for (int t = 0; t < threads; t++) {
        batch_job_t *j = &jobs[t];
        j->lo = B * t / threads; j->hi = B * (t + 1) / threads;
        j->n = n; j->m = m; j->p = p; j->maxit = maxit;
        j->P = P; j->A = A; j->G = G; j->c = c; j->h = h; j->b = b; j->perm = perm;
        j->reltol = reltol; j->abstol = abstol; j->x = x; j->flags = flags; j->iters = iters;
        pthread_create(&tid[t], NULL, batch_worker, j);
    }
    for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
    return 0;
}

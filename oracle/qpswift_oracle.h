/*
 * qpswift_oracle.h -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * A from-scratch CPU restatement of the reference qpSWIFT interior-point solve
 * (prisma-lab/APF_quadruped, dogbot_controller/src/qpSWIFT/{qpSWIFT,Auxilary,ldl}.c).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * Parity pin: tests/test_oracle.py checks this restatement bit-for-bit against
 * golden vectors produced by the reference itself (oracle/_ref, compiled from the
 * reference C sources by oracle/Makefile) -- see tests/golden/make_golden.py.
 *
 * Not restated: SuiteSparse AMD ordering (amd_*.c).  The oracle takes the KKT
 * permutation as an input; the reference's own AMD permutation is recorded in the
 * golden fixtures, so parity is anchored on the reference's output.
 */
#ifndef QPSWIFT_ORACLE_H
#define QPSWIFT_ORACLE_H
#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_result {
    long   flag;        /* 0 optimal, 2 maxit (GlobalOptions.h:54-57)           */
    long   iters;       /* stats->IterationCount                                 */
    double fval;        /* stats->fval (value at the last top-of-loop x)         */
    double n_rx, n_ry, n_rz, n_mu;  /* last computed residual norms              */
    double alpha_p, alpha_d;        /* last step lengths                         */
    long   n_regularised;           /* pivots hit by the dynamic regularisation  */
    long   lnz;                     /* nnz(L) of the KKT factor                  */
} oracle_result;

/* Sparse entry point: mirrors QP_SETUP (qpSWIFT.c:60-234) + QP_SOLVE (:473-644).
 * CSC arrays as in the reference: P is n x n (full pattern, both triangles),
 * A is p x n (may be NULL / p == 0), G is m x n.  perm: KKT permutation of
 * length n+p+m, or NULL for the identity.  Outputs x[n], y[p], z[m], s[m]. */
int oracle_solve_csc(long n, long m, long p,
                     const long *Pjc, const long *Pir, const double *Ppr,
                     const long *Ajc, const long *Air, const double *Apr,
                     const long *Gjc, const long *Gir, const double *Gpr,
                     const double *c, const double *h, const double *b,
                     double sigma_d, const long *perm,
                     double reltol, double abstol, long maxit,
                     double *x, double *y, double *z, double *s,
                     oracle_result *res);

/* Dense entry point: mirrors QP_SETUP_dense (qpSWIFT.c:260-456), column-major
 * (ordering = 30) or row-major (ordering = 20) P[n*n], A[p*n], G[m*n]. */
int oracle_solve_dense(long n, long m, long p,
                       const double *P, const double *A, const double *G,
                       const double *c, const double *h, const double *b,
                       const long *perm, int ordering,
                       double reltol, double abstol, long maxit,
                       double *x, double *y, double *z, double *s,
                       oracle_result *res);

/* Batch helper used by the CPU baseline: B dense column-major QPs of one shape,
 * QP q's blocks at P + q*n*n etc., solved on `threads` host threads. */
int oracle_solve_dense_batch(long B, long n, long m, long p,
                             const double *P, const double *A, const double *G,
                             const double *c, const double *h, const double *b,
                             const long *perm, double reltol, double abstol,
                             long maxit, double *x, long *flags, long *iters,
                             int threads);

#ifdef __cplusplus
}
#endif
#endif

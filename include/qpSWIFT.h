/*
 * qpSWIFT.h -- source- and ABI-compatible replacement for qpSWIFT's public
 * header, backed by the gfx950 interior-point kernel of libqpswift_hip.so.
 *
 * dogbot_controller includes "qpSWIFT/qpSWIFT.h" (src/client/main.cpp:12) and
 * calls QP_SETUP_dense -> options override -> QP_SOLVE -> reads myQP->x
 * (main.cpp:1649-1663).  This header declares the same five entry points
 * (reference include/qpSWIFT/qpSWIFT.h:14-26) and the same structs with the same
 * field order and types (reference include/qpSWIFT/Auxilary.h:18-151,
 * qp_int = long and qp_real = double as in GlobalOptions.h:36-43), so the
 * controller can be rebuilt against this header, or relinked against
 * libqpswift_hip.so without recompiling.
 *
 * Behaviour (see INTEGRATION.md for the full list of differences):
 *   QP_SETUP / QP_SETUP_dense  build the pattern plan (KKT layout, ordering,
 *       elimination tree, generated kernels) on the host and cache it by sparsity
 *       pattern; the matrices are converted exactly as the reference does
 *       (dense -> CSC drops exact zeros).  Like the reference (qpSWIFT.c:447),
 *       setup leaves kkt_initialize's point in x, y, z, s: one device launch
 *       (QPSWIFT_HIP_SETUP_INIT=0 skips it: x, y, z, s then stay zero until the
 *       first QP_SOLVE, which runs the initial point itself -- one device solve
 *       per tick instead of two, at the price of that difference).
 *   QP_SOLVE  continues from the QP object's state as the reference does
 *       (qpSWIFT.c:502-601): its x, y, z, s, stats->IterationCount, stats->Flag
 *       and options->sigma, at most options->maxit more iterations, QP_MAXIT only
 *       when IterationCount reaches exactly maxit; the plan's warm-solve kernel
 *       runs on the current HIP device, then x, y, z, s, the statistics and
 *       options->sigma are written back.
 *   Device solves (setup's initial point, QP_SOLVE) go to a persistent solver:
 *       per kind (cold / warm) and solving thread, a wave launched ahead of the
 *       call polls a mailbox in mapped host memory, answers ONE request and
 *       leaves; each call launches the next call's wave while its own solves, so
 *       a call costs no stream synchronisation and no launch on its path.  A
 *       queued wave leaves after QPSWIFT_HIP_SERVE_IDLE_MS (default 20) without a
 *       call; a call later than half that relaunches.  (QPSWIFT_HIP_SERVE_LIFE_MS
 *       > 0, diagnostics only, keeps one wave answering request after request
 *       for that long -- measured to carry state between requests.)  Plans
 *       whose one-QP kernel is the tree or the exact lane kernel, and
 *       QPSWIFT_HIP_SERVE=0, launch + synchronise per call.  There is no CPU
 *       fallback: without a usable GPU it returns QP_FATAL and qpb_last_error()
 *       says why.
 *   Arithmetic: by default the fast kernels (FMA, reciprocal pivots; the
 *   wave-cooperative kernel where eligible), which factor with the same
 *   permutation, pivots and regularisations and agree with qpSWIFT to rounding.
 *   QPSWIFT_HIP_EXACT=1 in the environment selects the bit-faithful kernel (the
 *   reference's operation order, IEEE division, no FMA): bit-identical to
 *   qpSWIFT when given the same permutation, across repeated QP_SOLVE calls too.
 *   With Permut == NULL the KKT is ordered by this library's restatement of
 *   SuiteSparse AMD (amd_l_order with amd_l_defaults, src/qpSWIFT/qpSWIFT.c:
 *   424-440), which yields qpSWIFT's own permutation (bit-for-bit,
 *   tests/test_amd.py); stats->AMD_RESULT is then 0, and -3 when Permut is
 *   given, as in the reference.
 *   stats->kkt_time / ldl_numeric  device time (s_memrealtime, 100 MHz) of this
 *       call's factorisations + triangular solves / of the factorisations
 *       (accumulated over calls, reset by setup), measured inside the kernel
 *       (the reference times kktsolve_1/_2 and LDL_numeric on the host,
 *       qpSWIFT.c:554-586, Auxilary.c:476-484); tsetup and tsolve hold the host
 *       wall time of QP_SETUP* / QP_SOLVE.
 *   options->verbose > 0  the reference's messages (qpSWIFT.c:484-488, 506-509,
 *       598-641) on stdout, the per-iteration lines printed after the launch from
 *       the kernel's trace (up to 256 iterations per call; the tree kernel, used
 *       only for KKT systems beyond the wave kernel's range, traces pcost as nan).
 */
#ifndef QPSWIFT_HIP_DROPIN_H
#define QPSWIFT_HIP_DROPIN_H

#ifdef __cplusplus
extern "C" {
#endif

#ifndef qp_real
#define qp_real double
#endif
#ifndef qp_int
#define qp_int long
#endif

/* defaults (GlobalOptions.h:46-50) */
#define MAXIT (100)
#define RELTOL (1e-6)
#define ABSTOL (1e-6)
#define SIGMA (100)
#define VERBOSE (0)

/* exit flags (GlobalOptions.h:54-57) */
#define QP_OPTIMAL (0)
#define QP_KKTFAIL (1)
#define QP_MAXIT (2)
#define QP_FATAL (3)

/* dense input storage order for QP_SETUP_dense (GlobalOptions.h:59-60) */
#define ROW_MAJOR_ORDERING (20)
#define COLUMN_MAJOR_ORDERING (30)

/* compressed sparse column matrix: m rows, n columns (Auxilary.h:18-26) */
typedef struct smat {
    qp_int *jc;
    qp_int *ir;
    qp_real *pr;
    qp_int n;
    qp_int m;
    qp_int nnz;
} smat;

/* KKT system (Auxilary.h:31-50).  Here the symbolic members (kktmatrix pattern
 * and setup-time values, Parent, Lnz, Lp, Li, P, Pinv) are filled from the plan;
 * the numeric factor lives on the GPU only, so Lx, D, Y, b are zero-filled
 * buffers of the reference's sizes. */
typedef struct kkt {
    smat *kktmatrix;
    qp_real *b;
    qp_int *Parent;
    qp_int *Flag;
    qp_int *Lnz;
    qp_int *Li;
    qp_int *Lp;
    qp_int *Lti;
    qp_int *Ltp;
    qp_int *Pattern;
    qp_int *UPattern;
    qp_real *Y;
    qp_real *Lx;
    qp_real *D;
    qp_int *P;
    qp_int *Pinv;
} kkt;

/* statistics (Auxilary.h:55-84) */
typedef struct stats {
    qp_real tsetup;
    qp_real tsolve;
    qp_real kkt_time;
    qp_real ldl_numeric;
    qp_int IterationCount;
    qp_real n_rx;
    qp_real n_ry;
    qp_real n_rz;
    qp_real n_mu;
    qp_real alpha_p;
    qp_real alpha_d;
    qp_real fval;
    qp_int Flag;
    qp_int AMD_RESULT;
    qp_int resolve_kkt;
} stats;

/* settings (Auxilary.h:89-100); sigma and verbose: see the header comment */
typedef struct settings {
    qp_int maxit;
    qp_real reltol;
    qp_real abstol;
    qp_real sigma;
    qp_int verbose;
} settings;

/* solver object (Auxilary.h:106-151) */
typedef struct QP {
    qp_int n;
    qp_int m;
    qp_int p;
    qp_real sigma_d;
    qp_real mu;
    qp_real rho;
    qp_real *x;
    qp_real *y;
    qp_real *z;
    qp_real *s;
    qp_real *rx;
    qp_real *ry;
    qp_real *rz;
    qp_real *delta;
    qp_real *delta_x;
    qp_real *delta_y;
    qp_real *delta_z;
    qp_real *delta_s;
    qp_real *ds;
    qp_real *lambda;
    qp_real *temp;
    smat *P;
    qp_real *c;
    smat *G;
    qp_real *h;
    smat *A;
    qp_real *b;
    smat *At;
    smat *Gt;
    kkt *kkt;
    settings *options;
    stats *stats;
} QP;

/* qpSWIFT.h:14 -- CSC inputs (P full, both triangles), all borrowed */
QP *QP_SETUP(qp_int n, qp_int m, qp_int p, qp_int *Pjc, qp_int *Pir, qp_real *Ppr,
             qp_int *Ajc, qp_int *Air, qp_real *Apr, qp_int *Gjc, qp_int *Gir, qp_real *Gpr,
             qp_real *c, qp_real *h, qp_real *b, qp_real sigma_d, qp_int *Permut);

/* qpSWIFT.h:17 -- dense inputs (copied); c, h, b borrowed */
QP *QP_SETUP_dense(qp_int n, qp_int m, qp_int p, qp_real *Ppr, qp_real *Apr, qp_real *Gpr,
                   qp_real *c, qp_real *h, qp_real *b, qp_int *Permut, int ordering);

/* qpSWIFT.h:20 */
qp_int QP_SOLVE(QP *myQP);

/* qpSWIFT.h:23,26 */
void QP_CLEANUP(QP *myQP);
void QP_CLEANUP_dense(QP *myQP);

#ifdef __cplusplus
}
#endif
#endif

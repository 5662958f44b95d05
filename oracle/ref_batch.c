/*
 * ref_batch.c -- TEST INFRASTRUCTURE ONLY: a pthread batch driver around the
 * reference qpSWIFT (oracle/_ref/libqpswift_ref.so), used as the CPU baseline of
 * bench.py.  Each QP is solved exactly as dogbot_controller does per tick
 * (main.cpp:1649-1656): QP_SETUP_dense -> reltol/abstol override -> QP_SOLVE,
 * followed by QP_CLEANUP_dense.  Compiled against the reference's own headers by
 * oracle/Makefile (`make ref`); output lands in oracle/_ref/.
 */
#include <pthread.h>
#include <string.h>

#include "qpSWIFT/qpSWIFT.h"

typedef struct {
    long lo, hi, n, m, p;
    double *P, *A, *G, *c, *h, *b;
    double tol;
    double *x; long *flags, *iters;
} job_t;

static void *worker(void *arg) {
    job_t *j = (job_t *)arg;
    for (long q = j->lo; q < j->hi; q++) {
        QP *qp = QP_SETUP_dense(j->n, j->m, j->p, j->P + q * j->n * j->n, j->A + q * j->p * j->n,
                                j->G + q * j->m * j->n, j->c + q * j->n, j->h + q * j->m,
                                j->b + q * j->p, NULL, COLUMN_MAJOR_ORDERING);
        qp->options->reltol = j->tol;
        qp->options->abstol = j->tol;
        long f = QP_SOLVE(qp);
        if (j->x) memcpy(j->x + q * j->n, qp->x, sizeof(double) * (size_t)j->n);
        if (j->flags) j->flags[q] = f;
        if (j->iters) j->iters[q] = qp->stats->IterationCount;
        QP_CLEANUP_dense(qp);
    }
    return NULL;
}

int ref_solve_dense_batch(long B, long n, long m, long p, double *P, double *A, double *G,
                          double *c, double *h, double *b, double tol, double *x, long *flags,
                          long *iters, int threads) {
    pthread_t tid[256];
    job_t jobs[256];
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    for (int t = 0; t < threads; t++) {
        job_t *j = &jobs[t];
        j->lo = B * t / threads; j->hi = B * (t + 1) / threads;
        j->n = n; j->m = m; j->p = p; j->P = P; j->A = A; j->G = G; j->c = c; j->h = h; j->b = b;
        j->tol = tol; j->x = x; j->flags = flags; j->iters = iters;
        pthread_create(&tid[t], NULL, worker, j);
    }
    for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
    return 0;
}

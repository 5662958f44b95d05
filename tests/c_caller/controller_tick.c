/*
 * controller_tick.c -- a compiled C caller of the drop-in boundary
 * (include/qpSWIFT.h, linked against libqpswift_hip.so), replaying
 * dogbot_controller's per-tick call sequence (src/client/main.cpp:1649-1663):
 *
 *     myQP = QP_SETUP_dense(n, m, p, Q, A, D, c, C, b, NULL, COLUMN_MAJOR_ORDERING);
 *     myQP->options->reltol = tol;  myQP->options->abstol = tol;
 *     ExitCode = QP_SOLVE(myQP);
 *     x_(i) = myQP->x[i];
 *
 * plus QP_CLEANUP_dense (the controller never calls it and leaks every tick).
 * Input: a binary file  int64 n, m, p, ticks; double tol; then per tick the
 * column-major dense P[n*n], A[p*n], G[m*n] and c[n], h[m], b[p].
 * Output: one line per tick  "tick k exit E iters I amd R x x0 x1 ...".
 * Test infrastructure (tests/test_c_caller.py).
 */
#include <stdio.h>
#include <stdlib.h>

#include "qpSWIFT.h"

static void *read_n(FILE *f, size_t count, size_t size) {
    void *p = malloc(count * size + 8);
    if (!p || fread(p, size, count, f) != count) { fprintf(stderr, "short input\n"); exit(2); }
    return p;
}

int main(int argc, char **argv) {
    if (argc != 2) { fprintf(stderr, "usage: %s inputs.bin\n", argv[0]); return 2; }
    FILE *f = fopen(argv[1], "rb");
    if (!f) { perror(argv[1]); return 2; }
    long long hdr[4];
    double tol;
    if (fread(hdr, sizeof hdr[0], 4, f) != 4 || fread(&tol, sizeof tol, 1, f) != 1) return 2;
    const qp_int n = hdr[0], m = hdr[1], p = hdr[2];
    for (long long t = 0; t < hdr[3]; t++) {
        qp_real *Q = read_n(f, (size_t)(n * n), sizeof(qp_real));
        qp_real *A = read_n(f, (size_t)(p * n), sizeof(qp_real));
        qp_real *D = read_n(f, (size_t)(m * n), sizeof(qp_real));
        qp_real *c = read_n(f, (size_t)n, sizeof(qp_real));
        qp_real *C = read_n(f, (size_t)m, sizeof(qp_real));
        qp_real *b = read_n(f, (size_t)p, sizeof(qp_real));

        QP *myQP = QP_SETUP_dense(n, m, p, Q, p > 0 ? A : NULL, D, c, C, p > 0 ? b : NULL, NULL,
                                  COLUMN_MAJOR_ORDERING);
        myQP->options->reltol = tol;
        myQP->options->abstol = tol;
        qp_int ExitCode = QP_SOLVE(myQP);

        printf("tick %lld exit %ld iters %ld amd %ld x", t, (long)ExitCode, (long)myQP->stats->IterationCount,
               (long)myQP->stats->AMD_RESULT);
        for (qp_int i = 0; i < n; i++) printf(" %.17g", myQP->x[i]);
        printf("\n");
        QP_CLEANUP_dense(myQP);
        free(Q); free(A); free(D); free(c); free(C); free(b);
    }
    fclose(f);
    return 0;
}

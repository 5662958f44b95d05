// Operand layout of v_mfma_f64_4x4x4f64 (gfx950).  For each lane p of the wavefront:
// A = e_p (1 in lane p only), B = lane + 1.  D(l) = sum_k A[i(l)][k] B[k][j(l)] is non-zero
// exactly in the output lanes whose row is A-lane p's row (in A-lane p's block), and
// D(l) - 1 is the B-lane paired with A-lane p for output l's column.  Prints one line per p.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(double *out) {
    const int l = threadIdx.x;
    for (int p = 0; p < 64; p++) {
        const double a = (l == p) ? 1.0 : 0.0;
        out[p * 64 + l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, (double)(l + 1), 0.0, 0, 0, 0);
    }
}

int main() {
    double *d;
    hipMalloc(&d, 64 * 64 * sizeof(double));
    hipMemset(d, 0, 64 * 64 * sizeof(double));
    probe<<<1, 64>>>(d);
    static double h[64 * 64];
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    printf("A-lane p: output lane -> paired B-lane\n");
    for (int p = 0; p < 64; p++) {
        printf("p=%2d:", p);
        for (int l = 0; l < 64; l++)
            if (h[p * 64 + l] != 0.0) printf(" %d->%g", l, h[p * 64 + l] - 1);
        printf("\n");
    }
    return 0;
}

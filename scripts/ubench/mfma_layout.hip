// Operand layout of v_mfma_f64_4x4x4f64 (four 4x4x4 blocks, one per 16-lane row) on gfx950.
// For each lane p of a block: A = e_p (1 in lane p only), B = 2^(lane & 15).  Then
// D(l) = sum_k A[i(l)][k] B[k][j(l)] is non-zero exactly in the output lanes whose row i
// is the row of A-lane p, and its value names the B-lane paired with A-lane p for that
// output column.  Prints one line per p: the output lanes hit and log2 of their values.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>

__global__ void probe(double *out) {
    const int l = threadIdx.x;
    for (int p = 0; p < 16; p++) {
        const double a = ((l & 15) == p) ? 1.0 : 0.0;
        const double b = (double)(1 << (l & 15));
        out[p * 64 + l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
    }
}

int main() {
    double *d;
    hipMalloc(&d, 16 * 64 * sizeof(double));
    hipMemset(d, 0, 16 * 64 * sizeof(double));
    probe<<<1, 64>>>(d);
    double h[16 * 64];
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    printf("A-lane p: output lane -> B-lane (log2 D), block 0 (lanes 0-15); blocks 1-3 identical: %s\n", [&] {
        for (int p = 0; p < 16; p++)
            for (int l = 0; l < 16; l++)
                for (int b = 1; b < 4; b++)
                    if (h[p * 64 + l] != h[p * 64 + 16 * b + l]) return "no";
        return "yes";
    }());
    for (int p = 0; p < 16; p++) {
        printf("p=%2d:", p);
        for (int l = 0; l < 16; l++)
            if (h[p * 64 + l] != 0.0) printf(" %d->%d", l, (int)std::log2(h[p * 64 + l]));
        printf("\n");
    }
    return 0;
}

// Layout probe of v_mfma_f64_4x4x4f64 (four 4x4x4 blocks, one per 16-lane row) on gfx950:
// which lanes each output lane sums over for A and for B, and whether
// D2 = ones x (A x ones) is the full 16-lane sum of A in every lane of its row.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(double *out) {
    const int l = threadIdx.x;
    const double one = 1.0;
    // 1: A = l + 1, B = 1  -> D(l) = sum of A over the lanes of output l's row of A
    double d1 = __builtin_amdgcn_mfma_f64_4x4x4f64((double)(l + 1), one, 0.0, 0, 0, 0);
    // 2: A = 1, B = l + 1  -> D(l) = sum of B over the lanes of output l's column of B
    double d2 = __builtin_amdgcn_mfma_f64_4x4x4f64(one, (double)(l + 1), 0.0, 0, 0, 0);
    // 3: powers of two to identify the summed lanes exactly (within a 16-lane block)
    double d3 = __builtin_amdgcn_mfma_f64_4x4x4f64((double)(1 << (l & 15)), one, 0.0, 0, 0, 0);
    double d4 = __builtin_amdgcn_mfma_f64_4x4x4f64(one, (double)(1 << (l & 15)), 0.0, 0, 0, 0);
    // 5: the two-step total: ones x (A x ones)
    double t1 = __builtin_amdgcn_mfma_f64_4x4x4f64((double)(1 << (l & 15)), one, 0.0, 0, 0, 0);
    double t2 = __builtin_amdgcn_mfma_f64_4x4x4f64(one, t1, 0.0, 0, 0, 0);
    double t3 = __builtin_amdgcn_mfma_f64_4x4x4f64(t1, one, 0.0, 0, 0, 0);
    out[l * 8 + 0] = d1; out[l * 8 + 1] = d2; out[l * 8 + 2] = d3; out[l * 8 + 3] = d4;
    out[l * 8 + 4] = t1; out[l * 8 + 5] = t2; out[l * 8 + 6] = t3;
}

int main() {
    double *d;
    hipMalloc(&d, 64 * 8 * sizeof(double));
    hipMemset(d, 0, 64 * 8 * sizeof(double));
    probe<<<1, 64>>>(d);
    double h[64 * 8];
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    printf("lane d1(A=l+1) d2(B=l+1) d3(A=2^l) d4(B=2^l) t1 t2=ones*t1 t3=t1*ones\n");
    for (int l = 0; l < 64; l++)
        printf("%2d %6.0f %6.0f %6.0f %6.0f %6.0f %6.0f %6.0f\n", l, h[l * 8], h[l * 8 + 1], h[l * 8 + 2], h[l * 8 + 3],
               h[l * 8 + 4], h[l * 8 + 5], h[l * 8 + 6]);
    return 0;
}

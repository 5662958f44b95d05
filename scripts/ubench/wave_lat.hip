// Single-wave latency / throughput microbenchmarks for the instruction mix of
// the wave kernel (gfx950): cycles per op from s_memtime around unrolled chains.
//   hipcc --offload-arch=gfx950 -O3 -o wave_lat wave_lat.hip && ./wave_lat
#include <hip/hip_runtime.h>
#include <cstdio>

#define N 64
#define REP8(x) x x x x x x x x
#define REP64(x) REP8(x) REP8(x) REP8(x) REP8(x) REP8(x) REP8(x) REP8(x) REP8(x)

__device__ __forceinline__ long long clk() {
    long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t));
    return t;
}

extern "C" __global__ void ub(double *out, double *sink, const double *in) {
    __shared__ double lds[1024];
    const int lane = threadIdx.x;
    double a = in[lane], b = in[lane + 64], c = in[lane + 128];
    double x = a, y = b, z = c, w = a + b, u = b + c, v = a + c, p = a * b, q = b * c;
    int k = 0;                 // result slot (never an asm operand)
    int sc = lane, sd = lane + 1, se = lane + 2;   // scratch registers for the asm tests
    typedef int i4 __attribute__((ext_vector_type(4)));
    i4 t[4] = {};
    long long t0, t1;
#define TIME(name, body)                                                        \
    __builtin_amdgcn_s_waitcnt(0);                                              \
    t0 = clk();                                                                 \
    body;                                                                       \
    __builtin_amdgcn_s_waitcnt(0);                                              \
    t1 = clk();                                                                 \
    if (lane == 0) out[k] = (double)(t1 - t0) / N;                              \
    k++;
    // 0: dependent f64 FMA chain
    TIME("fma_dep", REP64(asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b));))
    // 1: 4 independent FMA chains (per op)
    TIME("fma_ind4", REP8(REP8(asm volatile("v_fma_f64 %0, %0, %4, %5\n\tv_fma_f64 %1, %1, %4, %5\n\tv_fma_f64 %2, %2, %4, %5\n\tv_fma_f64 %3, %3, %4, %5" : "+v"(x), "+v"(y), "+v"(z), "+v"(w) : "v"(a), "v"(b));)))
    // 2: dependent fmac_dpp row_newbcast (s_nop 1 + fmac)
    TIME("fmac_dpp_dep", REP64(asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %0, %1 row_newbcast:3 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(y) : "v"(a));))
    // 3: independent fmac_dpp (same source, 8 destinations)
    TIME("fmac_dpp_ind", REP8(asm volatile("v_fmac_f64_dpp %0, %8, %9 row_newbcast:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                                          "v_fmac_f64_dpp %1, %8, %9 row_newbcast:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                                          "v_fmac_f64_dpp %2, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                                          "v_fmac_f64_dpp %3, %8, %9 row_newbcast:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                                          "v_fmac_f64_dpp %4, %8, %9 row_newbcast:5 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                                          "v_fmac_f64_dpp %5, %8, %9 row_newbcast:6 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                                          "v_fmac_f64_dpp %6, %8, %9 row_newbcast:7 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                                          "v_fmac_f64_dpp %7, %8, %9 row_newbcast:8 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                                          : "+v"(x), "+v"(y), "+v"(z), "+v"(w), "+v"(u), "+v"(v), "+v"(p), "+v"(q) : "v"(a), "v"(b));))
    // 4: dependent v_mov_b64_dpp + fmac
    TIME("mov_dpp_fmac_dep", REP64(asm volatile("s_nop 1\n\tv_mov_b64_dpp %1, %0 row_newbcast:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\tv_fmac_f64 %0, %1, %2" : "+v"(z), "=&v"(u) : "v"(a));))
    // 5: dependent rcp_f64
    TIME("rcp_dep", REP64(asm volatile("v_rcp_f64 %0, %0" : "+v"(w));))
    // 6: accvgpr read pair + fma (dependent through fma)
    {
        double ag = a;
        asm volatile("v_accvgpr_write_b32 a0, %0\n\tv_accvgpr_write_b32 a1, %1" :: "v"((int)__builtin_bit_cast(long long, ag)), "v"((int)(__builtin_bit_cast(long long, ag) >> 32)) : "a0", "a1");
        TIME("accread2_fma", REP64(asm volatile("v_accvgpr_read_b32 %1, a0\n\tv_accvgpr_read_b32 %2, a1\n\tv_fma_f64 %0, %0, %3, %4" : "+v"(x), "=&v"(sc), "=&v"(sd) : "v"(a), "v"(b) : "a0", "a1");))
    }
    // 7: LDS store -> load round trip (dependent)
    TIME("lds_roundtrip", REP64(asm volatile("ds_write_b64 %1, %0\n\ts_waitcnt lgkmcnt(0)\n\tds_read_b64 %0, %2\n\ts_waitcnt lgkmcnt(0)" : "+v"(x) : "v"(lane * 8), "v"(0));))
    // 8: LDS broadcast read latency (dependent address chain is not possible; read + wait)
    TIME("lds_read_wait", REP64(asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(y) : "v"(0));))
    // 9: 8 LDS b128 broadcast reads then one wait (per read)
    TIME("lds_read_b128_x8", REP8(asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:16\n\tds_read_b128 %2, %4 offset:32\n\tds_read_b128 %3, %4 offset:48\n\t"
                                              "ds_read_b128 %0, %4 offset:64\n\tds_read_b128 %1, %4 offset:80\n\tds_read_b128 %2, %4 offset:96\n\tds_read_b128 %3, %4 offset:112\n\ts_waitcnt lgkmcnt(0)"
                                              : "=v"(t[0]), "=v"(t[1]), "=v"(t[2]), "=v"(t[3]) : "v"(0));))  // types approximate; timing only
    // 10: readlane x2 -> fma with sgpr operand (dependent chain through x)
    TIME("readlane_add_dep", REP64(asm volatile("v_readlane_b32 s20, %0, 3\n\tv_add_u32 %0, s20, %0" : "+v"(sc) :: "s20");))
    // 11: quad_perm reduction stage f64 (2 x mov_b32_dpp + add), dependent
    TIME("qperm_add_dep", REP64(asm volatile("s_nop 1\n\tv_mov_b32_dpp %1, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                                            "v_mov_b32_dpp %2, %3 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(sc), "=&v"(sd), "=&v"(se) : "v"(sc));))
    // 12: independent 32-bit VALU (v_cndmask) throughput
    {
        int i0 = lane, i1 = lane + 1, i2 = lane + 2, i3 = lane + 3;
        TIME("valu32_ind", REP8(REP8(asm volatile("v_add_u32 %0, %0, %4\n\tv_add_u32 %1, %1, %4\n\tv_add_u32 %2, %2, %4\n\tv_add_u32 %3, %3, %4" : "+v"(i0), "+v"(i1), "+v"(i2), "+v"(i3) : "v"(lane));)))
        sink[lane + 64] = i0 + i1 + i2 + i3;
    }
    // 13: dependent f64 add
    TIME("add_dep", REP64(asm volatile("v_add_f64 %0, %0, %1" : "+v"(u) : "v"(a));))
    // 14: dependent f64 mul
    TIME("mul_dep", REP64(asm volatile("v_mul_f64 %0, %0, %1" : "+v"(v) : "v"(a));))
    // 15: s_memtime overhead (empty)
    TIME("empty", ;)
    // 16: dependent v_cndmask_b32 pair (64-bit select)
    TIME("cndmask64_dep", REP64(asm volatile("v_cmp_lt_f64 vcc, %0, %1\n\tv_cndmask_b32 %2, %2, %3, vcc" : "+v"(p), "+v"(q), "+v"(sc) : "v"(lane) : "vcc");))
    // 17: v_mfma_f64_16x16x4_f64, dependent accumulator chain
    typedef double d4 __attribute__((ext_vector_type(4)));
    d4 m0 = {a, b, c, a}, m1 = {b, c, a, b}, m2 = m0, m3 = m1;
    TIME("mfma16_dep", REP64(asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(m0) : "v"(a), "v"(b));))
    // 18: 4 independent 16x16x4 accumulators (per MFMA)
    TIME("mfma16_ind4", REP8(REP8(asm volatile("v_mfma_f64_16x16x4_f64 %0, %4, %5, %0\n\tv_mfma_f64_16x16x4_f64 %1, %4, %5, %1\n\t"
                                              "v_mfma_f64_16x16x4_f64 %2, %4, %5, %2\n\tv_mfma_f64_16x16x4_f64 %3, %4, %5, %3"
                                              : "+v"(m0), "+v"(m1), "+v"(m2), "+v"(m3) : "v"(a), "v"(b));)))
    // 19: v_mfma_f64_4x4x4_4b_f64 (four 4x4 blocks per wave: one per 16-lane row), dependent
    double e0 = a, e1 = b, e2 = c, e3 = a + 1.0;
    TIME("mfma4_dep", REP64(asm volatile("v_mfma_f64_4x4x4_4b_f64 %0, %1, %2, %0" : "+v"(e0) : "v"(a), "v"(b));))
    // 20: 4 independent 4x4x4 accumulators (per MFMA)
    TIME("mfma4_ind4", REP8(REP8(asm volatile("v_mfma_f64_4x4x4_4b_f64 %0, %4, %5, %0\n\tv_mfma_f64_4x4x4_4b_f64 %1, %4, %5, %1\n\t"
                                             "v_mfma_f64_4x4x4_4b_f64 %2, %4, %5, %2\n\tv_mfma_f64_4x4x4_4b_f64 %3, %4, %5, %3"
                                             : "+v"(e0), "+v"(e1), "+v"(e2), "+v"(e3) : "v"(a), "v"(b));)))
    // 21: v_permlane32_swap_b32 pair (64-bit cross-half move) + dependent fma
    TIME("permlane32swap2_fma_dep", REP64(asm volatile("v_mov_b32 %1, %0\n\tv_permlane32_swap_b32 %0, %1\n\tv_fma_f64 %2, %2, %3, %3"
                                                   : "+v"(sc), "=&v"(sd), "+v"(x) : "v"(a));))
    // 22: independent f64 FMA, 8 accumulators (per op): FP64 issue rate of one wave
    TIME("fma_ind8", REP8(asm volatile("v_fma_f64 %0, %0, %8, %9\n\tv_fma_f64 %1, %1, %8, %9\n\tv_fma_f64 %2, %2, %8, %9\n\tv_fma_f64 %3, %3, %8, %9\n\t"
                                       "v_fma_f64 %4, %4, %8, %9\n\tv_fma_f64 %5, %5, %8, %9\n\tv_fma_f64 %6, %6, %8, %9\n\tv_fma_f64 %7, %7, %8, %9"
                                       : "+v"(x), "+v"(y), "+v"(z), "+v"(w), "+v"(u), "+v"(v), "+v"(p), "+v"(q) : "v"(a), "v"(b));))
    // 23: s_nop 1 throughput
    TIME("s_nop1", REP64(asm volatile("s_nop 1");))
    // 24: v_fmac_f64 with an SGPR-pair operand fed by two v_readlane_b32 (dependent through the readlanes)
    TIME("readlane2_fmac_dep", REP64(asm volatile("v_readlane_b32 s20, %0, 3\n\tv_readlane_b32 s21, %1, 3\n\tv_fma_f64 %2, s[20:21], %3, %2"
                                                  : "+v"(sc), "+v"(sd), "+v"(y) : "v"(a) : "s20", "s21");))
    // 25: three interleaved dependent fmac_dpp chains, no s_nop (2 VALU between a write and its DPP read), per op
    TIME("fmac_dpp_3chains", REP64(asm volatile("v_fmac_f64_dpp %0, %0, %3 row_newbcast:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                                                "v_fmac_f64_dpp %1, %1, %3 row_newbcast:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                                                "v_fmac_f64_dpp %2, %2, %3 row_newbcast:3 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                                                : "+v"(u), "+v"(v), "+v"(p) : "v"(a));))
    // 26: v_rcp_f64 + 2 Newton FMAs, dependent (a pivot reciprocal)
    TIME("rcp_newton_dep", REP64(asm volatile("v_rcp_f64 %1, %0\n\tv_fma_f64 %2, -%0, %1, 1.0\n\tv_fma_f64 %0, %2, %1, %1"
                                              : "+v"(w), "=&v"(x), "=&v"(y));))
    sink[lane + 128] = m0.x + m1.y + m2.z + m3.w + e0 + e1 + e2 + e3;
    sink[lane] = x + y + z + w + u + v + p + q + t[0].x + t[1].y + t[2].z + t[3].w + sc + sd + se + lds[lane];
}

int main() {
    const char *names[] = {"fma_dep", "fma_ind4(per op)", "fmac_dpp_dep(+nop1)", "fmac_dpp_ind(per op)", "mov_dpp+fmac_dep(+nop1)",
                           "rcp_dep", "accread2+fma_dep", "lds_wr_rd_roundtrip", "lds_read_wait", "lds_read_b128(per read, 8 in flight)",
                           "readlane+add_u32 chain", "qperm 2xmov_dpp", "valu32_ind(per op)", "add_f64_dep", "mul_f64_dep", "memtime_overhead(total)",
                           "cmp+cndmask_dep", "mfma_f64_16x16x4_dep", "mfma_f64_16x16x4_ind4(per op)", "mfma_f64_4x4x4_4b_dep",
                           "mfma_f64_4x4x4_4b_ind4(per op)", "mov+permlane32_swap+fma_dep", "fma_f64_ind8(per op)", "s_nop1",
                           "readlane2+fma(sgpr)_dep", "fmac_dpp 3 chains no nop(per op)", "rcp+2fma_dep"};
    const int K = 27;
    double *d_out, *d_sink, *d_in, h_in[192], h_out[32];
    for (int i = 0; i < 192; i++) h_in[i] = 1.0 + 1e-9 * i;
    hipMalloc(&d_out, 32 * 8); hipMalloc(&d_sink, 192 * 8); hipMalloc(&d_in, 192 * 8);
    hipMemcpy(d_in, h_in, 192 * 8, hipMemcpyHostToDevice);
    hipMemset(d_out, 0xff, 32 * 8);
    for (int r = 0; r < 3; r++) {
        hipLaunchKernelGGL(ub, dim3(1), dim3(64), 0, 0, d_out, d_sink, d_in);
        hipError_t e = hipDeviceSynchronize();
        if (e != hipSuccess || hipGetLastError() != hipSuccess) { printf("error: %s\n", hipGetErrorString(e)); return 1; }
    }
    hipMemcpy(h_out, d_out, K * 8, hipMemcpyDeviceToHost);
    // operations per timed unit (the device divides by N = 64 units)
    const double per[] = {1, 4, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 4, 1, 1, 1.0 / 64, 1, 1, 4, 1, 4, 1, 1, 1, 1, 3, 1};
    for (int i = 0; i < K; i++) printf("%-40s %8.2f cycles\n", names[i], h_out[i] / per[i]);
    return 0;
}

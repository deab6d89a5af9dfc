// VALU issue cost per wave64 instruction on gfx950 (cycles, s_memtime): one
// wave per SIMD, 8 independent chains of the same instruction.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
#define R8(S) S S S S S S S S
#define R64(S) R8(S) R8(S) R8(S) R8(S) R8(S) R8(S) R8(S) R8(S)

#define BENCH(NAME, INIT, BODY, OUT)                                                   \
__global__ void NAME(float* o, unsigned long long* t) {                               \
    INIT                                                                               \
    unsigned long long t0, t1;                                                         \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0) :: "memory");       \
    for (int it = 0; it < 4; ++it) { R64(BODY) }                                       \
    asm volatile("s_waitcnt vmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1) :: "memory"); \
    o[blockIdx.x * blockDim.x + threadIdx.x] = OUT;                                     \
    if ((threadIdx.x & 63) == 0) { t[2 * (threadIdx.x >> 6)] = t0; t[2 * (threadIdx.x >> 6) + 1] = t1; } \
}
// each BODY = 8 instructions (8 chains)
#define V8F float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
#define OUT8F (a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7)
#define OP1(op) asm volatile(op " %0, %0\n" op " %1, %1\n" op " %2, %2\n" op " %3, %3\n" op " %4, %4\n" op " %5, %5\n" op " %6, %6\n" op " %7, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
#define OP2(op) asm volatile(op " %0, %0, %1\n" op " %1, %1, %2\n" op " %2, %2, %3\n" op " %3, %3, %4\n" op " %4, %4, %5\n" op " %5, %5, %6\n" op " %6, %6, %7\n" op " %7, %7, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
BENCH(b_fma, V8F, asm volatile("v_fma_f32 %0, %0, %0, %1\nv_fma_f32 %1, %1, %1, %2\nv_fma_f32 %2, %2, %2, %3\nv_fma_f32 %3, %3, %3, %4\nv_fma_f32 %4, %4, %4, %5\nv_fma_f32 %5, %5, %5, %6\nv_fma_f32 %6, %6, %6, %7\nv_fma_f32 %7, %7, %7, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));, OUT8F)
BENCH(b_log, V8F, OP1("v_log_f32"), OUT8F)
BENCH(b_sin, V8F, OP1("v_sin_f32"), OUT8F)
BENCH(b_sqrt, V8F, OP1("v_sqrt_f32"), OUT8F)
BENCH(b_rcp, V8F, OP1("v_rcp_f32"), OUT8F)
BENCH(b_exp, V8F, OP1("v_exp_f32"), OUT8F)
BENCH(b_mullo, V8F, OP2("v_mul_lo_u32"), OUT8F)
BENCH(b_mulhi, V8F, OP2("v_mul_hi_u32"), OUT8F)
BENCH(b_xor3, V8F, OP2("v_xor_b32"), OUT8F)
BENCH(b_dpp, V8F, asm volatile("v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\nv_mov_b32_dpp %1, %2 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\nv_mov_b32_dpp %2, %3 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\nv_mov_b32_dpp %3, %4 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\nv_mov_b32_dpp %4, %5 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\nv_mov_b32_dpp %5, %6 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\nv_mov_b32_dpp %6, %7 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\nv_mov_b32_dpp %7, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));, OUT8F)
BENCH(b_pkfma, double a0 = threadIdx.x; double a1 = a0 + 1; double a2 = a0 + 2; double a3 = a0 + 3; double a4 = a0 + 4; double a5 = a0 + 5; double a6 = a0 + 6; double a7 = a0 + 7;,
      asm volatile("v_pk_fma_f32 %0, %0, %0, %1\nv_pk_fma_f32 %1, %1, %1, %2\nv_pk_fma_f32 %2, %2, %2, %3\nv_pk_fma_f32 %3, %3, %3, %4\nv_pk_fma_f32 %4, %4, %4, %5\nv_pk_fma_f32 %5, %5, %5, %6\nv_pk_fma_f32 %6, %6, %6, %7\nv_pk_fma_f32 %7, %7, %7, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));, (float)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7))
BENCH(b_addf64, double a0 = threadIdx.x; double a1 = a0 + 1; double a2 = a0 + 2; double a3 = a0 + 3; double a4 = a0 + 4; double a5 = a0 + 5; double a6 = a0 + 6; double a7 = a0 + 7;,
      asm volatile("v_add_f64 %0, %0, %1\nv_add_f64 %1, %1, %2\nv_add_f64 %2, %2, %3\nv_add_f64 %3, %3, %4\nv_add_f64 %4, %4, %5\nv_add_f64 %5, %5, %6\nv_add_f64 %6, %6, %7\nv_add_f64 %7, %7, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));, (float)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7))
BENCH(b_fmaf64, double a0 = threadIdx.x; double a1 = a0 + 1; double a2 = a0 + 2; double a3 = a0 + 3; double a4 = a0 + 4; double a5 = a0 + 5; double a6 = a0 + 6; double a7 = a0 + 7;,
      asm volatile("v_fma_f64 %0, %0, %1, %2\nv_fma_f64 %1, %1, %2, %3\nv_fma_f64 %2, %2, %3, %4\nv_fma_f64 %3, %3, %4, %5\nv_fma_f64 %4, %4, %5, %6\nv_fma_f64 %5, %5, %6, %7\nv_fma_f64 %6, %6, %7, %0\nv_fma_f64 %7, %7, %0, %1" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));, (float)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7))
BENCH(b_cvtf64, V8F double d0 = 0; double d1 = 0; double d2 = 0; double d3 = 0; double d4 = 0; double d5 = 0; double d6 = 0; double d7 = 0;,
      asm volatile("v_cvt_f64_f32 %0, %8\nv_cvt_f64_f32 %1, %9\nv_cvt_f64_f32 %2, %10\nv_cvt_f64_f32 %3, %11\nv_cvt_f64_f32 %4, %12\nv_cvt_f64_f32 %5, %13\nv_cvt_f64_f32 %6, %14\nv_cvt_f64_f32 %7, %15" : "=v"(d0), "=v"(d1), "=v"(d2), "=v"(d3), "=v"(d4), "=v"(d5), "=v"(d6), "=v"(d7) : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5), "v"(a6), "v"(a7)); a0 += (float)d0; a1 += (float)d1;, OUT8F)
__global__ void b_mad64(float* o, unsigned long long* t) {
    unsigned long long a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    unsigned m = 0xD2511F53u ^ threadIdx.x, mm = threadIdx.x * 7u;
    unsigned long long t0, t1;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0) :: "memory");
    for (int it = 0; it < 4; ++it) { R64(asm volatile("v_mad_u64_u32 %0, s[100:101], %8, %9, %0\nv_mad_u64_u32 %1, s[100:101], %8, %9, %1\nv_mad_u64_u32 %2, s[100:101], %8, %9, %2\nv_mad_u64_u32 %3, s[100:101], %8, %9, %3\nv_mad_u64_u32 %4, s[100:101], %8, %9, %4\nv_mad_u64_u32 %5, s[100:101], %8, %9, %5\nv_mad_u64_u32 %6, s[100:101], %8, %9, %6\nv_mad_u64_u32 %7, s[100:101], %8, %9, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(m), "v"(mm) : "s100", "s101");) }
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1) :: "memory");
    o[blockIdx.x * blockDim.x + threadIdx.x] = (float)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);
    if ((threadIdx.x & 63) == 0) { t[2 * (threadIdx.x >> 6)] = t0; t[2 * (threadIdx.x >> 6) + 1] = t1; }
}
typedef void (*kfn)(float*, unsigned long long*);
int main() {
    float* o; unsigned long long *t, h[128];
    CK(hipMalloc(&o, 1 << 20)); CK(hipMalloc(&t, 4096));
    struct { const char* n; kfn f; } ks[] = {{"v_fma_f32", b_fma}, {"v_pk_fma_f32", b_pkfma}, {"v_log_f32", b_log},
        {"v_sin_f32", b_sin}, {"v_sqrt_f32", b_sqrt}, {"v_rcp_f32", b_rcp}, {"v_exp_f32", b_exp},
        {"v_mul_lo_u32", b_mullo}, {"v_mul_hi_u32", b_mulhi}, {"v_xor_b32", b_xor3}, {"v_mov_b32_dpp", b_dpp},
        {"v_add_f64", b_addf64}, {"v_fma_f64", b_fmaf64}, {"v_cvt_f64_f32(+2 f32)", b_cvtf64}, {"v_mad_u64_u32", b_mad64}};
    for (auto& k : ks) {
        for (int waves : {1, 2, 4}) {   // waves per SIMD: block of 256*waves threads on one CU
            for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(k.f, dim3(1), dim3(256 * waves), 0, 0, o, t);
            CK(hipDeviceSynchronize());
            const int nw = 4 * waves;
            CK(hipMemcpy(h, t, 16 * nw, hipMemcpyDeviceToHost));
            unsigned long long mn = ~0ull, mx = 0, w0 = h[1] - h[0];
            for (int i = 0; i < nw; ++i) { mn = h[2 * i] < mn ? h[2 * i] : mn; mx = h[2 * i + 1] > mx ? h[2 * i + 1] : mx; }
            const double per = 4.0 * 64 * 8;
            printf("%-24s waves/SIMD=%d  wave0 cycles/instr %.2f   all-waves span: SIMD cycles per wave-instr %.2f\n",
                   k.n, waves, w0 / per, (double)(mx - mn) / per / waves);
        }
    }
    return 0;
}

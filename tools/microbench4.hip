// Instruction-fetch cost: straight-line code (~N distinct VALU ops) vs the same
// op count from a small loop, one wave, cycles via s_memtime.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
#define F4(a,b,c,d) a = fmaf(a, 1.0001f, 0.5f); b = fmaf(b, 0.9999f, 0.25f); c = fmaf(c, 1.0002f, 0.125f); d = fmaf(d, 0.9998f, 0.0625f);
#define F16(a,b,c,d) F4(a,b,c,d) F4(b,c,d,a) F4(c,d,a,b) F4(d,a,b,c)
#define F64(a,b,c,d) F16(a,b,c,d) F16(a,b,c,d) F16(a,b,c,d) F16(a,b,c,d)
#define F256(a,b,c,d) F64(a,b,c,d) F64(a,b,c,d) F64(a,b,c,d) F64(a,b,c,d)
__global__ void k_straight(float* o, unsigned long long* t) {
    float a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
    unsigned long long t0, t1;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0) :: "memory");
    F256(a,b,c,d) F256(a,b,c,d) F256(a,b,c,d) F256(a,b,c,d)   // 4096 fma
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1) :: "memory");
    o[threadIdx.x] = a + b + c + d;
    if (threadIdx.x == 0) t[blockIdx.x] = t1 - t0;
}
__global__ void k_loop(float* o, unsigned long long* t, int n) {
    float a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
    unsigned long long t0, t1;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0) :: "memory");
    for (int i = 0; i < n; ++i) { F64(a,b,c,d) }
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1) :: "memory");
    o[threadIdx.x] = a + b + c + d;
    if (threadIdx.x == 0) t[blockIdx.x] = t1 - t0;
}
int main() {
    float* o; unsigned long long *t, h[4];
    CK(hipMalloc(&o, 4096)); CK(hipMalloc(&t, 4096));
    for (int r = 0; r < 3; ++r) {
        hipLaunchKernelGGL(k_straight, dim3(1), dim3(64), 0, 0, o, t);
        CK(hipDeviceSynchronize()); CK(hipMemcpy(h, t, 8, hipMemcpyDeviceToHost));
        printf("straight-line 4096 fma: %llu cycles (%.2f cyc/op)\n", h[0], h[0] / 4096.0);
        hipLaunchKernelGGL(k_loop, dim3(1), dim3(64), 0, 0, o, t, 64);
        CK(hipDeviceSynchronize()); CK(hipMemcpy(h, t, 8, hipMemcpyDeviceToHost));
        printf("loop     4096 fma: %llu cycles (%.2f cyc/op)\n", h[0], h[0] / 4096.0);
    }
    return 0;
}

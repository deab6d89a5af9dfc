// Dependent-load latency on MI355X, in shader cycles (s_memtime) and ns
// (s_memrealtime, 100 MHz): L2-warm vs data just written by another kernel.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_fill(int* buf, int n, int stride) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        buf[i] = (i + stride) % n;
}
__global__ void k_chase(const int* buf, int hops, unsigned long long* out) {
    if (threadIdx.x != 0) return;
    int idx = blockIdx.x * 4096;
    unsigned long long t0, t1, r0, r1;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0) :: "memory");
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r0) :: "memory");
    for (int h = 0; h < hops; ++h) {
        idx = __builtin_nontemporal_load(buf + idx);
    }
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1) :: "memory");
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r1) :: "memory");
    out[blockIdx.x * 3 + 0] = t1 - t0;
    out[blockIdx.x * 3 + 1] = r1 - r0;
    out[blockIdx.x * 3 + 2] = idx;
}
__global__ void k_lds_chase(int hops, unsigned long long* out) {
    __shared__ int l[1024];
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) l[i] = (i * 37 + 11) & 1023;
    __syncthreads();
    if (threadIdx.x != 0) return;
    int idx = 0;
    unsigned long long t0, t1;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0) :: "memory");
    for (int h = 0; h < hops; ++h) idx = l[idx];
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1) :: "memory");
    out[0] = t1 - t0; out[1] = idx;
}

int main() {
    const int n = 1 << 24;
    int* buf; unsigned long long *out, h[64];
    CK(hipMalloc(&buf, n * 4)); CK(hipMalloc(&out, 4096));
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, buf, n, 4099 * 16 + 1);
    CK(hipDeviceSynchronize());
    const int hops = 64;
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k_chase, dim3(4), dim3(64), 0, 0, buf, hops, out);   // cold/warm
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h, out, 12 * 8, hipMemcpyDeviceToHost));
        printf("chase rep %d (after fill=%d): %.0f cyc/hop  %.0f ns/hop\n", rep, rep == 0, (double)h[0] / hops,
               (double)h[1] * 10.0 / hops);
    }
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_chase, dim3(4), dim3(64), 0, 0, buf, hops, out);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h, out, 12 * 8, hipMemcpyDeviceToHost));
        printf("chase warm again: %.0f cyc/hop  %.0f ns/hop  -> clock %.2f GHz\n", (double)h[0] / hops,
               (double)h[1] * 10.0 / hops, (double)h[0] / ((double)h[1] * 10.0));
    }
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, buf, n, 4099 * 16 + 1);   // rewrite
    hipLaunchKernelGGL(k_chase, dim3(4), dim3(64), 0, 0, buf, hops, out);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h, out, 12 * 8, hipMemcpyDeviceToHost));
    printf("chase right after a producer kernel: %.0f cyc/hop  %.0f ns/hop\n", (double)h[0] / hops, (double)h[1] * 10.0 / hops);
    hipLaunchKernelGGL(k_lds_chase, dim3(1), dim3(256), 0, 0, 256, out);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h, out, 16, hipMemcpyDeviceToHost));
    printf("LDS dependent read: %.0f cyc\n", (double)h[0] / 256);
    return 0;
}

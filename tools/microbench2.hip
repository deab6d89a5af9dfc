// Producer -> consumer latency across a kernel boundary (records written by 256
// blocks, read by 7 blocks x 256 threads x 16 float4 loads), vs. reading a
// buffer nobody wrote since, vs. kernarg-dependent first loads.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_produce(float4* rec, int n4) {   // 256 blocks x 256 threads
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x)
        rec[i] = make_float4(i, 1, 2, 3);
}
__global__ void k_consume(const float4* __restrict__ rec, float* out, int stride4) {
    const int tid = threadIdx.x;
    float4 acc = make_float4(0, 0, 0, 0);
    float4 x[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = rec[(size_t)(tid / 8 + 32 * (i & 7)) * stride4 + (tid & 7) + (i >> 3) * 8 + blockIdx.x * 9];
#pragma unroll
    for (int i = 0; i < 16; ++i) { acc.x += x[i].x; acc.y += x[i].y; }
    if (acc.x == 1234.5f) out[tid] = acc.y;
}
__global__ void k_stamp(unsigned long long* t, const float4* __restrict__ rec, int stride4) {
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    float4 v = rec[(size_t)threadIdx.x * stride4 + blockIdx.x];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { t[blockIdx.x * 2] = t1 - t0; t[blockIdx.x * 2 + 1] = (unsigned long long)v.x; }
}

int main() {
    const int nrec = 256, P4 = 57;   // 228 floats per record
    float4 *rec, *rec2; float* out; unsigned long long* ts;
    CK(hipMalloc(&rec, nrec * P4 * 16)); CK(hipMalloc(&rec2, nrec * P4 * 16)); CK(hipMalloc(&out, 4096));
    CK(hipMalloc(&ts, 4096));
    hipStream_t s; CK(hipStreamCreate(&s));
    hipLaunchKernelGGL(k_produce, dim3(256), dim3(256), 0, s, rec2, nrec * P4);
    unsigned long long h[32];
    for (int it = 0; it < 200; ++it) {
        hipLaunchKernelGGL(k_produce, dim3(256), dim3(256), 0, s, rec, nrec * P4);
        hipLaunchKernelGGL(k_consume, dim3(7), dim3(256), 0, s, rec, out, P4);     // fresh data
        hipLaunchKernelGGL(k_consume, dim3(7), dim3(256), 0, s, rec2, out, P4);    // untouched data
        hipLaunchKernelGGL(k_produce, dim3(256), dim3(256), 0, s, rec, nrec * P4);
        hipLaunchKernelGGL(k_stamp, dim3(8), dim3(64), 0, s, ts, rec, P4);         // one load, fresh
        hipLaunchKernelGGL(k_stamp, dim3(8), dim3(64), 0, s, ts + 16, rec2, P4);   // one load, old
    }
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(h, ts, sizeof(h), hipMemcpyDeviceToHost));
    printf("single-load latency cycles: fresh");
    for (int b = 0; b < 8; ++b) printf(" %llu", h[2 * b]);
    printf(" | untouched");
    for (int b = 0; b < 8; ++b) printf(" %llu", h[16 + 2 * b]);
    printf("\n");
    return 0;
}

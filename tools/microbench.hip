// Launch/latency microbenchmarks on MI355X to size the fixed costs of a tiny
// control step (kernarg size, dependent global round trips, host-mapped writes).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

struct Big { float v[600]; };   // 2.4 KB of kernel arguments
__global__ void k_empty(int x) { if (x == 12345) asm volatile("s_nop 0"); }
__global__ void k_bigarg(Big b, float* out) { if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = b.v[599] + b.v[7]; }
__global__ void k_chain(const float* __restrict__ in, float* out, int hops) {
    // dependent global loads: pointer chase through `in`
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    int idx = 0;
    for (int i = 0; i < hops; ++i) idx = (int)in[idx];
    out[0] = (float)idx;
}
__global__ void k_hostwrite(double* hout) { if (threadIdx.x == 0) hout[blockIdx.x] = 1.0 + blockIdx.x; }
__global__ void k_grid(float* out) {  // 256 blocks x 512 threads, trivial work
    out[blockIdx.x * blockDim.x + threadIdx.x] = threadIdx.x;
}

int main() {
    float *d, *o; double* h; double* hd;
    CK(hipMalloc(&d, 1 << 24)); CK(hipMalloc(&o, 1 << 24));
    std::vector<float> idx(1 << 20);
    for (int i = 0; i < (1 << 20); ++i) idx[i] = (float)((i * 4099 + 77777) % (1 << 20));
    CK(hipMemcpy(d, idx.data(), idx.size() * 4, hipMemcpyHostToDevice));
    CK(hipHostMalloc((void**)&h, 4096, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostGetDevicePointer((void**)&hd, h, 0));
    hipStream_t s; CK(hipStreamCreate(&s));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    Big b{}; b.v[599] = 1; b.v[7] = 2;
    auto bench = [&](const char* name, auto launch) {
        for (int i = 0; i < 50; ++i) launch();
        CK(hipStreamSynchronize(s));
        const int N = 2000;
        auto t0 = std::chrono::steady_clock::now();
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < N; ++i) launch();
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        auto t1 = std::chrono::steady_clock::now();
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-28s gpu %.2f us/launch   host %.2f us/launch\n", name, 1e3 * ms / N,
               std::chrono::duration<double, std::micro>(t1 - t0).count() / N);
        // single launch + sync round trip
        auto t2 = std::chrono::steady_clock::now();
        for (int i = 0; i < 200; ++i) { launch(); CK(hipStreamSynchronize(s)); }
        auto t3 = std::chrono::steady_clock::now();
        printf("%-28s launch+sync %.2f us\n", name, std::chrono::duration<double, std::micro>(t3 - t2).count() / 200);
        return 0;
    };
    bench("empty", [&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, 0); });
    bench("bigarg 2.4KB", [&] { hipLaunchKernelGGL(k_bigarg, dim3(1), dim3(64), 0, s, b, o); });
    bench("chain 1 hop", [&] { hipLaunchKernelGGL(k_chain, dim3(1), dim3(64), 0, s, d, o, 1); });
    bench("chain 4 hops", [&] { hipLaunchKernelGGL(k_chain, dim3(1), dim3(64), 0, s, d, o, 4); });
    bench("chain 16 hops", [&] { hipLaunchKernelGGL(k_chain, dim3(1), dim3(64), 0, s, d, o, 16); });
    bench("hostwrite 7 blocks", [&] { hipLaunchKernelGGL(k_hostwrite, dim3(7), dim3(64), 0, s, hd); });
    bench("grid 256x512", [&] { hipLaunchKernelGGL(k_grid, dim3(256), dim3(512), 0, s, o); });
    bench("empty+empty", [&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, 0);
                               hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, 0); });
    return 0;
}

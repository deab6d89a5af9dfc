// Host-side launch cost on this stack: enqueue time per hipLaunchKernelGGL for
// kernel-argument structs of 16 B .. 4 KB, plus hipSetDevice / hipEventRecord.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
template <int N> struct Arg { int v[N / 4]; };
template <int N> __global__ void k_empty(const Arg<N> a, int* sink) { if (a.v[0] == 12345 && threadIdx.x == 9999) sink[0] = a.v[N / 4 - 1]; }
__global__ void k_scalar(int a, int b, float* p) { if (a == 12345 && threadIdx.x == 9999) p[b] = 0; }
using clk = std::chrono::high_resolution_clock;
template <int N> double bench(hipStream_t s, int n) {
    Arg<N> a = {};
    for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(k_empty<N>, dim3(28), dim3(256), 0, s, a, nullptr);
    (void)hipStreamSynchronize(s);
    auto t0 = clk::now();
    for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_empty<N>, dim3(28), dim3(256), 0, s, a, nullptr);
    auto t1 = clk::now();
    (void)hipStreamSynchronize(s);
    auto t2 = clk::now();
    printf("kernarg %5d B: enqueue %.2f us/launch, total %.2f us/launch\n", N,
           std::chrono::duration<double, std::micro>(t1 - t0).count() / n,
           std::chrono::duration<double, std::micro>(t2 - t0).count() / n);
    return 0;
}
int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const int n = 2000;
    bench<16>(s, n); bench<256>(s, n); bench<1024>(s, n); bench<2560>(s, n); bench<4096>(s, n);
    {
        auto t0 = clk::now();
        for (int i = 0; i < n; ++i) (void)hipSetDevice(0);
        auto t1 = clk::now();
        printf("hipSetDevice: %.3f us\n", std::chrono::duration<double, std::micro>(t1 - t0).count() / n);
        hipEvent_t ev; CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        t0 = clk::now();
        for (int i = 0; i < n; ++i) (void)hipEventRecord(ev, s);
        t1 = clk::now();
        (void)hipStreamSynchronize(s);
        auto t2 = clk::now();
        printf("hipEventRecord: enqueue %.3f us, total %.3f us\n", std::chrono::duration<double, std::micro>(t1 - t0).count() / n,
               std::chrono::duration<double, std::micro>(t2 - t0).count() / n);
        t0 = clk::now();
        for (int i = 0; i < n; ++i) (void)hipGetLastError();
        t1 = clk::now();
        printf("hipGetLastError: %.3f us\n", std::chrono::duration<double, std::micro>(t1 - t0).count() / n);
    }
    {   // alternating two kernels (like rollout/finalize)
        Arg<1024> a = {}; Arg<256> b = {};
        auto t0 = clk::now();
        for (int i = 0; i < n; ++i) {
            hipLaunchKernelGGL(k_empty<1024>, dim3(256), dim3(512), 0, s, a, nullptr);
            hipLaunchKernelGGL(k_empty<256>, dim3(28), dim3(512), 0, s, b, nullptr);
        }
        auto t1 = clk::now();
        (void)hipStreamSynchronize(s);
        auto t2 = clk::now();
        printf("alternating pair: enqueue %.2f us/pair, total %.2f us/pair\n",
               std::chrono::duration<double, std::micro>(t1 - t0).count() / n,
               std::chrono::duration<double, std::micro>(t2 - t0).count() / n);
    }
    {   // graph of the pair
        hipGraph_t g; hipGraphExec_t ge;
        Arg<1024> a = {}; Arg<256> b = {};
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        hipLaunchKernelGGL(k_empty<1024>, dim3(256), dim3(512), 0, s, a, nullptr);
        hipLaunchKernelGGL(k_empty<256>, dim3(28), dim3(512), 0, s, b, nullptr);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int i = 0; i < 50; ++i) CK(hipGraphLaunch(ge, s));
        (void)hipStreamSynchronize(s);
        auto t0 = clk::now();
        for (int i = 0; i < n; ++i) (void)hipGraphLaunch(ge, s);
        auto t1 = clk::now();
        (void)hipStreamSynchronize(s);
        auto t2 = clk::now();
        printf("graph pair: enqueue %.2f us/pair, total %.2f us/pair\n",
               std::chrono::duration<double, std::micro>(t1 - t0).count() / n,
               std::chrono::duration<double, std::micro>(t2 - t0).count() / n);
    }
    return 0;
}

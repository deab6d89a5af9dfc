// Floor of a back-to-back kernel sequence on MI355X: n launches of an empty kernel, and of
// an alternating pair, between one HIP event pair (tools/ only; the step of the MPPI
// engine is a rollout + finalize pair).
//   hipcc --offload-arch=gfx950 -O3 -o tools/mb8.bin tools/microbench8.hip && ./tools/mb8.bin
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_empty(int* p) { if (p && threadIdx.x == 1u << 20) p[0] = 1; }
__global__ void k_empty2(int* p) { if (p && threadIdx.x == 1u << 20) p[1] = 1; }

int main() {
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int grids[3] = {28, 256, 1024};
    for (int gi = 0; gi < 3; ++gi) {
        const int g = grids[gi];
        for (int rep = 0; rep < 2; ++rep) {
            const int n = 400;
            for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(k_empty, dim3(g), dim3(256), 0, s, nullptr);
            (void)hipEventRecord(a, s);
            for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_empty, dim3(g), dim3(256), 0, s, nullptr);
            (void)hipEventRecord(b, s);
            (void)hipEventSynchronize(b);
            float ms1 = 0;
            (void)hipEventElapsedTime(&ms1, a, b);
            (void)hipEventRecord(a, s);
            for (int i = 0; i < n / 2; ++i) {
                hipLaunchKernelGGL(k_empty, dim3(g), dim3(512), 0, s, nullptr);
                hipLaunchKernelGGL(k_empty2, dim3(28), dim3(256), 0, s, nullptr);
            }
            (void)hipEventRecord(b, s);
            (void)hipEventSynchronize(b);
            float ms2 = 0;
            (void)hipEventElapsedTime(&ms2, a, b);
            printf("grid %4d x 256: empty kernel %.2f us each back to back; pair (grid x 512, 28 x 256) %.2f us per pair\n",
                   g, 1e3f * ms1 / n, 1e3f * ms2 / (n / 2));
        }
    }
    return 0;
}

// Kernel-start load latency on MI355X (tools/ only): how long after a wave starts does the
// first value arrive from (a) the kernel-argument segment (written by the host for this
// launch), (b) a device buffer no kernel has written for a while, (c) a device buffer the
// previous kernel on the stream wrote from every XCD (as u_prev / the records are), and
// (d) the same buffer read a second time in the same wave (L2 hit).  Each wave of a 256-block
// grid stamps s_memrealtime (100 MHz) at its start and after each load's value is consumed;
// the host reports medians over the waves and over back-to-back launches.
//   hipcc --offload-arch=gfx950 -O3 -o tools/mb9.bin tools/microbench9.hip && ./tools/mb9.bin
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

struct Big { unsigned v[256]; };   // a 1 KB kernel-argument block, like the rollout's

__device__ __forceinline__ unsigned long long rt() {
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    __builtin_amdgcn_sched_barrier(0);
    return t;
}

__global__ void __launch_bounds__(256) k_writer(unsigned* buf, unsigned tag) {
    // every block (all XCDs) writes its slice: the next kernel's reads miss in their L2
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    buf[i] = tag + i;
}

__global__ void __launch_bounds__(256) k_probe(const Big args, const unsigned* cold, const unsigned* fresh,
                                              unsigned long long* out, unsigned* sink) {
    const unsigned long long t0 = rt();
    // (a) kernel-argument word far from the preloaded ones
    unsigned a = args.v[200 + (blockIdx.x & 7)];
    asm volatile("" : "+v"(a));
    const unsigned long long t1 = rt();
    // (b) cold device buffer (scalar load)
    unsigned b = cold[(blockIdx.x & 7) * 16];
    asm volatile("" : "+v"(b));
    const unsigned long long t2 = rt();
    // (c) buffer the previous kernel wrote (vector load, per lane)
    unsigned c = fresh[blockIdx.x * blockDim.x + threadIdx.x];
    asm volatile("" : "+v"(c));
    const unsigned long long t3 = rt();
    // (d) a neighbouring line of (c), same wave, second touch of the same page
    unsigned d = fresh[((blockIdx.x + 1) % gridDim.x) * blockDim.x + threadIdx.x];
    asm volatile("" : "+v"(d));
    const unsigned long long t4 = rt();
    if (threadIdx.x == 0) {
        unsigned long long* o = out + (size_t)blockIdx.x * 4;
        o[0] = t1 - t0; o[1] = t2 - t1; o[2] = t3 - t2; o[3] = t4 - t3;
    }
    if (a + b + c + d == 0xFFFFFFFFu) sink[0] = 1;
}

int main() {
    const int nb = 256, nt = 256, reps = 200;
    unsigned *cold, *fresh, *sink;
    unsigned long long* out;
    (void)hipMalloc(&cold, 1 << 20);
    (void)hipMalloc(&fresh, (size_t)nb * nt * 4);
    (void)hipMalloc(&sink, 64);
    (void)hipMalloc(&out, (size_t)nb * 4 * 8);
    (void)hipMemset(cold, 0, 1 << 20);
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    Big args;
    for (int i = 0; i < 256; ++i) args.v[i] = i;
    std::vector<unsigned long long> h((size_t)nb * 4);
    std::vector<double> med[4];
    for (int r = 0; r < reps; ++r) {
        hipLaunchKernelGGL(k_writer, dim3(nb), dim3(nt), 0, s, fresh, (unsigned)r);
        hipLaunchKernelGGL(k_probe, dim3(nb), dim3(nt), 0, s, args, cold, fresh, out, sink);
        (void)hipStreamSynchronize(s);
        (void)hipMemcpy(h.data(), out, h.size() * 8, hipMemcpyDeviceToHost);
        for (int j = 0; j < 4; ++j) {
            std::vector<double> x;
            for (int b = 0; b < nb; ++b) x.push_back(10.0 * (double)h[(size_t)b * 4 + j]);
            std::nth_element(x.begin(), x.begin() + x.size() / 2, x.end());
            med[j].push_back(x[x.size() / 2]);
        }
    }
    const char* names[4] = {"kernel-argument word (fresh per launch)", "device buffer, untouched for a while (s_load)",
                            "device buffer the previous kernel wrote on all XCDs (vector load)",
                            "second line of that buffer, same wave"};
    for (int j = 0; j < 4; ++j) {
        std::vector<double> x = med[j];
        std::sort(x.begin(), x.end());
        printf("%-66s median %6.0f ns  p10 %6.0f  p90 %6.0f\n", names[j], x[x.size() / 2], x[x.size() / 10],
               x[x.size() * 9 / 10]);
    }
    return 0;
}

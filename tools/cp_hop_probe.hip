// cp_hop_probe.hip -- tools/, not shipped.  Latency of the hand-offs a one-finalize RCCL step would
// need (the RCCL exchange): a running kernel on stream A signals a word, stream B's
// hipStreamWaitValue32 releases a kernel (standing in for the collective), hipStreamWriteValue32
// then releases the still-running kernel on A, which polls the word.  Compared with the plain
// kernel boundary on one stream (end stamp of one kernel -> start stamp of the next).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/_bin/cp_hop_probe tools/cp_hop_probe.hip
//   tools/_bin/cp_hop_probe [iterations]
//
// Part 3 replaces B's kernel with the real collective: a 1-rank RCCL communicator's
// ncclAllReduce of the C4 shard's 660-float slot (librccl.so.1 by dlopen, as the engine loads it).
//
// Stamps are s_memrealtime (100 MHz).  Every spin has a 20 ms deadline, so a lost release ends
// the kernel (reported as a timeout) instead of hanging the GPU.
#include <hip/hip_runtime.h>

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

typedef unsigned long long u64;

__global__ void k_stamp(u64* t) {
    if (threadIdx.x == 0) t[0] = __builtin_amdgcn_s_memrealtime();
}

// stream A's kernel: stamp, signal `go` = i, wait for `back` >= i, stamp
__global__ void k_signal_wait(uint32_t* go, uint32_t* back, uint32_t i, u64* t) {
    if (threadIdx.x != 0) return;
    t[0] = __builtin_amdgcn_s_memrealtime();
    __hip_atomic_store(go, i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const u64 t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t v = 0;
    for (;;) {
        v = __hip_atomic_load(back, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (v >= i) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > 2000000ull) break;   // 20 ms
        __builtin_amdgcn_s_sleep(1);
    }
    t[1] = __builtin_amdgcn_s_memrealtime();
    t[2] = v;
}

static void report(const char* name, std::vector<double> x) {
    std::sort(x.begin(), x.end());
    const size_t n = x.size();
    printf("%-44s n=%zu  p10 %6.2f  p50 %6.2f  p90 %6.2f us\n", name, n, x[n / 10], x[n / 2], x[n * 9 / 10]);
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 300;
    int can = 0;
    CK(hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, 0));
    printf("hipDeviceAttributeCanUseStreamWaitValue = %d\n", can);
    hipStream_t A, B;
    CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
    uint32_t *go = nullptr, *back = nullptr;
    CK(hipExtMallocWithFlags((void**)&go, 8, hipMallocSignalMemory));
    CK(hipExtMallocWithFlags((void**)&back, 8, hipDeviceMallocFinegrained));
    CK(hipMemset(go, 0, 4));
    CK(hipMemset(back, 0, 4));
    u64* t = nullptr;
    CK(hipMalloc(&t, 64 * sizeof(u64)));
    CK(hipMemset(t, 0, 64 * sizeof(u64)));
    CK(hipDeviceSynchronize());
    u64 h[64];
    u64* hbuf = h;

    // 1. the plain boundary: two kernels back to back on one stream
    std::vector<double> bnd;
    for (int i = 0; i < iters; ++i) {
        hipLaunchKernelGGL(k_stamp, dim3(1), dim3(64), 0, A, t);
        hipLaunchKernelGGL(k_stamp, dim3(1), dim3(64), 0, A, t + 1);
        CK(hipStreamSynchronize(A));
        CK(hipMemcpy(h, t, 2 * sizeof(u64), hipMemcpyDeviceToHost));
        bnd.push_back((double)(h[1] - h[0]) * 0.01);
    }
    report("same-stream kernel boundary (start->start)", bnd);

    // 2. the cross-stream round trip
    std::vector<double> out, back_us, total;
    int timeouts = 0;
    for (int i = 1; i <= iters; ++i) {
        CK(hipStreamWaitValue32(B, go, (uint32_t)i, hipStreamWaitValueGte, 0xFFFFFFFFu));
        hipLaunchKernelGGL(k_stamp, dim3(1), dim3(64), 0, B, t + 8);
        CK(hipStreamWriteValue32(B, back, (uint32_t)i, 0));
        hipLaunchKernelGGL(k_signal_wait, dim3(1), dim3(64), 0, A, go, back, (uint32_t)i, t);
        CK(hipStreamSynchronize(A));
        CK(hipStreamSynchronize(B));
        CK(hipMemcpy(h, t, 16 * sizeof(u64), hipMemcpyDeviceToHost));
        if (h[2] < (u64)i) { ++timeouts; continue; }
        out.push_back((double)(h[8] - h[0]) * 0.01);
        back_us.push_back((double)(h[1] - h[8]) * 0.01);
        total.push_back((double)(h[1] - h[0]) * 0.01);
    }
    printf("timeouts: %d of %d\n", timeouts, iters);
    if (!out.empty()) {
        report("signal -> WaitValue -> B's kernel start", out);
        report("B's kernel start -> WriteValue -> A sees", back_us);
        report("round trip (A signals .. A released)", total);
    }

    // 3. the same round trip with the 1-rank all-reduce in place of B's kernel
    void* lib = dlopen("librccl.so.1", RTLD_NOW);
    if (!lib) lib = dlopen("librccl.so", RTLD_NOW);
    if (!lib) { printf("librccl not loadable: %s\n", dlerror()); return 0; }
    auto get_id = (ncclResult_t(*)(ncclUniqueId*))dlsym(lib, "ncclGetUniqueId");
    auto init = (ncclResult_t(*)(ncclComm_t*, int, ncclUniqueId, int))dlsym(lib, "ncclCommInitRank");
    auto ar = (ncclResult_t(*)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                               hipStream_t))dlsym(lib, "ncclAllReduce");
    auto destroy = (ncclResult_t(*)(ncclComm_t))dlsym(lib, "ncclCommDestroy");
    if (!get_id || !init || !ar || !destroy) { printf("librccl lacks an entry point\n"); return 0; }
    ncclUniqueId id;
    ncclComm_t comm;
    if (get_id(&id) != ncclSuccess || init(&comm, 1, id, 0) != ncclSuccess) { printf("rccl init failed\n"); return 0; }
    float* slot = nullptr;
    CK(hipMalloc(&slot, 660 * sizeof(float)));
    CK(hipMemset(slot, 0, 660 * sizeof(float)));
    for (int i = 0; i < 20; ++i) ar(slot, slot, 660, ncclFloat32, ncclSum, comm, B);   // connection setup
    CK(hipStreamSynchronize(B));
    std::vector<double> rt, bnd_ar;
    timeouts = 0;
    for (int i = iters + 1; i <= 2 * iters; ++i) {
        CK(hipStreamWaitValue32(B, go, (uint32_t)i, hipStreamWaitValueGte, 0xFFFFFFFFu));
        ar(slot, slot, 660, ncclFloat32, ncclSum, comm, B);
        CK(hipStreamWriteValue32(B, back, (uint32_t)i, 0));
        hipLaunchKernelGGL(k_signal_wait, dim3(1), dim3(64), 0, A, go, back, (uint32_t)i, t);
        CK(hipStreamSynchronize(A));
        CK(hipStreamSynchronize(B));
        CK(hipMemcpy(hbuf, t, 16 * sizeof(u64), hipMemcpyDeviceToHost));
        if (hbuf[2] < (u64)i) { ++timeouts; continue; }
        rt.push_back((double)(hbuf[1] - hbuf[0]) * 0.01);
    }
    printf("timeouts (rccl): %d of %d\n", timeouts, iters);
    if (!rt.empty()) report("round trip with ncclAllReduce (1 rank, 660 floats)", rt);
    // the reference point: kernel -> all-reduce -> kernel on ONE stream, start of the first to start of the last
    for (int i = 0; i < iters; ++i) {
        hipLaunchKernelGGL(k_stamp, dim3(1), dim3(64), 0, B, t);
        ar(slot, slot, 660, ncclFloat32, ncclSum, comm, B);
        hipLaunchKernelGGL(k_stamp, dim3(1), dim3(64), 0, B, t + 1);
        CK(hipStreamSynchronize(B));
        CK(hipMemcpy(hbuf, t, 2 * sizeof(u64), hipMemcpyDeviceToHost));
        bnd_ar.push_back((double)(hbuf[1] - hbuf[0]) * 0.01);
    }
    report("same stream: kernel -> ncclAllReduce -> kernel", bnd_ar);
    destroy(comm);
    CK(hipFree(slot));
    CK(hipFree(t));
    CK(hipFree(go));
    CK(hipFree(back));
    return 0;
}

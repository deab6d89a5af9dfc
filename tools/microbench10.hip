// Host dispatch cost, HIP launch vs. raw AQL packets on an HSA queue of our own (tools/ only).
// The same two kernels (a 256-block "rollout-shaped" and an 8-block "finalize-shaped" one,
// with 1 KB and 0.5 KB argument blocks) alternate, each dependent on the one before
// (barrier bit), n pairs back to back:
//   HIP:  hipLaunchKernelGGL per kernel (kernel arguments copied per launch)
//   AQL:  kernel objects from this file's own code object (loaded through the HSA loader),
//         kernel arguments written once into device memory, per kernel only the 64 B packet
//         (system memory ring) and one doorbell store; "AQL-1" rings the doorbell once per
//         batch.  Completion: an HSA signal on the last packet.
//   hipcc --offload-arch=gfx950 -O3 --cuda-device-only -c --no-gpu-bundle-output -o tools/mb10.co tools/microbench10.hip
//   hipcc --offload-arch=gfx950 -O3 -o tools/mb10.bin tools/microbench10.hip -lhsa-runtime64 && ./tools/mb10.bin tools/mb10.co
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

struct ArgBig { unsigned v[256]; };
struct ArgMid { unsigned v[120]; };

extern "C" __global__ void __launch_bounds__(512) k_big(const ArgBig a, unsigned* out) {
    if (threadIdx.x == 0) out[blockIdx.x] = a.v[0] + a.v[255] + blockIdx.x;
}
extern "C" __global__ void __launch_bounds__(512) k_mid(const ArgMid a, unsigned* out) {
    if (threadIdx.x == 0) out[1024 + blockIdx.x] = a.v[0] + out[blockIdx.x];
}
// the dispatch id the command processor hands the wave (user SGPRs), per launch in order
// (the LLVM intrinsic by its name: clang has no builtin for it)
extern "C" __device__ unsigned long long mppi_dispatch_id(void) __asm("llvm.amdgcn.dispatch.id");
extern "C" __global__ void __launch_bounds__(64) k_id(unsigned long long* ids, unsigned slot) {
    if (threadIdx.x == 0 && blockIdx.x == 0) ids[slot] = mppi_dispatch_id();
}

#ifndef __HIP_DEVICE_COMPILE__
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)
#define HK(x) do { hsa_status_t s_ = (x); if (s_ != HSA_STATUS_SUCCESS) { const char* m_; hsa_status_string(s_, &m_); printf("%s: %s\n", #x, m_); return 1; } } while (0)
using clk = std::chrono::steady_clock;
static double us(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); }

static hsa_agent_t g_gpu;
static bool g_found = false;
static hsa_status_t find_gpu(hsa_agent_t a, void*) {
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_GPU && !g_found) { g_gpu = a; g_found = true; }
    return HSA_STATUS_SUCCESS;
}

struct KObj { uint64_t obj; uint32_t kas, gss, pss; };

static int get_kernel(hsa_executable_t ex, const char* name, KObj* k) {
    hsa_executable_symbol_t s;
    HK(hsa_executable_get_symbol_by_name(ex, name, &g_gpu, &s));
    HK(hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k->obj));
    HK(hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &k->kas));
    HK(hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &k->gss));
    HK(hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &k->pss));
    return 0;
}

static inline void put_packet(hsa_queue_t* q, const KObj& k, void* karg, uint32_t blocks, uint16_t threads,
                              hsa_signal_t done, bool ring, bool system_release) {
    const uint64_t idx = hsa_queue_add_write_index_relaxed(q, 1);
    while (idx - hsa_queue_load_read_index_scacquire(q) >= q->size) { }
    hsa_kernel_dispatch_packet_t* p = (hsa_kernel_dispatch_packet_t*)q->base_address + (idx & (q->size - 1));
    p->workgroup_size_x = threads; p->workgroup_size_y = 1; p->workgroup_size_z = 1; p->reserved0 = 0;
    p->grid_size_x = blocks * threads; p->grid_size_y = 1; p->grid_size_z = 1;
    p->private_segment_size = k.pss; p->group_segment_size = k.gss;
    p->kernel_object = k.obj; p->kernarg_address = karg; p->reserved2 = 0;
    p->completion_signal = done;
    const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) | (1 << HSA_PACKET_HEADER_BARRIER) |
                            (HSA_FENCE_SCOPE_AGENT << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                            ((system_release ? HSA_FENCE_SCOPE_SYSTEM : HSA_FENCE_SCOPE_AGENT) << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
    const uint32_t hs = (uint32_t)header | (1u << 16);   // setup: 1 dimension
    __atomic_store_n((uint32_t*)p, hs, __ATOMIC_RELEASE);
    if (ring) hsa_signal_store_relaxed(q->doorbell_signal, (hsa_signal_value_t)idx);
}

int main(int argc, char** argv) {
    if (argc < 2) { printf("usage: mb10.bin code_object\n"); return 1; }
    CK(hipSetDevice(0));
    unsigned* out;
    CK(hipMalloc(&out, 8192 * 4));
    CK(hipMemset(out, 0, 8192 * 4));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    ArgBig ab = {}; ArgMid am = {};
    for (int i = 0; i < 256; ++i) ab.v[i] = i;
    for (int i = 0; i < 120; ++i) am.v[i] = 7 * i;
    const int n = 2000, reps = 5;

    HK(hsa_init());
    HK(hsa_iterate_agents(find_gpu, nullptr));
    if (!g_found) { printf("no GPU agent\n"); return 1; }
    FILE* f = fopen(argv[1], "rb");
    if (!f) { printf("cannot open %s\n", argv[1]); return 1; }
    std::vector<char> co;
    { char buf[65536]; size_t r; while ((r = fread(buf, 1, sizeof buf, f)) > 0) co.insert(co.end(), buf, buf + r); fclose(f); }
    hsa_code_object_reader_t rd;
    HK(hsa_code_object_reader_create_from_memory(co.data(), co.size(), &rd));
    hsa_executable_t ex;
    HK(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &ex));
    HK(hsa_executable_load_agent_code_object(ex, g_gpu, rd, nullptr, nullptr));
    HK(hsa_executable_freeze(ex, nullptr));
    KObj kb, km;
    if (get_kernel(ex, "k_big.kd", &kb) || get_kernel(ex, "k_mid.kd", &km)) return 1;
    printf("k_big: kernarg %u B, lds %u; k_mid: kernarg %u B\n", kb.kas, kb.gss, km.kas);
    hsa_queue_t* q;
    HK(hsa_queue_create(g_gpu, 4096, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q));
    // kernel arguments: written once, in device memory
    char* kdev;
    CK(hipMalloc(&kdev, 4096));
    std::vector<char> kh(4096, 0);
    memcpy(kh.data(), &ab, sizeof ab); memcpy(kh.data() + sizeof ab, &out, 8);
    memcpy(kh.data() + 2048, &am, sizeof am); memcpy(kh.data() + 2048 + sizeof am, &out, 8);
    CK(hipMemcpy(kdev, kh.data(), 4096, hipMemcpyHostToDevice));
    hsa_signal_t done;
    HK(hsa_signal_create(1, 0, nullptr, &done));
    hsa_signal_t none = {0};

    for (int r = 0; r < reps; ++r) {
        // HIP
        for (int i = 0; i < 50; ++i) {
            hipLaunchKernelGGL(k_big, dim3(256), dim3(512), 0, s, ab, out);
            hipLaunchKernelGGL(k_mid, dim3(8), dim3(512), 0, s, am, out);
        }
        CK(hipStreamSynchronize(s));
        auto t0 = clk::now();
        for (int i = 0; i < n; ++i) {
            hipLaunchKernelGGL(k_big, dim3(256), dim3(512), 0, s, ab, out);
            hipLaunchKernelGGL(k_mid, dim3(8), dim3(512), 0, s, am, out);
        }
        auto t1 = clk::now();
        CK(hipStreamSynchronize(s));
        auto t2 = clk::now();
        printf("HIP    pair: enqueue %.2f us, total %.2f us per pair\n", us(t0, t1) / n, us(t0, t2) / n);
        // AQL, doorbell per packet / once per batch
        for (int mode = 0; mode < 2; ++mode) {
            hsa_signal_store_relaxed(done, 1);
            auto a0 = clk::now();
            for (int i = 0; i < n; ++i) {
                const bool last = i == n - 1;
                put_packet(q, kb, kdev, 256, 512, none, mode == 0, false);
                put_packet(q, km, kdev + 2048, 8, 512, last ? done : none, mode == 0 || last, last);
            }
            auto a1 = clk::now();
            while (hsa_signal_wait_scacquire(done, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_ACTIVE) != 0) { }
            auto a2 = clk::now();
            printf("AQL-%s pair: enqueue %.2f us, total %.2f us per pair\n", mode == 0 ? "n" : "1", us(a0, a1) / n,
                   us(a0, a2) / n);
        }
    }
    {   // dispatch ids: packet write index vs the id the waves see
        KObj ki;
        if (get_kernel(ex, "k_id.kd", &ki)) return 1;
        unsigned long long* ids;
        CK(hipMalloc(&ids, 64 * 8));
        CK(hipMemset(ids, 0, 64 * 8));
        struct { unsigned long long* p; unsigned slot; unsigned pad; } ia[8];
        char* kid;
        CK(hipMalloc(&kid, 8 * 64));
        for (int i = 0; i < 8; ++i) { ia[i].p = ids; ia[i].slot = (unsigned)i; ia[i].pad = 0; }
        std::vector<char> kb8(8 * 64, 0);
        for (int i = 0; i < 8; ++i) memcpy(kb8.data() + 64 * i, &ia[i], sizeof ia[i]);
        CK(hipMemcpy(kid, kb8.data(), kb8.size(), hipMemcpyHostToDevice));
        hsa_signal_store_relaxed(done, 1);
        std::vector<uint64_t> widx;
        for (int i = 0; i < 8; ++i) {
            widx.push_back(hsa_queue_load_write_index_relaxed(q));
            put_packet(q, ki, kid + 64 * i, 1, 64, i == 7 ? done : none, true, i == 7);
        }
        while (hsa_signal_wait_scacquire(done, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_ACTIVE) != 0) { }
        std::vector<unsigned long long> h8(8);
        CK(hipMemcpy(h8.data(), ids, 64, hipMemcpyDeviceToHost));
        for (int i = 0; i < 8; ++i) printf("packet write index %llu -> dispatch id %llu\n", (unsigned long long)widx[i], h8[i]);
    }
    // result check: k_mid reads what k_big wrote (dependency honoured)
    std::vector<unsigned> h(8192);
    CK(hipMemcpy(h.data(), out, 8192 * 4, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int b = 0; b < 256; ++b) bad += h[b] != 0u + 255u + (unsigned)b;
    for (int b = 0; b < 8; ++b) bad += h[1024 + b] != 0u + h[b];
    printf("check: %s\n", bad ? "MISMATCH" : "ok");
    hsa_signal_destroy(done);
    hsa_queue_destroy(q);
    hsa_executable_destroy(ex);
    hsa_code_object_reader_destroy(rd);
    return bad != 0;
}
#endif

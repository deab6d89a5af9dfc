// mppi_aql.cpp -- native dispatch of the control step: raw AQL kernel-dispatch packets on an
// HSA queue of the engine's own (see mppi_aql.h).
//
// Why: hipLaunchKernel costs the host 2.4-3.3 us per launch on the MI355X boxes (kernel-
// argument marshalling and a device-memory copy of the argument block each time), and a
// (rollout, finalize) pair alternating 8-9 us (tools/microbench10.hip,
// profiles/r03/microbench_aql_dispatch.txt) -- the same order as the GPU's 9.6 us C3 step,
// so mppi_run_steps ran host-bound in some batches (profiles/r03/final_r03b: 5.2-8.2 us of
// enqueue per step, 9.96-10.9 us per step).  Here the argument blocks are written once into
// device memory; per step the host writes two 64 B packets into the queue's ring and stores
// the doorbell: 0.57 us per pair, and the GPU side runs the dependent pair back to back.
//
// The kernels are the library's own: build.py writes each kernel translation unit's gfx950
// code object next to the library (<library>.<unit>.co); they are loaded once per device
// through the HSA loader, and a launch's symbol comes from the launcher itself (mppi_device.h
// go(), capture mode), so native and HIP dispatch run the same code with the same arguments.
#include "mppi_aql.h"

#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <immintrin.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <map>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace {

thread_local mppi::LaunchDesc* t_capture = nullptr;

struct Kern {
    uint64_t obj = 0;
    uint32_t kas = 0, gss = 0, pss = 0;
};

// one device's loaded code objects (process-wide; executables live as long as the process)
struct Device {
    bool tried = false, ok = false;
    std::string why;
    hsa_agent_t agent{};
    std::vector<hsa_executable_t> exes;
    std::unordered_map<std::string, Kern> syms;
    // device memory the host can write (large BAR): the control calls' argument blocks
    bool vis_pool_ok = false;
    hsa_amd_memory_pool_t vis_pool{};
    hsa_agent_t cpu{};
    std::string vis_pool_kind;
    hsa_amd_hdp_flush_t hdp{};
};

hsa_status_t first_cpu(hsa_agent_t a, void* data) {
    hsa_device_type_t t;
    if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_CPU) {
        *(hsa_agent_t*)data = a;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}

struct PoolPick {
    hsa_agent_t cpu;
    int best_rank;   // 3 kernarg-init, 2 fine-grained, 1 coarse-grained (CPU-accessible in every case)
    hsa_amd_memory_pool_t pool;
};
hsa_status_t pick_pool(hsa_amd_memory_pool_t pool, void* data) {
    auto* pk = (PoolPick*)data;
    hsa_amd_segment_t seg;
    uint32_t flags = 0;
    bool alloc = false;
    hsa_amd_memory_pool_access_t acc = HSA_AMD_MEMORY_POOL_ACCESS_NEVER_ALLOWED;
    if (hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) != HSA_STATUS_SUCCESS ||
        seg != HSA_AMD_SEGMENT_GLOBAL)
        return HSA_STATUS_SUCCESS;
    if (hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags) != HSA_STATUS_SUCCESS ||
        hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc) != HSA_STATUS_SUCCESS ||
        !alloc)
        return HSA_STATUS_SUCCESS;
    if (hsa_amd_agent_memory_pool_get_info(pk->cpu, pool, HSA_AMD_AGENT_MEMORY_POOL_INFO_ACCESS, &acc) !=
            HSA_STATUS_SUCCESS || acc == HSA_AMD_MEMORY_POOL_ACCESS_NEVER_ALLOWED)
        return HSA_STATUS_SUCCESS;
    const int rank = (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT) ? 3
                     : (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED) ? 2 : 1;
    if (rank > pk->best_rank) { pk->best_rank = rank; pk->pool = pool; }
    return HSA_STATUS_SUCCESS;
}
std::mutex g_mu;
std::map<int, Device> g_dev;

const char* const kUnits[] = {"mppi_rollout_drone", "mppi_rollout_arm", "mppi_rollout_arm_h32", "mppi_rollout_arm32",
                              "mppi_rollout_wb",
                              "mppi_rollout_quad", "mppi_finalize"};

std::string hsa_msg(hsa_status_t s) {
    const char* m = nullptr;
    if (hsa_status_string(s, &m) != HSA_STATUS_SUCCESS || !m) return "HSA status " + std::to_string((int)s);
    return m;
}

struct AgentMatch {
    uint32_t domain, bdf;
    bool found;
    hsa_agent_t agent;
};
hsa_status_t match_agent(hsa_agent_t a, void* data) {
    auto* m = (AgentMatch*)data;
    hsa_device_type_t t;
    if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS || t != HSA_DEVICE_TYPE_GPU)
        return HSA_STATUS_SUCCESS;
    uint32_t bdf = 0, dom = 0;
    if (hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
    if (hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom) != HSA_STATUS_SUCCESS) dom = 0;
    if (bdf == m->bdf && dom == m->domain && !m->found) { m->agent = a; m->found = true; }
    return HSA_STATUS_SUCCESS;
}

// directory + stem of this library: the code objects sit next to it
bool library_stem(std::string* stem) {
    Dl_info info;
    if (!dladdr((void*)&match_agent, &info) || !info.dli_fname) return false;
    std::string p = info.dli_fname;
    if (p.size() > 3 && p.compare(p.size() - 3, 3, ".so") == 0) p.resize(p.size() - 3);
    *stem = p;
    return true;
}

bool read_file(const std::string& path, std::vector<char>* out) {
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) return false;
    char buf[1 << 16];
    size_t r;
    while ((r = fread(buf, 1, sizeof buf, f)) > 0) out->insert(out->end(), buf, buf + r);
    fclose(f);
    return !out->empty();
}

// caller holds g_mu
Device* device_for(int ordinal) {
    Device& d = g_dev[ordinal];
    if (d.tried) return &d;
    d.tried = true;
    char bus[64] = {0};
    unsigned dom = 0, b = 0, dv = 0, fn = 0;
    if (hipDeviceGetPCIBusId(bus, (int)sizeof bus, ordinal) != hipSuccess ||
        sscanf(bus, "%x:%x:%x.%x", &dom, &b, &dv, &fn) != 4) {
        d.why = "no PCI bus id for HIP device " + std::to_string(ordinal);
        return &d;
    }
    hsa_status_t st = hsa_init();   // reference-counted: HIP initialised the runtime already
    if (st != HSA_STATUS_SUCCESS) { d.why = "hsa_init: " + hsa_msg(st); return &d; }
    AgentMatch m{dom, (b << 8) | (dv << 3) | fn, false, {}};
    hsa_iterate_agents(match_agent, &m);
    if (!m.found) { d.why = std::string("no HSA agent at ") + bus; return &d; }
    d.agent = m.agent;
    std::string stem;
    if (!library_stem(&stem)) { d.why = "cannot locate the library's own path"; return &d; }
    for (const char* u : kUnits) {
        const std::string path = stem + "." + u + ".co";
        std::vector<char> co;
        if (!read_file(path, &co)) { d.why = "missing code object " + path + " (python -m quadrotor_manipulator_mppi_amd.build)"; return &d; }
        hsa_code_object_reader_t rd;
        hsa_executable_t ex;
        if ((st = hsa_code_object_reader_create_from_memory(co.data(), co.size(), &rd)) != HSA_STATUS_SUCCESS ||
            (st = hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &ex)) !=
                HSA_STATUS_SUCCESS) {
            d.why = "loading " + path + ": " + hsa_msg(st);
            return &d;
        }
        // the reader's buffer must outlive the executable: keep it (process lifetime)
        static std::vector<std::vector<char>> keep;
        keep.push_back(std::move(co));
        if ((st = hsa_executable_load_agent_code_object(ex, d.agent, rd, nullptr, nullptr)) != HSA_STATUS_SUCCESS ||
            (st = hsa_executable_freeze(ex, nullptr)) != HSA_STATUS_SUCCESS) {
            d.why = "loading " + path + ": " + hsa_msg(st);
            return &d;
        }
        d.exes.push_back(ex);
    }
    // a GPU memory pool the host can write directly (large BAR), for the control calls'
    // rollout arguments; without one they go to pinned host memory
    hsa_agent_t cpu{};
    if (hsa_iterate_agents(first_cpu, &cpu) == HSA_STATUS_INFO_BREAK && !getenv("MPPI_AQL_CALL_HOSTMEM")) {
        PoolPick pk{cpu, 0, {}};
        hsa_amd_agent_iterate_memory_pools(d.agent, pick_pool, &pk);
        if (pk.best_rank > 0 &&
            hsa_agent_get_info(d.agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_HDP_FLUSH, &d.hdp) == HSA_STATUS_SUCCESS &&
            d.hdp.HDP_MEM_FLUSH_CNTL) {
            d.vis_pool_ok = true;
            d.vis_pool = pk.pool;
            d.cpu = cpu;
            d.vis_pool_kind = pk.best_rank == 3 ? "device kernarg pool" : pk.best_rank == 2 ? "device fine-grained"
                                                                                             : "device coarse-grained";
        }
    }
    d.ok = true;
    return &d;
}

// caller holds g_mu
bool lookup(Device* d, const char* name, Kern* k, std::string* err) {
    std::string sym = std::string(name) + ".kd";
    auto it = d->syms.find(sym);
    if (it != d->syms.end()) { *k = it->second; return true; }
    for (hsa_executable_t ex : d->exes) {
        hsa_executable_symbol_t s;
        if (hsa_executable_get_symbol_by_name(ex, sym.c_str(), &d->agent, &s) != HSA_STATUS_SUCCESS) continue;
        Kern r;
        if (hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &r.obj) != HSA_STATUS_SUCCESS ||
            hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &r.kas) != HSA_STATUS_SUCCESS ||
            hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &r.gss) != HSA_STATUS_SUCCESS ||
            hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &r.pss) != HSA_STATUS_SUCCESS)
            break;
        d->syms[sym] = r;
        *k = r;
        return true;
    }
    *err = "kernel " + sym + " not in the code objects";
    return false;
}

}  // namespace

extern "C" mppi::LaunchDesc* mppi_capture_target(void) { return t_capture; }

namespace mppi_aql {

constexpr uint32_t kQueueSize = 4096;   // packets (256 KB ring)
constexpr size_t kArgSlot = 4096;       // bytes per argument block: [rollout | finalize | call finalize]
// control calls rotate through this many rollout argument blocks (each call a fresh address,
// as HIP's own kernel-argument ring: no copy of an earlier call's block can sit in a cache)
constexpr uint32_t kCallSlots = 16;
// the batch path's (rollout, finalize) argument pair: re-uploads rotate over this many pairs
constexpr uint32_t kBatchSlots = 4;

struct Step {
    Device* dev = nullptr;
    hsa_queue_t* q = nullptr;
    hsa_signal_t done{0};                 // outstanding batches; each batch's last packet decrements it
    std::atomic<int> qerr{0};             // HSA status of an asynchronous queue error
    unsigned char* d_args = nullptr;      // device: the control call's finalize at 0, then kBatchSlots
                                          // (rollout, finalize) pairs for batches
    uint32_t batch_slot = 0;              // the pair the batches use now
    unsigned char* h_call = nullptr;      // the control calls' rollout arguments: kCallSlots blocks in
    unsigned char* h_call_dev = nullptr;  //   host-writable device memory (else pinned host memory),
    bool call_vis = false;                //   host and device addresses; call_vis = device memory
    uint32_t call_slot = 0;
    mppi::LaunchDesc fin_call{};          // what the call's finalize block holds
    Kern kc_r, kc_f;
    bool call_valid = false;
    bool call_unread = false;             // the last call's outputs not yet seen (step_call_read)
    mppi::LaunchDesc roll{}, fin{};       // what the device blocks hold (step word as uploaded)
    Kern kr, kf;
    uint32_t step_off = 0, step_word = 0; // the resident rollout's dispatch-id relative step word
    bool valid = false;
    int64_t outstanding = 0;              // batches dispatched and not yet waited for
    unsigned char* d_touch = nullptr;     // step_touch: two 64 B argument blocks, then its 16 B output
    Kern kt;
    // the queue is single-producer: every function below that writes packets or waits holds this
    // (recursive: step_call and step_prepare wait inside), so the engine's prewarm thread
    // (step_touch) and the control calls never write packets at the same time
    std::recursive_mutex mu;
};

void set_capture(mppi::LaunchDesc* d) { t_capture = d; }

static void queue_error(hsa_status_t status, hsa_queue_t*, void* data) {
    ((Step*)data)->qerr.store((int)status);
}

static bool probe_dispatch_ids(Step* s, std::string* why);

Step* step_create(int device, std::string* why) {
    Device* d = nullptr;
    {   // (g_mu only around the device table: the probe below takes it for its symbol lookup)
        std::lock_guard<std::mutex> lk(g_mu);
        d = device_for(device);
        if (!d->ok) { *why = d->why; return nullptr; }
    }
    Step* s = new Step();
    s->dev = d;
    hsa_status_t st = hsa_queue_create(d->agent, kQueueSize, HSA_QUEUE_TYPE_SINGLE, queue_error, s, UINT32_MAX,
                                       UINT32_MAX, &s->q);
    if (st != HSA_STATUS_SUCCESS) { *why = "hsa_queue_create: " + hsa_msg(st); delete s; return nullptr; }
    if ((st = hsa_signal_create(0, 0, nullptr, &s->done)) != HSA_STATUS_SUCCESS) {
        *why = "hsa_signal_create: " + hsa_msg(st);
        hsa_queue_destroy(s->q);
        delete s;
        return nullptr;
    }
    if (d->vis_pool_ok) {   // host-writable device memory for the calls' argument blocks
        void* p = nullptr;
        if (hsa_amd_memory_pool_allocate(d->vis_pool, kCallSlots * kArgSlot, 0, &p) == HSA_STATUS_SUCCESS) {
            if (hsa_amd_agents_allow_access(1, &d->cpu, nullptr, p) == HSA_STATUS_SUCCESS) {
                s->h_call = s->h_call_dev = (unsigned char*)p;
                s->call_vis = true;
            } else {
                hsa_amd_memory_pool_free(p);
            }
        }
    }
    if (hipMalloc(&s->d_args, (1 + 2 * kBatchSlots) * kArgSlot) != hipSuccess ||
        (!s->call_vis &&
         (hipHostMalloc((void**)&s->h_call, kCallSlots * kArgSlot, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
          hipHostGetDevicePointer((void**)&s->h_call_dev, s->h_call, 0) != hipSuccess))) {
        *why = "allocating the argument blocks failed";
        if (s->d_args) (void)hipFree(s->d_args);
        if (s->h_call) { if (s->call_vis) hsa_amd_memory_pool_free(s->h_call); else (void)hipHostFree(s->h_call); }
        hsa_signal_destroy(s->done);
        hsa_queue_destroy(s->q);
        delete s;
        return nullptr;
    }
    if (!probe_dispatch_ids(s, why)) {   // the queue's dispatch ids are not its packet indices
        if (!step_destroy(s)) *why += " (and the probe's queue did not drain)";
        return nullptr;
    }
    // step_touch's argument blocks and scratch output, here on the creating thread (whose device
    // is the queue's): the prewarm thread that touches never selects a device
    {
        std::lock_guard<std::mutex> lk(g_mu);
        if (!lookup(s->dev, "k_dispatch_probe", &s->kt, why)) { (void)step_destroy(s); return nullptr; }
    }
    unsigned char h[128] = {};
    if (hipMalloc(&s->d_touch, 3 * 64) != hipSuccess) {
        s->d_touch = nullptr;
        *why = "touch buffer";
        (void)step_destroy(s);
        return nullptr;
    }
    unsigned char* outs[2] = {s->d_touch + 128, s->d_touch + 136};
    memcpy(h, &outs[0], 8);
    memcpy(h + 64, &outs[1], 8);
    if (hipMemcpy(s->d_touch, h, sizeof h, hipMemcpyHostToDevice) != hipSuccess) {
        *why = "touch upload";
        (void)step_destroy(s);
        return nullptr;
    }
    return s;
}

bool step_destroy(Step* s) {
    if (!s) return true;
    std::string e;
    if (s->outstanding && step_wait(s, 60000, &e) != 0) {
        // kernels may still run against the argument blocks (and the engine's buffers): stop the
        // queue and leak its memory rather than free what the device may still touch
        hsa_queue_inactivate(s->q);
        fprintf(stderr, "[mppi aql] queue did not drain at destroy (%s): its buffers are leaked\n", e.c_str());
        return false;
    }
    hsa_signal_destroy(s->done);
    hsa_queue_destroy(s->q);
    (void)hipFree(s->d_args);
    if (s->d_touch) (void)hipFree(s->d_touch);
    if (s->call_vis) hsa_amd_memory_pool_free(s->h_call); else (void)hipHostFree(s->h_call);
    delete s;
    return true;
}

bool step_busy(Step* s) {
    if (!s) return false;
    std::lock_guard<std::recursive_mutex> qlk(s->mu);
    return s->outstanding > 0;
}

// a launch's argument block against the kernel's: only explicit arguments (no hidden ones),
// LDS within the CU's 160 KB.  (Scratch: the packet carries the kernel's private segment size;
// the runtime backs the queue's scratch on demand, as for HIP's own queues.)
static bool check_launch(const mppi::LaunchDesc& l, const Kern& k, std::string* err) {
    if (k.kas < l.arg_bytes || k.kas - l.arg_bytes >= 16 || k.kas > kArgSlot) {
        *err = std::string(l.symbol) + ": kernel-argument segment " + std::to_string(k.kas) + " B vs " +
               std::to_string(l.arg_bytes) + " B packed";
        return false;
    }
    if (k.gss + l.lds > 160 * 1024) { *err = std::string(l.symbol) + ": LDS over 160 KB"; return false; }
    for (int i = 0; i < 3; ++i)
        if (l.grid[i] == 0 || l.block[i] == 0) { *err = std::string(l.symbol) + ": empty grid"; return false; }
    if ((uint64_t)l.block[0] * l.block[1] * l.block[2] > 1024) { *err = "block over 1024 threads"; return false; }
    return true;
}

static bool same_launch(const mppi::LaunchDesc& a, const mppi::LaunchDesc& b, uint32_t skip_off) {
    if (strcmp(a.symbol, b.symbol) != 0 || memcmp(a.grid, b.grid, sizeof a.grid) != 0 ||
        memcmp(a.block, b.block, sizeof a.block) != 0 || a.lds != b.lds || a.arg_bytes != b.arg_bytes)
        return false;
    if (skip_off >= a.arg_bytes || a.arg_bytes - skip_off < 4) return memcmp(a.args, b.args, a.arg_bytes) == 0;
    return memcmp(a.args, b.args, skip_off) == 0 &&
           memcmp(a.args + skip_off + 4, b.args + skip_off + 4, a.arg_bytes - skip_off - 4) == 0;
}

static unsigned char* batch_args(Step* s) { return s->d_args + (1 + 2 * (size_t)s->batch_slot) * kArgSlot; }

int step_prepare(Step* s, const mppi::LaunchDesc& roll, const mppi::LaunchDesc& fin, uint32_t step,
                 uint32_t step_off, std::string* err) {
    std::lock_guard<std::recursive_mutex> qlk(s->mu);
    // the next rollout's packet index (the queue holds (rollout, finalize) pairs only, so
    // rollouts sit at indices of one parity and (index >> 1) counts pairs)
    const uint32_t word = step - (uint32_t)(hsa_queue_load_write_index_relaxed(s->q) >> 1);
    if (s->valid && s->step_word == word && s->step_off == step_off && same_launch(roll, s->roll, step_off) &&
        same_launch(fin, s->fin, ~0u))
        return 0;
    if (getenv("MPPI_AQL_PROFILE") && s->valid) {   // diagnostics: why the blocks are re-uploaded
        int first = -1;
        for (uint32_t i = 0; i < roll.arg_bytes && i < s->roll.arg_bytes; ++i)
            if ((i < step_off || i >= step_off + 4) && roll.args[i] != s->roll.args[i]) { first = (int)i; break; }
        int ffirst = -1;
        for (uint32_t i = 0; i < fin.arg_bytes && i < s->fin.arg_bytes; ++i)
            if (fin.args[i] != s->fin.args[i]) { ffirst = (int)i; break; }
        fprintf(stderr, "[mppi aql] re-upload: word %u vs %u, rollout args differ at %d, finalize at %d, sym %d/%d\n", word,
                s->step_word, first, ffirst, strcmp(roll.symbol, s->roll.symbol), strcmp(fin.symbol, s->fin.symbol));
    }
    Kern kr, kf;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        if (!lookup(s->dev, roll.symbol, &kr, err) || !lookup(s->dev, fin.symbol, &kf, err)) return -2;
    }
    if (!check_launch(roll, kr, err) || !check_launch(fin, kf, err)) return -2;
    if (step_off + 4 > roll.arg_bytes) { *err = "step counter outside the rollout's arguments"; return -2; }
    // the queue may still be reading the blocks about to be overwritten
    if (s->outstanding && step_wait(s, 60000, err) != 0) return -1;
    std::vector<unsigned char> h(2 * kArgSlot, 0);
    memcpy(h.data(), roll.args, roll.arg_bytes);
    memcpy(h.data() + step_off, &word, 4);
    memcpy(h.data() + kArgSlot, fin.args, fin.arg_bytes);
    // a fresh pair of blocks for every upload (no cached copy of an earlier upload can be read)
    s->batch_slot = (s->batch_slot + 1) % kBatchSlots;
    if (hipMemcpy(batch_args(s), h.data(), h.size(), hipMemcpyHostToDevice) != hipSuccess) {
        *err = "uploading the argument blocks failed";
        s->valid = false;
        return -1;
    }
    s->roll = roll;
    s->fin = fin;
    s->kr = kr;
    s->kf = kf;
    s->step_off = step_off;
    s->step_word = word;
    s->valid = true;
    return 0;
}

// One kernel-dispatch packet: body first, then header + setup in one release store (the
// packet processor may read the slot as soon as the header says KERNEL_DISPATCH).
// Packet fence scopes (0 none, 1 agent, 2 system): rollout acquire, rollout release, finalize
// acquire, finalize release.  What one kernel of the step reads from the other is written
// through at device scope and drained before the writing waves end (the rollouts' record
// bodies, headers and handed-over vehicle constants, mppi_rollout.h drain_stores; the
// finalize's u_prev), and read with device-scope loads that bypass the L1 (mppi_device.h
// ld_dev / kAuxDev).  So no packet of a batch needs a release, whose end-of-kernel L2
// writeback cost up to ~0.8 us per C3 step, and only a submission's FIRST packet acquires
// (agent scope: what the host and the HIP stream wrote since the last batch -- argument
// blocks, state, target), which saves ~0.28 us per C3 step over an acquire on every packet
// (tools/probes.py fences).  Nothing a batch writes to device memory stays dirty in an L2
// either: the values read only after a batch (the costs S, the readback copies of w_eps, the
// stored noise) are written through at device scope as well (mppi_device.h st_dev / st_dev_run).
// Plain stores would leave them dirty across the release-free packets, and since which XCD runs
// a block is not fixed from step to step (MI355X_MICROARCH.md, "Workgroup dispatch, XCD
// placement"), two L2s could hold dirty copies of one line from different steps, written back in
// an undefined order (tests/test_gpu_aql.py, the small-K batch readback test).
// Diagnostics: MPPI_AQL_FENCES = four digits for the packets after the first.
static int g_fence[4] = {-1, -1, -1, -1};
static void load_fences() {
    if (g_fence[0] >= 0) return;
    const char* f = getenv("MPPI_AQL_FENCES");
    const char* def = "0000";
    for (int i = 0; i < 4; ++i) g_fence[i] = (f && strlen(f) == 4 && f[i] >= '0' && f[i] <= '2') ? f[i] - '0' : def[i] - '0';
}
static const int kScope[3] = {HSA_FENCE_SCOPE_NONE, HSA_FENCE_SCOPE_AGENT, HSA_FENCE_SCOPE_SYSTEM};

static inline void put(hsa_queue_t* q, const Kern& k, const mppi::LaunchDesc& l, void* args, hsa_signal_t sig,
                       int acquire, int release, bool barrier = true) {
    const uint64_t idx = hsa_queue_add_write_index_relaxed(q, 1);
    while (idx - hsa_queue_load_read_index_scacquire(q) >= q->size) _mm_pause();
    auto* p = (hsa_kernel_dispatch_packet_t*)q->base_address + (idx & (q->size - 1));
    p->workgroup_size_x = (uint16_t)l.block[0];
    p->workgroup_size_y = (uint16_t)l.block[1];
    p->workgroup_size_z = (uint16_t)l.block[2];
    p->reserved0 = 0;
    p->grid_size_x = l.grid[0] * l.block[0];
    p->grid_size_y = l.grid[1] * l.block[1];
    p->grid_size_z = l.grid[2] * l.block[2];
    p->private_segment_size = k.pss;
    p->group_segment_size = k.gss + l.lds;
    p->kernel_object = k.obj;
    p->kernarg_address = args;
    p->reserved2 = 0;
    p->completion_signal = sig;
    // each kernel waits for the one before (barrier bit) and sees its writes (agent-scope
    // acquire); the batch's last one releases to system scope (the outputs in host memory)
    const uint16_t header =
        (uint16_t)((HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) | ((barrier ? 1 : 0) << HSA_PACKET_HEADER_BARRIER) |
                   (kScope[acquire] << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                   (kScope[release] << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
    const uint32_t setup = 3u << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
    __atomic_store_n((uint32_t*)p, (uint32_t)header | (setup << 16), __ATOMIC_RELEASE);
}

// The rollout's Philox step is arg + (dispatch id >> 1) under native dispatch: this holds only
// while the dispatch id the packet processor hands the waves equals the packet's index in this
// queue.  A tool that intercepts the queue (rocprofv3 --pmc injects its counter packets, and the
// packets the application writes are copied to another queue) breaks that silently: steps would
// repeat or be skipped.  So every new queue first runs two probe packets (k_dispatch_probe writes
// its dispatch id) and is used only when both ids equal their packet indices; otherwise the
// engine keeps HIP launches (mppi_dispatch_info says why).
static bool probe_dispatch_ids(Step* s, std::string* why) {
    Kern k;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        if (!lookup(s->dev, "k_dispatch_probe", &k, why)) return false;
    }
    unsigned long long* d_ids = nullptr;
    if (hipMalloc(&d_ids, 2 * sizeof(unsigned long long)) != hipSuccess) { *why = "probe buffer"; return false; }
    // the two packets' argument blocks (one pointer each) in the batch slots' space
    unsigned long long* args[2] = {d_ids, d_ids + 1};
    std::vector<unsigned char> h(2 * kArgSlot, 0);
    memcpy(h.data(), &args[0], 8);
    memcpy(h.data() + kArgSlot, &args[1], 8);
    bool ok = hipMemset(d_ids, 0xFF, 2 * sizeof(unsigned long long)) == hipSuccess &&
              hipMemcpy(s->d_args + kArgSlot, h.data(), h.size(), hipMemcpyHostToDevice) == hipSuccess;
    if (!ok) { (void)hipFree(d_ids); *why = "probe upload"; return false; }
    mppi::LaunchDesc l{};
    snprintf(l.symbol, sizeof l.symbol, "k_dispatch_probe");
    l.grid[0] = l.grid[1] = l.grid[2] = 1;
    l.block[0] = 64; l.block[1] = l.block[2] = 1;
    l.arg_bytes = 8;
    uint64_t idx[2];
    hsa_signal_add_relaxed(s->done, 1);
    ++s->outstanding;
    for (int i = 0; i < 2; ++i) {
        idx[i] = hsa_queue_load_write_index_relaxed(s->q);
        put(s->q, k, l, s->d_args + (1 + i) * kArgSlot, i == 1 ? s->done : hsa_signal_t{0}, 2, i == 1 ? 2 : 0);
    }
    hsa_signal_store_screlease(s->q->doorbell_signal, (hsa_signal_value_t)idx[1]);
    std::string err;
    unsigned long long got[2] = {~0ull, ~0ull};
    if (step_wait(s, 10000, &err) != 0) {   // (buffer leaked: may be in use)
        char b[160];
        snprintf(b, sizeof b, " [signal %ld, read index %llu, write index %llu]", (long)hsa_signal_load_relaxed(s->done),
                 (unsigned long long)hsa_queue_load_read_index_relaxed(s->q),
                 (unsigned long long)hsa_queue_load_write_index_relaxed(s->q));
        *why = "dispatch-id probe: " + err + b;
        return false;
    }
    ok = hipMemcpy(got, d_ids, sizeof got, hipMemcpyDeviceToHost) == hipSuccess;
    (void)hipFree(d_ids);
    if (!ok) { *why = "dispatch-id probe readback"; return false; }
    if (const char* sk = getenv("MPPI_AQL_PROBE_SKEW")) {   // test hook: the refusal path (tests/test_gpu_aql.py)
        got[0] += (unsigned long long)atoll(sk);
        got[1] += (unsigned long long)atoll(sk);
    }
    if (got[0] != idx[0] || got[1] != idx[1]) {
        char b[256];
        snprintf(b, sizeof b, "the queue's dispatch ids (%llu, %llu) are not its packet indices (%llu, %llu): "
                 "intercepted by a tool", got[0], got[1], (unsigned long long)idx[0], (unsigned long long)idx[1]);
        *why = b;
        return false;
    }
    return true;
}

std::unique_lock<std::recursive_mutex> step_guard(Step* s) { return std::unique_lock<std::recursive_mutex>(s->mu); }

int step_dispatch(Step* s, int n, std::string* err, bool overlap) {
    std::lock_guard<std::recursive_mutex> qlk(s->mu);
    if (!s->valid) { *err = "step_dispatch before step_prepare"; return -1; }
    if (n <= 0) return 0;
    if (s->qerr.load()) { *err = "native queue error: " + hsa_msg((hsa_status_t)s->qerr.load()); return -1; }
    hsa_signal_add_relaxed(s->done, 1);   // this batch's completion
    ++s->outstanding;
    const hsa_signal_t none{0};
    void* ra = batch_args(s);
    void* fa = batch_args(s) + kArgSlot;
    load_fences();
    for (int i = 0; i < n; ++i) {
        const bool last = i == n - 1;
        put(s->q, s->kr, s->roll, ra, none, i == 0 ? std::max(1, g_fence[0]) : g_fence[0], g_fence[1],
            !(overlap && i > 0));
        put(s->q, s->kf, s->fin, fa, last ? s->done : none, g_fence[2], last ? 2 : g_fence[3]);
        // the doorbell takes the index of the last packet written
        hsa_signal_store_screlease(s->q->doorbell_signal, (hsa_signal_value_t)hsa_queue_load_write_index_relaxed(s->q) - 1);
    }
    return 0;
}

int step_call(Step* s, const mppi::LaunchDesc& roll, const mppi::LaunchDesc& fin, uint32_t step,
              uint32_t step_off, uint32_t seq_off, uint32_t* seq, std::string* err) {
    std::lock_guard<std::recursive_mutex> qlk(s->mu);
    if (s->qerr.load()) { *err = "native queue error: " + hsa_msg((hsa_status_t)s->qerr.load()); return -1; }
    static const bool prof = getenv("MPPI_AQL_PROFILE") != nullptr;   // diagnostics: phases of a call
    static double pacc[4] = {0, 0, 0, 0};
    static long pcn = 0;
    auto now = [] { return std::chrono::steady_clock::now(); };
    const auto p0 = now();
    Kern kr, kf;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        if (!lookup(s->dev, roll.symbol, &kr, err) || !lookup(s->dev, fin.symbol, &kf, err)) return -2;
    }
    if (!check_launch(roll, kr, err) || !check_launch(fin, kf, err)) return -2;
    if (step_off + 4 > roll.arg_bytes || seq_off + 4 > roll.arg_bytes) { *err = "call words outside the arguments"; return -2; }
    // the host block is rewritten below: the previous call's rollout must have read it.  The
    // engine reads every call's outputs before the next call (its flag: that rollout has run),
    // so only an unread call waits; a queued batch does not read this block.
    if (s->call_unread && s->outstanding && step_wait(s, 60000, err) != 0) return -1;
    if (!s->call_valid || !same_launch(fin, s->fin_call, ~0u)) {
        if (s->outstanding && step_wait(s, 60000, err) != 0) return -1;
        std::vector<unsigned char> h(kArgSlot, 0);
        memcpy(h.data(), fin.args, fin.arg_bytes);
        if (hipMemcpy(s->d_args, h.data(), kArgSlot, hipMemcpyHostToDevice) != hipSuccess) {
            *err = "uploading the call's finalize arguments failed";
            s->call_valid = false;
            return -1;
        }
        s->fin_call = fin;
        s->call_valid = true;
    }
    s->kc_r = kr;
    s->kc_f = kf;
    const uint64_t r = hsa_queue_load_write_index_relaxed(s->q);   // this call's rollout packet
    const uint32_t word = step - (uint32_t)(r >> 1);
    *seq = 0x80000000u | (uint32_t)(r >> 1);
    const uint32_t slot = s->call_slot++ % kCallSlots;
    unsigned char* blk = s->h_call + (size_t)slot * kArgSlot;
    alignas(16) unsigned char tmp[kArgSlot];
    memcpy(tmp, roll.args, roll.arg_bytes);
    memcpy(tmp + step_off, &word, 4);
    memcpy(tmp + seq_off, seq, 4);
    const uint32_t nb = (roll.arg_bytes + 63) & ~63u;   // whole 64 B lines
    memset(tmp + roll.arg_bytes, 0, nb - roll.arg_bytes);
    const auto p1 = now();
    memcpy(blk, tmp, nb);
    const auto p2 = now();
    if (s->call_vis) {
        // device memory written through the BAR: drain the write-combining buffers, flush the
        // host data path and read the flush register back (the writes have landed) before the
        // packet can send the command processor to the block
        _mm_sfence();
        volatile uint32_t* f = s->dev->hdp.HDP_MEM_FLUSH_CNTL;
        *f = 1u;
        (void)*f;
    }
    std::atomic_thread_fence(std::memory_order_release);
    const auto p3 = now();
    hsa_signal_add_relaxed(s->done, 1);
    ++s->outstanding;
    s->call_unread = true;
    const hsa_signal_t none{0};
    load_fences();
    put(s->q, kr, roll, s->h_call_dev + (size_t)slot * kArgSlot, none, std::max(1, g_fence[0]), g_fence[1]);
    put(s->q, kf, fin, s->d_args, s->done, g_fence[2], 2);
    hsa_signal_store_screlease(s->q->doorbell_signal, (hsa_signal_value_t)hsa_queue_load_write_index_relaxed(s->q) - 1);
    if (prof) {
        const auto p4 = now();
        pacc[0] += std::chrono::duration<double, std::micro>(p1 - p0).count();
        pacc[1] += std::chrono::duration<double, std::micro>(p2 - p1).count();
        pacc[2] += std::chrono::duration<double, std::micro>(p3 - p2).count();
        pacc[3] += std::chrono::duration<double, std::micro>(p4 - p3).count();
        if (++pcn % 1000 == 0)
            fprintf(stderr, "[mppi aql] step_call (us): lookups+checks %.2f  block write %.2f  flush+readback %.2f  packets %.2f\n",
                    pacc[0] / pcn, pacc[1] / pcn, pacc[2] / pcn, pacc[3] / pcn);
    }
    return 0;
}

int step_touch(Step* s, bool if_free, std::string* err) {
    std::unique_lock<std::recursive_mutex> qlk(s->mu, std::defer_lock);
    if (if_free) {
        if (!qlk.try_lock()) return 1;
    } else {
        qlk.lock();
    }
    if (s->qerr.load()) { *err = "native queue error: " + hsa_msg((hsa_status_t)s->qerr.load()); return -1; }
    mppi::LaunchDesc l{};
    l.grid[0] = l.grid[1] = l.grid[2] = 1;
    l.block[0] = 64; l.block[1] = l.block[2] = 1;
    l.arg_bytes = 8;
    // a pair, so rollouts keep their packet-index parity; the next batch re-uploads its step word
    hsa_signal_add_relaxed(s->done, 1);
    ++s->outstanding;
    put(s->q, s->kt, l, s->d_touch, hsa_signal_t{0}, 1, 0);
    put(s->q, s->kt, l, s->d_touch + 64, s->done, 0, 0);
    hsa_signal_store_screlease(s->q->doorbell_signal, (hsa_signal_value_t)hsa_queue_load_write_index_relaxed(s->q) - 1);
    return 0;
}

void step_ring(Step* s) {
    const uint64_t w = hsa_queue_load_write_index_relaxed(s->q);
    if (w) hsa_signal_store_screlease(s->q->doorbell_signal, (hsa_signal_value_t)(w - 1));
}

int step_error(Step* s) { return s ? s->qerr.load() : 0; }

const char* step_call_memory(Step* s) {
    return !s ? "" : s->call_vis ? s->dev->vis_pool_kind.c_str() : "pinned host memory";
}

void step_call_read(Step* s) {
    if (!s) return;
    std::lock_guard<std::recursive_mutex> qlk(s->mu);
    s->call_unread = false;
}

int step_wait(Step* s, int timeout_ms, std::string* err) {
    if (!s) return 0;
    std::lock_guard<std::recursive_mutex> qlk(s->mu);
    if (!s->outstanding) return 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        if (hsa_signal_load_scacquire(s->done) == 0) break;
        if (s->qerr.load()) {
            *err = "native queue error: " + hsa_msg((hsa_status_t)s->qerr.load());
            return -1;
        }
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms)) {
            *err = "native dispatch: no completion after " + std::to_string(timeout_ms) + " ms";
            return -1;
        }
        _mm_pause();
    }
    s->outstanding = 0;
    s->call_unread = false;
    return 0;
}

}  // namespace mppi_aql

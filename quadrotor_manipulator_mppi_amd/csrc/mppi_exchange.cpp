// mppi_exchange.cpp -- the sharded step's exchanges: the
// engine-owned RCCL communicator (one SUM all-reduce of the ranks' zero-padded partial-record slots
// per step, between the rollout's PACK and the FINAL) and the peer exchange (no collective: every
// k_finalize block stores its partial into every rank's IPC-mapped region and combines the ranks'
// partials from its own).  Rank 0's RCCL id and the regions' IPC handles travel over
// torch.distributed (distributed.py); nothing here talks to another process except through RCCL
// and the mapped regions.
#include <dlfcn.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "mppi_engine.h"

using namespace mppi;

namespace mppi_host {

const Rccl& rccl() {
    static const Rccl r = [] {
        Rccl x;
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW);
        if (!h) h = dlopen("librccl.so", RTLD_NOW);
        if (!h) { x.why = dlerror() ? dlerror() : "librccl.so.1 not found"; return x; }
        x.get_unique_id = (decltype(x.get_unique_id))dlsym(h, "ncclGetUniqueId");
        x.init_rank = (decltype(x.init_rank))dlsym(h, "ncclCommInitRank");
        x.all_reduce = (decltype(x.all_reduce))dlsym(h, "ncclAllReduce");
        x.destroy = (decltype(x.destroy))dlsym(h, "ncclCommDestroy");
        x.err = (decltype(x.err))dlsym(h, "ncclGetErrorString");
        x.init_rank_config = (decltype(x.init_rank_config))dlsym(h, "ncclCommInitRankConfig");
        x.async_error = (decltype(x.async_error))dlsym(h, "ncclCommGetAsyncError");
        x.abort = (decltype(x.abort))dlsym(h, "ncclCommAbort");
        x.count = (decltype(x.count))dlsym(h, "ncclCommCount");
        x.user_rank = (decltype(x.user_rank))dlsym(h, "ncclCommUserRank");
        x.ok = x.get_unique_id && x.init_rank && x.all_reduce && x.destroy && x.err && x.init_rank_config &&
               x.async_error && x.abort && x.count && x.user_rank;
        if (!x.ok) x.why = "librccl.so.1 lacks an nccl* entry point";
        return x;
    }();
    return r;
}

void exchange_release(mppi_engine* e) {
    if (e->comm) rccl().destroy(e->comm);
    e->comm = nullptr;
    for (void* q : e->x_opened) if (q) (void)hipIpcCloseMemHandle(q);
    e->x_opened.clear();
}

// Wait for a non-blocking communicator to leave ncclInProgress, at most until `deadline`.
ncclResult_t comm_wait(const Rccl& r, ncclComm_t comm, std::chrono::steady_clock::time_point deadline,
                       bool* timed_out) {
    *timed_out = false;
    for (;;) {
        ncclResult_t st = ncclInProgress;
        const ncclResult_t q = r.async_error(comm, &st);
        if (q != ncclSuccess) return q;
        if (st != ncclInProgress) return st;
        if (std::chrono::steady_clock::now() >= deadline) { *timed_out = true; return ncclInProgress; }
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
}
int init_timeout_ms() {
    const char* s = getenv("MPPI_COMM_INIT_TIMEOUT_MS");
    return (s && atoi(s) > 0) ? atoi(s) : 60000;
}

}  // namespace mppi_host

using namespace mppi_host;

extern "C" {

mppi_status mppi_exchange_slot_floats(mppi_engine* e, int64_t* n) {
    if (!e || !n) return fail(MPPI_ERR_INVALID_ARG, "null argument");
    *n = (int64_t)e->V * e->dp.P;
    return MPPI_OK;
}

mppi_status mppi_bind_exchange(mppi_engine* e, float* d) {
    if (!e) return fail(MPPI_ERR_INVALID_ARG, "null engine");
    if (e->comm) return fail(MPPI_ERR_STATE, "the engine owns a communicator and its exchange buffer");
    if (use_device(e)) return MPPI_ERR_HIP;
    e->d_exchange = d;
    return upload_pack_tail(e);
}

mppi_status mppi_comm_unique_id(uint8_t* id) {
    if (!id) return fail(MPPI_ERR_INVALID_ARG, "null id");
    const Rccl& r = rccl();
    if (!r.ok) return fail(MPPI_ERR_COMM, "RCCL unavailable: %s", r.why.c_str());
    static_assert(sizeof(ncclUniqueId) == MPPI_COMM_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId u;
    const ncclResult_t rc = r.get_unique_id(&u);
    if (rc != ncclSuccess) return fail(MPPI_ERR_COMM, "ncclGetUniqueId: %s", r.err(rc));
    std::memcpy(id, &u, sizeof(u));
    return MPPI_OK;
}

mppi_status mppi_comm_available(void) {
    const Rccl& r = rccl();
    if (!r.ok) return fail(MPPI_ERR_COMM, "RCCL unavailable: %s", r.why.c_str());
    return MPPI_OK;
}

// Collective over all shard engines (one per process and GPU): every rank calls it
// with the same id, rank = cfg.shard_rank, world = cfg.shard_count.  The communicator is
// made non-blocking (ncclCommInitRankConfig, blocking = 0) and polled until it is ready or
// `timeout_ms` passes; then it is aborted and the call fails with MPPI_ERR_COMM, so a rank
// whose peers never join returns instead of hanging in the init (distributed.py then
// moves every rank to the torch.distributed collective).  The engine then owns the
// exchange buffer and runs the per-step all-reduce itself (mppi_exchange; inside
// mppi_step / mppi_run_steps).
mppi_status mppi_comm_init_ex(mppi_engine* e, const uint8_t* id, int32_t timeout_ms) {
    if (!e || !id) return fail(MPPI_ERR_INVALID_ARG, "null argument");
    if (e->comm) return fail(MPPI_ERR_STATE, "communicator already initialised");
    const Rccl& r = rccl();
    if (!r.ok) return fail(MPPI_ERR_COMM, "RCCL unavailable: %s", r.why.c_str());
    if (use_device(e)) return MPPI_ERR_HIP;
    if (timeout_ms <= 0) timeout_ms = init_timeout_ms();
    const size_t n = (size_t)e->cfg.shard_count * e->V * e->dp.P;
    HIP_TRY(hipMalloc(&e->d_xown, n * sizeof(float)));
    HIP_TRY(hipMemsetAsync(e->d_xown, 0, n * sizeof(float), e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
    ncclComm_t comm = nullptr;
    ncclResult_t rc = r.init_rank_config(&comm, e->cfg.shard_count, u, e->cfg.shard_rank, &cfg);
    bool timed_out = false;
    if ((rc == ncclSuccess || rc == ncclInProgress) && comm) rc = comm_wait(r, comm, deadline, &timed_out);
    if (rc != ncclSuccess || !comm) {
        if (comm) (void)r.abort(comm);   // also ends RCCL's bootstrap thread of a half-made comm
        (void)hipFree(e->d_xown);
        e->d_xown = nullptr;
        if (timed_out)
            return fail(MPPI_ERR_COMM, "ncclCommInitRankConfig(rank %d of %d): not ready after %d ms (aborted)",
                        e->cfg.shard_rank, e->cfg.shard_count, (int)timeout_ms);
        return fail(MPPI_ERR_COMM, "ncclCommInitRankConfig(rank %d of %d): %s", e->cfg.shard_rank,
                    e->cfg.shard_count, r.err(rc));
    }
    e->comm = comm;
    e->d_exchange = e->d_xown;
    return upload_pack_tail(e);
}

mppi_status mppi_comm_init(mppi_engine* e, const uint8_t* id) { return mppi_comm_init_ex(e, id, 0); }

mppi_status mppi_comm_info(mppi_engine* e, int32_t* nranks, int32_t* rank) {
    if (!e || !nranks || !rank) return fail(MPPI_ERR_INVALID_ARG, "null argument");
    if (!e->comm) return fail(MPPI_ERR_STATE, "mppi_comm_info needs mppi_comm_init");
    int c = 0, u = 0;
    ncclResult_t rc = rccl().count(e->comm, &c);
    if (rc == ncclSuccess) rc = rccl().user_rank(e->comm, &u);
    if (rc != ncclSuccess) return fail(MPPI_ERR_COMM, "ncclCommCount/UserRank: %s", rccl().err(rc));
    *nranks = c;
    *rank = u;
    return MPPI_OK;
}

// The step's one collective: SUM all-reduce of the zero-padded slots on the engine
// stream, between mppi_rollout (which packed this shard's slot) and mppi_finalize.
mppi_status mppi_exchange(mppi_engine* e) {
    if (!e) return fail(MPPI_ERR_INVALID_ARG, "null engine");
    if (!e->comm) return fail(MPPI_ERR_STATE, "mppi_exchange needs mppi_comm_init");
    if (use_device(e)) return MPPI_ERR_HIP;
    const size_t n = (size_t)e->cfg.shard_count * e->V * e->dp.P;
    ncclResult_t rc = rccl().all_reduce(e->d_exchange, e->d_exchange, n, ncclFloat32, ncclSum, e->comm,
                                        e->stream);
    if (rc == ncclInProgress) {   // non-blocking communicator (mppi_comm_init_ex): the enqueue
                                  // finishes asynchronously (first call: lazy connection setup)
        bool timed_out = false;
        rc = comm_wait(rccl(), e->comm,
                       std::chrono::steady_clock::now() + std::chrono::milliseconds(init_timeout_ms()), &timed_out);
        if (timed_out) return fail(MPPI_ERR_COMM, "ncclAllReduce: not enqueued after %d ms", init_timeout_ms());
    }
    if (rc != ncclSuccess) return fail(MPPI_ERR_COMM, "ncclAllReduce: %s", rccl().err(rc));
    return MPPI_OK;
}

// ---------------------------------------------------------------- peer exchange
// An upper bound of the finalize's blocks: its grid.x is 8 XCD lanes x dim groups x t-slices
// (mppi_launch_finalize), and the dim groups are A / MPPI_FIN_XCDS rounded up, at most A (the
// kernel indexes the region with its own grid, so any build's fits)
static size_t fin_blocks(const mppi_engine* e) { return (size_t)8 * e->A * e->fin_ts * e->V; }

mppi_status mppi_peer_open(mppi_engine* e, uint8_t* handle) {
    if (!e || !handle) return fail(MPPI_ERR_INVALID_ARG, "null argument");
    if (e->V != 1) return fail(MPPI_ERR_STATE, "peer exchange: one vehicle per engine (V = %d)", e->V);
    if (e->cfg.shard_count > kMaxPeers)
        return fail(MPPI_ERR_STATE, "peer exchange: at most %d ranks (%d)", kMaxPeers, e->cfg.shard_count);
    if (e->comm || e->d_exchange) return fail(MPPI_ERR_STATE, "peer exchange: the engine already has an exchange");
    if (e->d_xregion) return fail(MPPI_ERR_STATE, "peer exchange: region already open");
    if (use_device(e)) return MPPI_ERR_HIP;
    const size_t bytes = (kXCtl + 2 * (size_t)e->cfg.shard_count * fin_blocks(e) * kXW) * sizeof(unsigned long long);
    // uncached: the words other GPUs store into it are never behind a stale line of this GPU's L2
    void* p = nullptr;
    hipError_t r = hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached);
    if (r != hipSuccess) {
        (void)hipGetLastError();
        HIP_TRY(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocFinegrained));
    }
    e->d_xregion = (unsigned long long*)p;
    e->x_bytes = bytes;
    HIP_TRY(hipMemset(p, 0, bytes));   // tags 0: no step's (bit 31 is set in every tag); no timeout reports
    hipIpcMemHandle_t h;
    static_assert(sizeof(h) == MPPI_PEER_HANDLE_BYTES, "hipIpcMemHandle_t size");
    HIP_TRY(hipIpcGetMemHandle(&h, p));
    std::memcpy(handle, &h, sizeof(h));
    return MPPI_OK;
}

// the regions' device addresses (past their control words), in rank order, into the finalize's
// tail (both connects)
static mppi_status peer_bind(mppi_engine* e, std::vector<unsigned long long*> ptrs) {
    const int n = e->cfg.shard_count, me = e->cfg.shard_rank;
    for (auto& p : ptrs) p += kXCtl;
    if (!e->d_xpeers) HIP_TRY(hipMalloc(&e->d_xpeers, kMaxPeers * sizeof(void*)));
    HIP_TRY(hipMemcpy(e->d_xpeers, ptrs.data(), n * sizeof(void*), hipMemcpyHostToDevice));
    if (!e->d_xdec) {
        HIP_TRY(hipMalloc(&e->d_xdec, 2 * fin_blocks(e) * sizeof(unsigned long long)));
        HIP_TRY(hipMemset(e->d_xdec, 0, 2 * fin_blocks(e) * sizeof(unsigned long long)));
    }
    FinParams& f = e->fp;
    f.xpeers = e->d_xpeers; f.xlocal = xdata(e); f.xn = n; f.xme = me; f.xdec = e->d_xdec;
    FinTail t[2] = {tail_of(f, 0), tail_of(f, 2)};
    t[0].wraw = t[0].wsmooth = nullptr;   // (as at create: the step's FINAL stores no readback copies)
    HIP_TRY(hipStreamSynchronize(e->stream));
    HIP_TRY(hipMemcpy(e->d_tail + kTailFinal, &t[0], sizeof(FinTail), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(e->d_tail + kTailReadback, &t[1], sizeof(FinTail), hipMemcpyHostToDevice));
    e->peer = true;
    e->call_cached = false;
    return MPPI_OK;
}

mppi_status mppi_peer_connect(mppi_engine* e, const uint8_t* handles) {
    if (!e || !handles) return fail(MPPI_ERR_INVALID_ARG, "null argument");
    if (!e->d_xregion) return fail(MPPI_ERR_STATE, "mppi_peer_connect before mppi_peer_open");
    if (e->peer) return fail(MPPI_ERR_STATE, "peer exchange already connected");
    if (use_device(e)) return MPPI_ERR_HIP;
    const int n = e->cfg.shard_count, me = e->cfg.shard_rank;
    std::vector<unsigned long long*> ptrs(n, nullptr);
    e->x_opened.assign(n, nullptr);
    for (int r = 0; r < n; ++r) {
        if (r == me) { ptrs[r] = e->d_xregion; continue; }
        hipIpcMemHandle_t h;
        std::memcpy(&h, handles + (size_t)r * MPPI_PEER_HANDLE_BYTES, sizeof(h));
        void* q = nullptr;
        const hipError_t rc = hipIpcOpenMemHandle(&q, h, hipIpcMemLazyEnablePeerAccess);
        if (rc != hipSuccess) {
            for (void*& o : e->x_opened) if (o) { (void)hipIpcCloseMemHandle(o); o = nullptr; }
            return fail(MPPI_ERR_HIP, "peer exchange: opening rank %d's region: %s", r, hipGetErrorString(rc));
        }
        e->x_opened[r] = q;
        ptrs[r] = (unsigned long long*)q;
    }
    return peer_bind(e, ptrs);
}

mppi_status mppi_peer_region(mppi_engine* e, uint64_t* device_address) {
    if (!e || !device_address) return fail(MPPI_ERR_INVALID_ARG, "null argument");
    if (!e->d_xregion) return fail(MPPI_ERR_STATE, "mppi_peer_region before mppi_peer_open");
    *device_address = (uint64_t)(uintptr_t)e->d_xregion;
    return MPPI_OK;
}

mppi_status mppi_peer_connect_ptrs(mppi_engine* e, const uint64_t* device_addresses) {
    if (!e || !device_addresses) return fail(MPPI_ERR_INVALID_ARG, "null argument");
    if (!e->d_xregion) return fail(MPPI_ERR_STATE, "mppi_peer_connect_ptrs before mppi_peer_open");
    if (e->peer) return fail(MPPI_ERR_STATE, "peer exchange already connected");
    if (use_device(e)) return MPPI_ERR_HIP;
    const int n = e->cfg.shard_count, me = e->cfg.shard_rank;
    if (device_addresses[me] != (uint64_t)(uintptr_t)e->d_xregion)
        return fail(MPPI_ERR_INVALID_ARG, "mppi_peer_connect_ptrs: entry %d is not this engine's region", me);
    std::vector<unsigned long long*> ptrs(n, nullptr);
    for (int r = 0; r < n; ++r) {
        if (!device_addresses[r]) return fail(MPPI_ERR_INVALID_ARG, "mppi_peer_connect_ptrs: null region of rank %d", r);
        ptrs[r] = (unsigned long long*)(uintptr_t)device_addresses[r];
    }
    return peer_bind(e, ptrs);
}

// Connection check before the first step (distributed.py), three phases with a barrier between
// each: 0 stores a pattern word into this rank's slot of every rank's region through the mapping
// (a copy); 1 checks that this rank's region holds every rank's word and clears it; 2 runs the
// finalize's own store-and-poll over the regions in a one-wave kernel (k_peer_probe: every rank's
// tagged word must arrive within 2 s) and clears the region again.
mppi_status mppi_peer_probe(mppi_engine* e, int32_t phase) {
    if (!e) return fail(MPPI_ERR_INVALID_ARG, "null engine");
    if (!e->peer) return fail(MPPI_ERR_STATE, "mppi_peer_probe before mppi_peer_connect");
    if (use_device(e)) return MPPI_ERR_HIP;
    const int n = e->cfg.shard_count, me = e->cfg.shard_rank;
    const size_t slot = fin_blocks(e) * kXW;   // words per (parity, rank)
    if (phase == 2) {
        unsigned long long* d_got = nullptr;
        HIP_TRY(hipMalloc(&d_got, kMaxPeers * sizeof(unsigned long long)));
        const uint32_t tag = 0x3C3C0000u;   // (bit 31 clear: never a step's tag)
        int rc = mppi_launch_peer_probe(e->d_xpeers, xdata(e), n, me, slot, tag, kPeerWaitTicks, d_got, e->stream);
        std::vector<unsigned long long> got(kMaxPeers, 0ull);
        hipError_t he = rc == 0 ? hipStreamSynchronize(e->stream) : (hipError_t)rc;
        if (he == hipSuccess) he = hipMemcpy(got.data(), d_got, n * sizeof(unsigned long long), hipMemcpyDeviceToHost);
        (void)hipFree(d_got);
        if (he != hipSuccess) return fail(MPPI_ERR_HIP, "peer probe kernel: %s", hipGetErrorString(he));
        HIP_TRY(hipMemset(e->d_xregion, 0, e->x_bytes));
        HIP_TRY(hipDeviceSynchronize());
        e->x_connected = 0;
        for (int r = 0; r < n; ++r) {
            if ((uint32_t)(got[r] >> 32) != (tag | (uint32_t)r))
                return fail(MPPI_ERR_COMM, "peer exchange: rank %d's word did not reach this rank's region in the "
                                           "kernel probe (%016llx)", r, got[r]);
            ++e->x_connected;
        }
        return MPPI_OK;
    }
    auto pattern = [](int r, int d) { return (0x5A5A0000ull | (unsigned)(16 * r + d)) << 32 | 0x3F800000ull; };
    if (phase == 0) {
        std::vector<unsigned long long*> ptrs(n);
        HIP_TRY(hipMemcpy(ptrs.data(), e->d_xpeers, n * sizeof(void*), hipMemcpyDeviceToHost));
        for (int d = 0; d < n; ++d) {
            const unsigned long long w = pattern(me, d);
            HIP_TRY(hipMemcpy(ptrs[d] + (size_t)me * slot, &w, sizeof(w), hipMemcpyHostToDevice));
        }
        return MPPI_OK;
    }
    std::vector<unsigned long long> got(n);
    for (int r = 0; r < n; ++r)
        HIP_TRY(hipMemcpy(&got[r], xdata(e) + (size_t)r * slot, sizeof(got[r]), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemset(e->d_xregion, 0, e->x_bytes));
    HIP_TRY(hipDeviceSynchronize());
    for (int r = 0; r < n; ++r)
        if (got[r] != pattern(r, me))
            return fail(MPPI_ERR_COMM, "peer exchange: rank %d's probe word did not arrive (%016llx)", r, got[r]);
    return MPPI_OK;
}

// The exchange's failure state.  sticky: this engine's own timeout word (a step tag, 0 = none;
// mapped host memory, no device access).  reports (may be NULL): the control words of this rank's
// region, one per rank (a step tag << 32 | 1 from every rank that gave a step up since the last
// reset; a device-to-host copy of kMaxPeers words, after waiting for the engine's work).
mppi_status mppi_peer_status(mppi_engine* e, uint32_t* sticky, uint64_t* reports, uint32_t* epoch) {
    if (!e) return fail(MPPI_ERR_INVALID_ARG, "null engine");
    if (!e->d_xregion) return fail(MPPI_ERR_STATE, "mppi_peer_status before mppi_peer_open");
    if (reports) {
        if (use_device(e)) return MPPI_ERR_HIP;
        HIP_TRY(hipStreamSynchronize(e->stream));
        HIP_TRY(hipMemcpy(reports, e->d_xregion, kMaxPeers * sizeof(uint64_t), hipMemcpyDeviceToHost));
    }
    if (sticky) *sticky = sticky_timeout(e);
    if (epoch) *epoch = e->x_epoch;
    return MPPI_OK;
}

// The connection as the kernel probe saw it and the torn word (mppi_dev.h, "All or nothing within a rank"): connected = the
// ranks whose tagged word reached this rank's region in mppi_peer_probe's phase 2 (0 before it).
mppi_status mppi_peer_info(mppi_engine* e, int32_t* connected, int32_t* rank, uint32_t* torn) {
    if (!e) return fail(MPPI_ERR_INVALID_ARG, "null engine");
    if (!e->d_xregion) return fail(MPPI_ERR_STATE, "mppi_peer_info before mppi_peer_open");
    if (connected) *connected = e->x_connected;
    if (rank) *rank = e->cfg.shard_rank;
    if (torn) *torn = e->h_out ? *(const volatile uint32_t*)(e->h_out + off_xerr(e) + 4) : 0u;
    return MPPI_OK;
}

// Diagnostic (not part of the public header): the next FINAL's finalize block `block` stalls `ms`
// milliseconds before it stores its partial into the peers' regions (once; the word is then
// cleared by the kernel).  The stall word is allocated at the first call, so an engine that never
// calls this carries a null pointer (no load in the kernel).  tests/test_gpu_peer.py.
int32_t mppi_debug_peer_stall(mppi_engine* e, int32_t block, int32_t ms) {
    if (!e || block < 0 || block > 0xFFFF || ms < 0 || ms > 60000) return fail(MPPI_ERR_INVALID_ARG, "bad arguments");
    if (!e->peer) return fail(MPPI_ERR_STATE, "mppi_debug_peer_stall before mppi_peer_connect");
    if (use_device(e)) return MPPI_ERR_HIP;
    if (!e->d_xstall) {
        HIP_TRY(hipMalloc(&e->d_xstall, sizeof(uint32_t)));
        e->fp.xstall = e->d_xstall;
        FinTail t = tail_of(e->fp, 0);
        t.wraw = t.wsmooth = nullptr;   // (as at create)
        HIP_TRY(hipStreamSynchronize(e->stream));
        HIP_TRY(hipMemcpy(e->d_tail + kTailFinal, &t, sizeof(FinTail), hipMemcpyHostToDevice));
        e->call_cached = e->batch_cached = false;
    }
    const uint32_t w = ms ? ((uint32_t)ms << 16) | (uint32_t)block : 0u;
    HIP_TRY(hipMemcpy(e->d_xstall, &w, sizeof(w), hipMemcpyHostToDevice));
    return MPPI_OK;
}

// Collective recovery after a timeout (distributed.py ShardedEngine.resync): every rank has
// synchronised its engine and passed a barrier, so no kernel writes into any region; each rank
// clears its own region (partials and timeout reports) and its sticky word, and takes the step
// counter and exchange epoch every rank agreed on; a second barrier follows before any rank steps.
mppi_status mppi_peer_reset(mppi_engine* e, uint32_t step, uint32_t epoch) {
    if (!e) return fail(MPPI_ERR_INVALID_ARG, "null engine");
    if (!e->peer) return fail(MPPI_ERR_STATE, "mppi_peer_reset before mppi_peer_connect");
    if (use_device(e)) return MPPI_ERR_HIP;
    HIP_TRY(hipStreamSynchronize(e->stream));
    HIP_TRY(hipMemset(e->d_xregion, 0, e->x_bytes));
    if (e->d_xdec) HIP_TRY(hipMemset(e->d_xdec, 0, 2 * fin_blocks(e) * sizeof(unsigned long long)));
    HIP_TRY(hipDeviceSynchronize());
    *(volatile uint32_t*)(e->h_out + off_xerr(e)) = 0u;       // the sticky word
    *(volatile uint32_t*)(e->h_out + off_xerr(e) + 4) = 0u;   // the torn word
    e->step_ctr = step;
    e->x_epoch = epoch;
    return build_vehicle_consts(e);
}

// n back-to-back all-reduces of the exchange slots on the engine stream between one event
// pair (collective: every rank calls it with the same n).  The slots are summed in place,
// so the call leaves the exchange buffer scaled by shard_count^n: run a step after it.
mppi_status mppi_exchange_timing(mppi_engine* e, int32_t n, double* allreduce_us) {
    if (!e || n <= 0 || !allreduce_us) return fail(MPPI_ERR_INVALID_ARG, "mppi_exchange_timing: bad arguments");
    if (!e->comm) return fail(MPPI_ERR_STATE, "mppi_exchange_timing needs mppi_comm_init");
    if (use_device(e)) return MPPI_ERR_HIP;
    hipEvent_t ev[2] = {nullptr, nullptr};
    mppi_status st = MPPI_OK;
    float ms = 0.0f;
    HIP_TRY(hipEventCreate(&ev[0]));
    if (hipEventCreate(&ev[1]) != hipSuccess) { (void)hipEventDestroy(ev[0]); return fail(MPPI_ERR_HIP, "hipEventCreate"); }
    if (hipEventRecord(ev[0], e->stream) != hipSuccess) st = fail(MPPI_ERR_HIP, "hipEventRecord");
    for (int i = 0; i < n && st == MPPI_OK; ++i) st = mppi_exchange(e);
    if (st == MPPI_OK && (hipEventRecord(ev[1], e->stream) != hipSuccess || hipEventSynchronize(ev[1]) != hipSuccess ||
                          hipEventElapsedTime(&ms, ev[0], ev[1]) != hipSuccess))
        st = fail(MPPI_ERR_HIP, "exchange timing events failed");
    if (st == MPPI_OK) *allreduce_us = 1e3 * ms / n;
    (void)hipEventDestroy(ev[0]);
    (void)hipEventDestroy(ev[1]);
    return st;
}

}  // extern "C"

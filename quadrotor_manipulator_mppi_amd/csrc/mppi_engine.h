// mppi_engine.h -- the engine object behind include/mppi_hip.h and the host-side helpers its
// translation units share.  Internal: not part of the public ABI.
//
// The host side of libmppi_hip.so is split by concern:
//   mppi_host_math.cpp   error state, config defaults and validation, the reference's fp32 tensor
//                        builders (joint origins, base and target rotations), SavGol taps, host FK
//   mppi_engine.cpp      create / destroy, buffers, state and target uploads, readbacks, timing
//   mppi_step.cpp        the control step: rollout, finalize, outputs, native (AQL) batches and calls
//   mppi_exchange.cpp    the sharded step's exchanges: the engine-owned RCCL communicator and the
//                        peer exchange (regions, connect, probe, status, reset)
//   mppi_prewarm.cpp     the opt-in prewarm thread (mppi_set_prewarm)
//
// Threads.  Every entry point of one engine is called from one thread at a time (the Python
// wrapper serialises them), except the prewarm thread, which reads only the atomics marked for it
// below (call_t, call_n, pw_*) and e->aql once pw_native has been stored with release after it.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "mppi_aql.h"
#include "mppi_dev.h"

struct mppi_engine {
    mppi_config cfg;
    int K, H, A, V, nq, qoff, state_dim, out_dim, C, threads;
    int64_t out_bytes;
    mppi::DevParams dp;
    mppi::FinParams fp;
    float sg_taps[mppi::kMaxW];
    float fixedM[12];                   // product of the leading fixed joints (folded into base)
    hipStream_t own_stream = nullptr, stream = nullptr;
    float* d_sigma = nullptr;
    mppi::JointDev* d_joints = nullptr;
    mppi::VehicleConst* d_vc = nullptr;
    float* d_u_prev = nullptr;
    float* d_noise_in = nullptr;
    uint32_t step_ctr = 0;              // Philox counter word; +1 per finalized step
    uint32_t out_seq = 0;               // completion-flag value of the step read_outputs waits for
    // a native control call's launch descriptions, reused while only the state changes
    bool call_cached = false;
    int call_threads = 0;
    mppi::DevParams call_p{};
    mppi::FinParams call_f{};
    mppi::LaunchDesc call_roll{}, call_fin{};
    // a native batch's launch descriptions, reused while the step's parameters are unchanged
    bool batch_cached = false;
    int batch_threads = 0;
    mppi::DevParams batch_p{};
    mppi::FinParams batch_f{};
    mppi::LaunchDesc batch_roll{}, batch_fin{};
    std::vector<double> rec_out;        // a read step's outputs assembled from its tagged records
    std::vector<float> rec_u0, rec_stats;
    std::vector<float> fk_O, fk_ax;     // the joints' origins and unit axes for check_reach's host FK
    uint32_t seq_ctr = 0;               // last completion-flag value handed out: monotonic and
                                        // independent of step_ctr (mppi_set_step_counter rewinds that)
    bool event_wait = false;            // MPPI_EVENT_WAIT=1: wait on ev_out instead of polling flags
    bool no_flag_dbg = false;           // MPPI_DEBUG_NO_FLAG=1 (diagnostics, with MPPI_EVENT_WAIT=1): no step
                                        // writes the completion flag, so the last step runs like the others
    int out_dbg = 0;                    // MPPI_DEBUG_OUT (diagnostics): 1 = unread steps write their outputs
                                        // to device scratch, 2 = mppi_kernel_timing writes to mapped host memory
    float* d_traj = nullptr;
    float* d_noise_out = nullptr;
    float* d_S = nullptr;
    float* d_hdr = nullptr;     // (V,nb,4) block record headers
    float* d_rdata = nullptr;   // (V,A,nb,H) block record bodies
    int fin_ts = 1, fin_tsz = 8;   // finalize t-slices
    unsigned char* d_out = nullptr;   // device scratch in h_out's layout (mppi_kernel_timing's outputs)
    mppi::FinTail* d_tail = nullptr;  // [kTailSlots] the finalize's tail parameters per launch kind
    float* d_wraw = nullptr;
    float* d_wsmooth = nullptr;
    float* d_w = nullptr;
    float* d_sinv = nullptr;      // extra cost terms: Sigma^-1 (A,A)
    float* d_gamma = nullptr;     //   gamma^t (H)
    float* d_jtraj = nullptr;     //   joint tracking target (V,H,nq)
    float* d_exchange = nullptr;
    ncclComm_t comm = nullptr;          // engine-owned RCCL communicator (mppi_comm_init)
    float* d_xown = nullptr;            // its exchange buffer (shard_count * V * P floats)
    bool peer = false;                  // peer exchange connected (mppi_peer_connect): no PACK, no collective
    int x_connected = 0;                // ranks whose word the kernel probe received (mppi_peer_probe phase 2)
    unsigned long long* d_xregion = nullptr;   // this rank's exchange region (uncached device memory)
    size_t x_bytes = 0;
    std::vector<void*> x_opened;        // the other ranks' regions, IPC-mapped
    unsigned long long** d_xpeers = nullptr;   // (shard_count) region pointers, device resident
    uint32_t x_epoch = 0;               // the exchange epoch in the tags (mppi_dev.h peer_tag): moved by
                                        // mppi_set_step_counter and mppi_peer_reset on a connected engine
    uint32_t* d_xstall = nullptr;       // diagnostics (mppi_debug_peer_stall): a finalize block's stall
    unsigned long long* d_xdec = nullptr;   // the peer exchange's commit marks (2 parities x finalize blocks)
    bool overlap = false;               // MPPI_OVERLAP=1 (experiment): native batches dispatch each rollout
                                        // while the finalize before it runs (mppi_device.h kNoiseOverlap)
    uint32_t* d_ovl = nullptr;          // its (V, A, fin_ts) step counters, one per finalize block
    mppi::VehicleConst* h_vc = nullptr; // pinned staging
    unsigned char* h_out = nullptr;     // pinned + mapped: k_finalize writes it directly
    unsigned char* h_out_dev = nullptr; // device view of h_out
    hipEvent_t ev_vc = nullptr, ev_out = nullptr;
    bool vc_pending = false, state_set = false, out_pending = false;
    std::vector<float> tpos, tquat;
    std::vector<double> state;
    // timing
    bool timing = false;
    std::vector<hipEvent_t> ev_pool;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> roll_pairs, fin_pairs;
    double roll_ms = 0.0, fin_ms = 0.0;
    unsigned long long* d_stamps = nullptr;    // MPPI_STAMPS diagnostics
    unsigned long long* d_fstamps = nullptr;
    std::vector<double> fstamp_sum;
    int64_t fstamp_n = 0;
    std::vector<double> stamp_sum;
    int64_t stamp_n = 0;
    double clk_sum = 0.0;
    int64_t roll_n = 0, fin_n = 0;
    // native dispatch of mppi_run_steps (mppi_aql.cpp): MPPI_DISPATCH = hip | aql | auto (default)
    mppi_aql::Step* aql = nullptr;
    int aql_mode = 2;                   // 0 hip, 1 aql (required), 2 auto (aql when available)
    bool aql_tried = false;             // step_create attempted (its failure is final for the engine)
    bool aql_off = false;               // this engine's launches are not dispatchable natively
    std::string aql_why = "no mppi_run_steps yet";   // why the last run went through HIP ("" = native)
    bool aql_out = false;               // the pending outputs come from a native batch
    bool aql_call = false;              // ... from a native control call (flags carry bit 31)
    bool calls_native = false;          // the last mppi_step went out as native packets
    double call_wait_us = 0.0;          // diagnostics (MPPI_AQL_PROFILE): the last call's flag wait
    // prewarm (mppi_set_prewarm, mppi_prewarm.cpp): a host thread learns the control calls' cadence
    // from their start times and touches the native queue through a window before each predicted call
    std::thread pw_thr;
    std::mutex pw_mu;                   // (for pw_cv only)
    std::condition_variable pw_cv;
    std::atomic<int32_t> pw_us{0};      // the window half-width; 0: off
    std::atomic<bool> pw_stop{false};
    std::atomic<int64_t> pw_touches{0};
    std::atomic<int64_t> call_t[8];     // steady-clock start of the last 8 control calls (ring)
    std::atomic<int64_t> call_n{0};     // control calls recorded
    bool pw_spin = false;               // diagnostics (MPPI_PREWARM_SPIN=1): spin between touches
    std::atomic<bool> pw_native{false}; // the last control call went out as native packets (release:
                                        // stored after e->aql, so the prewarm thread may read it)
};

namespace mppi_host {

// ------------------------------------------------------------- errors (mppi_host_math.cpp)
// Sets the calling thread's mppi_last_error string and returns st.
mppi_status fail(mppi_status st, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

#define HIP_TRY(expr)                                                                              \
    do {                                                                                           \
        hipError_t _e = (expr);                                                                    \
        if (_e != hipSuccess)                                                                      \
            return ::mppi_host::fail(MPPI_ERR_HIP, "%s failed: %s (%s:%d)", #expr,                \
                                     hipGetErrorString(_e), __FILE__, __LINE__);                   \
    } while (0)

// ------------------------------------------- reference fp32 builders (mppi_host_math.cpp)
int nq_of(const mppi_config& c);
mppi_status validate(const mppi_config& c);
void rpy_to_R(float r, float p, float y, float* R);
void joint_origin(const mppi_joint& j, float* T16);
void unit_axis(const mppi_joint& j, float* a);
void base_from_xyzquat(const double* b, bool f64, float* T16);
void quat_xyzw_to_R(const float* q, float* R);
void euler_zyx(const float* m, float* ypr);
int savgol_taps(int window, int order, float* c);
void bake_joint(const mppi_joint& j, mppi::JointDev& d);
void mul34(const float* A, const float* B, float* C);
void fk_consts(const mppi_joint* joints, int nj, float* O16s, float* axes);
void host_fk_c(const mppi_joint* joints, int nj, const float* O16s, const float* axes, const double* q,
               const double* xyzquat, bool f64, float* out16);
void host_fk(const mppi_joint* joints, int nj, const double* q, const double* xyzquat, bool f64, float* out16);

// ------------------------------------------------------------ engine (mppi_engine.cpp)
// the step goes through the exchange slots: several shards, or an engine-owned communicator (a
// one-rank communicator runs the same pack -> all-reduce -> combine).  A shard connected by the
// peer exchange steps like an unsharded engine: its finalize does the exchange.
inline bool sharded(const mppi_engine* e) { return (e->cfg.shard_count > 1 || e->comm) && !e->peer; }
mppi::FinTail tail_of(const mppi::FinParams& f, int32_t mode);
void pack_fields(const mppi_engine* e, mppi::FinParams& f);
mppi_status upload_pack_tail(mppi_engine* e);
int traj_pitch(const mppi_engine* e);
size_t traj_floats(const mppi_engine* e);
mppi_status aql_join(mppi_engine* e);
mppi_status use_device(mppi_engine* e);
mppi_status build_vehicle_consts(mppi_engine* e);
void quad_outputs(const mppi_engine* e, const double* s, const float* u0, double* out);
mppi_status upload_consts(mppi_engine* e);
hipEvent_t pool_event(mppi_engine* e);
mppi_status drain_timing(mppi_engine* e);

// mapped output buffer layout (h_out): outputs, u0, stats, then the tagged records of a read step
// (k_finalize): per vehicle, 2 per dim -- (o1, u0, seq), (o2, nan flag, seq) -- and one
// (rho, eta, ess, seq), 16 B each, each written by ONE store; the host polls their tags and takes
// the values from the records themselves
inline size_t off_u0(const mppi_engine* e) { return ((size_t)e->V * e->out_dim * sizeof(double) + 15) & ~size_t(15); }
inline size_t off_stats(const mppi_engine* e) {
    return (off_u0(e) + (size_t)e->V * e->A * sizeof(float) + 15) & ~size_t(15);
}
inline size_t off_flags(const mppi_engine* e) { return off_stats(e) + (size_t)e->V * 16; }
inline size_t rec_count(const mppi_engine* e) { return (size_t)e->V * (2 * e->A + 1); }
// the peer exchange's sticky timeout word (16 B after the records): the step tag of a finalize
// block that gave a step up, written by that block, cleared only by the host (mppi_peer_reset)
inline size_t off_xerr(const mppi_engine* e) { return off_flags(e) + rec_count(e) * 16; }
inline uint32_t sticky_timeout(const mppi_engine* e) {
    return e->h_out ? *(const volatile uint32_t*)(e->h_out + off_xerr(e)) : 0u;
}
// this rank's exchange region past its control words (mppi_dev.h kXCtl): the partials' base
inline unsigned long long* xdata(const mppi_engine* e) { return e->d_xregion + mppi::kXCtl; }

// -------------------------------------------------------------- step (mppi_step.cpp)
// the rollout's per-block partial records (DevParams::hdr / rdata layout)
void block_records(const mppi_engine* e, mppi::FinParams& f);
// the finalize's record source: the rollout blocks' records, or the exchange slots of a shard
void final_records(const mppi_engine* e, mppi::FinParams& f);

// ------------------------------------------------------ exchange (mppi_exchange.cpp)
// RCCL, resolved at the first mppi_comm_* call (dlopen: the library loads and its single-GPU
// paths run without RCCL; inside a torch process this binds the librccl.so.1 torch already
// loaded, so there is one RCCL per process).
struct Rccl {
    bool ok = false;
    std::string why;
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                               hipStream_t) = nullptr;
    ncclResult_t (*destroy)(ncclComm_t) = nullptr;
    const char* (*err)(ncclResult_t) = nullptr;
    // the non-blocking init with a deadline (mppi_comm_init_ex) and the communicator's own
    // view of its size (mppi_comm_info)
    ncclResult_t (*init_rank_config)(ncclComm_t*, int, ncclUniqueId, int, ncclConfig_t*) = nullptr;
    ncclResult_t (*async_error)(ncclComm_t, ncclResult_t*) = nullptr;
    ncclResult_t (*abort)(ncclComm_t) = nullptr;
    ncclResult_t (*count)(const ncclComm_t, int*) = nullptr;
    ncclResult_t (*user_rank)(const ncclComm_t, int*) = nullptr;
};
const Rccl& rccl();
// the engine's exchange resources (communicator, mapped peer regions), released by mppi_destroy
void exchange_release(mppi_engine* e);

// ------------------------------------------------------- prewarm (mppi_prewarm.cpp)
void note_call(mppi_engine* e);      // mppi_step entry (the caller's thread)
void prewarm_stop(mppi_engine* e);   // joins the thread (mppi_destroy, mppi_set_prewarm)
int prewarm_plan(const int64_t* t, int m, int64_t win, int64_t* start, int64_t* end);

// MPPI_STAMPS diagnostics: stamp indices in program order and the phase each difference measures
// (see the STAMP calls in mppi_rollout.h / mppi_finalize.hip).
inline const std::vector<int> kRollStampOrder = {0, 9, 10, 8, 1, 2, 3, 4, 5, 11, 6, 12, 7};
inline const char* const kRollStampNames[] = {"", "loads(waited)", "philox0", "lds-writes(waited)", "barrier",
                                              "noise", "integrator", "fk+cost", "S+softmin", "deposit",
                                              "combine-barrier", "fw", "record"};
inline const std::vector<int> kFinStampOrder = {0, 7, 8, 1, 2, 3, 4, 5, 6};
inline const char* const kFinStampNames[] = {"", "loads-issued", "accum(last chunk)", "wave-fold", "barrier",
                                             "combine", "w_eps", "savgol", "update+outputs"};

}  // namespace mppi_host

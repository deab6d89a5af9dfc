// mppi_capi.cpp -- host side of libmppi_hip.so: the C-ABI of include/mppi_hip.h.
//
// Owns the engine (device buffers allocated once at create, no allocation in
// the step), bakes the per-joint / per-vehicle fp32 constants exactly the way
// the reference builds its tensors, and sequences the two kernels of a step on
// one HIP stream.  See DESIGN.md for the data layout and the kernel roofline.
#include <dlfcn.h>
#include <emmintrin.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <sys/prctl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "mppi_aql.h"
#include "mppi_dev.h"

using namespace mppi;

namespace {

thread_local std::string g_err;

// RCCL, resolved at the first mppi_comm_* call (dlopen: the library loads and its
// single-GPU paths run without RCCL; inside a torch process this binds the
// librccl.so.1 torch already loaded, so there is one RCCL per process).
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

mppi_status fail(mppi_status st, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return st;
}

#define HIP_TRY(expr)                                                                              \
    do {                                                                                           \
        hipError_t _e = (expr);                                                                    \
        if (_e != hipSuccess)                                                                      \
            return fail(MPPI_ERR_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e),      \
                        __FILE__, __LINE__);                                                       \
    } while (0)

int pow2ceil(int x) {
    int p = 1;
    while (p < x) p <<= 1;
    return p;
}

int nq_of(const mppi_config& c) {
    if (c.model == MPPI_MODEL_ARM) return c.n_action;
    if (c.model == MPPI_MODEL_WHOLEBODY) return c.n_action - 3;
    return 0;
}

// ----------------------------------------------------- reference fp32 builders
// rotation_matrix_rpy (transformation_matrix.py:4-25): every product is a 0-d
// fp32 tensor op, evaluated left to right.
void rpy_to_R(float r, float p, float y, float* R) {
    const float cr = cosf(r), sr = sinf(r), cp = cosf(p), sp = sinf(p), cy = cosf(y), sy = sinf(y);
    volatile float t;   // keep every intermediate an fp32 rounding (no contraction)
    t = cy * cp; R[0] = t;
    t = cy * sp; t = t * sr; { volatile float u = sy * cr; R[1] = t - u; }
    t = cy * sp; t = t * cr; { volatile float u = sy * sr; R[2] = t + u; }
    t = sy * cp; R[3] = t;
    t = sy * sp; t = t * sr; { volatile float u = cy * cr; R[4] = t + u; }
    t = sy * sp; t = t * cr; { volatile float u = cy * sr; R[5] = t - u; }
    R[6] = -sp;
    t = cp * sr; R[7] = t;
    t = cp * cr; R[8] = t;
}

void joint_origin(const mppi_joint& j, float* T16) {
    float R[9];
    rpy_to_R(j.rpy[0], j.rpy[1], j.rpy[2], R);
    std::memset(T16, 0, 16 * sizeof(float));
    for (int i = 0; i < 3; ++i)
        for (int k = 0; k < 3; ++k) T16[4 * i + k] = R[3 * i + k];
    T16[3] = j.xyz[0]; T16[7] = j.xyz[1]; T16[11] = j.xyz[2];
    T16[15] = 1.0f;
}

void unit_axis(const mppi_joint& j, float* a) {
    float x = 1.0f, y = 0.0f, z = 0.0f;
    if (j.has_axis) { x = j.axis[0]; y = j.axis[1]; z = j.axis[2]; }
    const float n = sqrtf(x * x + y * y + z * z);
    if (!(n >= 1e-12f)) { a[0] = 1.0f; a[1] = 0.0f; a[2] = 0.0f; return; }
    a[0] = x / n; a[1] = y / n; a[2] = z / n;
}

// xyzquat_to_matrix (urdf_fk.py:30-55) in the state dtype, rounded into fp32.
template <typename T>
void base_from_xyzquat_t(const double* b, float* T16) {
    const T qx = (T)b[3], qy = (T)b[4], qz = (T)b[5], qw = (T)b[6];
    volatile T a, c;
    std::memset(T16, 0, 16 * sizeof(float));
    a = (T)1 - (T)2 * (qy * qy); a = a - (T)2 * (qz * qz); T16[0] = (float)a;
    a = ((T)2 * qx) * qy; c = ((T)2 * qz) * qw; T16[1] = (float)(a - c);
    a = ((T)2 * qx) * qz; c = ((T)2 * qy) * qw; T16[2] = (float)(a + c);
    a = ((T)2 * qx) * qy; c = ((T)2 * qz) * qw; T16[4] = (float)(a + c);
    a = (T)1 - (T)2 * (qx * qx); a = a - (T)2 * (qz * qz); T16[5] = (float)a;
    a = ((T)2 * qy) * qz; c = ((T)2 * qx) * qw; T16[6] = (float)(a - c);
    a = ((T)2 * qx) * qz; c = ((T)2 * qy) * qw; T16[8] = (float)(a - c);
    a = ((T)2 * qy) * qz; c = ((T)2 * qx) * qw; T16[9] = (float)(a + c);
    a = (T)1 - (T)2 * (qx * qx); a = a - (T)2 * (qy * qy); T16[10] = (float)a;
    T16[3] = (float)(T)b[0]; T16[7] = (float)(T)b[1]; T16[11] = (float)(T)b[2];
    T16[15] = 1.0f;
}

// quaternion_to_matrix with xyzw input (rotation_conversions.py:45-75), fp32.
void quat_xyzw_to_R(const float* q, float* R) {
    const float i = q[0], j = q[1], k = q[2], r = q[3];
    volatile float s = i * i;
    s = s + j * j; s = s + k * k; s = s + r * r;
    const float ts = 2.0f / s;
    volatile float u;
    u = j * j + k * k; R[0] = 1.0f - ts * u;
    u = i * j - k * r; R[1] = ts * u;
    u = i * k + j * r; R[2] = ts * u;
    u = i * j + k * r; R[3] = ts * u;
    u = i * i + k * k; R[4] = 1.0f - ts * u;
    u = j * k - i * r; R[5] = ts * u;
    u = i * k - j * r; R[6] = ts * u;
    u = j * k + i * r; R[7] = ts * u;
    u = i * i + j * j; R[8] = 1.0f - ts * u;
}

// ZYX Euler (rotation_conversions.py:277-319): returns (yaw, pitch, roll).
void euler_zyx(const float* m, float* ypr) {
    float v = -m[6];
    v = std::min(1.0f, std::max(-1.0f, v));
    ypr[1] = asinf(v);
    ypr[0] = atan2f(m[3], m[0]);
    ypr[2] = atan2f(m[7], m[8]);
}

// Savitzky-Golay smoothing taps (svg_filter.py:50-55): first row of
// inv(A^T A) A^T for the Vandermonde A on x = -h..h (fp64 solve, fp32 taps).
int savgol_taps(int window, int order, float* c) {
    if (window < 1 || window % 2 == 0 || window > kMaxW || order < 0 || order >= window) return -1;
    const int h = window / 2, n = order + 1;
    double M[16][16] = {}, Minv[16][16] = {};
    for (int r = 0; r < n; ++r)
        for (int s = 0; s < n; ++s) {
            double acc = 0.0;
            for (int x = -h; x <= h; ++x) acc += std::pow((double)x, r) * std::pow((double)x, s);
            M[r][s] = acc;
        }
    for (int r = 0; r < n; ++r) Minv[r][r] = 1.0;
    for (int col = 0; col < n; ++col) {   // Gauss-Jordan with partial pivoting
        int piv = col;
        for (int r = col + 1; r < n; ++r)
            if (std::fabs(M[r][col]) > std::fabs(M[piv][col])) piv = r;
        for (int s = 0; s < n; ++s) { std::swap(M[col][s], M[piv][s]); std::swap(Minv[col][s], Minv[piv][s]); }
        const double d = M[col][col];
        for (int s = 0; s < n; ++s) { M[col][s] /= d; Minv[col][s] /= d; }
        for (int r = 0; r < n; ++r) {
            if (r == col) continue;
            const double f = M[r][col];
            for (int s = 0; s < n; ++s) { M[r][s] -= f * M[col][s]; Minv[r][s] -= f * Minv[col][s]; }
        }
    }
    for (int x = -h; x <= h; ++x) {
        double acc = 0.0;
        for (int s = 0; s < n; ++s) acc += Minv[0][s] * std::pow((double)x, s);
        c[x + h] = (float)acc;
    }
    return 0;
}

void bake_joint(const mppi_joint& j, JointDev& d) {
    std::memset(&d, 0, sizeof(d));
    d.type = j.type;
    d.q_index = j.q_index;
    float T16[16];
    joint_origin(j, T16);
    for (int i = 0; i < 12; ++i) d.O[i] = T16[i];
    unit_axis(j, d.ax);
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) d.axx[3 * r + c] = d.ax[r] * d.ax[c];
    d.axis_z = (d.ax[0] == 0.0f && d.ax[1] == 0.0f && d.ax[2] == 1.0f) ? 1 : 0;
}

// C = A * B for 3x4 affine rows (implicit last row 0 0 0 1), fp32.
void mul34(const float* A, const float* B, float* C) {
    float r[12];
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 4; ++j) {
            float acc = A[4 * i] * B[j] + A[4 * i + 1] * B[4 + j] + A[4 * i + 2] * B[8 + j];
            if (j == 3) acc += A[4 * i + 3];
            r[4 * i + j] = acc;
        }
    }
    std::memcpy(C, r, sizeof(r));
}

// The joints' constant parts for the host FK: origin transforms (rpy -> R: six libm trig calls per
// joint) and unit axes.  An engine computes them once (mppi_create); per control call they were
// ~1.5 us of check_reach's ~2 us.
void fk_consts(const mppi_joint* joints, int nj, float* O16s, float* axes) {
    for (int n = 0; n < nj; ++n) {
        joint_origin(joints[n], O16s + 16 * n);
        unit_axis(joints[n], axes + 3 * n);
    }
}

// Host FK at one joint vector (check_reach path, urdf_fk.py:60-75 +
// urdfparser.py:166-206): cos/sin in the state dtype, transforms in fp32.
void host_fk_c(const mppi_joint* joints, int nj, const float* O16s, const float* axes, const double* q,
               const double* xyzquat, bool f64, float* out16) {
    float T[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    auto mul = [](const float* A, const float* B, float* C) {
        float r[16];
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) {
                float acc = 0.0f;
                for (int k = 0; k < 4; ++k) acc += A[4 * i + k] * B[4 * k + j];
                r[4 * i + j] = acc;
            }
        std::memcpy(C, r, sizeof(r));
    };
    for (int n = 0; n < nj; ++n) {
        const mppi_joint& j = joints[n];
        const float* O = O16s + 16 * n;
        const float* a = axes + 3 * n;
        float L[16];
        if (j.type == MPPI_JOINT_REVOLUTE && j.q_index >= 0) {
            const double qv = f64 ? q[j.q_index] : (double)(float)q[j.q_index];
            float c, s;
            if (f64) { c = (float)std::cos(qv); s = (float)std::sin(qv); }
            else { c = cosf((float)qv); s = sinf((float)qv); }
            const float omc = 1.0f - c;
            float R[16] = {c + a[0] * a[0] * omc, a[0] * a[1] * omc - a[2] * s, a[0] * a[2] * omc + a[1] * s, 0,
                           a[1] * a[0] * omc + a[2] * s, c + a[1] * a[1] * omc, a[1] * a[2] * omc - a[0] * s, 0,
                           a[2] * a[0] * omc - a[1] * s, a[2] * a[1] * omc + a[0] * s, c + a[2] * a[2] * omc, 0,
                           0, 0, 0, 1};
            mul(O, R, L);
        } else if (j.type == MPPI_JOINT_PRISMATIC && j.q_index >= 0) {
            const float qf = (float)q[j.q_index];
            float S[16] = {1, 0, 0, a[0] * qf, 0, 1, 0, a[1] * qf, 0, 0, 1, a[2] * qf, 0, 0, 0, 1};
            mul(O, S, L);
        } else {
            std::memcpy(L, O, sizeof(L));
        }
        mul(T, L, T);
    }
    float B[16];
    if (f64) base_from_xyzquat_t<double>(xyzquat, B);
    else base_from_xyzquat_t<float>(xyzquat, B);
    mul(B, T, out16);
}

void host_fk(const mppi_joint* joints, int nj, const double* q, const double* xyzquat, bool f64, float* out16) {
    std::vector<float> O((size_t)16 * nj), ax((size_t)3 * nj);
    fk_consts(joints, nj, O.data(), ax.data());
    host_fk_c(joints, nj, O.data(), ax.data(), q, xyzquat, f64, out16);
}

}  // namespace

// =============================================================================
// MPPI_STAMPS diagnostics: stamp indices in program order and the phase each
// difference measures (see the STAMP calls in mppi_rollout.hip / mppi_finalize.hip).
static const std::vector<int> kRollStampOrder = {0, 9, 10, 8, 1, 2, 3, 4, 5, 11, 6, 12, 7};
static const char* const kRollStampNames[] = {"", "loads(waited)", "philox0", "lds-writes(waited)", "barrier",
                                              "noise", "integrator", "fk+cost", "S+softmin", "deposit",
                                              "combine-barrier", "fw", "record"};
static const std::vector<int> kFinStampOrder = {0, 7, 8, 1, 2, 3, 4, 5, 6};
static const char* const kFinStampNames[] = {"", "loads-issued", "accum(last chunk)", "wave-fold", "barrier",
                                             "combine", "w_eps", "savgol", "update+outputs"};

struct mppi_engine {
    mppi_config cfg;
    int K, H, A, V, nq, qoff, state_dim, out_dim, C, threads;
    int64_t out_bytes;
    DevParams dp;
    FinParams fp;
    float sg_taps[kMaxW];
    float fixedM[12];                   // product of the leading fixed joints (folded into base)
    hipStream_t own_stream = nullptr, stream = nullptr;
    float* d_sigma = nullptr;
    JointDev* d_joints = nullptr;
    VehicleConst* d_vc = nullptr;
    float* d_u_prev = nullptr;
    float* d_noise_in = nullptr;
    uint32_t step_ctr = 0;              // Philox counter word; +1 per finalized step
    uint32_t out_seq = 0;               // completion-flag value of the step read_outputs waits for
    // a native control call's launch descriptions, reused while only the state changes
    bool call_cached = false;
    int call_threads = 0;
    DevParams call_p{};
    FinParams call_f{};
    LaunchDesc call_roll{}, call_fin{};
    // a native batch's launch descriptions, reused while the step's parameters are unchanged
    bool batch_cached = false;
    int batch_threads = 0;
    DevParams batch_p{};
    FinParams batch_f{};
    LaunchDesc batch_roll{}, batch_fin{};
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
    FinTail* d_tail = nullptr;        // [kTailSlots] the finalize's tail parameters per launch kind
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
    unsigned long long* d_xregion = nullptr;   // this rank's exchange region (uncached device memory)
    size_t x_bytes = 0;
    std::vector<void*> x_opened;        // the other ranks' regions, IPC-mapped
    unsigned long long** d_xpeers = nullptr;   // (shard_count) region pointers, device resident
    uint32_t x_epoch = 0;               // the exchange epoch in the tags (mppi_dev.h peer_tag): moved by
                                        // mppi_set_step_counter and mppi_peer_reset on a connected engine
    VehicleConst* h_vc = nullptr;       // pinned staging
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
    // prewarm (mppi_set_prewarm): a host thread learns the control calls' cadence from their start
    // times and touches the native queue through a window before each predicted call
    std::thread pw_thr;
    std::mutex pw_mu;                   // (for pw_cv only)
    std::condition_variable pw_cv;
    std::atomic<int32_t> pw_us{0};      // the window half-width; 0: off
    std::atomic<bool> pw_stop{false};
    std::atomic<int64_t> pw_touches{0};
    std::atomic<int64_t> call_t[8];     // steady-clock start of the last 8 control calls (ring)
    std::atomic<int64_t> call_n{0};     // control calls recorded
    bool pw_spin = false;               // diagnostics (MPPI_PREWARM_SPIN=1): spin between touches
    std::atomic<bool> pw_native{false}; // the last control call went out as native packets
};

namespace {

// the step goes through the exchange slots: several shards, or an engine-owned
// communicator (a one-rank communicator runs the same pack -> all-reduce -> combine).  A shard
// connected by the peer exchange steps like an unsharded engine: its finalize does the exchange.
bool sharded(const mppi_engine* e) { return (e->cfg.shard_count > 1 || e->comm) && !e->peer; }

FinTail tail_of(const FinParams& f, int32_t mode) {
    FinTail t;
    std::memset(&t, 0, sizeof(t));
    t.coef = f.coef; t.dt = f.dt; t.dt2 = f.dt2;
    t.mode = mode; t.model = f.model; t.qoff = f.qoff; t.nq = f.nq; t.state_f64 = f.state_f64;
    t.out_dim = f.out_dim; t.window = f.window;
    t.u_prev = f.u_prev; t.vc = f.vc;
    t.out = f.out; t.u0 = f.u0; t.stats = f.stats; t.flags = f.flags; t.wraw = f.wraw; t.wsmooth = f.wsmooth;
    t.dst = f.dst; t.xbase = f.xbase; t.xslot = f.xslot; t.nslots = f.nslots; t.myslot = f.myslot; t.P = f.P;
    t.xpeers = f.xpeers; t.xlocal = f.xlocal; t.xn = f.xn; t.xme = f.xme; t.xerr = f.xerr;
    std::memcpy(t.sg, f.sg, sizeof(t.sg));
    return t;
}

// a shard's PACK fields (mppi_rollout) into FinParams, and into the PACK tail copy
void pack_fields(const mppi_engine* e, FinParams& f) {
    const size_t slot = (size_t)e->V * e->dp.P;
    f.mode = 1;
    f.dst = e->d_exchange ? e->d_exchange + slot * e->cfg.shard_rank : nullptr;
    f.xbase = e->d_exchange; f.xslot = (int64_t)slot;
    f.nslots = e->cfg.shard_count; f.myslot = e->cfg.shard_rank;
}
mppi_status upload_pack_tail(mppi_engine* e) {
    FinParams f = e->fp;
    pack_fields(e, f);
    const FinTail t = tail_of(f, 1);
    // a PACK of an earlier step may still be reading the old tail on the engine's stream
    // (a non-blocking torch stream: the blocking copy below is not ordered against it)
    HIP_TRY(hipStreamSynchronize(e->stream));
    HIP_TRY(hipMemcpy(e->d_tail + kTailPack, &t, sizeof(t), hipMemcpyHostToDevice));
    return MPPI_OK;
}

// Trajectory planes: k_rollout rows (one rollout's H steps) are padded to 64 B, hp = H
// rounded up to 16 floats, and written whole.  With H = 100 the unpadded rows left partial
// 64 B sectors at both ends of every wave store, which the write-through stores hand to HBM
// as masked writes: arm K=4096 rollout 20.3 us at H = 100 vs 13.4 at H = 128
// (profiles/r02/ab_traj_row_pitch.txt).  k_rollout_quad writes t-major (C,H,Kp) planes,
// its rows (one step's K samples) padded the same way: Kp = K rounded up to 16.
int traj_pitch(const mppi_engine* e) {
    return e->cfg.model == MPPI_MODEL_QUADROTOR ? (e->K + 15) & ~15 : (e->H + 15) & ~15;
}
size_t traj_floats(const mppi_engine* e) {   // all vehicles' planes
    const size_t plane = e->cfg.model == MPPI_MODEL_QUADROTOR ? (size_t)traj_pitch(e) * e->H
                                                               : (size_t)e->K * traj_pitch(e);
    return (size_t)e->V * e->C * plane;
}

// Native batches are not ordered with the engine's HIP stream: every entry point that touches
// the device (use_device) first waits for them.
mppi_status aql_join(mppi_engine* e) {
    if (e->aql && mppi_aql::step_busy(e->aql)) {
        std::string err;
        if (mppi_aql::step_wait(e->aql, 60000, &err) != 0) return fail(MPPI_ERR_HIP, "%s", err.c_str());
    }
    return MPPI_OK;
}

mppi_status use_device(mppi_engine* e) {
    HIP_TRY(hipSetDevice(e->cfg.device));
    return aql_join(e);
}

size_t off_u0(const mppi_engine* e) { return ((size_t)e->V * e->out_dim * sizeof(double) + 15) & ~size_t(15); }
size_t off_stats(const mppi_engine* e) { return (off_u0(e) + (size_t)e->V * e->A * sizeof(float) + 15) & ~size_t(15); }
// tagged output records of a read step (k_finalize): per vehicle, 2 per dim -- (o1, u0, seq),
// (o2, nan flag, seq) -- and one (rho, eta, ess, seq), 16 B each, each written by ONE store;
// the host polls their tags and takes the values from the records themselves
size_t off_flags(const mppi_engine* e) { return off_stats(e) + (size_t)e->V * 16; }
size_t rec_count(const mppi_engine* e) { return (size_t)e->V * (2 * e->A + 1); }
// the peer exchange's sticky timeout word (16 B after the records): the step tag of a finalize
// block that gave a step up, written by that block, cleared only by the host (mppi_peer_reset)
size_t off_xerr(const mppi_engine* e) { return off_flags(e) + rec_count(e) * 16; }
uint32_t sticky_timeout(const mppi_engine* e) {
    return e->h_out ? *(const volatile uint32_t*)(e->h_out + off_xerr(e)) : 0u;
}
// this rank's exchange region past its control words (mppi_dev.h kXCtl): the partials' base
unsigned long long* xdata(const mppi_engine* e) { return e->d_xregion + kXCtl; }

mppi_status build_vehicle_consts(mppi_engine* e) {
    const mppi_config& c = e->cfg;
    for (int v = 0; v < e->V; ++v) {
        VehicleConst& vc = e->h_vc[v];
        std::memset(&vc, 0, sizeof(vc));
        for (int j = 0; j < kMaxJ; ++j) { vc.qc[j] = c.q_center[j]; vc.qlo[j] = c.q_lower[j]; vc.qhi[j] = c.q_upper[j]; }
        const double* s = e->state.data() + (size_t)v * e->state_dim;
        std::memcpy(vc.tpos, &e->tpos[3 * v], 3 * sizeof(float));
        std::memcpy(&vc._pad[2], &e->x_epoch, sizeof(uint32_t));   // the exchange epoch (kVcEpochWord)
        quat_xyzw_to_R(&e->tquat[4 * v], vc.tR);
        if (c.model == MPPI_MODEL_DRONE) {
            for (int a = 0; a < 3; ++a) {
                vc.pos0f[a] = (float)s[a]; vc.vel0f[a] = (float)s[3 + a];
                vc.pos0[a] = vc.pos0f[a]; vc.vel0[a] = vc.vel0f[a];
            }
        } else if (c.model == MPPI_MODEL_QUADROTOR) {   // xyz rpy | v omega (float32 tensors)
            for (int a = 0; a < 6; ++a) {
                vc.pos0f[a] = (float)s[a]; vc.vel0f[a] = (float)s[6 + a];
                vc.pos0[a] = vc.pos0f[a]; vc.vel0[a] = vc.vel0f[a];
            }
        } else if (c.model == MPPI_MODEL_ARM) {
            float T16[16];
            if (c.state_f64) base_from_xyzquat_t<double>(s, T16);
            else base_from_xyzquat_t<float>(s, T16);
            mul34(T16, e->fixedM, vc.base);
            for (int a = 0; a < e->nq; ++a) {
                const double q = s[7 + a], qd = s[7 + e->nq + a];
                vc.pos0f[a] = (float)q; vc.vel0f[a] = (float)qd;
                vc.pos0[a] = c.state_f64 ? q : (double)vc.pos0f[a];
                vc.vel0[a] = c.state_f64 ? qd : (double)vc.vel0f[a];
            }
        } else {   // whole-body: base pos(3) quat(4) q(nq) base vel(3) qd(nq)
            float qf[4] = {(float)s[3], (float)s[4], (float)s[5], (float)s[6]};
            float Rq[9], ypr[3], R[9];
            quat_xyzw_to_R(qf, Rq);
            euler_zyx(Rq, ypr);
            rpy_to_R(ypr[2], ypr[1], ypr[0], R);   // transformation_matrix.py:148-187
            float B[12] = {R[0], R[1], R[2], 0.0f, R[3], R[4], R[5], 0.0f, R[6], R[7], R[8], 0.0f};
            mul34(B, e->fixedM, vc.base);    // translation column: R * M_t; p(k,t) added on device
            for (int a = 0; a < 3; ++a) {
                vc.pos0f[a] = (float)s[a]; vc.vel0f[a] = (float)s[7 + e->nq + a];
            }
            for (int a = 0; a < e->nq; ++a) {
                vc.pos0f[3 + a] = (float)s[7 + a]; vc.vel0f[3 + a] = (float)s[7 + e->nq + 3 + a];
            }
            for (int a = 0; a < e->A; ++a) { vc.pos0[a] = vc.pos0f[a]; vc.vel0[a] = vc.vel0f[a]; }
        }
    }
    return MPPI_OK;
}

// QUADROTOR outputs: the model's first step (k_rollout_quad, t = 0) under the new u[0],
// in fp32 as the device / the reference's float32 tensors: x_des = (p, rpy) and
// v_des = (v, omega) after one step (the drone returns the same pair, drone_mppi.py:168-175).
void quad_outputs(const mppi_engine* e, const double* s, const float* u0, double* out) {
    const DevParams& p = e->dp;
    const float dt = p.dt;
    float x[12];
    for (int i = 0; i < 12; ++i) x[i] = (float)s[i];
    const float sr = std::sin(x[3]), cr = std::cos(x[3]), sp = std::sin(x[4]), cp = std::cos(x[4]);
    const float sy = std::sin(x[5]), cy = std::cos(x[5]);
    const float tp = sp / cp;
    const float r02 = cy * sp * cr + sy * sr, r12 = sy * sp * cr - cy * sr, r22 = cp * cr;
    const float wx = x[9], wy = x[10], wz = x[11];
    const float dr = wx + sr * tp * wy + cr * tp * wz;
    const float dpi = cr * wy - sr * wz;
    const float dya = sr / cp * wy + cr / cp * wz;
    out[0] = x[0] + dt * x[6]; out[1] = x[1] + dt * x[7]; out[2] = x[2] + dt * x[8];
    out[3] = x[3] + dt * dr; out[4] = x[4] + dt * dpi; out[5] = x[5] + dt * dya;
    const float thr = u0[0];
    out[6] = x[6] + dt * (p.q_inv_m * (r02 * thr - p.q_kd * x[6]));
    out[7] = x[7] + dt * (p.q_inv_m * (r12 * thr - p.q_kd * x[7]));
    out[8] = x[8] + dt * (-p.q_g + p.q_inv_m * (r22 * thr - p.q_kd * x[8]));
    out[9] = wx + dt * (p.q_iinv[0] * u0[1]);
    out[10] = wy + dt * (p.q_iinv[1] * u0[2]);
    out[11] = wz + dt * (p.q_iinv[2] * u0[3]);
}

mppi_status upload_consts(mppi_engine* e) {
    if (e->vc_pending) {   // the previous copy out of the staging buffer must be done
        HIP_TRY(hipEventSynchronize(e->ev_vc));
        e->vc_pending = false;
    }
    mppi_status st = build_vehicle_consts(e);
    if (st != MPPI_OK) return st;
    if (e->V == 1) return MPPI_OK;   // passed by value in the kernel arguments
    HIP_TRY(hipMemcpyAsync(e->d_vc, e->h_vc, sizeof(VehicleConst) * e->V, hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipEventRecord(e->ev_vc, e->stream));
    e->vc_pending = true;
    return MPPI_OK;
}

hipEvent_t pool_event(mppi_engine* e) {
    if (!e->ev_pool.empty()) {
        hipEvent_t ev = e->ev_pool.back();
        e->ev_pool.pop_back();
        return ev;
    }
    hipEvent_t ev = nullptr;
    (void)hipEventCreate(&ev);
    return ev;
}

mppi_status drain_timing(mppi_engine* e) {
    for (auto* vec : {&e->roll_pairs, &e->fin_pairs}) {
        for (auto& pr : *vec) {
            HIP_TRY(hipEventSynchronize(pr.second));
            float ms = 0.0f;
            HIP_TRY(hipEventElapsedTime(&ms, pr.first, pr.second));
            if (vec == &e->roll_pairs) { e->roll_ms += ms; ++e->roll_n; }
            else { e->fin_ms += ms; ++e->fin_n; }
            e->ev_pool.push_back(pr.first);
            e->ev_pool.push_back(pr.second);
        }
        vec->clear();
    }
    return MPPI_OK;
}

mppi_status validate(const mppi_config& c) {
    if (c.model < 0 || c.model > 3) return fail(MPPI_ERR_INVALID_ARG, "unknown model %d", c.model);
    if (c.n_vehicles < 1 || c.n_samples < 1 || c.n_horizon < 2 || c.n_horizon > MPPI_MAX_HORIZON)
        return fail(MPPI_ERR_INVALID_ARG, "bad sizes V=%d K=%d H=%d", c.n_vehicles, c.n_samples, c.n_horizon);
    if (c.model == MPPI_MODEL_DRONE && c.n_action != 3)
        return fail(MPPI_ERR_INVALID_ARG, "DRONE needs n_action=3");
    if (c.model == MPPI_MODEL_ARM && c.n_action != 7)
        return fail(MPPI_ERR_INVALID_ARG, "ARM kernels are built for the 7-DoF Kinova chain (n_action 7, got %d)",
                    c.n_action);
    if (c.model == MPPI_MODEL_WHOLEBODY && c.n_action != 10)
        return fail(MPPI_ERR_INVALID_ARG, "WHOLEBODY kernels are built for 3 + 7 dims (n_action 10, got %d)",
                    c.n_action);
    if (c.model == MPPI_MODEL_QUADROTOR) {
        if (c.n_action != 4) return fail(MPPI_ERR_INVALID_ARG, "QUADROTOR needs n_action=4 (thrust + 3 torques)");
        if (c.n_horizon > 64) return fail(MPPI_ERR_INVALID_ARG, "QUADROTOR supports H <= 64 (got %d)", c.n_horizon);
        if (!(c.quad_mass > 0.0f) || !(c.quad_inertia[0] > 0.0f) || !(c.quad_inertia[1] > 0.0f) ||
            !(c.quad_inertia[2] > 0.0f))
            return fail(MPPI_ERR_INVALID_ARG, "QUADROTOR needs a positive mass and inertia");
    }
    if (c.model == MPPI_MODEL_ARM || c.model == MPPI_MODEL_WHOLEBODY) {
        if (c.n_joints < 1 || c.n_joints > MPPI_MAX_JOINTS)
            return fail(MPPI_ERR_INVALID_ARG, "n_joints=%d", c.n_joints);
        const int nq = nq_of(c);
        for (int j = 0; j < c.n_joints; ++j) {
            const mppi_joint& jj = c.joints[j];
            if (jj.type < 0 || jj.type > 2) return fail(MPPI_ERR_INVALID_ARG, "joint %d: bad type", j);
            if (jj.type != MPPI_JOINT_FIXED && (jj.q_index < 0 || jj.q_index >= nq))
                return fail(MPPI_ERR_INVALID_ARG, "joint %d: q_index %d outside [0,%d)", j, jj.q_index, nq);
        }
    }
    const int half = c.savgol_window / 2;
    if (c.savgol_window % 2 != 1 || c.savgol_window > kMaxW)
        return fail(MPPI_ERR_INVALID_ARG, "Window size must be odd (and <= %d).", kMaxW);
    if (c.savgol_order >= c.savgol_window)
        return fail(MPPI_ERR_INVALID_ARG, "Polyorder must be less than window size.");
    if (c.n_horizon <= half)
        return fail(MPPI_ERR_INVALID_ARG, "Padding (%d) is too large for data length (%d).", half, c.n_horizon);
    if (!(c.lambda_ > 0.0) || !(c.dt > 0.0)) return fail(MPPI_ERR_INVALID_ARG, "lambda and dt must be > 0");
    if (c.shard_count < 1 || c.shard_rank < 0 || c.shard_rank >= c.shard_count)
        return fail(MPPI_ERR_INVALID_ARG, "shard %d/%d", c.shard_rank, c.shard_count);
    if (c.vehicle_offset < 0 || c.vehicle_offset + c.n_vehicles > 32768)
        return fail(MPPI_ERR_INVALID_ARG, "vehicle_offset %d: the fleet-wide vehicle index must stay below 32768",
                    c.vehicle_offset);
    if (c.cost_terms & ~0x1F) return fail(MPPI_ERR_INVALID_ARG, "unknown cost_terms bits 0x%x", c.cost_terms);
    if (c.cost_terms && (c.model == MPPI_MODEL_DRONE || c.model == MPPI_MODEL_QUADROTOR))
        return fail(MPPI_ERR_INVALID_ARG, "cost_terms apply to the ARM / WHOLEBODY CostManager (not DRONE)");
    if (c.block_threads && (c.block_threads % 64 || c.block_threads > 512))
        return fail(MPPI_ERR_INVALID_ARG, "block_threads must be a multiple of 64 <= 512");
    return MPPI_OK;
}

}  // namespace

// =============================================================================
extern "C" {

int32_t mppi_abi_version(void) { return MPPI_ABI_VERSION; }
// error reporting for the host dynamics TU (mppi_dynamics.cpp); not in the public header
mppi_status mppi_fail_dyn(mppi_status st, const char* msg) { return fail(st, "%s", msg); }
const char* mppi_last_error(void) { return g_err.c_str(); }

void mppi_struct_sizes(int32_t* c, int32_t* j, int32_t* s) {
    if (c) *c = (int32_t)sizeof(mppi_config);
    if (j) *j = (int32_t)sizeof(mppi_joint);
    if (s) *s = (int32_t)sizeof(mppi_stats);
}

void mppi_config_default(mppi_config* c, int32_t model) {
    std::memset(c, 0, sizeof(*c));
    c->model = model;
    c->n_vehicles = 1;
    c->n_horizon = 32;
    c->dt = 0.01;
    c->lambda_ = 0.1;
    c->savgol_order = 2;
    c->seed = 0x5EEDULL;
    c->shard_count = 1;
    c->store_trajectory = 1;
    c->reach_tol = 0.005f;
    if (model == MPPI_MODEL_DRONE) {            // drone_mppi.py:16-35, 87-107, 160
        c->n_samples = 1000; c->n_action = 3;
        for (int a = 0; a < 3; ++a) c->sigma[a * 3 + a] = 30.0f;
        c->w_stage_pos = 100.0f; c->w_term_pos = 20.0f;
        c->savgol_window = 5;
    } else if (model == MPPI_MODEL_QUADROTOR) {  // the drone controller's sizes and cost (drone_mppi.py:16-35,
        c->n_samples = 1000; c->n_action = 4;     // 87-107, 160); Sigma is build-defined: 30 N on the thrust
        c->sigma[0] = 30.0f;                      // (the drone's 30), 1 N m on each torque
        for (int a = 1; a < 4; ++a) c->sigma[a * 4 + a] = 1.0f;
        c->w_stage_pos = 100.0f; c->w_term_pos = 20.0f;
        c->savgol_window = 5;
    } else {                                     // mppi.py:37-75; cost_manager.py:25-28
        c->n_samples = 100;
        c->n_action = (model == MPPI_MODEL_ARM) ? 7 : 10;
        const int A = c->n_action;
        for (int a = 0; a < A; ++a) c->sigma[a * A + a] = 0.1f;
        if (model == MPPI_MODEL_WHOLEBODY) {
            c->n_horizon = 64;
            for (int a = 0; a < 3; ++a) c->sigma[a * A + a] = 30.0f;
        }
        c->w_stage_pos = 50.0f; c->w_stage_ori = 30.0f; c->w_term_pos = 40.0f; c->w_term_ori = 30.0f;
        c->savgol_window = 9;
        c->check_reach = (model == MPPI_MODEL_ARM);
        c->state_f64 = (model == MPPI_MODEL_ARM);
    }
    // extra CostManager terms, off as in the reference (cost_manager.py:83-87); weights
    // cost_manager.py:21-43, targets / limits joint_space_cost.py:16,71-72
    c->cost_terms = 0;
    c->w_covar = 0.1f; c->cost_alpha = 0.1f; c->cost_gamma = 0.98f;
    c->w_center = 1.0f; c->w_joint_track = 1.0f; c->w_action = 0.01f; c->joint_limit_penalty = 1e10f;
    const float qc[7] = {0.0f, 0.0f, 0.0f, (float)((-3.0718 - 0.0698) / 2), 0.0f, (float)((3.7525 - 0.0175) / 2), 0.0f};
    const float lo[7] = {-6.2832f, 0.8203f, -6.2832f, 0.5236f, -6.2832f, 1.1345f, -6.2832f};
    const float hi[7] = {6.2832f, 5.4629f, 6.2832f, 5.7596f, 6.2832f, 5.1487f, 6.2832f};
    for (int j = 0; j < MPPI_MAX_JOINTS; ++j) {
        c->q_center[j] = j < 7 ? qc[j] : 0.0f;
        c->q_lower[j] = j < 7 ? lo[j] : -INFINITY;
        c->q_upper[j] = j < 7 ? hi[j] : INFINITY;
    }
    c->quad_mass = 14.7f;                                  // drone.urdf:15-16
    c->quad_inertia[0] = 1.57f; c->quad_inertia[1] = 3.93f; c->quad_inertia[2] = 2.59f;
    c->quad_kd = 0.0f;
    c->quad_gravity = 9.81f;
}

int32_t mppi_state_dim(const mppi_config* c) {
    const int nq = nq_of(*c);
    if (c->model == MPPI_MODEL_DRONE) return 6;
    if (c->model == MPPI_MODEL_QUADROTOR) return 12;
    if (c->model == MPPI_MODEL_ARM) return 7 + 2 * nq;
    return 7 + nq + 3 + nq;
}

int32_t mppi_output_dim(const mppi_config* c) {
    const int nq = nq_of(*c);
    if (c->model == MPPI_MODEL_DRONE) return 6;
    if (c->model == MPPI_MODEL_QUADROTOR) return 12;
    if (c->model == MPPI_MODEL_ARM) return 2 * nq;
    return 6 + 2 * nq;
}

int32_t mppi_traj_channels(const mppi_config* c) {
    if (c->model == MPPI_MODEL_DRONE) return 3;
    if (c->model == MPPI_MODEL_QUADROTOR) return 6;
    return c->n_action + 16;
}

int64_t mppi_rollout_bytes(const mppi_config* c) {
    // algorithmic bytes of one rollout launch: trajectory planes written
    // (+ injected eps read, + eps written when stored) + S + partial records
    const int64_t KH = (int64_t)c->n_vehicles * c->n_samples * c->n_horizon;
    const int64_t C = (c->model == MPPI_MODEL_DRONE) ? 3 : (c->model == MPPI_MODEL_QUADROTOR) ? 6 : c->n_action + 12;
    int64_t b = 0;
    if (c->store_trajectory) b += KH * C * 4;
    if (c->noise_mode == MPPI_NOISE_INJECTED) b += KH * c->n_action * 4;
    if (c->store_noise) b += KH * c->n_action * 4;
    b += (int64_t)c->n_vehicles * c->n_samples * 4;
    return b;
}

void mppi_joint_origin(const mppi_joint* j, float* T16) { joint_origin(*j, T16); }

void mppi_base_transform(const double* xyzquat, int32_t f64, float* T16) {
    if (f64) base_from_xyzquat_t<double>(xyzquat, T16);
    else base_from_xyzquat_t<float>(xyzquat, T16);
}

void mppi_target_rotation(const float* q, float* R9) { quat_xyzw_to_R(q, R9); }

int32_t mppi_savgol_coefficients(int32_t window, int32_t order, float* c) { return savgol_taps(window, order, c); }

mppi_status mppi_host_fk(const mppi_joint* joints, int32_t nj, const double* q, const double* xyzquat,
                         int32_t f64, float* T16) {
    if (!joints || nj < 0 || nj > MPPI_MAX_JOINTS || !q || !xyzquat || !T16)
        return fail(MPPI_ERR_INVALID_ARG, "mppi_host_fk: bad arguments");
    host_fk(joints, nj, q, xyzquat, f64 != 0, T16);
    return MPPI_OK;
}

mppi_status mppi_create(const mppi_config* cfg, mppi_engine** out) {
    if (!cfg || !out) return fail(MPPI_ERR_INVALID_ARG, "null argument");
    *out = nullptr;
    mppi_status st = validate(*cfg);
    if (st != MPPI_OK) return st;
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (cfg->device < 0 || cfg->device >= ndev)
        return fail(MPPI_ERR_INVALID_ARG, "device %d not present (%d HIP devices)", cfg->device, ndev);

    mppi_engine* e = new mppi_engine();
    e->cfg = *cfg;
    if (e->cfg.model == MPPI_MODEL_WHOLEBODY) e->cfg.state_f64 = 0;
    const mppi_config& c = e->cfg;
    e->K = c.n_samples; e->H = c.n_horizon; e->A = c.n_action; e->V = c.n_vehicles;
    e->nq = nq_of(c);
    e->qoff = (c.model == MPPI_MODEL_WHOLEBODY) ? 3 : 0;
    e->state_dim = mppi_state_dim(&c);
    e->out_dim = mppi_output_dim(&c);
    e->C = (c.model == MPPI_MODEL_DRONE) ? 3 : (c.model == MPPI_MODEL_QUADROTOR) ? 6 : e->A + 12;
    e->tpos.assign((size_t)3 * e->V, 0.0f);
    e->fk_O.assign((size_t)16 * std::max(0, (int)e->cfg.n_joints), 0.0f);
    e->fk_ax.assign((size_t)3 * std::max(0, (int)e->cfg.n_joints), 0.0f);
    fk_consts(e->cfg.joints, e->cfg.n_joints, e->fk_O.data(), e->fk_ax.data());
    e->tquat.assign((size_t)4 * e->V, 0.0f);
    for (int v = 0; v < e->V; ++v) e->tquat[4 * v + 3] = 1.0f;
    e->state.assign((size_t)e->state_dim * e->V, 0.0);

    // ---- geometry
    const int H = e->H;
    const int L = (H > 32) ? 64 : 32;
    const int nch = (H + 63) / 64;
    if (nch != 1 && nch != 2 && nch != 4) {
        delete e;
        return fail(MPPI_ERR_INVALID_ARG, "H=%d: supported horizons are <= 128 or 193..256", H);
    }
    const int R = 64 / L;
    e->threads = c.block_threads ? c.block_threads : 512;
    const int nw = e->threads / 64;
    const int groups = (e->K + nw * R - 1) / (nw * R);
    int nb = c.blocks_per_vehicle;
    // auto: one block per group (iters == 1: the single-group kernel) while the grid is at
    // most 512 blocks (2 per CU); above that >= 2 groups per block (the looping kernel; the
    // prologue and the block combine are amortised, fewer records for the finalize),
    // capped at 1024 blocks in total.  Re-measured on MI355X in round 5 (tools/probes.py geom,
    // profiles/r05/geom): WB K=8192 step pair 17.6 us at 512 looping blocks vs 19.5-20.7 at 1024
    // single-group blocks (whose finalize also reads twice the records) and 18.3 at 256; K=65536
    // best at 1024 (85.2-86.1 us pairs vs 87.6-92.9 at 512, 89.1+ with 256-thread blocks).
    if (nb <= 0) {
        nb = (groups * e->V <= 512) ? groups : std::min(std::max(1, groups / 2), std::max(1, 1024 / e->V));
    }
    nb = std::min(nb, groups);
    int iters = (groups + nb - 1) / nb;
    // a block's cost run (iters * nw * R samples) is staged in LDS for one write-through store
    // (k_rollout): at most kMaxCostRun floats, more blocks otherwise
    iters = std::min(iters, std::max(1, kMaxCostRun / cost_run_stride(nw * R)));
    nb = (groups + iters - 1) / iters;
    if (c.model == MPPI_MODEL_QUADROTOR) {   // k_rollout_quad: 16 rollouts (4 lanes each) per dynamics
        e->threads = 256;                     // wave; 1 dynamics wave per block up to 1024 blocks, else 4
        iters = ((e->K + 15) / 16 * e->V <= 1024) ? 1 : 4;   // (carried in DevParams::iters)
        nb = (e->K + 16 * iters - 1) / (16 * iters);
    }
    if (nb > 4096) { delete e; return fail(MPPI_ERR_INVALID_ARG, "too many rollout blocks (%d)", nb); }
    const int P = (kHdr + e->A * H + 3) & ~3;
    // the rollout kernels address one vehicle's trajectory planes through a buffer
    // resource (32-bit byte offsets) and the record bodies with 32-bit indices
    if (c.store_trajectory && (uint64_t)e->C * ((e->K + 15) & ~15) * ((H + 15) & ~15) * sizeof(float) > 0xFFFFFFFFull) {
        const int C = e->C, K = e->K;
        delete e;
        return fail(MPPI_ERR_INVALID_ARG, "trajectory of one vehicle (C=%d x K=%d x H=%d floats) exceeds 4 GiB: "
                    "disable store_trajectory or shard the samples", C, K, H);
    }
    if ((uint64_t)e->V * e->A * nb * H >= 0x80000000ull) {
        const int V = e->V, A = e->A;
        delete e;
        return fail(MPPI_ERR_INVALID_ARG, "record bodies (V=%d x A=%d x %d blocks x H=%d = %llu floats) exceed 2^31",
                    V, A, nb, H, (unsigned long long)V * A * nb * H);
    }

    if (savgol_taps(c.savgol_window, c.savgol_order, e->sg_taps) != 0) {
        delete e;
        return fail(MPPI_ERR_INVALID_ARG, "bad SavGol window/order");
    }

#define CREATE_TRY(expr)                                                                  \
    do {                                                                                  \
        hipError_t _e = (expr);                                                           \
        if (_e != hipSuccess) {                                                           \
            fail(MPPI_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(_e));            \
            mppi_destroy(e);                                                              \
            return MPPI_ERR_HIP;                                                          \
        }                                                                                 \
    } while (0)

    CREATE_TRY(hipSetDevice(c.device));
    CREATE_TRY(hipStreamCreateWithFlags(&e->own_stream, hipStreamNonBlocking));
    e->stream = e->own_stream;
    CREATE_TRY(hipEventCreateWithFlags(&e->ev_vc, hipEventDisableTiming));
    CREATE_TRY(hipEventCreateWithFlags(&e->ev_out, hipEventDisableTiming));
    const size_t KH = (size_t)e->V * e->K * H;
    CREATE_TRY(hipMalloc(&e->d_joints, sizeof(JointDev) * kMaxJ));
    CREATE_TRY(hipMalloc(&e->d_vc, sizeof(VehicleConst) * e->V));
    CREATE_TRY(hipMalloc(&e->d_u_prev, sizeof(float) * e->V * H * e->A));
    CREATE_TRY(hipMalloc(&e->d_S, sizeof(float) * e->V * e->K));
    CREATE_TRY(hipMalloc(&e->d_w, sizeof(float) * e->V * e->K));
    CREATE_TRY(hipMalloc(&e->d_hdr, sizeof(float) * (size_t)e->V * nb * 4));
    CREATE_TRY(hipMalloc(&e->d_rdata, sizeof(float) * (size_t)e->V * e->A * nb * H));
    CREATE_TRY(hipMalloc(&e->d_wraw, sizeof(float) * e->V * H * e->A));
    CREATE_TRY(hipMalloc(&e->d_wsmooth, sizeof(float) * e->V * H * e->A));
    if (c.store_trajectory) CREATE_TRY(hipMalloc(&e->d_traj, sizeof(float) * traj_floats(e)));
    if (c.store_noise) CREATE_TRY(hipMalloc(&e->d_noise_out, sizeof(float) * KH * e->A));
    e->out_bytes = (int64_t)(off_xerr(e) + 16);
    CREATE_TRY(hipMalloc(&e->d_out, e->out_bytes));
    CREATE_TRY(hipHostMalloc((void**)&e->h_out, e->out_bytes, hipHostMallocMapped | hipHostMallocCoherent));
    CREATE_TRY(hipHostGetDevicePointer((void**)&e->h_out_dev, e->h_out, 0));
    std::memset(e->h_out, 0, e->out_bytes);
    CREATE_TRY(hipMalloc(&e->d_sigma, sizeof(float) * kMaxA * kMaxA));
    CREATE_TRY(hipMemcpy(e->d_sigma, c.sigma, sizeof(float) * e->A * e->A, hipMemcpyHostToDevice));
    if (c.cost_terms) {   // Sigma^-1 (covar_cost.py:21), gamma^t (action_cost.py:21), tracking target
        std::vector<double> m(e->A * 2 * e->A, 0.0);
        const int A = e->A, W2 = 2 * A;
        for (int i = 0; i < A; ++i) {
            for (int j = 0; j < A; ++j) m[i * W2 + j] = c.sigma[i * A + j];
            m[i * W2 + A + i] = 1.0;
        }
        for (int col = 0; col < A; ++col) {   // Gauss-Jordan, partial pivoting, fp64
            int piv = col;
            for (int r = col + 1; r < A; ++r)
                if (std::fabs(m[r * W2 + col]) > std::fabs(m[piv * W2 + col])) piv = r;
            if (std::fabs(m[piv * W2 + col]) < 1e-30) { mppi_destroy(e); return fail(MPPI_ERR_INVALID_ARG, "Sigma is singular"); }
            for (int j = 0; j < W2; ++j) std::swap(m[col * W2 + j], m[piv * W2 + j]);
            const double d = m[col * W2 + col];
            for (int j = 0; j < W2; ++j) m[col * W2 + j] /= d;
            for (int r = 0; r < A; ++r)
                if (r != col) {
                    const double f2 = m[r * W2 + col];
                    for (int j = 0; j < W2; ++j) m[r * W2 + j] -= f2 * m[col * W2 + j];
                }
        }
        std::vector<float> sinv(A * A), gam(H);
        for (int i = 0; i < A; ++i)
            for (int j = 0; j < A; ++j) sinv[i * A + j] = (float)m[i * W2 + A + j];
        for (int t = 0; t < H; ++t) gam[t] = std::pow(c.cost_gamma, (float)t);
        CREATE_TRY(hipMalloc(&e->d_sinv, sizeof(float) * A * A));
        CREATE_TRY(hipMalloc(&e->d_gamma, sizeof(float) * H));
        CREATE_TRY(hipMalloc(&e->d_jtraj, sizeof(float) * (size_t)e->V * H * std::max(1, e->nq)));
        CREATE_TRY(hipMemcpy(e->d_sinv, sinv.data(), sizeof(float) * A * A, hipMemcpyHostToDevice));
        CREATE_TRY(hipMemcpy(e->d_gamma, gam.data(), sizeof(float) * H, hipMemcpyHostToDevice));
        CREATE_TRY(hipMemset(e->d_jtraj, 0, sizeof(float) * (size_t)e->V * H * std::max(1, e->nq)));
    }
    CREATE_TRY(hipHostMalloc((void**)&e->h_vc, sizeof(VehicleConst) * e->V, hipHostMallocDefault));
    CREATE_TRY(hipMemsetAsync(e->d_u_prev, 0, sizeof(float) * e->V * H * e->A, e->stream));
    CREATE_TRY(hipMemsetAsync(e->d_out, 0, e->out_bytes, e->stream));

    std::vector<JointDev> jd(kMaxJ);
    for (int j = 0; j < c.n_joints; ++j) bake_joint(c.joints[j], jd[j]);
    // fold the leading fixed joints of the chain into the per-vehicle base transform
    const float I12[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
    std::memcpy(e->fixedM, I12, sizeof(I12));
    int j0 = 0;
    while (c.model != MPPI_MODEL_DRONE && j0 < c.n_joints && jd[j0].type == MPPI_JOINT_FIXED) {
        mul34(e->fixedM, jd[j0].O, e->fixedM);
        ++j0;
    }
    CREATE_TRY(hipMemcpy(e->d_joints, jd.data(), sizeof(JointDev) * kMaxJ, hipMemcpyHostToDevice));
    CREATE_TRY(hipStreamSynchronize(e->stream));
#undef CREATE_TRY

    DevParams& p = e->dp;
    std::memset(&p, 0, sizeof(p));
    p.model = c.model; p.V = e->V; p.K = e->K; p.H = H; p.A = e->A;
    p.L = L; p.R = R; p.nch = nch; p.nb = nb; p.iters = iters;
    p.nq = e->nq; p.qoff = e->qoff; p.nj = c.n_joints;
    // (the vehicle offset in the high half: the rollouts' fleet-wide Philox vehicle key)
    p.noise_mode = c.noise_mode | (c.vehicle_offset << 16); p.state_f64 = c.state_f64;
    p.store_traj = c.store_trajectory; p.store_noise = c.store_noise;
    bool diag = true;
    for (int a = 0; a < e->A; ++a)
        for (int b = 0; b < e->A; ++b) {
            if (a == b) p.sdiag[a] = c.sigma[a * e->A + b];
            else if (c.sigma[a * e->A + b] != 0.0f) diag = false;
        }
    p.sigma_diag = diag;
    p.sigma = e->d_sigma;
    p.j0 = j0;
    {   // fast FK path: the unfolded chain is exactly nq revolute-z joints in q order
        bool fast = c.model != MPPI_MODEL_DRONE && (c.n_joints - j0) == e->nq;
        for (int j = j0; fast && j < c.n_joints; ++j)
            fast = jd[j].type == MPPI_JOINT_REVOLUTE && jd[j].axis_z && jd[j].q_index == j - j0;
        p.chain_fast = fast;
        if (fast && e->nq == 7 && c.n_joints - j0 == 7) {   // Kinova origin table (mppi_dev.h kKinova)
            bool kin = true;
            for (int j = 0; kin && j < 7; ++j) {
                const float* O = jd[j0 + j].O;
                const KinOrigin& k = kKinova[j];
                for (int col = 0; kin && col < 3; ++col)
                    for (int row = 0; kin && row < 3; ++row) {
                        const float want = (row == k.p[col]) ? (float)k.s[col] : 0.0f;
                        kin = std::fabs(O[4 * row + col] - want) <= 1e-6f;
                    }
                for (int d = 0; kin && d < 3; ++d) kin = ((k.tmask >> d) & 1) ? true : (O[4 * d + 3] == 0.0f);
            }
            if (kin && !getenv("MPPI_NO_KINOVA_PATH")) p.chain_fast = 2;
        }
    }
    p.P = P; p.C = e->C; p.hp = traj_pitch(e);
    p.seed_lo = (uint32_t)c.seed; p.seed_hi = (uint32_t)(c.seed >> 32);
    p.k_offset = (int64_t)c.shard_rank * e->K;
    p.dt = (float)c.dt; p.dt2 = (float)(c.dt * c.dt); p.dt_d = c.dt;
    p.coef = (float)(-1.0 / c.lambda_);
    p.w_sp = c.w_stage_pos; p.w_so = c.w_stage_ori; p.w_tp = c.w_term_pos; p.w_to = c.w_term_ori;
    p.joints = e->d_joints;
    p.cost_terms = c.cost_terms;
    p.w_cov = (float)((double)c.w_covar * (c.lambda_ * (1.0 - (double)c.cost_alpha)));   // covar_cost.py:15,24
    p.w_cen = c.w_center; p.w_jt = c.w_joint_track; p.w_act = c.w_action; p.lim_pen = c.joint_limit_penalty;
    p.sinv = e->d_sinv; p.gamma_t = e->d_gamma; p.jtraj = e->d_jtraj;
    p.q_inv_m = (float)(1.0 / (double)c.quad_mass);   // 1/self.m as a Python float, used in fp32
    for (int d = 0; d < 3; ++d) p.q_iinv[d] = (float)(1.0 / (double)c.quad_inertia[d]);
    p.q_kd = c.quad_kd; p.q_g = c.quad_gravity; p.q_literal_jinv = c.quad_literal_jinv ? 1 : 0;
    p.vc = e->d_vc; p.u_prev = e->d_u_prev;
    p.traj = e->d_traj; p.noise_out = e->d_noise_out; p.S = e->d_S; p.hdr = e->d_hdr; p.rdata = e->d_rdata;
#ifdef MPPI_STAMPS
    if (getenv("MPPI_STAMPS")) {
        const size_t nwaves = (size_t)e->V * nb * (e->threads / 64);
        if (hipMalloc(&e->d_stamps, nwaves * kStamps * 8) == hipSuccess) p.stamps = e->d_stamps;
        e->stamp_sum.assign(kStamps, 0.0);
        // FINAL's blocks, then a shard's PACK blocks (mppi_debug_fstamps)
        (void)hipMalloc(&e->d_fstamps, 2 * (size_t)e->V * e->A * ((H + 7) / 8) * kStamps * 8);
        e->fstamp_sum.assign(kStamps, 0.0);
    }
#endif

    FinParams& f = e->fp;
    std::memset(&f, 0, sizeof(f));
    f.model = c.model; f.V = e->V; f.H = H; f.A = e->A; f.nq = e->nq; f.qoff = e->qoff;
    f.state_f64 = c.state_f64; f.P = P;
    // (diagnostics: MPPI_FIN_TSZ = t per finalize slice, for the slice-count / fetch trade-off
    // measured in profiles/r05/finalize_fetch; 8 is the measured best)
    if (const char* z = getenv("MPPI_FIN_TSZ")) {
        const int tz = atoi(z);
        if (tz >= 1 && tz + 2 * (c.savgol_window / 2) <= 64) e->fin_tsz = tz;
    }
    f.tsz = e->fin_tsz; f.ts = e->fin_ts = (H + e->fin_tsz - 1) / e->fin_tsz;
    f.window = c.savgol_window; f.half = c.savgol_window / 2;
    for (int j = 0; j < c.savgol_window; ++j) f.sg[j] = e->sg_taps[c.savgol_window - 1 - j];
    f.coef = p.coef; f.dt = p.dt; f.dt2 = p.dt2; f.dt_d = c.dt;
    f.u_prev = e->d_u_prev; f.vc = e->d_vc;
    f.out = (double*)e->h_out_dev;
    f.u0 = (float*)(e->h_out_dev + off_u0(e));
    f.stats = (float*)(e->h_out_dev + off_stats(e));
    f.flags = (uint32_t*)(e->h_out_dev + off_flags(e));
    f.xerr = (uint32_t*)(e->h_out_dev + off_xerr(e));
    f.wraw = e->d_wraw; f.wsmooth = e->d_wsmooth; f.out_dim = e->out_dim;
    if (const char* dbg = getenv("MPPI_FIN_DEBUG")) f.dbg = atoi(dbg);
    e->event_wait = getenv("MPPI_EVENT_WAIT") && atoi(getenv("MPPI_EVENT_WAIT")) != 0;
    e->no_flag_dbg = e->event_wait && getenv("MPPI_DEBUG_NO_FLAG") && atoi(getenv("MPPI_DEBUG_NO_FLAG")) != 0;
    e->out_dbg = getenv("MPPI_DEBUG_OUT") ? atoi(getenv("MPPI_DEBUG_OUT")) : 0;
    if (const char* d = getenv("MPPI_DISPATCH")) e->aql_mode = !strcmp(d, "hip") ? 0 : !strcmp(d, "aql") ? 1 : 2;
    f.stamps = e->d_fstamps;
    {   // the finalize's tail parameters, one device copy per launch kind (constant for the
        // engine's life): the control step's FINAL, a shard's PACK, and FINAL into the device
        // scratch outputs (mppi_kernel_timing, probes)
        FinTail t[kTailSlots];
        t[kTailFinal] = tail_of(f, 0);
        t[kTailPack] = tail_of(f, 1);
        t[kTailScratch] = tail_of(f, 0);
        t[kTailScratch].out = (double*)e->d_out;
        t[kTailScratch].u0 = (float*)(e->d_out + off_u0(e));
        t[kTailScratch].stats = (float*)(e->d_out + off_stats(e));
        t[kTailScratch].flags = (uint32_t*)(e->d_out + off_flags(e));
        t[kTailScratch].xerr = (uint32_t*)(e->d_out + off_xerr(e));
        t[kTailScratch].wraw = nullptr;
        t[kTailScratch].wsmooth = nullptr;
        // the step's FINAL stores no readback copies of w_eps: mppi_get_weighted_noise recomputes
        // them from the last step's records (READBACK), so the step's tail carries no extra stores
        t[kTailFinal].wraw = nullptr;
        t[kTailFinal].wsmooth = nullptr;
        t[kTailReadback] = tail_of(f, 2);
        hipError_t te = hipMalloc(&e->d_tail, sizeof(t));
        if (te == hipSuccess) te = hipMemcpy(e->d_tail, t, sizeof(t), hipMemcpyHostToDevice);
        if (te != hipSuccess) {
            fail(MPPI_ERR_HIP, "finalize tail parameters: %s", hipGetErrorString(te));
            mppi_destroy(e);
            return MPPI_ERR_HIP;
        }
        f.tail = e->d_tail + kTailFinal;
    }
    *out = e;
    return MPPI_OK;
}

namespace { void prewarm_stop(mppi_engine* e); }

void mppi_destroy(mppi_engine* e) {
    if (!e) return;
    prewarm_stop(e);   // the prewarm thread first: it writes packets into the native queue
    (void)hipSetDevice(e->cfg.device);
    // the native queue first: its last batch may still write the buffers freed below (stamps
    // included).  A queue that does not drain leaves them leaked rather than freed under it.
    if (e->aql && !mppi_aql::step_destroy(e->aql)) {
        fprintf(stderr, "[mppi] mppi_destroy: the engine's native queue did not drain; its device buffers are leaked\n");
        return;
    }
    e->aql = nullptr;
    if (e->d_stamps && e->stamp_n) {
        fprintf(stderr, "[mppi stamps] rollout avg cycles per wave over %lld waves:", (long long)e->stamp_n);
        for (size_t i = 1; i < kRollStampOrder.size(); ++i)
            fprintf(stderr, " %s=%.0f", kRollStampNames[i], e->stamp_sum[i] / e->stamp_n);
        fprintf(stderr, "\n[mppi stamps] finalize avg cycles per block over %lld blocks:", (long long)e->fstamp_n);
        for (size_t i = 1; i < kFinStampOrder.size(); ++i)
            fprintf(stderr, " %s=%.0f", kFinStampNames[i], e->fstamp_sum[i] / std::max<int64_t>(1, e->fstamp_n));
        fprintf(stderr, "\n");
    }
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    for (auto& pr : e->roll_pairs) { (void)hipEventDestroy(pr.first); (void)hipEventDestroy(pr.second); }
    for (auto& pr : e->fin_pairs) { (void)hipEventDestroy(pr.first); (void)hipEventDestroy(pr.second); }
    for (auto ev : e->ev_pool) (void)hipEventDestroy(ev);
    if (e->comm) rccl().destroy(e->comm);
    for (void* q : e->x_opened) if (q) (void)hipIpcCloseMemHandle(q);
    void* dev[] = {e->d_xregion, e->d_xpeers, e->d_sigma, e->d_joints, e->d_vc, e->d_u_prev, e->d_noise_in, e->d_traj, e->d_noise_out,
                   e->d_S, e->d_hdr, e->d_rdata, e->d_out, e->d_wraw, e->d_wsmooth, e->d_w,
                   e->d_sinv, e->d_gamma, e->d_jtraj, e->d_xown, e->d_tail, e->d_stamps, e->d_fstamps};
    for (void* p : dev) if (p) (void)hipFree(p);
    if (e->h_out) (void)hipHostFree(e->h_out);
    if (e->h_vc) (void)hipHostFree(e->h_vc);
    if (e->ev_vc) (void)hipEventDestroy(e->ev_vc);
    if (e->ev_out) (void)hipEventDestroy(e->ev_out);
    if (e->own_stream) (void)hipStreamDestroy(e->own_stream);
    delete e;
}

// ---------------------------------------------------------------- prewarm (the node's idle gaps)
// At the node's cadence (rospy.Rate(100), kinova.py:101) the engine's queue sits empty ~10 ms
// between calls, and a call on a queue idle for more than ~50-100 us runs ~6-7 us longer than
// back to back; a pair of one-wave packets on the same queue 20-50 us before the call removes
// that, a touch 100 us or more before it does not, nor does a touch on another queue or the
// doorbell alone (profiles/r05/prewarm/).  So the thread predicts the next call from the median
// interval of the last calls and, from pw_us before the prediction until the call starts (or
// pw_us after it), touches the queue every kTouchNs.  Calls back to back or slower than 1 s get
// no touches; nothing the engine computes changes (the touch writes a scratch word only).
namespace {
constexpr int64_t kTouchNs = 25000;

int64_t steady_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

void note_call(mppi_engine* e) {   // mppi_step entry (the caller's thread)
    if (!e->pw_us.load(std::memory_order_relaxed)) return;
    const int64_t n = e->call_n.load(std::memory_order_relaxed);
    e->call_t[n % 8].store(steady_ns(), std::memory_order_relaxed);
    e->call_n.store(n + 1, std::memory_order_release);
}

// The next window from the last m (<= 8) call starts t[] (oldest first): the median interval P
// predicts the call at t[m-1] + P, the window is [that - win, that + win].  0: no window (fewer
// than 4 calls, P < 4 windows -- back to back -- or P > 1 s); 1: *start / *end set.
int prewarm_plan(const int64_t* t, int m, int64_t win, int64_t* start, int64_t* end) {
    if (m < 4) return 0;
    int64_t d[8];
    for (int i = 1; i < m; ++i) d[i - 1] = t[i] - t[i - 1];
    std::nth_element(d, d + (m - 1) / 2, d + (m - 1));
    const int64_t P = d[(m - 1) / 2];
    if (P < 4 * win || P > 1000000000) return 0;
    *start = t[m - 1] + P - win;
    *end = t[m - 1] + P + win;
    return 1;
}

void prewarm_loop(mppi_engine* e) {
    prctl(PR_SET_TIMERSLACK, 1000UL, 0UL, 0UL, 0UL);   // this thread's sleeps end ~1 us after their deadline
    std::unique_lock<std::mutex> lk(e->pw_mu);
    auto nap = [&](int64_t ns) { e->pw_cv.wait_for(lk, std::chrono::nanoseconds(ns), [&] { return e->pw_stop.load(); }); };
    while (!e->pw_stop.load()) {
        const int64_t win = (int64_t)e->pw_us.load() * 1000;
        const int64_t n = e->call_n.load(std::memory_order_acquire);
        // pw_native (acquire) first: a native call stored it (release) after e->aql was set, so the
        // pointer is read only once its write is visible here.  HIP-launched calls: nothing to warm.
        if (n < 4 || !e->pw_native.load(std::memory_order_acquire) || !e->aql) { nap(2000000); continue; }
        const int m = (int)std::min<int64_t>(n, 8);
        int64_t t[8], start = 0, end = 0;
        for (int i = 0; i < m; ++i) t[i] = e->call_t[(n - m + i) % 8].load(std::memory_order_relaxed);
        const int64_t now = steady_ns();
        if (!prewarm_plan(t, m, win, &start, &end) || now > end) { nap(2000000); continue; }   // no cadence, or the call is late
        if (now < start - 200000) { nap(start - 100000 - now); continue; }           // (then look again)
        lk.unlock();   // through the window: a touch, then sleep to the next (the host keeps its core)
        int64_t next = start;
        while (!e->pw_stop.load(std::memory_order_relaxed) && e->call_n.load(std::memory_order_acquire) == n) {
            const int64_t tn = steady_ns();
            if (tn > end) break;
            if (tn >= next) {
                std::string err;
                if (mppi_aql::step_touch(e->aql, true, &err) == 0) e->pw_touches.fetch_add(1, std::memory_order_relaxed);
                next = tn + kTouchNs;
            }
            if (e->pw_spin) _mm_pause();
            else std::this_thread::sleep_for(std::chrono::nanoseconds(std::max<int64_t>(1000, next - steady_ns())));
        }
        lk.lock();
        if (e->call_n.load(std::memory_order_acquire) == n) nap(1000000);   // the window passed without the call
    }
}

void prewarm_stop(mppi_engine* e) {
    if (!e->pw_thr.joinable()) return;
    {
        std::lock_guard<std::mutex> lk(e->pw_mu);
        e->pw_stop.store(true);
    }
    e->pw_cv.notify_all();
    e->pw_thr.join();
    e->pw_stop.store(false);
}
}  // namespace

mppi_status mppi_set_prewarm(mppi_engine* e, int32_t window_us) {
    if (!e) return fail(MPPI_ERR_INVALID_ARG, "null engine");
    if (window_us != 0 && (window_us < 50 || window_us > 5000))
        return fail(MPPI_ERR_INVALID_ARG, "prewarm window %d us: 0 (off) or 50 .. 5000", window_us);
    prewarm_stop(e);
    e->pw_us.store(window_us);
    e->call_n.store(0);
    const char* spin = getenv("MPPI_PREWARM_SPIN");
    e->pw_spin = spin && spin[0] == '1';
    if (window_us) e->pw_thr = std::thread(prewarm_loop, e);
    return MPPI_OK;
}

mppi_status mppi_get_prewarm(mppi_engine* e, int32_t* window_us, int64_t* touches) {
    if (!e || !window_us || !touches) return fail(MPPI_ERR_INVALID_ARG, "null argument");
    *window_us = e->pw_us.load();
    *touches = e->pw_touches.load();
    return MPPI_OK;
}

mppi_status mppi_set_stream(mppi_engine* e, void* s) {
    if (!e) return fail(MPPI_ERR_INVALID_ARG, "null engine");
    if (use_device(e)) return MPPI_ERR_HIP;
    HIP_TRY(hipStreamSynchronize(e->stream));
    e->stream = s ? (hipStream_t)s : e->own_stream;
    return MPPI_OK;
}

mppi_status mppi_set_joint_trajectory(mppi_engine* e, int32_t v, const float* traj) {
    if (!e || v < 0 || v >= e->V) return fail(MPPI_ERR_INVALID_ARG, "mppi_set_joint_trajectory: bad arguments");
    if (!e->d_jtraj) return fail(MPPI_ERR_STATE, "engine created without cost_terms");
    if (use_device(e)) return MPPI_ERR_HIP;
    const size_t n = (size_t)e->H * e->nq;
    float* dst = e->d_jtraj + (size_t)v * n;
    if (traj) HIP_TRY(hipMemcpyAsync(dst, traj, n * sizeof(float), hipMemcpyHostToDevice, e->stream));
    else HIP_TRY(hipMemsetAsync(dst, 0, n * sizeof(float), e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    return MPPI_OK;
}

mppi_status mppi_set_target(mppi_engine* e, int32_t v, const float* pos, const float* quat) {
    if (!e || !pos || v < 0 || v >= e->V) return fail(MPPI_ERR_INVALID_ARG, "mppi_set_target: bad arguments");
    std::memcpy(&e->tpos[3 * v], pos, 3 * sizeof(float));
    if (quat) std::memcpy(&e->tquat[4 * v], quat, 4 * sizeof(float));
    if (e->state_set) {
        if (use_device(e)) return MPPI_ERR_HIP;
        return upload_consts(e);
    }
    return MPPI_OK;
}

mppi_status mppi_set_u_prev(mppi_engine* e, const float* u) {
    if (!e || !u) return fail(MPPI_ERR_INVALID_ARG, "null argument");
    if (use_device(e)) return MPPI_ERR_HIP;
    HIP_TRY(hipMemcpyAsync(e->d_u_prev, u, sizeof(float) * e->V * e->H * e->A, hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    return MPPI_OK;
}

mppi_status mppi_get_u_prev(mppi_engine* e, float* u) {
    if (!e || !u) return fail(MPPI_ERR_INVALID_ARG, "null argument");
    if (use_device(e)) return MPPI_ERR_HIP;
    HIP_TRY(hipMemcpyAsync(u, e->d_u_prev, sizeof(float) * e->V * e->H * e->A, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    return MPPI_OK;
}

mppi_status mppi_set_state(mppi_engine* e, const double* state) {
    if (!e || !state) return fail(MPPI_ERR_INVALID_ARG, "null argument");
    if (use_device(e)) return MPPI_ERR_HIP;
    std::memcpy(e->state.data(), state, sizeof(double) * e->state.size());
    e->state_set = true;
    return upload_consts(e);
}

mppi_status mppi_set_step_counter(mppi_engine* e, uint32_t step) {
    if (!e) return fail(MPPI_ERR_INVALID_ARG, "null engine");
    if (use_device(e)) return MPPI_ERR_HIP;
    e->step_ctr = step;
    if (e->peer) {   // a new exchange epoch: words left in the regions under the old counter never match
        ++e->x_epoch;
        return build_vehicle_consts(e);   // (V == 1: the constants ride in the kernel arguments)
    }
    return MPPI_OK;
}

mppi_status mppi_get_step_counter(mppi_engine* e, uint32_t* step) {
    if (!e || !step) return fail(MPPI_ERR_INVALID_ARG, "null argument");
    *step = e->step_ctr;
    return MPPI_OK;
}

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

namespace {
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
}  // namespace

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
    FinParams& f = e->fp;
    f.xpeers = e->d_xpeers; f.xlocal = xdata(e); f.xn = n; f.xme = me;
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
        for (int r = 0; r < n; ++r)
            if ((uint32_t)(got[r] >> 32) != (tag | (uint32_t)r))
                return fail(MPPI_ERR_COMM, "peer exchange: rank %d's word did not reach this rank's region in the "
                                           "kernel probe (%016llx)", r, got[r]);
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
    HIP_TRY(hipDeviceSynchronize());
    *(volatile uint32_t*)(e->h_out + off_xerr(e)) = 0u;
    e->step_ctr = step;
    e->x_epoch = epoch;
    return build_vehicle_consts(e);
}

// the rollout's per-block partial records (DevParams::hdr / rdata layout)
static void block_records(const mppi_engine* e, FinParams& f) {
    const int64_t nb = e->dp.nb, H = e->H;
    f.nrec = (int32_t)nb;
    f.hdr = e->d_hdr; f.hdr_vs = nb * 4; f.hdr_rs = 4;
    f.dat = e->d_rdata; f.d_vs = (int64_t)e->A * nb * H; f.d_as = nb * H; f.d_rs = H;
}

// The finalize's record source: the rollout blocks' records, or the exchange slots of a shard.
static void final_records(const mppi_engine* e, FinParams& f) {
    if (sharded(e)) {   // slots [shard][v][P]: header then N[a][t]
        const int64_t P = e->dp.P;
        f.nrec = e->cfg.shard_count;
        f.hdr = e->d_exchange; f.hdr_vs = P; f.hdr_rs = (int64_t)e->V * P;
        f.dat = e->d_exchange + kHdr; f.d_vs = P; f.d_as = e->H; f.d_rs = (int64_t)e->V * P;
    } else {
        block_records(e, f);
    }
}

mppi_status mppi_rollout(mppi_engine* e, const float* d_noise) {
    if (!e) return fail(MPPI_ERR_INVALID_ARG, "null engine");
    if (!e->state_set) return fail(MPPI_ERR_STATE, "mppi_rollout before mppi_set_state");
    if (e->cfg.noise_mode == MPPI_NOISE_INJECTED && !d_noise)
        return fail(MPPI_ERR_INVALID_ARG, "INJECTED noise mode needs a device noise buffer");
    if (sharded(e) && !e->d_exchange)
        return fail(MPPI_ERR_STATE, "shard_count > 1 needs mppi_bind_exchange or mppi_comm_init");
    if (use_device(e)) return MPPI_ERR_HIP;
    DevParams p = e->dp;
    p.noise_in = d_noise;
    p.vc0 = e->h_vc[0];
    p.step_ctr = e->step_ctr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (e->timing) { e0 = pool_event(e); e1 = pool_event(e); HIP_TRY(hipEventRecord(e0, e->stream)); }
    int rc = mppi_launch_rollout(&p, e->threads, e->stream);
    if (rc != 0) return fail(MPPI_ERR_HIP, "rollout launch failed (%d: %s)", rc,
                             rc > 0 ? hipGetErrorString((hipError_t)rc) : "no kernel for this model/A/H");
    if (e->timing) {
        HIP_TRY(hipEventRecord(e1, e->stream));
        e->roll_pairs.emplace_back(e0, e1);
        if (e->roll_pairs.size() >= 2048) { mppi_status st = drain_timing(e); if (st) return st; }
    }
    if (sharded(e)) {   // fold this shard's block records into its exchange slot
        FinParams f = e->fp;
        pack_fields(e, f);
        f.tail = e->d_tail + kTailPack;
        if (f.stamps) f.stamps += (size_t)e->V * e->A * e->fin_ts * kStamps;   // diagnostics: PACK's own blocks
        block_records(e, f);
        rc = mppi_launch_finalize(&f, e->stream);
        if (rc != 0) return fail(MPPI_ERR_HIP, "pack launch failed (%d)", rc);
    }
    return MPPI_OK;
}

// record_out: mark the outputs' completion with ev_out (read_outputs waits on it).
// Back-to-back steps (mppi_run_steps) mark only the last one: an event record is
// a queue packet of its own, ~1 us of device time per step.
static mppi_status finalize_impl(mppi_engine* e, bool record_out) {
    if (use_device(e)) return MPPI_ERR_HIP;
    FinParams f = e->fp;
    f.mode = 0;
    f.seq = 0u;   // no completion flag (and no fence) for unread steps
    if (record_out && !e->no_flag_dbg) {   // a fresh value per read step, never 0 (the flags start zeroed):
                                           // the flags the previous read step left can never satisfy this
                                           // step's wait
        f.seq = ++e->seq_ctr & 0x7FFFFFFFu;   // (bit 31: native control calls' numbers)
        if (f.seq == 0u) f.seq = ++e->seq_ctr & 0x7FFFFFFFu;
    }
    final_records(e, f);
    if (e->out_dbg == 1 && !record_out) f.tail = e->d_tail + kTailScratch;   // diagnostic (MPPI_DEBUG_OUT)
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (e->timing) { e0 = pool_event(e); e1 = pool_event(e); HIP_TRY(hipEventRecord(e0, e->stream)); }
    int rc = mppi_launch_finalize(&f, e->stream);
    if (rc != 0) return fail(MPPI_ERR_HIP, "finalize launch failed (%d)", rc);
    if (e->timing) { HIP_TRY(hipEventRecord(e1, e->stream)); e->fin_pairs.emplace_back(e0, e1); }
    if (record_out) e->out_seq = f.seq;
    if (record_out) HIP_TRY(hipEventRecord(e->ev_out, e->stream));   // outputs land in mapped host memory
    ++e->step_ctr;
    e->out_pending = record_out;
    e->aql_out = false;
    e->aql_call = false;
    return MPPI_OK;
}

mppi_status mppi_finalize(mppi_engine* e) {
    if (!e) return fail(MPPI_ERR_INVALID_ARG, "null engine");
    return finalize_impl(e, true);
}

// True when every output record of the pending read step carries its sequence number (the
// tag is each record's last word; k_finalize writes a record with one 16 B store).
static bool records_tagged(const mppi_engine* e, uint32_t want) {
    const volatile uint32_t* r = (const volatile uint32_t*)(e->h_out + off_flags(e));
    const size_t n = rec_count(e);
    for (size_t i = 0; i < n; ++i)
        if (r[4 * i + 3] != want) return false;
    return true;
}

// One output record, read with one aligned 16 B load (atomic on x86-64 processors with AVX),
// so its values and its tag come from the same store.  false: the tag is not this step's.
static inline bool load_record(const mppi_engine* e, size_t i, uint32_t want, uint32_t (&w)[4]) {
    const __m128i x = _mm_load_si128((const __m128i*)(e->h_out + off_flags(e)) + i);
    _mm_storeu_si128((__m128i*)w, x);
    return w[3] == want;
}

// Wait for the finalised step's outputs.  k_finalize writes them into mapped host memory
// as tagged records (the step's sequence number in each), so the host sees completion by
// polling host memory instead of waking on the output event (which also trails the kernel
// by one queue packet).  The event stays the backstop: it is queried every few hundred
// polls, which also surfaces a faulted queue as an error.
static mppi_status wait_outputs(mppi_engine* e) {
    if (e->aql_out) return aql_join(e);   // a native batch: its completion signal (system-scope release)
    if (e->aql_call) {   // a native control call: its flags, the queue's error state as the backstop
        const uint32_t want = e->out_seq;
        const auto t0 = std::chrono::steady_clock::now();
        for (uint64_t it = 1;; ++it) {
            if (records_tagged(e, want)) break;
            if ((it & 255u) == 0) {
                if (const int q = mppi_aql::step_error(e->aql)) return fail(MPPI_ERR_HIP, "native queue error %d", q);
                if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60))
                    return fail(MPPI_ERR_HIP, "native control call: no outputs after 60 s");
            }
            __builtin_ia32_pause();
        }
        std::atomic_thread_fence(std::memory_order_acquire);
        mppi_aql::step_call_read(e->aql);
        e->call_wait_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        return MPPI_OK;
    }
    if (!e->event_wait) {
        const uint32_t want = e->out_seq;
        for (uint64_t it = 1;; ++it) {
            if (records_tagged(e, want)) {
                std::atomic_thread_fence(std::memory_order_acquire);
                return MPPI_OK;
            }
            if ((it & 255u) == 0) {
                const hipError_t q = hipEventQuery(e->ev_out);
                if (q == hipSuccess) break;
                if (q != hipErrorNotReady) return fail(MPPI_ERR_HIP, "waiting for the step: %s", hipGetErrorString(q));
            }
            __builtin_ia32_pause();
        }
    }
    HIP_TRY(hipEventSynchronize(e->ev_out));
    return MPPI_OK;
}

// The read step's outputs from its records into host staging in the plain arrays' layout
// (qdes/vdes or x/v per dim, u0, stats).  The plain arrays are the base (the quadrotor's
// outputs are formed on the host from u0).
static mppi_status assemble_records(mppi_engine* e) {
    const int V = e->V, A = e->A, od = e->out_dim, model = e->cfg.model;
    const uint32_t want = e->out_seq;
    e->rec_out.assign((const double*)e->h_out, (const double*)e->h_out + (size_t)V * od);
    e->rec_u0.resize((size_t)V * A);
    e->rec_stats.resize((size_t)V * 4);
    const int qoff = (model == MPPI_MODEL_WHOLEBODY) ? 3 : 0, nq = A - qoff;
    uint32_t w[4];
    for (int v = 0; v < V; ++v) {
        const size_t r0 = (size_t)v * (2 * A + 1);
        for (int a = 0; a < A; ++a) {
            double o1, o2;
            if (!load_record(e, r0 + 2 * a, want, w)) return fail(MPPI_ERR_STATE, "output record (%d,%d) not tagged", v, a);
            std::memcpy(&o1, w, 8);
            std::memcpy(&e->rec_u0[(size_t)v * A + a], &w[2], 4);
            if (!load_record(e, r0 + 2 * a + 1, want, w)) return fail(MPPI_ERR_STATE, "output record (%d,%d) not tagged", v, a);
            std::memcpy(&o2, w, 8);
            {   // the step's nan / exchange-timeout flag: the largest over every dim's record (a
                // peer-exchange block that gave the step up flags its own dim: any dim counts)
                float nf;
                std::memcpy(&nf, &w[2], 4);
                float& st3 = e->rec_stats[(size_t)v * 4 + 3];
                st3 = (a == 0 || nf > st3 || std::isnan(nf)) ? nf : st3;
            }
            double* ov = e->rec_out.data() + (size_t)v * od;
            if (model == MPPI_MODEL_QUADROTOR) continue;
            if (model == MPPI_MODEL_DRONE || (model == MPPI_MODEL_WHOLEBODY && a < 3)) {
                ov[a] = o1; ov[3 + a] = o2;
            } else {
                const int base = (model == MPPI_MODEL_WHOLEBODY) ? 6 : 0, j = a - qoff;
                ov[base + j] = o1; ov[base + nq + j] = o2;
            }
        }
        if (!load_record(e, r0 + 2 * A, want, w)) return fail(MPPI_ERR_STATE, "stats record %d not tagged", v);
        std::memcpy(&e->rec_stats[(size_t)v * 4], w, 12);
    }
    return MPPI_OK;
}

mppi_status mppi_read_outputs(mppi_engine* e, double* out, float* u0, mppi_stats* stats) {
    if (!e) return fail(MPPI_ERR_INVALID_ARG, "null engine");
    if (!e->out_pending) return fail(MPPI_ERR_STATE, "no finalised step to read");
    if (e->aql_call) HIP_TRY(hipSetDevice(e->cfg.device));   // (its flags, not the queue's drain)
    else if (use_device(e)) return MPPI_ERR_HIP;
    {   mppi_status st = wait_outputs(e);
        if (st != MPPI_OK) return st; }
    if (e->d_stamps) {   // diagnostic: average phase cycles over all waves
        const size_t nwaves = (size_t)e->V * e->dp.nb * (e->threads / 64);
        std::vector<unsigned long long> st(nwaves * kStamps);
        HIP_TRY(hipMemcpy(st.data(), e->d_stamps, st.size() * 8, hipMemcpyDeviceToHost));
        for (size_t w = 0; w < nwaves; ++w) {
            const unsigned long long* x = &st[w * kStamps];
            for (size_t i = 1; i < kRollStampOrder.size(); ++i)
                e->stamp_sum[i] += (double)(x[kRollStampOrder[i]] - x[kRollStampOrder[i - 1]]);
        }
        e->stamp_n += (int64_t)nwaves;
        const size_t nfb = (size_t)e->V * e->A * e->fin_ts;
        std::vector<unsigned long long> fs(nfb * kStamps);
        HIP_TRY(hipMemcpy(fs.data(), e->d_fstamps, fs.size() * 8, hipMemcpyDeviceToHost));
        for (size_t b = 0; b < nfb; ++b) {
            const unsigned long long* x = &fs[b * kStamps];
            for (size_t i = 1; i < kFinStampOrder.size(); ++i)
                e->fstamp_sum[i] += (double)(x[kFinStampOrder[i]] - x[kFinStampOrder[i - 1]]);
        }
        e->fstamp_n += (int64_t)nfb;
    }
    const double* o = (const double*)e->h_out;
    const float* uu = (const float*)(e->h_out + off_u0(e));
    const float* st = (const float*)(e->h_out + off_stats(e));
    if (!e->aql_out && e->out_seq != 0u) {   // a read step: its values from its tagged records
        mppi_status rs = assemble_records(e);
        if (rs != MPPI_OK) return rs;
        o = e->rec_out.data();
        uu = e->rec_u0.data();
        st = e->rec_stats.data();
    }
    if (out) std::memcpy(out, o, sizeof(double) * e->V * e->out_dim);
    if (out && e->cfg.model == MPPI_MODEL_QUADROTOR)
        for (int v = 0; v < e->V; ++v)
            quad_outputs(e, e->state.data() + (size_t)v * e->state_dim, uu + (size_t)v * e->A, out + (size_t)v * e->out_dim);
    if (u0) std::memcpy(u0, uu, sizeof(float) * e->V * e->A);
    bool nonfinite = false;
    for (int v = 0; v < e->V; ++v) {
        int reach = 0;
        if (e->cfg.check_reach && e->cfg.model == MPPI_MODEL_ARM) {   // mppi.py:95-120 (host FK)
            const double* s = e->state.data() + (size_t)v * e->state_dim;
            const double* qdes = o + (size_t)v * e->out_dim;
            float T16[16];
            host_fk_c(e->cfg.joints, e->cfg.n_joints, e->fk_O.data(), e->fk_ax.data(), qdes, s, e->cfg.state_f64 != 0,
                      T16);
            const float err = std::fabs(T16[3] - e->tpos[3 * v]) + std::fabs(T16[7] - e->tpos[3 * v + 1]) +
                              std::fabs(T16[11] - e->tpos[3 * v + 2]);
            reach = err < e->cfg.reach_tol;
        }
        // 2: a peer-exchange step given up (a rank's timeout: u_prev kept) -- this step's flag or
        // any step's since the exchange was last reset (the sticky word: every block, every step)
        const int nf = (st[4 * v + 3] >= 2.0f || (e->peer && sticky_timeout(e) != 0u)) ? 2
                       : ((st[4 * v + 3] > 0.0f) || !std::isfinite(st[4 * v]) || !std::isfinite(uu[(size_t)v * e->A]));
        nonfinite |= nf;
        if (stats) {
            stats[v].rho = st[4 * v];
            stats[v].eta = st[4 * v + 1];
            stats[v].ess = st[4 * v + 2];
            stats[v].nonfinite = nf;
            stats[v].reach = reach;
            stats[v]._pad = 0;
        }
    }
    (void)nonfinite;   // the reference propagates NaN silently; callers read stats.nonfinite
    return MPPI_OK;
}

static mppi_status control_call_aql(mppi_engine* e, const double* state, bool* used);

mppi_status mppi_step(mppi_engine* e, const double* state, const float* h_noise, double* out, float* u0,
                      mppi_stats* stats) {
    if (!e) return fail(MPPI_ERR_INVALID_ARG, "null engine");
    note_call(e);
    if (sharded(e) && !e->comm)
        return fail(MPPI_ERR_STATE, "mppi_step on a shard needs mppi_comm_init (or use the split phases)");
    mppi_status st;
    if (e->cfg.noise_mode == MPPI_NOISE_PHILOX && e->V == 1 && !sharded(e)) {   // one vehicle: native packets
        bool used = false;
        static const bool prof = getenv("MPPI_AQL_PROFILE") != nullptr;   // diagnostics: host phases of a call
        const auto c0 = std::chrono::steady_clock::now();
        if ((st = control_call_aql(e, state, &used)) != MPPI_OK) return st;
        e->calls_native = used;
        e->pw_native.store(used, std::memory_order_release);
        if (used) {
            if (!prof) return mppi_read_outputs(e, out, u0, stats);
            const auto c1 = std::chrono::steady_clock::now();
            st = mppi_read_outputs(e, out, u0, stats);
            const auto c2 = std::chrono::steady_clock::now();
            static double acc[3] = {0, 0, 0};
            static long cn = 0;
            const double pre = std::chrono::duration<double, std::micro>(c1 - c0).count();
            const double rd = std::chrono::duration<double, std::micro>(c2 - c1).count();
            acc[0] += pre; acc[1] += e->call_wait_us; acc[2] += rd - e->call_wait_us;
            if (++cn % 1000 == 0)
                fprintf(stderr, "[mppi aql] per call (us): before the doorbell %.2f  flag wait %.2f  outputs + check_reach %.2f\n",
                        acc[0] / cn, acc[1] / cn, acc[2] / cn);
            return st;
        }
    }
    e->calls_native = false;
    e->pw_native.store(false, std::memory_order_relaxed);   // (HIP launches: nothing to prewarm)
    if (state && (st = mppi_set_state(e, state)) != MPPI_OK) return st;
    const float* dn = nullptr;
    if (e->cfg.noise_mode == MPPI_NOISE_INJECTED) {
        if (!h_noise) return fail(MPPI_ERR_INVALID_ARG, "INJECTED noise mode needs noise");
        const size_t n = (size_t)e->V * e->K * e->H * e->A;
        if (use_device(e)) return MPPI_ERR_HIP;
        if (!e->d_noise_in) HIP_TRY(hipMalloc(&e->d_noise_in, n * sizeof(float)));
        HIP_TRY(hipMemcpyAsync(e->d_noise_in, h_noise, n * sizeof(float), hipMemcpyHostToDevice, e->stream));
        dn = e->d_noise_in;
    }
    if ((st = mppi_rollout(e, dn)) != MPPI_OK) return st;
    if (e->comm && (st = mppi_exchange(e)) != MPPI_OK) return st;
    if ((st = mppi_finalize(e)) != MPPI_OK) return st;
    return mppi_read_outputs(e, out, u0, stats);
}

// why this engine's mppi_run_steps cannot go native (nullptr: it can)
// A batch (mppi_run_steps) may carry the stamps / no-flag diagnostics natively (the timeline
// build measures the native step that way); a control call waits on the flags, so it may not.
static const char* aql_ineligible(const mppi_engine* e, bool batch = false) {
    if (e->aql_mode == 0) return "MPPI_DISPATCH=hip";
    if (sharded(e)) return "sharded step (its collective runs on the HIP stream)";
    if (e->timing) return "per-launch timing events (mppi_enable_timing)";
    if (e->d_stamps && !batch) return "stamps diagnostics";
    if (e->out_dbg || (e->no_flag_dbg && !batch)) return "output diagnostics";
    return nullptr;
}

// The rollout's step counter word: its third argument (seed_lo, seed_hi, step, ...), the same
// position in k_rollout and k_rollout_quad (mppi_rollout.h, mppi_rollout_quad.hip).  Under
// native dispatch it is relative to the dispatch id (kNoiseStepFromId in the noise-mode word).
constexpr uint32_t kRollStepOff = 8;
constexpr int32_t kNoiseStepFromId = 0x100;   // = mppi_device.h

// n steps as native AQL packets (mppi_aql.cpp).  *used = false: the caller runs them through
// HIP (auto mode, native dispatch unavailable for this engine; e->aql_why says why).
// the engine's native queue, created on first use; false when native dispatch is off for it
static bool aql_ready(mppi_engine* e) {
    if (e->aql_off) return false;
    if (!e->aql && !e->aql_tried) {
        e->aql_tried = true;
        std::string why;
        if (hipSetDevice(e->cfg.device) == hipSuccess) e->aql = mppi_aql::step_create(e->cfg.device, &why);
        else why = "hipSetDevice failed";
        if (!e->aql) e->aql_why = why;
    }
    if (!e->aql) e->aql_off = true;
    return e->aql != nullptr;
}

static mppi_status run_steps_aql(mppi_engine* e, int32_t n, bool* used) {
    *used = false;
    if (const char* why = aql_ineligible(e, true)) { e->aql_why = why; return MPPI_OK; }
    if (!aql_ready(e)) return e->aql_mode == 1 ? fail(MPPI_ERR_STATE, "native dispatch: %s", e->aql_why.c_str()) : MPPI_OK;
    HIP_TRY(hipSetDevice(e->cfg.device));
    static const bool prof = getenv("MPPI_AQL_PROFILE") != nullptr;   // diagnostics: host phase times
    static double pt[4] = {0, 0, 0, 0};
    static long pn = 0;
    auto now = [] { return std::chrono::steady_clock::now(); };
    const auto c0 = now();
    // HIP work still queued on the engine's stream (uploads, an earlier HIP-path step) first
    const hipError_t q = hipStreamQuery(e->stream);
    if (q == hipErrorNotReady) HIP_TRY(hipStreamSynchronize(e->stream));
    else if (q != hipSuccess) return fail(MPPI_ERR_HIP, "engine stream: %s", hipGetErrorString(q));
    // the two launches exactly as the HIP path makes them, described instead of launched (and
    // the description reused while nothing in it changed: the capture formats both kernels'
    // symbol names and packs ~2 KB of arguments, ~0.4 us per batch)
    const auto c1 = now();
    LaunchDesc& roll = e->batch_roll;
    LaunchDesc& fin = e->batch_fin;
    DevParams p = e->dp;
    p.noise_in = nullptr;
    p.vc0 = e->h_vc[0];
    p.step_ctr = 0u;                      // (set by step_prepare: relative to the dispatch id)
    p.noise_mode |= kNoiseStepFromId;
    FinParams f = e->fp;
    f.mode = 0;
    f.seq = 0u;   // completion: the batch's signal, not a flag
    final_records(e, f);
    if (!(e->batch_cached && e->batch_threads == e->threads && std::memcmp(&p, &e->batch_p, sizeof(p)) == 0 &&
          std::memcmp(&f, &e->batch_f, sizeof(f)) == 0)) {
        e->batch_cached = false;
        mppi_aql::set_capture(&roll);
        int rc = mppi_launch_rollout(&p, e->threads, e->stream);
        if (rc == 0) {
            mppi_aql::set_capture(&fin);
            rc = mppi_launch_finalize(&f, e->stream);
        }
        mppi_aql::set_capture(nullptr);
        if (rc != 0) return fail(MPPI_ERR_HIP, "describing the step's launches failed (%d)", rc);
        e->batch_p = p;
        e->batch_f = f;
        e->batch_threads = e->threads;
        e->batch_cached = true;
    }
    std::string err;
    const auto c2 = now();
    const auto guard = mppi_aql::step_guard(e->aql);   // (no prewarm touch between prepare and dispatch)
    const int pr = mppi_aql::step_prepare(e->aql, roll, fin, e->step_ctr, kRollStepOff, &err);
    const auto c3 = now();
    if (pr == -2) {   // not dispatchable natively (a kernel the code objects lack, hidden arguments)
        e->aql_off = true;
        e->aql_why = err;
        return e->aql_mode == 1 ? fail(MPPI_ERR_STATE, "native dispatch: %s", err.c_str()) : MPPI_OK;
    }
    if (pr != 0 || mppi_aql::step_dispatch(e->aql, n, &err) != 0)
        return fail(MPPI_ERR_HIP, "native dispatch: %s", err.c_str());
    if (prof) {
        const auto c4 = now();
        const std::chrono::steady_clock::time_point cs[5] = {c0, c1, c2, c3, c4};
        for (int i = 0; i < 4; ++i) pt[i] += std::chrono::duration<double, std::micro>(cs[i + 1] - cs[i]).count();
        if (++pn % 200 == 0)
            fprintf(stderr, "[mppi aql] per batch (us): stream query %.2f  capture %.2f  prepare %.2f  packets %.2f\n",
                    pt[0] / pn, pt[1] / pn, pt[2] / pn, pt[3] / pn);
    }
    e->step_ctr += (uint32_t)n;
    e->out_pending = true;
    e->aql_out = true;
    e->aql_call = false;
    e->aql_why.clear();
    *used = true;
    return MPPI_OK;
}

// One control call (V == 1) as a native (rollout, finalize) pair: the state goes into the
// rollout's arguments in pinned host memory (its vehicle constants), the finalize's arguments
// stay resident, and the call's completion flags carry a bit-31 sequence number the host
// wrote next to the constants (mppi_aql.h step_call).  *used = false: the HIP path runs it.
static mppi_status control_call_aql(mppi_engine* e, const double* state, bool* used) {
    *used = false;
    if (aql_ineligible(e) || e->event_wait) return MPPI_OK;
    if (!aql_ready(e)) return e->aql_mode == 1 ? fail(MPPI_ERR_STATE, "native dispatch: %s", e->aql_why.c_str())
                                               : MPPI_OK;
    static const bool prof = getenv("MPPI_AQL_PROFILE") != nullptr;   // diagnostics: host phases
    static double pacc[4] = {0, 0, 0, 0};
    static long pcn = 0;
    const auto q0 = std::chrono::steady_clock::now();
    HIP_TRY(hipSetDevice(e->cfg.device));
    const auto q1 = std::chrono::steady_clock::now();
    if (state) {   // mppi_set_state's work for one vehicle: host-side constants only
        std::memcpy(e->state.data(), state, sizeof(double) * e->state.size());
        e->state_set = true;
        mppi_status st = build_vehicle_consts(e);
        if (st != MPPI_OK) return st;
    }
    if (!e->state_set) return fail(MPPI_ERR_STATE, "mppi_step before mppi_set_state");
    const auto q2 = std::chrono::steady_clock::now();
    {   // HIP work queued on the engine's stream first (0.1 us when there is none)
        const hipError_t q = hipStreamQuery(e->stream);
        if (q == hipErrorNotReady) HIP_TRY(hipStreamSynchronize(e->stream));
        else if (q != hipSuccess) return fail(MPPI_ERR_HIP, "engine stream: %s", hipGetErrorString(q));
    }
    const auto q3 = std::chrono::steady_clock::now();
    DevParams p = e->dp;
    p.noise_in = nullptr;
    p.vc0 = e->h_vc[0];
    p.step_ctr = 0u;
    p.noise_mode |= kNoiseStepFromId;
    FinParams f = e->fp;
    f.mode = 0;
    f.seq = kSeqFromVc;
    final_records(e, f);
    // The launch descriptions of the previous call are reused when only the state changed:
    // the state lives in the vehicle constants (DevParams::vc0, inside the rollout's last
    // argument), which are patched in; anything else that differs re-captures (the capture
    // formats both kernels' symbol names and packs ~2 KB of arguments: ~0.4 us per call).
    LaunchDesc& roll = e->call_roll;
    LaunchDesc& fin = e->call_fin;
    constexpr size_t kVo = offsetof(DevParams, vc0), kVn = sizeof(VehicleConst);
    const bool hit = e->call_cached && e->call_threads == e->threads &&
                     std::memcmp(&p, &e->call_p, kVo) == 0 &&
                     std::memcmp((const char*)&p + kVo + kVn, (const char*)&e->call_p + kVo + kVn,
                                 sizeof(DevParams) - kVo - kVn) == 0 &&
                     std::memcmp(&f, &e->call_f, sizeof(FinParams)) == 0;
    if (hit) {
        std::memcpy(roll.args + roll.arg_bytes - sizeof(DevParams) + kVo, &p.vc0, kVn);
    } else {
        e->call_cached = false;
        mppi_aql::set_capture(&roll);
        int rc = mppi_launch_rollout(&p, e->threads, e->stream);
        if (rc == 0) {
            mppi_aql::set_capture(&fin);
            rc = mppi_launch_finalize(&f, e->stream);
        }
        mppi_aql::set_capture(nullptr);
        if (rc != 0) return fail(MPPI_ERR_HIP, "describing the step's launches failed (%d)", rc);
        e->call_p = p;
        e->call_f = f;
        e->call_threads = e->threads;
        e->call_cached = true;
    }
    if (prof) {
        const auto q4 = std::chrono::steady_clock::now();
        const std::chrono::steady_clock::time_point qs[5] = {q0, q1, q2, q3, q4};
        for (int i = 0; i < 4; ++i) pacc[i] += std::chrono::duration<double, std::micro>(qs[i + 1] - qs[i]).count();
        if (++pcn % 1000 == 0)
            fprintf(stderr, "[mppi aql] call setup (us): hipSetDevice %.2f  vehicle constants %.2f  stream query %.2f  "
                            "capture %.2f\n", pacc[0] / pcn, pacc[1] / pcn, pacc[2] / pcn, pacc[3] / pcn);
    }
    // the vehicle constants' spare word inside the rollout's last argument (DevParams by value)
    const uint32_t seq_off = roll.arg_bytes - (uint32_t)sizeof(DevParams) + (uint32_t)offsetof(DevParams, vc0) +
                             (uint32_t)offsetof(VehicleConst, _pad);
    std::string err;
    uint32_t seq = 0;
    const int pr = mppi_aql::step_call(e->aql, roll, fin, e->step_ctr, kRollStepOff, seq_off, &seq, &err);
    if (pr == -2) {
        e->aql_off = true;
        e->aql_why = err;
        return e->aql_mode == 1 ? fail(MPPI_ERR_STATE, "native dispatch: %s", err.c_str()) : MPPI_OK;
    }
    if (pr != 0) return fail(MPPI_ERR_HIP, "native dispatch: %s", err.c_str());
    ++e->step_ctr;
    e->out_seq = seq;
    e->out_pending = true;
    e->aql_out = false;
    e->aql_call = true;
    *used = true;
    return MPPI_OK;
}

mppi_status mppi_run_steps(mppi_engine* e, int32_t n) {
    if (!e || n < 0) return fail(MPPI_ERR_INVALID_ARG, "mppi_run_steps: bad arguments");
    if (sharded(e) && !e->comm) return fail(MPPI_ERR_STATE, "mppi_run_steps on a shard needs mppi_comm_init");
    if (e->cfg.noise_mode != MPPI_NOISE_PHILOX) return fail(MPPI_ERR_STATE, "mppi_run_steps needs device noise");
    if (!e->state_set) return fail(MPPI_ERR_STATE, "mppi_run_steps before mppi_set_state");
    if (n == 0) return MPPI_OK;
    bool used = false;
    mppi_status st = run_steps_aql(e, n, &used);
    if (st != MPPI_OK || used) return st;
    for (int i = 0; i < n; ++i) {
        mppi_status st = mppi_rollout(e, nullptr);
        if (st != MPPI_OK) return st;
        if (e->comm && (st = mppi_exchange(e)) != MPPI_OK) return st;
        if ((st = finalize_impl(e, i == n - 1)) != MPPI_OK) return st;
    }
    return MPPI_OK;
}

mppi_status mppi_kernel_timing_ex(mppi_engine* e, int32_t n, double* rollout_us, double* finalize_us,
                                  double* pair_us) {
    if (!e || n <= 0 || !rollout_us || !finalize_us)
        return fail(MPPI_ERR_INVALID_ARG, "mppi_kernel_timing: bad arguments");
    if (e->cfg.noise_mode != MPPI_NOISE_PHILOX) return fail(MPPI_ERR_STATE, "mppi_kernel_timing needs device noise");
    if (!e->state_set) return fail(MPPI_ERR_STATE, "mppi_kernel_timing before mppi_set_state");
    if (sharded(e) && !e->d_exchange)
        return fail(MPPI_ERR_STATE, "mppi_kernel_timing on a shard needs its exchange buffer");
    if (use_device(e)) return MPPI_ERR_HIP;
    const size_t ub = sizeof(float) * e->V * e->H * e->A;
    float* saved = nullptr;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    mppi_status st = MPPI_OK;
    DevParams p = e->dp;
    p.vc0 = e->h_vc[0];
    p.step_ctr = e->step_ctr;
    FinParams f = e->fp;
    f.mode = 0;
    f.seq = 0u;   // the throughput path's finalize (no completion flag)
    final_records(e, f);
    // the timing loop's outputs go to device scratch (same layout as the mapped host
    // buffer), so a pending read_outputs / get_weighted_noise still returns the last
    // real step; u_prev is restored below (the trajectory and S are overwritten).  On a
    // shard the finalize combines the exchange slots as they stand (no collective here).
    f.out = (double*)e->d_out;
    f.u0 = (float*)(e->d_out + off_u0(e));
    f.stats = (float*)(e->d_out + off_stats(e));
    f.flags = (uint32_t*)(e->d_out + off_flags(e));
    f.wraw = nullptr;
    f.wsmooth = nullptr;
    f.tail = e->d_tail + kTailScratch;   // (the same outputs, from the kernel's device-resident copy)
    if (e->out_dbg == 2) f.tail = e->d_tail + kTailFinal;   // diagnostic: outputs into mapped host memory
    float ms0 = 0.0f, ms1 = 0.0f, ms2 = 0.0f;
    int rc = 0;
#define KT_TRY(expr)                                                                        \
    do {                                                                                    \
        hipError_t _e = (expr);                                                             \
        if (_e != hipSuccess) { st = fail(MPPI_ERR_HIP, "%s: %s", #expr, hipGetErrorString(_e)); goto done; } \
    } while (0)
    KT_TRY(hipMalloc(&saved, ub));
    for (auto& x : ev) KT_TRY(hipEventCreate(&x));
    KT_TRY(hipMemcpyAsync(saved, e->d_u_prev, ub, hipMemcpyDeviceToDevice, e->stream));
    KT_TRY(hipEventRecord(ev[0], e->stream));
    for (int i = 0; i < n && rc == 0; ++i) rc = mppi_launch_rollout(&p, e->threads, e->stream);
    KT_TRY(hipEventRecord(ev[1], e->stream));
    for (int i = 0; i < n && rc == 0; ++i) rc = mppi_launch_finalize(&f, e->stream);
    KT_TRY(hipEventRecord(ev[2], e->stream));
    // the kernels as a control step runs them: rollout after finalize (u_prev and the
    // records just written, cold in the other XCDs' L2)
    for (int i = 0; i < n && rc == 0 && pair_us; ++i) {
        rc = mppi_launch_rollout(&p, e->threads, e->stream);
        if (rc == 0) rc = mppi_launch_finalize(&f, e->stream);
    }
    KT_TRY(hipEventRecord(ev[3], e->stream));
    KT_TRY(hipMemcpyAsync(e->d_u_prev, saved, ub, hipMemcpyDeviceToDevice, e->stream));
    KT_TRY(hipStreamSynchronize(e->stream));
    if (rc != 0) { st = fail(MPPI_ERR_HIP, "kernel launch failed (%d)", rc); goto done; }
    KT_TRY(hipEventElapsedTime(&ms0, ev[0], ev[1]));
    KT_TRY(hipEventElapsedTime(&ms1, ev[1], ev[2]));
    KT_TRY(hipEventElapsedTime(&ms2, ev[2], ev[3]));
    *rollout_us = 1e3 * ms0 / n;
    *finalize_us = 1e3 * ms1 / n;
    if (pair_us) *pair_us = 1e3 * ms2 / n;
#undef KT_TRY
done:
    for (auto x : ev) if (x) (void)hipEventDestroy(x);
    if (saved) (void)hipFree(saved);
    return st;
}

#ifdef MPPI_PROBE
// tools-only (MPPI_PROBE builds): average time of n repetitions of a kernel sequence
//   mode 0: rollout, empty kernel   1: rollout, rollout of one block   2: rollout, finalize
//   3: empty kernel                 4: rollout of one block            5: rollout
extern "C" int mppi_launch_boundary(float* scratch, int blocks, void* stream);
extern "C" mppi_status mppi_probe_sequence(mppi_engine* e, int32_t n, int32_t mode, double* us) {
    if (use_device(e)) return MPPI_ERR_HIP;
    DevParams p = e->dp;
    p.vc0 = e->h_vc[0];
    p.step_ctr = e->step_ctr;
    DevParams p1 = p;
    p1.nb = 1;
    FinParams f = e->fp;
    f.mode = 0; f.seq = 0u;
    final_records(e, f);
    f.out = (double*)e->d_out; f.u0 = (float*)(e->d_out + off_u0(e)); f.stats = (float*)(e->d_out + off_stats(e));
    f.flags = (uint32_t*)(e->d_out + off_flags(e)); f.wraw = nullptr; f.wsmooth = nullptr;
    f.tail = e->d_tail + kTailScratch;
    const int fb = 8 * ((e->A + 7) / 8) * ((e->H + 7) / 8) * e->V;
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    (void)hipEventRecord(a, e->stream);
    for (int i = 0; i < n; ++i) {
        if (mode <= 2 || mode == 5) mppi_launch_rollout(&p, e->threads, e->stream);
        if (mode == 0 || mode == 3) mppi_launch_boundary((float*)e->d_out, fb, e->stream);
        if (mode == 1 || mode == 4) mppi_launch_rollout(&p1, e->threads, e->stream);
        if (mode == 2) mppi_launch_finalize(&f, e->stream);
    }
    (void)hipEventRecord(b, e->stream);
    (void)hipEventSynchronize(b);
    float ms = 0.0f;
    (void)hipEventElapsedTime(&ms, a, b);
    *us = 1e3 * ms / n;
    (void)hipEventDestroy(a); (void)hipEventDestroy(b);
    return MPPI_OK;
}
#endif

mppi_status mppi_kernel_timing(mppi_engine* e, int32_t n, double* rollout_us, double* finalize_us) {
    return mppi_kernel_timing_ex(e, n, rollout_us, finalize_us, nullptr);
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

mppi_status mppi_dispatch_info(mppi_engine* e, char* buf, int32_t len) {
    if (!e || !buf || len <= 0) return fail(MPPI_ERR_INVALID_ARG, "mppi_dispatch_info: bad arguments");
    snprintf(buf, (size_t)len, "%s%s; calls: %s%s%s", e->aql_why.empty() ? "aql" : "hip: ", e->aql_why.c_str(),
             e->calls_native ? "aql (arguments in " : "hip", e->calls_native ? mppi_aql::step_call_memory(e->aql) : "",
             e->calls_native ? ")" : "");
    return MPPI_OK;
}

mppi_status mppi_synchronize(mppi_engine* e) {
    if (!e) return fail(MPPI_ERR_INVALID_ARG, "null engine");
    if (use_device(e)) return MPPI_ERR_HIP;
    // The last finalised step's completion flag is polled first (mapped host memory, a
    // few hundred ns behind the kernel); hipStreamSynchronize alone wakes the host
    // microseconds after the stream drains, which a short timed batch pays in full.
    if (e->out_pending && !e->event_wait && !e->aql_out) {
        mppi_status st = wait_outputs(e);
        if (st != MPPI_OK) return st;
    }
    HIP_TRY(hipStreamSynchronize(e->stream));
    if (e->peer)
        if (const uint32_t t = sticky_timeout(e))
            return fail(MPPI_ERR_PEER_TIMEOUT, "peer exchange: a step was given up (tag %08x): this rank's "
                                               "warm start may differ from its peers' until mppi_peer_reset", t);
    return MPPI_OK;
}

mppi_status mppi_get_costs(mppi_engine* e, float* S) {
    if (!e || !S) return fail(MPPI_ERR_INVALID_ARG, "null argument");
    if (use_device(e)) return MPPI_ERR_HIP;
    HIP_TRY(hipMemcpyAsync(S, e->d_S, sizeof(float) * e->V * e->K, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    return MPPI_OK;
}

mppi_status mppi_get_weights(mppi_engine* e, float* w) {
    if (!e || !w) return fail(MPPI_ERR_INVALID_ARG, "null argument");
    if (use_device(e)) return MPPI_ERR_HIP;
    int rc = mppi_launch_weights(e->d_S, e->fp.stats, e->d_w, e->V, e->K, e->dp.coef, e->stream);
    if (rc) return fail(MPPI_ERR_HIP, "weights launch failed (%d)", rc);
    HIP_TRY(hipMemcpyAsync(w, e->d_w, sizeof(float) * e->V * e->K, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    return MPPI_OK;
}

mppi_status mppi_get_noise(mppi_engine* e, float* eps) {
    if (!e || !eps) return fail(MPPI_ERR_INVALID_ARG, "null argument");
    if (!e->d_noise_out) return fail(MPPI_ERR_STATE, "engine created without store_noise");
    if (use_device(e)) return MPPI_ERR_HIP;
    HIP_TRY(hipMemcpyAsync(eps, e->d_noise_out, sizeof(float) * (size_t)e->V * e->K * e->H * e->A,
                           hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    return MPPI_OK;
}

mppi_status mppi_get_trajectory(mppi_engine* e, float* traj) {
    if (!e || !traj) return fail(MPPI_ERR_INVALID_ARG, "null argument");
    if (!e->d_traj) return fail(MPPI_ERR_STATE, "engine created without store_trajectory");
    if (use_device(e)) return MPPI_ERR_HIP;
    const size_t KH = (size_t)e->K * e->H, n = traj_floats(e);
    const size_t hp = (size_t)traj_pitch(e), plane = n / ((size_t)e->V * e->C);   // padded plane
    std::vector<float> soa(n);
    HIP_TRY(hipMemcpyAsync(soa.data(), e->d_traj, n * sizeof(float), hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    const int Cr = mppi_traj_channels(&e->cfg);
    const bool has_ee = e->cfg.model == MPPI_MODEL_ARM || e->cfg.model == MPPI_MODEL_WHOLEBODY;
    const int nstate = has_ee ? e->A : e->C;
    const bool t_major = e->cfg.model == MPPI_MODEL_QUADROTOR;   // (V,C,H,K) planes (k_rollout_quad)
    for (int v = 0; v < e->V; ++v)
        for (size_t i = 0; i < KH; ++i) {
            float* dst = traj + ((size_t)v * KH + i) * Cr;
            const size_t ii = t_major ? (i % e->H) * hp + i / e->H : (i / e->H) * hp + i % e->H;
            const float* src = soa.data() + (size_t)v * e->C * plane + ii;
            for (int c = 0; c < nstate; ++c) dst[c] = src[c * plane];
            if (has_ee) {
                float* ee = dst + nstate;
                for (int r = 0; r < 12; ++r) ee[r] = src[(nstate + r) * plane];
                ee[12] = 0.0f; ee[13] = 0.0f; ee[14] = 0.0f; ee[15] = 1.0f;
            }
        }
    return MPPI_OK;
}

mppi_status mppi_get_weighted_noise(mppi_engine* e, float* raw, float* smoothed) {
    if (!e) return fail(MPPI_ERR_INVALID_ARG, "null engine");
    if (use_device(e)) return MPPI_ERR_HIP;
    const size_t n = sizeof(float) * e->V * e->H * e->A;
    // w_eps and its SavGol of the records the last step combined (its block records, or the
    // shard's all-reduced exchange slots): k_finalize in READBACK mode, which writes only these.
    // The step's own finalize stores no readback copies (no stores that only a readback needs on
    // the latency path, and none left dirty in an XCD's L2 across a native batch).
    FinParams f = e->fp;
    f.mode = 2;
    f.seq = 0u;
    final_records(e, f);
    f.tail = e->d_tail + kTailReadback;
    const int rc = mppi_launch_finalize(&f, e->stream);
    if (rc != 0) return fail(MPPI_ERR_HIP, "weighted-noise readback launch failed (%d)", rc);
    if (raw) HIP_TRY(hipMemcpyAsync(raw, e->d_wraw, n, hipMemcpyDeviceToHost, e->stream));
    if (smoothed) HIP_TRY(hipMemcpyAsync(smoothed, e->d_wsmooth, n, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    return MPPI_OK;
}

mppi_status mppi_enable_timing(mppi_engine* e, int32_t enable) {
    if (!e) return fail(MPPI_ERR_INVALID_ARG, "null engine");
    if (use_device(e)) return MPPI_ERR_HIP;
    mppi_status st = drain_timing(e);
    if (st) return st;
    e->timing = enable != 0;
    e->roll_ms = e->fin_ms = 0.0;
    e->roll_n = e->fin_n = 0;
    return MPPI_OK;
}

mppi_status mppi_get_timing(mppi_engine* e, double* rms, double* fms, int64_t* rn, int64_t* fn) {
    if (!e) return fail(MPPI_ERR_INVALID_ARG, "null engine");
    if (use_device(e)) return MPPI_ERR_HIP;
    mppi_status st = drain_timing(e);
    if (st) return st;
    if (rms) *rms = e->roll_ms;
    if (fms) *fms = e->fin_ms;
    if (rn) *rn = e->roll_n;
    if (fn) *fn = e->fin_n;
    return MPPI_OK;
}

// Diagnostic (MPPI_STAMPS builds; not part of the public header): the raw per-wave stamps
// of the last rollout launch, kStamps uint64 per wave.  Returns the wave count (0 when the
// engine has no stamps) or a negative status.
int64_t mppi_debug_stamps(mppi_engine* e, unsigned long long* out, int64_t max_waves) {
    if (!e || !out) return MPPI_ERR_INVALID_ARG;
    if (!e->d_stamps) return 0;
    if (use_device(e)) return MPPI_ERR_HIP;
    const int64_t nwaves = std::min<int64_t>(max_waves, (int64_t)e->V * e->dp.nb * (e->threads / 64));
    if (hipStreamSynchronize(e->stream) != hipSuccess ||
        hipMemcpy(out, e->d_stamps, (size_t)nwaves * kStamps * 8, hipMemcpyDeviceToHost) != hipSuccess)
        return MPPI_ERR_HIP;
    return nwaves;
}

// Diagnostic (MPPI_STAMPS builds): the raw stamps of the last FINAL (which = 0) or PACK
// (which = 1) launch, kStamps uint64 per (vehicle, dim, t-slice) block.  Returns the block count.
int64_t mppi_debug_fstamps(mppi_engine* e, unsigned long long* out, int64_t max_blocks, int32_t which) {
    if (!e || !out || which < 0 || which > 1) return MPPI_ERR_INVALID_ARG;
    if (!e->d_fstamps) return 0;
    if (use_device(e)) return MPPI_ERR_HIP;
    const int64_t nb = (int64_t)e->V * e->A * e->fin_ts;
    const int64_t n = std::min<int64_t>(max_blocks, nb);
    if (hipStreamSynchronize(e->stream) != hipSuccess ||
        hipMemcpy(out, e->d_fstamps + (size_t)which * nb * kStamps, (size_t)n * kStamps * 8, hipMemcpyDeviceToHost) !=
            hipSuccess)
        return MPPI_ERR_HIP;
    return n;
}

// Diagnostic (not part of the public header): mppi_aql step_touch on the engine's own queue
// (tools/probes.py rate_split).  Same thread as the control calls.
int32_t mppi_debug_queue_touch(mppi_engine* e) {
    if (!e || !e->aql) return MPPI_ERR_INVALID_ARG;
    std::string err;
    const int r = mppi_aql::step_touch(e->aql, false, &err);
    return r == 0 ? MPPI_OK : fail(MPPI_ERR_HIP, "queue touch: %s", err.c_str());
}

// Diagnostic (host only, tests/test_capi_cpu.py): the prewarm thread's window for call starts
// t[0..m) in ns and a window of window_us: 1 and [*start, *end], or 0 (no window).
int32_t mppi_debug_prewarm_plan(const int64_t* t, int32_t m, int32_t window_us, int64_t* start, int64_t* end) {
    if (!t || !start || !end || m < 0 || m > 8) return MPPI_ERR_INVALID_ARG;
    return prewarm_plan(t, m, (int64_t)window_us * 1000, start, end);
}

// Diagnostic: mppi_aql step_ring (the doorbell again, no packet).
int32_t mppi_debug_queue_ring(mppi_engine* e) {
    if (!e || !e->aql) return MPPI_ERR_INVALID_ARG;
    mppi_aql::step_ring(e->aql);
    return MPPI_OK;
}

int32_t mppi_philox_words(int32_t A) {
    return A < 1 ? 0 : 4 * (A / 8) + ((A % 8) == 0 ? 0 : (A % 8) <= 4 ? 2 : 4);
}

mppi_status mppi_philox_normals(uint64_t seed, uint32_t step, int32_t vehicle, int64_t k0, int32_t K, int32_t H,
                                int32_t A, int32_t device, float* z, uint32_t* raw) {
    if (K < 1 || H < 1 || A < 1 || A > MPPI_MAX_ACTION || !z || !raw)
        return fail(MPPI_ERR_INVALID_ARG, "mppi_philox_normals: bad arguments");
    HIP_TRY(hipSetDevice(device));
    const size_t n = (size_t)K * H;
    const int nw = mppi_philox_words(A);   // raw Philox words per (k, t)
    float* dz = nullptr;
    uint32_t* dr = nullptr;
    HIP_TRY(hipMalloc(&dz, n * A * sizeof(float)));
    HIP_TRY(hipMalloc(&dr, n * nw * sizeof(uint32_t)));
    int rc = mppi_launch_philox(seed, step, vehicle, k0, K, H, A, dz, dr, nullptr);
    hipError_t e1 = hipMemcpy(z, dz, n * A * sizeof(float), hipMemcpyDeviceToHost);
    hipError_t e2 = hipMemcpy(raw, dr, n * nw * sizeof(uint32_t), hipMemcpyDeviceToHost);
    (void)hipFree(dz);
    (void)hipFree(dr);
    if (rc) return fail(MPPI_ERR_HIP, "philox launch failed (%d)", rc);
    if (e1 != hipSuccess || e2 != hipSuccess) return fail(MPPI_ERR_HIP, "philox copy failed");
    return MPPI_OK;
}

}  // extern "C"

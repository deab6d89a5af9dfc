// mppi_host_math.cpp -- host arithmetic of libmppi_hip.so (include/mppi_hip.h): the calling
// thread's error string, config defaults and validation, and the reference's fp32 tensor builders
// the engine bakes into its constants (joint origins, base and target rotations), the SavGol taps
// and the host FK of check_reach.  No device code; see mppi_engine.h for the file map.
#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "mppi_engine.h"

using namespace mppi;

namespace {
thread_local std::string g_err;

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

}  // namespace

namespace mppi_host {

mppi_status fail(mppi_status st, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return st;
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

void base_from_xyzquat(const double* b, bool f64, float* T16) {
    if (f64) base_from_xyzquat_t<double>(b, T16);
    else base_from_xyzquat_t<float>(b, T16);
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

}  // namespace mppi_host

using namespace mppi_host;

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

int32_t mppi_philox_words(int32_t A) {
    return A < 1 ? 0 : 4 * (A / 8) + ((A % 8) == 0 ? 0 : (A % 8) <= 4 ? 2 : 4);
}

}  // extern "C"

// mppi_kernels.hip -- gfx950 (CDNA4) kernels of the MPPI control step.
//
//   k_rollout   one launch per step: noise draw -> double-integrator rollout ->
//               FK chain -> per-rollout cost -> online-softmin partials.
//               Replaces standard_normal_noise.py:22-50, urdf_fk.py:79-108,
//               urdfparser.py:122-163, pose_cost.py:24-63 (arm) and
//               drone_mppi.py:40-107 (drone), mppi.py:184-188 (softmin).
//   k_finalize  one launch per step: combine the partial records, w_eps,
//               SavGol (svg_filter.py:13-90), u += w_eps, outputs
//               (mppi.py:144-158, drone_mppi.py:157-169).  The same kernel in
//               PACK mode folds a shard's records into its exchange slot.
//
// Lane mapping: a wave64 holds R = 64/L rollouts, one
// L-lane segment each, lane = timestep t (L = pow2 >= H, 16..64; H > 64 runs
// ceil(H/64) chunks per lane).  The two cumsums of the integrator are DPP
// segment scans in fp64 (torch's CPU cumsum accumulates in double); the FK
// chain, cost and softmin are lane-local; S_k is a segment reduction.
// Trajectories are stored as SoA planes (V,C,K,H): every store instruction of a
// wave writes 64 consecutive floats (256 B).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "mppi_dev.h"

using namespace mppi;

namespace {

// ----------------------------------------------------------------- DPP helpers
// dpp_ctrl encodings (GFX9): row_shr:n = 0x110+n, wave_shr:1 = 0x138,
// row_bcast:15 = 0x142, row_bcast:31 = 0x143.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ double dpp_f64(double x) {
    int lo = __double2loint(x), hi = __double2hiint(x);
    lo = __builtin_amdgcn_update_dpp(0, lo, CTRL, ROWMASK, 0xF, false);
    hi = __builtin_amdgcn_update_dpp(0, hi, CTRL, ROWMASK, 0xF, false);
    return __hiloint2double(hi, lo);
}
template <int CTRL, int ROWMASK>
__device__ __forceinline__ float dpp_f32(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, ROWMASK, 0xF, false));
}

// Inclusive prefix sum inside segments of L lanes (L in {16, 32, 64}).
__device__ __forceinline__ double seg_scan(double x, int L) {
    x += dpp_f64<0x111, 0xF>(x);
    x += dpp_f64<0x112, 0xF>(x);
    x += dpp_f64<0x114, 0xF>(x);
    x += dpp_f64<0x118, 0xF>(x);
    if (L >= 32) x += dpp_f64<0x142, 0xA>(x);
    if (L >= 64) x += dpp_f64<0x143, 0xC>(x);
    return x;
}

__device__ __forceinline__ double read_lane_f64(double x, int lane) {
    int lo = __builtin_amdgcn_readlane(__double2loint(x), lane);
    int hi = __builtin_amdgcn_readlane(__double2hiint(x), lane);
    return __hiloint2double(hi, lo);
}

// ------------------------------------------------------------------- Philox
__device__ __forceinline__ void philox10(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3,
                                         uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        const uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
        const uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    }
}

__device__ __forceinline__ float u01(uint32_t x) {   // (0,1), exact in fp32
    return ((float)(x >> 8) + 0.5f) * 5.9604644775390625e-8f;
}

// Box-Muller on the hardware transcendental units: v_log_f32 (log2),
// v_sqrt_f32, v_sin_f32 / v_cos_f32 (argument in revolutions).
__device__ __forceinline__ void box_muller(uint32_t a, uint32_t b, float& z0, float& z1) {
    const float u1 = u01(a), u2 = u01(b);
    const float r = __builtin_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u1));  // -2 ln u1
    z0 = r * __builtin_amdgcn_cosf(u2);
    z1 = r * __builtin_amdgcn_sinf(u2);
}

template <int NA>
__device__ __forceinline__ void draw_normals(float (&z)[NA], uint32_t kg, uint32_t t, uint32_t veh,
                                             uint32_t step, uint32_t s0, uint32_t s1) {
#pragma unroll
    for (int j = 0; j < (NA + 3) / 4; ++j) {
        uint32_t c0 = kg, c1 = t, c2 = (veh << 8) | (uint32_t)j, c3 = step;
        philox10(c0, c1, c2, c3, s0, s1);
        float a, b, c, d;
        box_muller(c0, c1, a, b);
        box_muller(c2, c3, c, d);
        if (4 * j + 0 < NA) z[4 * j + 0] = a;
        if (4 * j + 1 < NA) z[4 * j + 1] = b;
        if (4 * j + 2 < NA) z[4 * j + 2] = c;
        if (4 * j + 3 < NA) z[4 * j + 3] = d;
    }
}

// ---------------------------------------------------------------- FK helpers
struct Mat34 { float m[12]; };   // rows 0..2 of a homogeneous transform

// T <- T * [O3 | o]  (O a constant joint origin, uniform across the wave)
__device__ __forceinline__ void mul_affine(Mat34& T, const float* O) {
    Mat34 r;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float t0 = T.m[4 * i], t1 = T.m[4 * i + 1], t2 = T.m[4 * i + 2];
#pragma unroll
        for (int j = 0; j < 3; ++j) r.m[4 * i + j] = t0 * O[j] + t1 * O[4 + j] + t2 * O[8 + j];
        r.m[4 * i + 3] = t0 * O[3] + t1 * O[7] + t2 * O[11] + T.m[4 * i + 3];
    }
    T = r;
}

// T <- T * Rot(axis, q) for a revolute joint (Rodrigues, transformation_matrix.py:68-93)
__device__ __forceinline__ void mul_revolute(Mat34& T, const JointDev& J, float c, float s) {
    const float omc = 1.0f - c;
    if (J.axis_z) {   // R = [[c,-s,0],[s,c,0],[0,0,c+(1-c)]]
        const float r22 = c + omc;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const float a0 = T.m[4 * i], a1 = T.m[4 * i + 1];
            T.m[4 * i] = a0 * c + a1 * s;
            T.m[4 * i + 1] = a1 * c - a0 * s;
            T.m[4 * i + 2] = T.m[4 * i + 2] * r22;
        }
        return;
    }
    const float vx = J.ax[0], vy = J.ax[1], vz = J.ax[2];
    float R[9];
    R[0] = c + J.axx[0] * omc; R[1] = J.axx[1] * omc - vz * s; R[2] = J.axx[2] * omc + vy * s;
    R[3] = J.axx[3] * omc + vz * s; R[4] = c + J.axx[4] * omc; R[5] = J.axx[5] * omc - vx * s;
    R[6] = J.axx[6] * omc - vy * s; R[7] = J.axx[7] * omc + vx * s; R[8] = c + J.axx[8] * omc;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float a0 = T.m[4 * i], a1 = T.m[4 * i + 1], a2 = T.m[4 * i + 2];
#pragma unroll
        for (int j = 0; j < 3; ++j) T.m[4 * i + j] = a0 * R[j] + a1 * R[3 + j] + a2 * R[6 + j];
    }
}

// T <- T * Slide(axis * q) (transformation_matrix.py:38-55)
__device__ __forceinline__ void mul_prismatic(Mat34& T, const JointDev& J, float q) {
    const float d0 = J.ax[0] * q, d1 = J.ax[1] * q, d2 = J.ax[2] * q;
#pragma unroll
    for (int i = 0; i < 3; ++i)
        T.m[4 * i + 3] += T.m[4 * i] * d0 + T.m[4 * i + 1] * d1 + T.m[4 * i + 2] * d2;
}

// sin/cos of the joint angle.  fp32 state: the fp32 angle.  fp64 state: the
// reference evaluates cos/sin in fp64 and rounds into the fp32 transform
// (transformation_matrix.py:68-93 with q promoted by mppi.py:197), so split the
// double angle into hi+lo floats and correct to first order.
__device__ __forceinline__ void joint_sincos(double qd, float qf, bool f64, float& s, float& c) {
    if (!f64) { sincosf(qf, &s, &c); return; }
    const float qh = (float)qd;
    const float ql = (float)(qd - (double)qh);
    float sh, ch;
    sincosf(qh, &sh, &ch);
    s = fmaf(ch, ql, sh);
    c = fmaf(-sh, ql, ch);
}

// Pose cost of one (k,t): w_pos*||p - p*|| + w_ori*||eulerZYX(R^T R*)||
// (pose_cost.py:24-63; rotation_conversions.py:277-319; inv(R) of the
// orthonormal FK rotation taken as R^T).
__device__ __forceinline__ float pose_cost(const Mat34& T, const VehicleConst& vc, float wp, float wo) {
    const float dx = T.m[3] - vc.tpos[0], dy = T.m[7] - vc.tpos[1], dz = T.m[11] - vc.tpos[2];
    const float cp = __builtin_sqrtf(dx * dx + dy * dy + dz * dz);
    const float* tR = vc.tR;
    const float r00 = T.m[0] * tR[0] + T.m[4] * tR[3] + T.m[8] * tR[6];
    const float r10 = T.m[1] * tR[0] + T.m[5] * tR[3] + T.m[9] * tR[6];
    const float r20 = T.m[2] * tR[0] + T.m[6] * tR[3] + T.m[10] * tR[6];
    const float r21 = T.m[2] * tR[1] + T.m[6] * tR[4] + T.m[10] * tR[7];
    const float r22 = T.m[2] * tR[2] + T.m[6] * tR[5] + T.m[10] * tR[8];
    const float yaw = atan2f(r10, r00);
    const float pitch = asinf(fminf(fmaxf(-r20, -1.0f), 1.0f));
    const float roll = atan2f(r21, r22);
    const float co = __builtin_sqrtf(yaw * yaw + pitch * pitch + roll * roll);
    return wp * cp + wo * co;
}

}  // namespace

// =============================================================================
// k_rollout
// =============================================================================
template <int MODEL, int NA, int NCH>
__global__ void __launch_bounds__(512) k_rollout(const DevParams p) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int v = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, nw = blockDim.x >> 6;
    const int L = p.L, H = p.H, K = p.K;
    const int sub = lane / L, t0 = lane & (L - 1);
    const VehicleConst& vc = p.vc[v];
    const bool f64 = (MODEL == MPPI_MODEL_ARM) && p.state_f64;

    // ---- LDS: u_prev tile (H x A) of this vehicle, then wave partials
    float* u_lds = smem;
    const int HA = H * NA;
    for (int i = tid; i < HA; i += blockDim.x) u_lds[i] = p.u_prev[(size_t)v * HA + i];
    __syncthreads();

    const uint32_t step = p.step[0];
    float acc[NCH][NA];
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
        for (int a = 0; a < NA; ++a) acc[c][a] = 0.0f;
    float rho_w = INFINITY, eta_w = 0.0f, eta2_w = 0.0f;
    int nan_w = 0;

    for (int it = 0; it < p.iters; ++it) {
        const int g = blockIdx.x + it * p.nb;
        const int k = (g * nw + wid) * p.R + sub;
        const bool kval = k < K;
        const int64_t kg = p.k_offset + k;

        float eps[NCH][NA], act[NCH][NA];
        double posd[NCH][NA];
        float posf[NCH][NA];
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const int t = t0 + 64 * c;
            const bool val = kval && t < H;
            if (p.noise_mode == MPPI_NOISE_INJECTED) {
                const float* src = p.noise_in + (((size_t)v * K + k) * H + t) * NA;
#pragma unroll
                for (int a = 0; a < NA; ++a) eps[c][a] = val ? src[a] : 0.0f;
            } else {
                float z[NA];
                draw_normals<NA>(z, (uint32_t)kg, (uint32_t)t, (uint32_t)v, step, p.seed_lo, p.seed_hi);
                if (p.sigma_diag) {
#pragma unroll
                    for (int a = 0; a < NA; ++a) eps[c][a] = val ? z[a] * p.sigma[a * NA + a] : 0.0f;
                } else {
#pragma unroll
                    for (int b = 0; b < NA; ++b) {
                        float e = 0.0f;
#pragma unroll
                        for (int a = 0; a < NA; ++a) e += z[a] * p.sigma[a * NA + b];
                        eps[c][b] = val ? e : 0.0f;
                    }
                }
            }
#pragma unroll
            for (int a = 0; a < NA; ++a) act[c][a] = val ? u_lds[t * NA + a] + eps[c][a] : 0.0f;
            if (p.store_noise && val) {
                float* dst = p.noise_out + (((size_t)v * K + k) * H + t) * NA;
#pragma unroll
                for (int a = 0; a < NA; ++a) dst[a] = eps[c][a];
            }
        }

        // ---- double integrator (standard_normal_noise.py:41-48): two fp64
        //      segment scans per dim; roundings placed where torch rounds.
        {
#pragma clang fp contract(off)
#pragma unroll
            for (int a = 0; a < NA; ++a) {
                double carry1 = 0.0, carry2 = 0.0;
                double last_vel_d = 0.0;
                float last_vel_f = 0.0f;
#pragma unroll
                for (int c = 0; c < NCH; ++c) {
                    const float s1 = act[c][a] * p.dt;
                    double c1 = seg_scan((double)s1, L) + carry1;
                    if (NCH > 1) carry1 = read_lane_f64(c1, 63);
                    const float c1f = (float)c1;
                    float dqf = 0.0f;
                    double dqd = 0.0;
                    const float h2 = (0.5f * act[c][a]) * p.dt2;
                    if (!f64) {
                        const float velf = c1f + vc.vel0f[a];
                        float prev = dpp_f32<0x138, 0xF>(velf);     // wave_shr:1
                        if (t0 == 0) prev = (c == 0) ? vc.vel0f[a] : last_vel_f;
                        if (NCH > 1) last_vel_f = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(velf), 63));
                        dqf = prev * p.dt + h2;
                        dqd = (double)dqf;
                    } else {
                        const double vel = (double)c1f + vc.vel0[a];
                        double prev = dpp_f64<0x138, 0xF>(vel);
                        if (t0 == 0) prev = (c == 0) ? vc.vel0[a] : last_vel_d;
                        if (NCH > 1) last_vel_d = read_lane_f64(vel, 63);
                        dqd = prev * p.dt_d + (double)h2;
                    }
                    double c2 = seg_scan(dqd, L) + carry2;
                    if (NCH > 1) carry2 = read_lane_f64(c2, 63);
                    if (!f64) {
                        posf[c][a] = (float)c2 + vc.pos0f[a];
                        posd[c][a] = (double)posf[c][a];
                    } else {
                        posd[c][a] = c2 + vc.pos0[a];
                        posf[c][a] = (float)posd[c][a];
                    }
                }
            }
        }

        // ---- per-(k,t) model: FK + cost, trajectory planes
        float xs[NCH];   // per-t cost term
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const int t = t0 + 64 * c;
            const bool val = kval && t < H;
            const bool term = (t == H - 1);
            float x;
            if (MODEL == MPPI_MODEL_DRONE) {
                const float dx = posf[c][0] - vc.tpos[0], dy = posf[c][1] - vc.tpos[1],
                            dz = posf[c][2] - vc.tpos[2];
                x = dx * dx + dy * dy + dz * dz;
                if (p.store_traj && val) {
                    float* dst = p.traj + ((size_t)v * p.C * K + k) * H + t;
                    const size_t plane = (size_t)K * H;
                    dst[0] = posf[c][0]; dst[plane] = posf[c][1]; dst[2 * plane] = posf[c][2];
                }
            } else {
                Mat34 T;
                if (MODEL == MPPI_MODEL_ARM) {
#pragma unroll
                    for (int i = 0; i < 12; ++i) T.m[i] = vc.base[i];
                } else {   // whole-body: [R(rpy) | p_drone(k,t)]
#pragma unroll
                    for (int i = 0; i < 12; ++i) T.m[i] = vc.base[i];
                    T.m[3] = posf[c][0]; T.m[7] = posf[c][1]; T.m[11] = posf[c][2];
                }
                for (int jn = 0; jn < p.nj; ++jn) {
                    const JointDev& J = p.joints[jn];
                    mul_affine(T, J.O);
                    if (J.type == MPPI_JOINT_FIXED) continue;
                    // select the joint coordinate (q_index is wave-uniform)
                    double qd = 0.0; float qf = 0.0f;
#pragma unroll
                    for (int a = 0; a < NA - (MODEL == MPPI_MODEL_WHOLEBODY ? 3 : 0); ++a)
                        if (a == J.q_index) {
                            qd = posd[c][a + (MODEL == MPPI_MODEL_WHOLEBODY ? 3 : 0)];
                            qf = posf[c][a + (MODEL == MPPI_MODEL_WHOLEBODY ? 3 : 0)];
                        }
                    if (J.type == MPPI_JOINT_REVOLUTE) {
                        float s, cc;
                        joint_sincos(qd, qf, f64, s, cc);
                        mul_revolute(T, J, cc, s);
                    } else {
                        mul_prismatic(T, J, qf);
                    }
                }
                x = term ? pose_cost(T, vc, p.w_tp, p.w_to) : pose_cost(T, vc, p.w_sp, p.w_so);
                if (p.store_traj && val) {
                    const size_t plane = (size_t)K * H;
                    float* dst = p.traj + ((size_t)v * p.C * K + k) * H + t;
#pragma unroll
                    for (int a = 0; a < NA; ++a) dst[a * plane] = posf[c][a];
#pragma unroll
                    for (int i = 0; i < 12; ++i) dst[(NA + i) * plane] = T.m[i];
                }
            }
            xs[c] = val ? x : 0.0f;
        }

        // ---- S_k = fl(ws * sum_{t<H-1} x_t) + fl(wt * x_{H-1})  (segment reduction)
        double stage = 0.0;
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const int t = t0 + 64 * c;
            stage += (t < H - 1) ? (double)xs[c] : 0.0;
        }
        stage = seg_scan(stage, L);
        const int seg_base = lane & ~(L - 1);
        stage = __shfl(stage, seg_base + L - 1);
        float xterm = 0.0f;
#pragma unroll
        for (int c = 0; c < NCH; ++c)
            if (c == (H - 1) / 64) xterm = __shfl(xs[c], seg_base + ((H - 1) & 63));
        float S;
        if (MODEL == MPPI_MODEL_DRONE) S = (p.w_sp * (float)stage) + (p.w_tp * xterm);
        else S = (float)stage + xterm;
        if (!kval) S = INFINITY;
        if (kval && t0 == 0) p.S[(size_t)v * K + k] = S;

        // ---- online softmin (mppi.py:184-188) across this wave's rollouts
        const bool bad = kval && (S != S);
        nan_w |= __any(bad) ? 1 : 0;
        float m = bad ? INFINITY : S;
        for (int o = L; o < 64; o <<= 1) m = fminf(m, __shfl_xor(m, o));
        if (m < INFINITY) {
            const float rn = fminf(rho_w, m);
            const float f = (rho_w == INFINITY) ? 0.0f : __expf(p.coef * (rho_w - rn));
            const float e = (bad || !kval) ? 0.0f : __expf(p.coef * (S - rn));
            float es = (t0 == 0) ? e : 0.0f, e2 = es * es;
            for (int o = 1; o < 64; o <<= 1) { es += __shfl_xor(es, o); e2 += __shfl_xor(e2, o); }
            eta_w = eta_w * f + es;
            eta2_w = eta2_w * f * f + e2;
#pragma unroll
            for (int c = 0; c < NCH; ++c)
#pragma unroll
                for (int a = 0; a < NA; ++a) acc[c][a] = acc[c][a] * f + e * eps[c][a];
            rho_w = rn;
        }
    }

    // ---- fold the R segments of the wave (same rho_w): lanes t0 hold totals
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
        for (int a = 0; a < NA; ++a)
            for (int o = L; o < 64; o <<= 1) acc[c][a] += __shfl_xor(acc[c][a], o);

    // ---- cross-wave combine in LDS -> one partial record per block
    float* wsh = smem + ((HA + 3) & ~3);          // [nw][4 + NCH*64*NA]
    const int wstride = 4 + NCH * 64 * NA;
    float* mine = wsh + wid * wstride;
    if (lane == 0) { mine[0] = rho_w; mine[1] = eta_w; mine[2] = eta2_w; mine[3] = (float)nan_w; }
    if (sub == 0) {
#pragma unroll
        for (int c = 0; c < NCH; ++c)
#pragma unroll
            for (int a = 0; a < NA; ++a) mine[4 + (c * 64 + t0) * NA + a] = acc[c][a];
    }
    __syncthreads();
    float rho_b = INFINITY;
    for (int w = 0; w < nw; ++w) rho_b = fminf(rho_b, wsh[w * wstride]);
    float* rec = p.part + ((size_t)v * p.nb + blockIdx.x) * p.P;
    if (tid == 0) {
        float eta = 0.0f, eta2 = 0.0f, nanf = 0.0f;
        for (int w = 0; w < nw; ++w) {
            const float rw = wsh[w * wstride];
            const float f = (rw == INFINITY) ? 0.0f : __expf(p.coef * (rw - rho_b));
            eta += f * wsh[w * wstride + 1];
            eta2 += f * f * wsh[w * wstride + 2];
            nanf = fmaxf(nanf, wsh[w * wstride + 3]);
        }
        rec[0] = rho_b; rec[1] = eta; rec[2] = eta2; rec[3] = nanf;
    }
    // record body a-major: N[a*H + t]
    for (int i = tid; i < HA; i += blockDim.x) {
        const int a = i / H, t = i - a * H;
        const int c = t >> 6, tl = t & 63;
        float s = 0.0f;
        for (int w = 0; w < nw; ++w) {
            const float rw = wsh[w * wstride];
            const float f = (rw == INFINITY) ? 0.0f : __expf(p.coef * (rw - rho_b));
            s += f * wsh[w * wstride + 4 + (c * 64 + tl) * NA + a];
        }
        rec[kHdr + i] = s;
    }
}

// =============================================================================
// k_finalize: grid (A, V); block a owns action dim a of vehicle v.
// =============================================================================
constexpr int kFinThreads = 256;
constexpr int kMaxRec = 4096;

__global__ void __launch_bounds__(kFinThreads) k_finalize(const FinParams p) {
    __shared__ float f_lds[kMaxRec];
    __shared__ double red[kFinThreads];
    __shared__ float nsum[kFinThreads];
    __shared__ float wcol[MPPI_MAX_HORIZON + 2 * kMaxW];
    __shared__ float s_rho, s_nan;
    __shared__ double s_eta, s_eta2;
    const int a = blockIdx.x, v = blockIdx.y, tid = threadIdx.x;
    const int H = p.H, n = p.nrec;
    const float* recs = p.rec + (size_t)v * p.rec_vstride;

    // 1. rho = min over records; NaN flag
    float m = INFINITY, nanf = 0.0f;
    for (int r = tid; r < n; r += kFinThreads) {
        m = fminf(m, recs[(size_t)r * p.rec_rstride]);
        nanf = fmaxf(nanf, recs[(size_t)r * p.rec_rstride + 3]);
    }
    red[tid] = m;
    nsum[tid] = nanf;
    __syncthreads();
    for (int s = kFinThreads / 2; s > 0; s >>= 1) {
        if (tid < s) { red[tid] = fmin(red[tid], red[tid + s]); nsum[tid] = fmaxf(nsum[tid], nsum[tid + s]); }
        __syncthreads();
    }
    if (tid == 0) { s_rho = (float)red[0]; s_nan = nsum[0]; }
    __syncthreads();
    const float rho = s_rho;

    // 2. rescale factors and normalisers (fp64 accumulation, fixed order)
    double eta = 0.0, eta2 = 0.0;
    for (int r = tid; r < n; r += kFinThreads) {
        const float* rc = recs + (size_t)r * p.rec_rstride;
        const float f = (rc[0] == INFINITY) ? 0.0f : __expf(p.coef * (rc[0] - rho));
        f_lds[r] = f;
        eta += (double)f * rc[1];
        eta2 += (double)f * f * rc[2];
    }
    red[tid] = eta;
    __syncthreads();
    for (int s = kFinThreads / 2; s > 0; s >>= 1) { if (tid < s) red[tid] += red[tid + s]; __syncthreads(); }
    if (tid == 0) s_eta = red[0];
    __syncthreads();
    red[tid] = eta2;
    __syncthreads();
    for (int s = kFinThreads / 2; s > 0; s >>= 1) { if (tid < s) red[tid] += red[tid + s]; __syncthreads(); }
    if (tid == 0) s_eta2 = red[0];
    __syncthreads();

    // 3. N[t] = sum_r f_r N_r[a][t]: thread = (t, record group)
    const int groups = kFinThreads / H > 0 ? kFinThreads / H : 1;
    float acc_t[MPPI_MAX_HORIZON / kFinThreads + 1];
    const int tpt = (H + kFinThreads - 1) / kFinThreads;   // t per thread when H > threads
    for (int i = 0; i < tpt; ++i) acc_t[i] = 0.0f;
    if (H <= kFinThreads) {
        const int t = tid % H, gidx = tid / H;
        float s = 0.0f;
        if (gidx < groups)
            for (int r = gidx; r < n; r += groups)
                s += f_lds[r] * recs[(size_t)r * p.rec_rstride + kHdr + a * H + t];
        nsum[tid] = s;
        __syncthreads();
        if (tid < H) {
            float tot = 0.0f;
            for (int g = 0; g < groups; ++g) tot += nsum[g * H + tid];
            wcol[kMaxW + tid] = tot;
        }
    } else {
        for (int i = 0; i < tpt; ++i) {
            const int t = tid + i * kFinThreads;
            if (t >= H) break;
            float s = 0.0f;
            for (int r = 0; r < n; ++r) s += f_lds[r] * recs[(size_t)r * p.rec_rstride + kHdr + a * H + t];
            wcol[kMaxW + t] = s;
        }
    }
    __syncthreads();

    if (p.mode == 1) {   // PACK into this shard's exchange slot
        float* dst = p.dst + (size_t)v * p.P;
        if (a == 0 && tid == 0) {
            dst[0] = rho; dst[1] = (float)s_eta; dst[2] = (float)s_eta2; dst[3] = s_nan;
        }
        for (int t = tid; t < H; t += kFinThreads) dst[kHdr + a * H + t] = wcol[kMaxW + t];
        return;
    }

    // 4. FINAL: w_eps = N / eta; SavGol (symmetric pad); u += w_eps; outputs
    const float etaf = (s_nan > 0.0f) ? NAN : (float)s_eta;
    for (int t = tid; t < H; t += kFinThreads) {
        const float w = wcol[kMaxW + t] / etaf;
        wcol[kMaxW + t] = w;
        if (p.wraw) p.wraw[((size_t)v * H + t) * p.A + a] = w;
    }
    __syncthreads();
    const int hf = p.half;
    if (tid < hf) {   // [d_{h-1} .. d_0 | d | d_{N-1} .. d_{N-h}]
        wcol[kMaxW - 1 - tid] = wcol[kMaxW + tid];
        wcol[kMaxW + H + tid] = wcol[kMaxW + H - 1 - tid];
    }
    __syncthreads();
    float* up = p.u_prev + (size_t)v * H * p.A;
    const float uold0 = up[a];
    __syncthreads();
    for (int t = tid; t < H; t += kFinThreads) {
        float s = 0.0f;
        for (int j = 0; j < p.window; ++j) s += p.sg[j] * wcol[kMaxW - hf + t + j];
        if (p.wsmooth) p.wsmooth[((size_t)v * H + t) * p.A + a] = s;
        up[t * p.A + a] = up[t * p.A + a] + s;
    }
    __syncthreads();
    if (tid == 0) {
#pragma clang fp contract(off)
        const float u0 = up[a];
        p.u0[(size_t)v * p.A + a] = u0;
        const VehicleConst& vc = p.vc[v];
        double* out = p.out + (size_t)v * p.out_dim;
        const bool drone_dim = (p.model == MPPI_MODEL_DRONE) || (p.model == MPPI_MODEL_WHOLEBODY && a < 3);
        if (drone_dim) {   // drone_mppi.py:168-169
            const float x0 = vc.pos0f[a], v0 = vc.vel0f[a];
            const float xo = (x0 + v0 * p.dt) + (0.5f * u0) * p.dt2;
            const float vo = v0 + p.dt * u0;
            out[a] = xo;
            out[3 + a] = vo;
        } else {           // mppi.py:157-158 (qdes uses the OLD u_prev[0])
            const int j = a - p.qoff;
            const int base = (p.model == MPPI_MODEL_WHOLEBODY) ? 6 : 0;
            const float t1 = uold0 * p.dt;
            const float t2 = ((0.5f * u0) * p.dt) * p.dt;
            const float t3 = u0 * p.dt;
            if (p.state_f64 && p.model == MPPI_MODEL_ARM) {
                out[base + j] = (vc.pos0[a] + (double)t1) + (double)t2;
                out[base + p.nq + j] = vc.vel0[a] + (double)t3;
            } else {
                out[base + j] = (double)((vc.pos0f[a] + t1) + t2);
                out[base + p.nq + j] = (double)(vc.vel0f[a] + t3);
            }
        }
        if (a == 0) {
            const double e = s_eta, e2 = s_eta2;
            float* st = p.stats + (size_t)v * 4;
            st[0] = rho;
            st[1] = (float)e;
            st[2] = (e2 > 0.0) ? (float)(e * e / e2) : 0.0f;
            st[3] = s_nan;
            if (v == 0) p.step[0] = p.step[0] + 1u;
        }
    }
}

// w_k = exp(-(S_k - rho)/lambda) / eta  (mppi.py:184-191) -- readback only
__global__ void k_weights(const float* S, const float* stats, float* w, int V, int K, float coef) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= V * K) return;
    const int v = i / K;
    const float rho = stats[v * 4], eta = stats[v * 4 + 1];
    w[i] = expf(coef * (S[i] - rho)) / eta;
}

__global__ void k_philox(uint64_t seed, uint32_t step, int veh, int64_t k0, int K, int H, int A,
                         float* z, uint32_t* raw) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= K * H) return;
    const int k = i / H, t = i - k * H;
    const int nj = (A + 3) / 4;
    for (int j = 0; j < nj; ++j) {
        uint32_t c0 = (uint32_t)(k0 + k), c1 = (uint32_t)t, c2 = ((uint32_t)veh << 8) | (uint32_t)j, c3 = step;
        philox10(c0, c1, c2, c3, (uint32_t)seed, (uint32_t)(seed >> 32));
        uint32_t* rw = raw + ((size_t)i * nj + j) * 4;
        rw[0] = c0; rw[1] = c1; rw[2] = c2; rw[3] = c3;
        float n0, n1, n2, n3;
        box_muller(c0, c1, n0, n1);
        box_muller(c2, c3, n2, n3);
        const float nn[4] = {n0, n1, n2, n3};
        for (int q = 0; q < 4; ++q)
            if (4 * j + q < A) z[(size_t)i * A + 4 * j + q] = nn[q];
    }
}

// =============================================================================
// launchers
// =============================================================================
template <int MODEL, int NA, int NCH>
static int launch_rollout_t(const DevParams& p, int threads, hipStream_t s) {
    const int nw = threads / 64;
    const size_t lds = (size_t)(((p.H * NA + 3) & ~3) + nw * (4 + NCH * 64 * NA)) * sizeof(float);
    hipLaunchKernelGGL((k_rollout<MODEL, NA, NCH>), dim3(p.nb, p.V), dim3(threads), lds, s, p);
    return (int)hipGetLastError();
}

template <int MODEL, int NA>
static int dispatch_nch(const DevParams& p, int threads, hipStream_t s) {
    switch (p.nch) {
        case 1: return launch_rollout_t<MODEL, NA, 1>(p, threads, s);
        case 2: return launch_rollout_t<MODEL, NA, 2>(p, threads, s);
        case 4: return launch_rollout_t<MODEL, NA, 4>(p, threads, s);
        default: return -1;
    }
}

extern "C" int mppi_launch_rollout(const DevParams* p, int threads, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    switch (p->model) {
        case MPPI_MODEL_DRONE:
            if (p->A == 3) return dispatch_nch<MPPI_MODEL_DRONE, 3>(*p, threads, s);
            break;
        case MPPI_MODEL_ARM:
            if (p->A == 7) return dispatch_nch<MPPI_MODEL_ARM, 7>(*p, threads, s);
            if (p->A == 6) return dispatch_nch<MPPI_MODEL_ARM, 6>(*p, threads, s);
            break;
        case MPPI_MODEL_WHOLEBODY:
            if (p->A == 10) return dispatch_nch<MPPI_MODEL_WHOLEBODY, 10>(*p, threads, s);
            if (p->A == 9) return dispatch_nch<MPPI_MODEL_WHOLEBODY, 9>(*p, threads, s);
            break;
    }
    return -1;
}

extern "C" int mppi_launch_finalize(const FinParams* p, void* stream) {
    if (p->nrec > kMaxRec || p->H > MPPI_MAX_HORIZON) return -1;
    hipLaunchKernelGGL(k_finalize, dim3(p->A, p->V), dim3(kFinThreads), 0, (hipStream_t)stream, *p);
    return (int)hipGetLastError();
}

extern "C" int mppi_launch_weights(const float* S, const float* stats, float* w, int V, int K, float coef,
                                   void* stream) {
    const int n = V * K;
    hipLaunchKernelGGL(k_weights, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, S, stats, w, V,
                       K, coef);
    return (int)hipGetLastError();
}

extern "C" int mppi_launch_philox(uint64_t seed, uint32_t step, int vehicle, int64_t k0, int K, int H, int A,
                                  float* z, uint32_t* raw, void* stream) {
    const int n = K * H;
    hipLaunchKernelGGL(k_philox, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, seed, step,
                       vehicle, k0, K, H, A, z, raw);
    return (int)hipGetLastError();
}

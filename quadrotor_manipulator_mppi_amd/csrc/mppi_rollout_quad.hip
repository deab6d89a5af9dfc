// mppi_rollout_quad.hip -- gfx950 rollout kernel of the 6-DoF rigid-body quadrotor model
// (MPPI_MODEL_QUADROTOR).
//
// The reference ships this model only as commented-out code: the loop in
// drone_mppi.py:57-83 (thrust along body z, body torques, Euler-angle attitude)
// with the rotational Jacobian and rotation matrix of drone.py:114-154 and the
// inertial parameters of aerial_manipulation/urdf/drone.urdf:15-16.  It leaves m,
// I_inv, g and kd undefined; they are mppi_config.quad_* here.  Per sample k,
// following the commented loop (x_prev = (p, rpy), v_prev = (v, omega)):
//
//   step 0:  omega_0 = omega + dt I^-1 tau_0
//            v_0     = v + dt (g + (R(rpy) f_0 - kd v) / m)          f = (0, 0, thrust)
//            rpy_0   = rpy + dt J(rpy) omega                          (drone_mppi.py:70)
//            p_0     = p + dt v                                      (drone_mppi.py:71)
//   t >= 1:  omega_t = omega_{t-1} + dt I^-1 tau_t
//            rpy_t   = wrap(rpy_{t-1} + dt J(rpy_{t-1}) omega_t)      (:74-76)
//            v_t     = v_{t-1} + dt (g + (R(rpy_{t-1}) f_t - kd v_{t-1}) / m)   (:77)
//            p_t     = p_{t-1} + dt v_t                               (:78)
//
// J is the body-rate -> Euler-rate map of drone.py:114-124.  The commented loop
// applies inv(J) for t >= 1 and J at t = 0; the build uses J at every step
// (the inverse maps Euler rates to body rates, so it cannot
// integrate them).  wrap(x) = atan2(sin x, cos x) is taken as x - 2 pi rint(x / 2 pi).
// Cost: the drone's squared position cost (drone_mppi.py:87-107).
//
// The dynamics are sequential in t, so the lane mapping differs from k_rollout's
// (lane = timestep, prefix-scan integrator).  A block owns 64 rollouts:
//   1. all 4 waves draw the (64 x H) noise tile (Philox is counter-based, so no
//      sequential dependence) and u_prev into LDS;
//   2. wave 0 steps its 64 rollouts (lane = rollout) through t, the critical path;
//   3. all 4 waves form the block's online-softmin record
//      N[a][t] = sum_k exp(-(S_k - rho_b)/lambda) eps_k[t][a] (lane = t, 16 rollouts
//      per wave), written in k_rollout's record format, so k_finalize combines it
//      unchanged.  One record per block.
#include <type_traits>

#include "mppi_rollout.h"

namespace {

constexpr int kQA = 4;          // thrust, tau_x, tau_y, tau_z
constexpr int kQRow = 65;       // LDS row pitch in float4 (64 lanes + 1: no bank conflicts at lane = t)
constexpr int kQWaves = 4;      // waves per block: all draw the noise tile and form the record,
constexpr int kQThreads = 64 * kQWaves;   // wave 0 runs the sequential dynamics

__device__ __forceinline__ float wave_min_f32(float x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = fminf(x, __shfl_xor(x, o));
    return x;
}
__device__ __forceinline__ float wave_sum_f32(float x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    return x;
}

}  // namespace

template <bool VONE>
__global__ void __launch_bounds__(kQThreads) k_rollout_quad(const uint32_t seed_lo, const uint32_t seed_hi,
                                                            const uint32_t step_ctr, const uint32_t k_off,
                                                            const int32_t noise_mode, const int32_t H,
                                                            const float* __restrict__ u_prev, const DevParams pk) {
    extern __shared__ __attribute__((aligned(16))) float4 eps_lds[];   // [H][kQRow] eps, then [H] u_prev
    __shared__ float e_lds[64];
    __shared__ float4 part[kQWaves - 1][64];
    const DevParams& p = pk;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, v = blockIdx.y, b = blockIdx.x;
    const int K = p.K;
    const int kb = b * 64;                       // the block's 64 rollouts: kb .. kb+63
    float4* u_lds = eps_lds + H * kQRow;
    const VehicleConst& vc = VONE ? pk.vc0 : pk.vc[v];
    if (VONE && b == 0) {   // hand vc0 to the finalize (it reads vc[v])
        constexpr int kVCW = (int)(sizeof(VehicleConst) / 4);
        for (int i = tid; i < kVCW; i += kQThreads) ((int*)pk.vc)[i] = ((const int*)&pk.vc0)[i];
    }
    // ---- phase 1, all waves: u_prev and the (64 x H) noise tile into LDS.  Noise
    //      (standard_normal_noise.py:22-29 / drone_mppi.py:40-44): one Philox call per
    //      (k, t) gives its 4 normals, the same counter as k_rollout's j = 0 draw.
    const float4* up = reinterpret_cast<const float4*>(u_prev + (size_t)v * H * kQA);
    for (int t = tid; t < H; t += kQThreads) u_lds[t] = up[t];
    for (int i = tid; i < 64 * H; i += kQThreads) {
        const int kk = i & 63, t = i >> 6, k = kb + kk;
        const bool kval = k < K;
        float eps[kQA];
        if (noise_mode == MPPI_NOISE_INJECTED) {
            const int kc = kval ? k : K - 1;
            const float4 n = *reinterpret_cast<const float4*>(p.noise_in + (((size_t)v * K + kc) * H + t) * kQA);
            eps[0] = n.x; eps[1] = n.y; eps[2] = n.z; eps[3] = n.w;
        } else {
            float z[kQA];
            draw_normals<kQA>(z, k_off + (uint32_t)k, (uint32_t)t, (uint32_t)v, step_ctr, seed_lo, seed_hi);
            if (p.sigma_diag) {
#pragma unroll
                for (int a = 0; a < kQA; ++a) eps[a] = z[a] * p.sdiag[a];
            } else {
#pragma unroll
                for (int c = 0; c < kQA; ++c) {
                    float e = 0.0f;
#pragma unroll
                    for (int a = 0; a < kQA; ++a) e += z[a] * p.sigma[a * kQA + c];
                    eps[c] = e;
                }
            }
        }
#pragma unroll
        for (int a = 0; a < kQA; ++a) eps[a] = kval ? eps[a] : 0.0f;
        eps_lds[t * kQRow + kk] = make_float4(eps[0], eps[1], eps[2], eps[3]);
        if (p.store_noise && kval)
            *reinterpret_cast<float4*>(p.noise_out + (((size_t)v * K + k) * H + t) * kQA) =
                make_float4(eps[0], eps[1], eps[2], eps[3]);
    }
    __syncthreads();

    // ---- phase 2, wave 0: the sequential dynamics, lane = rollout
    if (wid == 0) {
        const int k = kb + lane;
        const bool kval = k < K;
        const float dt = p.dt, im = p.q_inv_m, kd = p.q_kd, g = p.q_g;
        const float ix = p.q_iinv[0], iy = p.q_iinv[1], iz = p.q_iinv[2];
        const float tx = vc.tpos[0], ty = vc.tpos[1], tz = vc.tpos[2];
        // state: position, Euler angles, world velocity, body rates
        float px = vc.pos0f[0], py = vc.pos0f[1], pz = vc.pos0f[2];
        float er = vc.pos0f[3], ep = vc.pos0f[4], ey = vc.pos0f[5];
        float vx = vc.vel0f[0], vy = vc.vel0f[1], vz = vc.vel0f[2];
        float wx = vc.vel0f[3], wy = vc.vel0f[4], wz = vc.vel0f[5];
        const float ox0 = wx, oy0 = wy, oz0 = wz;
        // trajectory planes t-major, (V, C, H, K): lane = rollout, so each store instruction
        // of a step writes 64 consecutive floats (the (V,C,K,H) planes of k_rollout would
        // scatter them H floats apart)
        const uint32_t plane_b = (uint32_t)K * (uint32_t)H * 4u;
        const __amdgpu_buffer_rsrc_t trs = traj_rsrc(pk.traj + (size_t)v * pk.C * K * H, plane_b, pk.C);
        const uint32_t koff = (uint32_t)k * 4u, tstep_b = (uint32_t)K * 4u;
        float stage = 0.0f, term = 0.0f;
        // one step; the first (FIRST) is peeled: it integrates the measured velocity and
        // rates (drone_mppi.py:65-70) and skips the angle wrap
        auto step = [&](const int t, auto first_c) {
            constexpr bool FIRST = decltype(first_c)::value;
            // v = u + eps (drone_mppi.py:144); f = (0, 0, thrust), tau (drone_mppi.py:59-60)
            const float4 ee = eps_lds[t * kQRow + lane], uu = u_lds[t];
            const float thr = uu.x + ee.x, t1 = uu.y + ee.y, t2 = uu.z + ee.z, t3 = uu.w + ee.w;
            // body rates: omega_t = omega_{t-1} + dt * (I^-1 tau_t)
            wx = wx + dt * (ix * t1);
            wy = wy + dt * (iy * t2);
            wz = wz + dt * (iz * t3);
            // attitude of the previous step: R (drone.py:126-154) and J (drone.py:114-124)
            float sr, cr, sp, cp, sy, cy;
            sincos_joint(er, sr, cr);
            sincos_joint(ep, sp, cp);
            sincos_joint(ey, sy, cy);
            // one hardware reciprocal (v_rcp_f32, <= 1 ulp) for tan and the 1/cos terms of J:
            // the IEEE division was ~10 ops on the one wave's serial chain; mul/add pairs
            // contract into FMAs (the dynamics are that chain's issue)
            const float ic = __builtin_amdgcn_rcpf(cp);
            const float tp = sp * ic;
            const float r02 = cy * sp * cr + sy * sr;
            const float r12 = sy * sp * cr - cy * sr;
            const float r22 = cp * cr;
            // Euler rates J(rpy) * omega; step 0 integrates the measured rates (drone_mppi.py:70)
            const float ox = FIRST ? ox0 : wx, oy = FIRST ? oy0 : wy, oz = FIRST ? oz0 : wz;
            const float dr = ox + sr * tp * oy + cr * tp * oz;
            const float dpi = cr * oy - sr * oz;
            const float dya = (sr * ic) * oy + (cr * ic) * oz;
            float nr = er + dt * dr, np_ = ep + dt * dpi, ny = ey + dt * dya;
            if (!FIRST) {   // atan2(sin x, cos x) (drone_mppi.py:76)
                nr = nr - 6.283185307179586f * __builtin_rintf(nr * 0.15915494309189535f);
                np_ = np_ - 6.283185307179586f * __builtin_rintf(np_ * 0.15915494309189535f);
                ny = ny - 6.283185307179586f * __builtin_rintf(ny * 0.15915494309189535f);
            }
            // translational: v_t = v_{t-1} + dt (g + (R f - kd v_{t-1}) / m); p_t = p_{t-1} + dt v
            const float ax_ = im * (r02 * thr - kd * vx);
            const float ay_ = im * (r12 * thr - kd * vy);
            const float az_ = -g + im * (r22 * thr - kd * vz);
            const float nvx = vx + dt * ax_, nvy = vy + dt * ay_, nvz = vz + dt * az_;
            // step 0 moves with the measured velocity (drone_mppi.py:71), later steps with v_t
            px = px + dt * (FIRST ? vx : nvx);
            py = py + dt * (FIRST ? vy : nvy);
            pz = pz + dt * (FIRST ? vz : nvz);
            vx = nvx; vy = nvy; vz = nvz;
            er = nr; ep = np_; ey = ny;
            if (p.store_traj && kval) {
                const uint32_t o = koff + (uint32_t)t * tstep_b;
                traj_store(trs, o, 0u, px); traj_store(trs, o, plane_b, py); traj_store(trs, o, 2u * plane_b, pz);
                traj_store(trs, o, 3u * plane_b, er); traj_store(trs, o, 4u * plane_b, ep);
                traj_store(trs, o, 5u * plane_b, ey);
            }
            // squared position error (drone_mppi.py:87-107)
            const float dx = px - tx, dy = py - ty, dz = pz - tz;
            const float x = dx * dx + dy * dy + dz * dz;
            if (t < H - 1) stage += x; else term = x;
        };
        step(0, std::true_type{});
        for (int t = 1; t < H; ++t) step(t, std::false_type{});
        const float S = kval ? (p.w_sp * stage) + (p.w_tp * term) : INFINITY;
        if (kval) p.S[(size_t)v * K + k] = S;
        // ---- online softmin over the block's 64 rollouts (mppi.py:184-188 / drone_mppi.py:111-130)
        const bool bad = S != S;
        const float rho = wave_min_f32(bad ? INFINITY : S);
        const float e = (kval && !bad && rho < INFINITY) ? __expf(p.coef * (S - rho)) : 0.0f;
        const float eta = wave_sum_f32(e), eta2 = wave_sum_f32(e * e);
        const float nanf = wave_sum_f32(bad && kval ? 1.0f : 0.0f) > 0.0f ? 1.0f : 0.0f;
        e_lds[lane] = e;
        if (lane == 0)
            *reinterpret_cast<float4*>(p.hdr + ((size_t)v * p.nb + b) * 4) = make_float4(rho, eta, eta2, nanf);
    }
    __syncthreads();
    // ---- phase 3, all waves: record N[a][t] = sum_k e_k eps_k[t][a], lane = t, wave w
    //      sums rollouts [16w, 16w + 16), wave 0 folds the partials and writes the record
    float4 n = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (lane < H) {
        const float4* row = eps_lds + lane * kQRow + wid * (64 / kQWaves);
#pragma unroll
        for (int j = 0; j < 64 / kQWaves; ++j) {
            const float w = e_lds[wid * (64 / kQWaves) + j];
            const float4 x = row[j];
            n.x = fmaf(w, x.x, n.x); n.y = fmaf(w, x.y, n.y); n.z = fmaf(w, x.z, n.z); n.w = fmaf(w, x.w, n.w);
        }
        if (wid > 0) part[wid - 1][lane] = n;
    }
    __syncthreads();
    if (wid == 0 && lane < H) {
#pragma unroll
        for (int w = 0; w < kQWaves - 1; ++w) {
            const float4 x = part[w][lane];
            n.x += x.x; n.y += x.y; n.z += x.z; n.w += x.w;
        }
        const size_t base = ((size_t)v * kQA * p.nb + b) * H + lane;
        const size_t as = (size_t)p.nb * H;
        p.rdata[base] = n.x; p.rdata[base + as] = n.y; p.rdata[base + 2 * as] = n.z; p.rdata[base + 3 * as] = n.w;
    }
}

extern "C" int mppi_launch_rollout_quad(const DevParams* p, int threads, void* stream) {
    (void)threads;   // 64 rollouts (kQWaves waves) per block
    if (p->H > 64 || p->A != kQA || p->nb * 64 < p->K) return -1;
    const size_t lds = (size_t)(p->H * kQRow + p->H) * sizeof(float4);
    hipStream_t s = (hipStream_t)stream;
    if (p->V == 1)
        hipLaunchKernelGGL(k_rollout_quad<true>, dim3(p->nb, p->V), dim3(kQThreads), lds, s, p->seed_lo, p->seed_hi,
                           p->step_ctr, (uint32_t)p->k_offset, p->noise_mode, p->H, p->u_prev, *p);
    else
        hipLaunchKernelGGL(k_rollout_quad<false>, dim3(p->nb, p->V), dim3(kQThreads), lds, s, p->seed_lo, p->seed_hi,
                           p->step_ctr, (uint32_t)p->k_offset, p->noise_mode, p->H, p->u_prev, *p);
    return (int)hipGetLastError();
}

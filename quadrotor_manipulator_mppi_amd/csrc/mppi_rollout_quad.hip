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
// applies inv(J) for t >= 1 and J at t = 0.  By default the build uses J at every step
// (the inverse maps Euler rates to body rates, so it cannot integrate them);
// mppi_config.quad_literal_jinv = 1 reproduces the loop as written (the closed form
// inv(J) = [[1, 0, -s_th], [0, c_ph, s_ph c_th], [0, -s_ph, c_ph c_th]]).
// wrap(x) = atan2(sin x, cos x) is taken as x - 2 pi rint(x / 2 pi).
// Cost: the drone's squared position cost (drone_mppi.py:87-107).
//
// The dynamics are sequential in t, so the lane mapping differs from k_rollout's
// (lane = timestep, prefix-scan integrator).  A block owns 16 rollouts:
//   1. all 4 waves draw the (16 x H) noise tile (Philox is counter-based, so no
//      sequential dependence) and u_prev into LDS;
//   2. wave 0 steps the 16 rollouts through t, FOUR lanes per rollout: lane j < 3 owns
//      axis j (position, velocity, Euler angle j, body rate j) and the sin/cos of its
//      own angle; quad_perm DPP broadcasts hand each lane the other two angles' sin/cos
//      and body rates.  One step is then ~35 instructions on the serial chain instead
//      of ~110 with one lane per rollout (lane 3 follows axis 2, masked);
//   3. wave 0 forms the block's online-softmin record
//      N[a][t] = sum_k exp(-(S_k - rho_b)/lambda) eps_k[t][a] (lane = t), written in
//      k_rollout's record format, so k_finalize combines it unchanged.  One record per
//      block.
#include <type_traits>

#include "mppi_rollout.h"

namespace {

constexpr int kQA = 4;                     // thrust, tau_x, tau_y, tau_z
constexpr int kQR = 16;                    // rollouts per dynamics wave (4 lanes each)
constexpr int kQWaves = 4;                 // all draw the noise tile; wave 0 steps the dynamics
constexpr int kQThreads = 64 * kQWaves;
// Block size NT: 512 threads for the one-dynamics-wave variant while the grid is at most
// 512 blocks (its phase-1 noise tile, 16 x H draws, then takes one draw per thread at
// H <= 32 on otherwise idle SIMDs: K=4096 H=32 rollout 7.99 -> 7.83 us, H=64 12.8 -> 12.2),
// else 256 (at 1024 blocks the extra waves only cost: K=16384 9.3 -> 9.5 us;
// profiles/r02/ab_quadrotor_block512.txt)
constexpr int kQThreadsWide = 512;

// lane SRC of every 4-lane group, to all four (DPP quad_perm [SRC, SRC, SRC, SRC])
template <int SRC>
__device__ __forceinline__ float qbc(float x) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), SRC * 0x55, 0xF, 0xF, false));
}
// per-lane select by a wave-uniform lane mask (m-lanes take b): a ternary on the lane's
// axis index compiled to divergent branches around each formula
__device__ __forceinline__ float lane_sel(float a, float b, uint64_t m) {
    float r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
    return r;
}
// sum over the 4 lanes of a group, in every lane
__device__ __forceinline__ float qsum(float x) {
    x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0xB1, 0xF, 0xF, false));   // [1,0,3,2]
    x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x4E, 0xF, 0xF, false));   // [2,3,0,1]
    return x;
}
}  // namespace

// NWD dynamics waves per block (1 or 4): 16 rollouts per block while the grid stays at most
// 1024 blocks (a small K spreads its noise tile and dynamics over the most CUs), 64 above
// (fewer records for the finalize: its record loop is sequential in chunks).
template <bool VONE, bool LIT, int NWD, int NT>
__global__ void __launch_bounds__(NT) k_rollout_quad(const uint32_t seed_lo, const uint32_t seed_hi,
                                                            const uint32_t step_arg, const uint32_t k_off,
                                                            const int32_t noise_arg, const int32_t H,
                                                            const float* __restrict__ u_prev, const DevParams pk) {
    static_assert(NWD == 1 || NWD == kQWaves, "dynamics waves per block");
    static_assert(NT == kQThreads || (NWD == 1 && NT == kQThreadsWide), "block size");
    constexpr int QR = kQR * NWD;              // rollouts per block
    constexpr int kQPitch = QR * kQA + 1;      // LDS floats per t row of the eps tile (odd: the record
                                               // phase's lane = t reads are bank-conflict free)
    extern __shared__ __attribute__((aligned(16))) float qlds[];   // eps tile [H+1][kQPitch], u_prev [H+1][4]
    __shared__ float e_lds[QR];
    __shared__ __attribute__((aligned(16))) float s_lds[QR];   // the costs, staged for st_dev_run
    __shared__ float wred[kQWaves][4];         // NWD > 1: the waves' (rho, eta, eta2, nan)
    __shared__ float4 part[kQWaves][64];       // NWD > 1: the waves' record partials (lane = t)
    const DevParams& p = pk;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, v = blockIdx.y, b = blockIdx.x;
    const int32_t noise_mode = noise_arg & 0xFF;
    const uint32_t step_ctr = step_of(step_arg, noise_arg);   // (native dispatch: from the dispatch id)
    const uint32_t vkey = (uint32_t)v + ((uint32_t)noise_arg >> 16);   // fleet-wide vehicle index (k_rollout)
    const int K = p.K;
    const int kb = b * QR;                       // the block's rollouts kb .. kb+QR-1
    float* const eps_t = qlds;
    float* const u_t = qlds + (H + 1) * kQPitch;
    const VehicleConst& vc = VONE ? pk.vc0 : pk.vc[v];
    if (VONE && b == 0) {   // hand vc0 to the finalize (it reads vc[v])
        constexpr int kVCW = (int)(sizeof(VehicleConst) / 4);
        for (int i = tid; i < kVCW; i += NT)   // (written through: k_rollout's drain_stores)
            __hip_atomic_store((int*)pk.vc + i, i == kVcStepWord ? (int)step_ctr : ((const int*)&pk.vc0)[i],
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // (+ the step: mppi_dev.h kVcStepWord)
    }
    // ---- phase 1, all waves: u_prev and the (16 x H) noise tile into LDS.  Noise
    //      (standard_normal_noise.py:22-29 / drone_mppi.py:40-44): the 4 normals of (k, t)
    //      are k_rollout's draw for 4 dims (one Philox2x32-10 call).
    // u_prev (H*4 <= 256 floats, one per thread) stays in flight across the draws, and the
    // dynamics phase's scalars are read here, so their loads share the noise phase's wait
    const float* up = u_prev + (size_t)v * H * kQA;
    const float u_r = (tid < H * kQA) ? ld_dev(up + tid) : 0.0f;   // (the previous finalize's; device scope)
    float x6[6], v6[6], tg3[3], ii3[3];
#pragma unroll
    for (int d = 0; d < 6; ++d) { x6[d] = uniform_f32(vc.pos0f[d]); v6[d] = uniform_f32(vc.vel0f[d]); }
#pragma unroll
    for (int d = 0; d < 3; ++d) { tg3[d] = uniform_f32(vc.tpos[d]); ii3[d] = p.q_iinv[d]; }
    float sdt = p.dt, sim = p.q_inv_m, skd = p.q_kd, sg = p.q_g, swsp = p.w_sp, swtp = p.w_tp, scoef = p.coef;
    const int sstore = p.store_traj;
    // one asm consumes them all: the loads issue together and are waited for once
    asm volatile("" : "+s"(x6[0]), "+s"(x6[1]), "+s"(x6[2]), "+s"(x6[3]), "+s"(x6[4]), "+s"(x6[5]),
                      "+s"(v6[0]), "+s"(v6[1]), "+s"(v6[2]), "+s"(v6[3]), "+s"(v6[4]), "+s"(v6[5]),
                      "+s"(tg3[0]), "+s"(tg3[1]), "+s"(tg3[2]), "+s"(ii3[0]), "+s"(ii3[1]), "+s"(ii3[2]),
                      "+s"(sdt), "+s"(sim), "+s"(skd), "+s"(sg), "+s"(swsp), "+s"(swtp), "+s"(scoef));
    for (int i = tid; i < QR * H; i += NT) {
        // rollouts past K replicate sample K-1 (noise and all): their lanes then compute and
        // store exactly K-1's values, so the dynamics need no store masks; weight 0 below
        const int r = i & (QR - 1), t = i / QR, k = kb + r;
        const bool kval = k < K;
        const int kc = kval ? k : K - 1;
        float eps[kQA];
        if (noise_mode == MPPI_NOISE_INJECTED) {
            const float4 n = *reinterpret_cast<const float4*>(p.noise_in + (((size_t)v * K + kc) * H + t) * kQA);
            eps[0] = n.x; eps[1] = n.y; eps[2] = n.z; eps[3] = n.w;
        } else {
            float z[kQA];
            draw_normals<kQA>(z, k_off + (uint32_t)kc, (uint32_t)t, vkey, step_ctr, seed_lo, seed_hi);
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
        float* dst = eps_t + t * kQPitch + r * kQA;
#pragma unroll
        for (int a = 0; a < kQA; ++a) dst[a] = eps[a];
        if (p.store_noise && kval) {   // (readback only: written through, st_dev)
            float* dst = p.noise_out + (((size_t)v * K + k) * H + t) * kQA;
#pragma unroll
            for (int a = 0; a < kQA; ++a) st_dev(dst + a, eps[a]);
        }
    }
    if (tid < H * kQA) u_t[tid] = u_r;
    __syncthreads();
    if (wid >= NWD) { drain_stores(); return; }

    // ---- phase 2, wave 0: the sequential dynamics, lane = (rollout r, axis j).  Lane 3
    //      follows axis 2 bit for bit and lanes past K replicate sample K-1, so every lane
    //      stores (duplicates write equal values to equal addresses) and no exec mask is
    //      set up per step.
    const int r = wid * kQR + (lane >> 2), j = lane & 3, jj = j < 3 ? j : 2;
    const int k = kb + r;
    const bool kval = k < K;
    const int kc = kval ? k : K - 1;
    constexpr uint64_t kM0 = 0x1111111111111111ull, kM1 = 0x2222222222222222ull;   // lanes of axis 0 / 1
    constexpr uint64_t kM2 = 0xCCCCCCCCCCCCCCCCull;                                  // axis 2 (and lane 3)
    auto axis = [&](const float* x3) { return lane_sel(lane_sel(x3[2], x3[1], kM1), x3[0], kM0); };
    const float dt = sdt, im = sim, kd = skd;
    const float gj = (j >= 2) ? -sg : 0.0f;      // g = (0, 0, -q_g)
    const float ij = axis(ii3), tg = axis(tg3);
    // this lane's axis of the state: position, Euler angle, world velocity, body rate
    float pj = axis(x6), ej = axis(x6 + 3), vj = axis(v6), wj = axis(v6 + 3);
    const float ox0 = v6[3], oy0 = v6[4], oz0 = v6[5];   // measured body rates
    // trajectory planes t-major, (V, C, H, Kp): lane (r, j) writes channel j (position) and
    // 3 + j (angle) of sample k; a store instruction covers 16 consecutive k (64 B) of 3
    // planes.  Rows are padded to Kp = K rounded up to 16 (pk.hp) and the lanes past K write
    // the pad (sample K-1's values), so a ragged K leaves no partial 64 B sector
    const int kp = pk.hp;
    const uint32_t plane_b = (uint32_t)kp * (uint32_t)H * 4u;
    const __amdgpu_buffer_rsrc_t trs = traj_rsrc(pk.traj + (size_t)v * pk.C * kp * H, plane_b, pk.C);
    const uint32_t off_p = (uint32_t)(k < kp ? k : kc) * 4u + (uint32_t)jj * plane_b, off_e = off_p + 3u * plane_b;
    const uint32_t tstep_b = (uint32_t)kp * 4u;
    const bool store = sstore != 0;
    float stage = 0.0f, term = 0.0f;
    const float a0 = (j == 0) ? 1.0f : 0.0f;   // J's column 0 is (1, 0, 0)
    // v = u + eps (drone_mppi.py:144): thrust and this axis' torque.  The LDS operands are
    // loaded one step ahead and added at their use, so the load latency hides behind a
    // step (the tile has a spare row H, never used).
    const float* rowp = eps_t + r * kQA;
    const float* urp = u_t;
    float pu0 = urp[0], pe0 = rowp[0], pu1 = urp[1 + jj], pe1 = rowp[1 + jj];
    auto step = [&](const int t, auto first_c, auto last_c) {
        constexpr bool FIRST = decltype(first_c)::value, LAST = decltype(last_c)::value;
        const float thr = pu0 + pe0, tau = pu1 + pe1;
        rowp += kQPitch;
        urp += kQA;
        pu0 = urp[0]; pe0 = rowp[0]; pu1 = urp[1 + jj]; pe1 = rowp[1 + jj];
        // body rate: omega_t = omega_{t-1} + dt * (I^-1 tau_t) (drone_mppi.py:65,72)
        wj = wj + dt * (ij * tau);
        // attitude of the previous step: sin/cos of this lane's angle, the others by DPP
        float sj, cj;
        sincos_joint(ej, sj, cj);
        const float sr = qbc<0>(sj), cr = qbc<0>(cj), sp = qbc<1>(sj), cp = qbc<1>(cj);
        const float sy = qbc<2>(sj), cy = qbc<2>(cj);
        // step 0 integrates the measured rates (drone_mppi.py:69), later steps omega_t
        const float ox = FIRST ? ox0 : qbc<0>(wj), oy = FIRST ? oy0 : qbc<1>(wj), oz = FIRST ? oz0 : qbc<2>(wj);
        // Euler rates of this lane's axis: J(rpy) omega (drone.py:114-124), or inv(J) omega
        // for t >= 1 in the literal mode (drone_mppi.py:73-75)
        float dj;
        if (LIT && !FIRST) {
            const float d0 = ox - sp * oz;
            const float d1 = cr * oy + (sr * cp) * oz;
            const float d2 = (cr * cp) * oz - sr * oy;
            dj = lane_sel(lane_sel(d2, d1, kM1), d0, kM0);
        } else {
            // row j of J as (A_j, B_j, C_j): (1, s_r t, c_r t), (0, c_r, -s_r), (0, s_r/c_p, c_r/c_p)
            // with t = s_p / c_p: B and C of rows 0 and 2 are (s_r, c_r) times f = (s_p or 1) / c_p
            const float ic = __builtin_amdgcn_rcpf(cp);   // one v_rcp_f32 (<= 1 ulp) for tan and 1/cos
            const float f = ic * lane_sel(1.0f, sp, kM0);
            const float Bj = lane_sel(sr * f, cr, kM1), Cj = lane_sel(cr * f, -sr, kM1);
            dj = fmaf(Cj, oz, fmaf(Bj, oy, a0 * ox));
        }
        float en = ej + dt * dj;
        if (!FIRST) en = en - 6.283185307179586f * __builtin_rintf(en * 0.15915494309189535f);   // atan2(sin, cos) (:76)
        // translational: v_t = v_{t-1} + dt (g + (R f - kd v_{t-1}) / m), f = (0, 0, thrust),
        // R(rpy_{t-1}) (drone.py:126-154); p_t = p_{t-1} + dt v
        // column 2 of R: (c_y s_p c_r + s_y s_r, s_y s_p c_r - c_y s_r, c_p c_r) as
        // P_j (s_p c_r) + Q_j s_r for rows 0, 1
        const float Pj = lane_sel(sy, cy, kM0), Qj = lane_sel(-cy, sy, kM0);
        const float rj = lane_sel(fmaf(Pj, sp * cr, Qj * sr), cp * cr, kM2);
        const float aj = gj + im * (rj * thr - kd * vj);
        const float nv = vj + dt * aj;
        pj = pj + dt * (FIRST ? vj : nv);   // step 0 moves with the measured velocity (:70)
        vj = nv;
        ej = en;
        if (store) {
            const uint32_t o = (uint32_t)t * tstep_b;
            traj_store(trs, off_p, o, pj);
            traj_store(trs, off_e, o, ej);
        }
        // squared position error of this axis (drone_mppi.py:87-107), summed over axes below
        const float dd = pj - tg;
        if (LAST) term = dd * dd; else stage = fmaf(dd, dd, stage);
    };
    using T_ = std::true_type;
    using F_ = std::false_type;
    step(0, T_{}, F_{});
    int t = 1;
    for (; t + 4 <= H - 1; t += 4) {   // unrolled: the LDS and store offsets fold into immediates
        step(t, F_{}, F_{}); step(t + 1, F_{}, F_{}); step(t + 2, F_{}, F_{}); step(t + 3, F_{}, F_{});
    }
    for (; t < H - 1; ++t) step(t, F_{}, F_{});
    step(H - 1, F_{}, T_{});
    // axes 0..2 of the rollout (lane 3 duplicates axis 2)
    stage = qbc<0>(stage) + qbc<1>(stage) + qbc<2>(stage);
    term = qbc<0>(term) + qbc<1>(term) + qbc<2>(term);
    const float S = kval ? (swsp * stage) + (swtp * term) : INFINITY;
    if (j == 0) s_lds[r] = S;
    // ---- online softmin over the block's rollouts (mppi.py:184-188 / drone_mppi.py:111-130)
    const bool mine = kval && j == 0, bad = S != S;
    float rho = wave_fold_all((mine && !bad) ? S : INFINITY, OpMin());
    float nanf = wave_fold_all(mine && bad ? 1.0f : 0.0f, OpMax());
    if constexpr (NWD > 1) {
        if (lane == 0) { wred[wid][0] = rho; wred[wid][3] = nanf; }
        __syncthreads();
#pragma unroll
        for (int w = 0; w < NWD; ++w) { rho = fminf(rho, wred[w][0]); nanf = fmaxf(nanf, wred[w][3]); }
    }
    const float e = (mine && !bad && rho < INFINITY) ? __expf(scoef * (S - rho)) : 0.0f;
    float eta = wave_fold_all(e, OpAdd()), eta2 = wave_fold_all(e * e, OpAdd());
    if (j == 0) e_lds[r] = e;
    wave_lds_handoff();
    {   // this wave's 16 costs as one write-through 64 B run (mppi_device.h st_dev_run)
        const int k0 = kb + wid * kQR, n = min(kQR, K - k0);
        if (lane < 4) st_dev_run(uniform_ptr(p.S + (size_t)v * K), (uint32_t)k0, s_lds + wid * kQR, n, lane);
    }
    // ---- record N[a][t] = sum_k e_k eps_k[t][a], lane = t (each wave its own 16 rollouts)
    float n[kQA] = {0.0f, 0.0f, 0.0f, 0.0f};
    if (lane < H) {
        const float* row = eps_t + lane * kQPitch + wid * kQR * kQA;
#pragma unroll
        for (int rr = 0; rr < kQR; ++rr) {
            const float w = e_lds[wid * kQR + rr];
#pragma unroll
            for (int a = 0; a < kQA; ++a) n[a] = fmaf(w, row[rr * kQA + a], n[a]);
        }
    }
    if constexpr (NWD > 1) {
        if (lane == 0) { wred[wid][1] = eta; wred[wid][2] = eta2; }
        if (wid > 0 && lane < H) part[wid][lane] = make_float4(n[0], n[1], n[2], n[3]);
        __syncthreads();
        if (wid != 0) { drain_stores(); return; }
        eta = 0.0f; eta2 = 0.0f;
#pragma unroll
        for (int w = 0; w < NWD; ++w) { eta += wred[w][1]; eta2 += wred[w][2]; }
        if (lane < H) {
#pragma unroll
            for (int w = 1; w < NWD; ++w) {
                const float4 x = part[w][lane];
                n[0] += x.x; n[1] += x.y; n[2] += x.z; n[3] += x.w;
            }
        }
    }
    if (lane == 0)
        wt_store4(uniform_ptr(p.hdr), ((uint32_t)v * (uint32_t)p.nb + (uint32_t)b) * 16u, make_float4(rho, eta, eta2, nanf));
    if (lane < H) {
        float* const rdata_v = uniform_ptr(p.rdata + (size_t)v * kQA * p.nb * H);
#pragma unroll
        for (int a = 0; a < kQA; ++a)
            wt_store(rdata_v, (((uint32_t)a * (uint32_t)p.nb + (uint32_t)b) * (uint32_t)H + (uint32_t)lane) * 4u, n[a]);
    }
    drain_stores();
}

extern "C" int mppi_launch_rollout_quad(const DevParams* p, int threads, void* stream) {
    (void)threads;   // block size chosen below; p->iters = dynamics waves per block (1 or 4)
    const int nwd = p->iters;
    if (p->H > 64 || p->A != kQA || (nwd != 1 && nwd != kQWaves) || p->nb * kQR * nwd < p->K) return -1;
    const size_t lds = (size_t)((p->H + 1) * (kQR * nwd * kQA + 1) + (p->H + 1) * kQA) * sizeof(float);
    hipStream_t s = (hipStream_t)stream;
    const bool wide = nwd == 1 && (size_t)p->nb * p->V <= 512;
#define MPPI_QUAD_GO(VO, LI, NW, NT)                                                                             \
    return go(k_rollout_quad<VO, LI, NW, NT>,                                                                    \
              [](char* b, size_t n) {                                                                            \
                  snprintf(b, n, "_Z14k_rollout_quadILb%dELb%dELi%dELi%dEEvjjjjiiPKfN4mppi9DevParamsE", (int)VO, \
                           (int)LI, NW, NT);                                                                     \
              },                                                                                                 \
              dim3(p->nb, p->V), dim3(NT), lds, s, p->seed_lo, p->seed_hi, p->step_ctr, (uint32_t)p->k_offset,   \
              p->noise_mode, p->H, p->u_prev, *p)
#define MPPI_QUAD_NW(VO, LI)                                                                                     \
    do {                                                                                                         \
        if (wide) MPPI_QUAD_GO(VO, LI, 1, kQThreadsWide);                                                        \
        else if (nwd == 1) MPPI_QUAD_GO(VO, LI, 1, kQThreads);                                                   \
        else MPPI_QUAD_GO(VO, LI, kQWaves, kQThreads);                                                           \
    } while (0)
    if (p->V == 1) {
        if (p->q_literal_jinv) MPPI_QUAD_NW(true, true); else MPPI_QUAD_NW(true, false);
    } else {
        if (p->q_literal_jinv) MPPI_QUAD_NW(false, true); else MPPI_QUAD_NW(false, false);
    }
#undef MPPI_QUAD_NW
#undef MPPI_QUAD_GO
    return -1;
}

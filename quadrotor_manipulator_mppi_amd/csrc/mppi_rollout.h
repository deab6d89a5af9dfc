// mppi_rollout.h -- gfx950 (CDNA4) rollout kernel of the MPPI control step (the
// template; instantiated per model in mppi_rollout_{drone,arm,arm32,wb}.hip so the
// translation units compile in parallel).
//
//   k_rollout   one launch per step: noise draw -> double-integrator rollout ->
//               FK chain -> per-rollout cost -> online-softmin partials.
//               Replaces standard_normal_noise.py:22-50, urdf_fk.py:79-108,
//               urdfparser.py:122-163, pose_cost.py:24-63 (arm) and
//               drone_mppi.py:40-107 (drone), mppi.py:184-188 (softmin).
//   (k_finalize, the second launch of a step, is in mppi_finalize.hip.)
//
// Lane mapping: a wave64 holds R = 64/L rollouts, one
// L-lane segment each, lane = timestep t (L = pow2 >= H, 16..64; H > 64 runs
// ceil(H/64) chunks per lane).  The two cumsums of the integrator run in a
// transposed lane map through the wave's LDS slot (integrate_lds; DPP segment scans
// for H > 64); the FK chain, cost and softmin are lane-local; S_k is a segment
// reduction.
// Trajectories are stored as SoA planes (V,C,K,H): every store instruction of a
// wave writes 64 consecutive floats (256 B).
#pragma once
#include "mppi_device.h"

// Timing knockouts for tools/ experiments only (MPPI_HIPCC_EXTRA=-DMPPI_KO=n; results are
// wrong in such a build): 1 drops the integrator scans, 2 the Philox draw, 4 the FK chain,
// 8 the pose cost, 16 the trajectory stores, 32 Box-Muller, 64 the block record body,
// 128 the u_prev loads (H*A <= 4 * block threads), 256 the prologue's block barrier (LDS
// staging read unsynchronised), 512 the end-of-wave store drain (the hand-off unordered).
#ifndef MPPI_KO
#define MPPI_KO 0
#endif
// waves per SIMD the rollout kernel is register-budgeted for (4: <= 128 VGPRs)
// NCH == 4 (H in 193..256) is budgeted for 2 waves (<= 256 VGPRs): at 4 it spilled
// 0.3-2 KB per lane and ran 2.3x slower (arm K=4096 H=256 40.7 -> 28.1 us, whole-body
// 81.8 -> 35.3 us); NCH == 2 keeps 4 (its 8-96 B spill is cheaper than 3 or 2 waves:
// arm H=128 13.6 us at 4, 16.7 at 3 and 2; profiles/r02/ab_rollout_occupancy_long_h.txt)
#ifndef MPPI_ROLL_OCC_NCH2
#define MPPI_ROLL_OCC_NCH2 4
#endif
// the extended (XC) NCH == 2 kernels likewise run best at 2 (whole-body K=8192 H=128 full
// Sigma 72.1 -> 43.6 us, arm 21.8 -> 19.3); XC NCH == 1 keeps 4 (2 and 3 measured slower;
// profiles/r02/ab_rollout_occupancy_xc.txt)
#ifndef MPPI_ROLL_OCC_NCH2_XC
#define MPPI_ROLL_OCC_NCH2_XC 2
#endif
#ifndef MPPI_ROLL_OCC_XC
#define MPPI_ROLL_OCC_XC 4
#endif
#ifndef MPPI_ROLL_OCC
#define MPPI_ROLL_OCC 4
#endif
// wave priority by remaining rollout groups (k_rollout, iters > 1)
#ifndef MPPI_PRIO
#define MPPI_PRIO 1
#endif
// experiment knob: the costs S as plain per-lane stores (round 3), not staged write-through runs
#ifndef MPPI_S_PLAIN
#define MPPI_S_PLAIN 0
#endif
// park eps in LDS across the FK and cost (k_rollout, NA >= 7) -- in the extended and the
// multi-chunk kernels only: the common one-chunk kernels keep it in registers (whole-body 89 -> 96
// VGPRs, still 5 waves per SIMD, no scratch; same-process A/B, mean of both orders,
// profiles/r05/eps_stash: C3 -0.10 us per step, whole-body K=8192 -0.22, K=65536 -1.7, V=8 fleet -1.7)
#ifndef MPPI_EPS_STASH
#define MPPI_EPS_STASH 1
#endif
// experiment knob: after the block-combine barrier the waves with no record element (and
// not wave 0, the header's) leave at once instead of computing the rescale factors too
#ifndef MPPI_COMB_EXIT
#define MPPI_COMB_EXIT 0
#endif

namespace {

// ------------------------------------------------------------------- Philox
// a ^ b ^ k in one VALU op: gfx950's v_bitop3_b32 with truth table 0x96 (three-input
// XOR).  The compiler emits two v_xor_b32 for it (there is no v_xor3 on gfx950).
__device__ __forceinline__ uint32_t xor3_sk(uint32_t a, uint32_t b, uint32_t k) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "s"(k));
    return r;
}

__device__ __forceinline__ void philox10(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3,
                                         uint32_t k0, uint32_t k1) {
    k0 = __builtin_amdgcn_readfirstlane(k0);   // the key is wave-uniform: keep it scalar
    k1 = __builtin_amdgcn_readfirstlane(k1);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) {   // key schedule in place (opaque scalar adds): hoisting 18 round keys
                   // would spill SGPRs in the rollout kernel
            asm volatile("s_add_u32 %0, %0, 0x9e3779b9" : "+s"(k0) :: "scc");
            asm volatile("s_add_u32 %0, %0, 0xbb67ae85" : "+s"(k1) :: "scc");
        }
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0;   // one v_mad_u64_u32 each
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t n0 = xor3_sk((uint32_t)(p1 >> 32), c1, k0), n2 = xor3_sk((uint32_t)(p0 >> 32), c3, k1);
        c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
    }
}

// s_setprio takes an immediate: min(r, 3) for a wave-uniform r
__device__ __forceinline__ void set_wave_prio(int r) {
    if (r >= 3) __builtin_amdgcn_s_setprio(3);
    else if (r == 2) __builtin_amdgcn_s_setprio(2);
    else if (r == 1) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
}

__device__ __forceinline__ float uniform_f32(float x) {   // wave-uniform value kept in an SGPR
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x)));
}

// One standard-normal pair per 32-bit Philox word (Box-Muller on the hardware
// transcendental units: v_log_f32 (log2), v_sqrt_f32, v_sin_f32 / v_cos_f32 with the
// argument in revolutions).  The radius takes the top 18 bits, u1 = (w>>14 + 1/2) 2^-18,
// the angle the low 14, u2 = ((w & 0x3fff) + 1/2) 2^-14 (midpoint grids: the radial CDF
// is off by <= 2^-19, the angle's midpoint rule by O(2^-28); the tail is cut at 5.1
// sigma, mass 3e-7).  One Philox4x32-10 call thus yields 8 normals: the 7 arm dims take
// one call and the 10 whole-body dims two (two words per pair took 2 and 3).
__device__ __forceinline__ void box_muller32(uint32_t w, float& z0, float& z1) {
    if (MPPI_KO & 32) { z0 = __uint_as_float((w & 0x3FFFFFu) | 0x3F800000u); z1 = z0 - 1.5f; return; }
    const float u1 = ((float)(w >> 14) + 0.5f) * 3.814697265625e-6f;      // 2^-18
    const float u2 = ((float)(w & 0x3FFFu) + 0.5f) * 6.103515625e-5f;     // 2^-14
    // -2 ln u1 lies in [1.3e-6, 26.3] (u1 >= 2^-19): the bare v_sqrt_f32 (1 ulp) needs none
    // of the denormal scaling and correction steps __builtin_sqrtf adds (~12 VALU)
    const float r = __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u1));
    z0 = r * __builtin_amdgcn_cosf(u2);
    z1 = r * __builtin_amdgcn_sinf(u2);
}

// Philox2x32-10 (Salmon et al., SC'11; Random123's philox2x32): one 32x32 -> 64 multiply
// per round instead of two, for the draws that need at most 2 words.
__device__ __forceinline__ void philox2x10(uint32_t& c0, uint32_t& c1, uint32_t k) {
    k = __builtin_amdgcn_readfirstlane(k);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) asm volatile("s_add_u32 %0, %0, 0x9e3779b9" : "+s"(k) :: "scc");
        const uint64_t p = (uint64_t)0xD256D193u * c0;   // one v_mad_u64_u32
        const uint32_t n0 = xor3_sk((uint32_t)(p >> 32), c1, k);
        c1 = (uint32_t)p;
        c0 = n0;
    }
}

// The key of the Philox2x32 draws: the 64-bit seed folded to 32 bits, plus the control
// step times the golden ratio (a bijection of the step for a fixed seed).
__host__ __device__ __forceinline__ uint32_t philox2_key(uint32_t seed_lo, uint32_t seed_hi, uint32_t step) {
    return (seed_lo ^ (seed_hi * 0x85EBCA6Bu)) + step * 0x9E3779B9u;
}
// Its second counter word: (veh<<8 | t) ^ (step<<16) (t < 256 = MPPI_MAX_HORIZON).  The step
// in the counter as well as in the key: two seeds whose folded 32-bit keys meet at some pair
// of steps still draw different words unless the steps are equal too.  The uniform part
// (veh<<8 ^ step<<16) is one scalar value, so the lane pays one OR, as before.
__host__ __device__ __forceinline__ uint32_t philox2_ctr1(uint32_t veh, uint32_t t, uint32_t step) {
    return t | ((veh << 8) ^ (step << 16));
}

// Standard normals z[a], a < NA, of sample kg at step t (noise):
//   * normals 8j .. 8j+7 (j < NA/8): Philox4x32-10 call j, counter (kg, t, veh<<8 | j, step),
//     key (seed lo, seed hi); word i gives the pair (8j+2i, 8j+2i+1);
//   * the r = NA mod 8 left over: r <= 4 -> one Philox2x32-10 call, counter
//     (kg, philox2_ctr1(veh, t, step)), key philox2_key(seed, step), its words giving pairs 8J.., 8J+2..
//     (J = NA/8); r >= 5 -> Philox4x32-10 call J as above.
// (the whole-body's 10 dims: one 4x32 call + one 2x32 call, 30 multiplies instead of 40)
// The draw in two halves (the rollout overlaps them with LDS latency, k_rollout): the
// Philox words of one (k, t) -- word 4j + i of call j, then the Philox2x32 words -- and the
// normals Box-Muller makes of them.
template <int NA>
constexpr int draw_words() {
    return 4 * (NA / 8 + ((NA % 8) >= 5 ? 1 : 0)) + (((NA % 8) >= 1 && (NA % 8) <= 4) ? 2 : 0);
}
template <int NA>
__device__ __forceinline__ void draw_philox(uint32_t (&w)[draw_words<NA>()], uint32_t kg, uint32_t t, uint32_t veh,
                                            uint32_t step, uint32_t s0, uint32_t s1) {
    constexpr int J = NA / 8, REM = NA % 8;
    constexpr int N4 = J + (REM >= 5 ? 1 : 0);   // Philox4x32 calls
#pragma unroll
    for (int j = 0; j < N4; ++j) {
        w[4 * j] = kg; w[4 * j + 1] = t; w[4 * j + 2] = (veh << 8) | (uint32_t)j; w[4 * j + 3] = step;
        if (!(MPPI_KO & 2)) philox10(w[4 * j], w[4 * j + 1], w[4 * j + 2], w[4 * j + 3], s0, s1);
    }
    if constexpr (REM >= 1 && REM <= 4) {
        w[4 * N4] = kg; w[4 * N4 + 1] = philox2_ctr1(veh, t, step);
        if (!(MPPI_KO & 2)) philox2x10(w[4 * N4], w[4 * N4 + 1], philox2_key(s0, s1, step));
    }
}
template <int NA>
__device__ __forceinline__ void draw_box_muller(const uint32_t (&w)[draw_words<NA>()], float (&z)[NA]) {
#pragma unroll
    for (int i = 0; 2 * i < NA; ++i) {   // word i gives normals 2i, 2i + 1 (both layouts above)
        float a, b;
        box_muller32(w[i], a, b);
        z[2 * i] = a;
        if (2 * i + 1 < NA) z[2 * i + 1] = b;
    }
}
template <int NA>
__device__ __forceinline__ void draw_normals(float (&z)[NA], uint32_t kg, uint32_t t, uint32_t veh,
                                             uint32_t step, uint32_t s0, uint32_t s1) {
    uint32_t w[draw_words<NA>()];
    draw_philox<NA>(w, kg, t, veh, step, s0, s1);
    draw_box_muller<NA>(w, z);
}

// Philox words one (k, t) draw consumes (the raw layout of k_philox / oracle.philox_normals)
__host__ __device__ constexpr int philox_words(int NA) {
    return 4 * (NA / 8) + ((NA % 8) == 0 ? 0 : (NA % 8) <= 4 ? 2 : 4);
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

// sin/cos of a joint angle.  The reference evaluates them in the state dtype
// (fp32, or fp64 when update_joint got float64 arrays, mppi.py:197) and rounds
// into the fp32 transform (transformation_matrix.py:68-93).  Cody-Waite
// reduction by pi/2 in fp64 (exact for |q| << 2^20), then minimax polynomials
// in fp32 on [-pi/4, pi/4] (Cephes sinf/cosf): ~25 VALU ops, <= 2 ulp, no
// large-argument path (ocml sincosf is ~130 ops with a Payne-Hanek branch).
__device__ __forceinline__ void sincos_poly(float x, int qd, float& s, float& c) {
    const float x2 = x * x;
    float sp = fmaf(x2, -1.9515295891e-4f, 8.3321608736e-3f);
    sp = fmaf(x2, sp, -1.6666654611e-1f);
    const float sn = fmaf(x * x2, sp, x);
    float cp = fmaf(x2, 2.443315711809948e-5f, -1.388731625493765e-3f);
    cp = fmaf(x2, cp, 4.166664568298827e-2f);
    const float cs = fmaf(x2 * x2, cp, fmaf(-0.5f, x2, 1.0f));
    qd &= 3;
    s = (qd & 1) ? cs : sn;
    c = (qd & 1) ? sn : cs;
    if (qd & 2) s = -s;
    if ((qd + 1) & 2) c = -c;
}

// Default: reduce the angle to f in [-1/2, 1/2] revolutions in the angle's own precision,
// then the hardware v_sin_f32 / v_cos_f32 of 2 pi f (2 transcendentals + 4 ops instead of
// ~20).  Measured on MI355X over random angles in [-3 pi, 3 pi]
// (tools/microbench7.hip, profiles/r01/sincos_accuracy.txt): max error 1.8e-7 (fp64
// angle) and 2.6e-7 (fp32 angle) absolute, vs 9e-8 for the polynomials -- 1e2 below the
// trajectory tolerances.  MPPI_SINCOS_POLY=1 selects the polynomials.
#ifndef MPPI_SINCOS_POLY
#define MPPI_SINCOS_POLY 0
#endif
__device__ __forceinline__ void sincos_joint(double q, float& s, float& c) {
    if (MPPI_SINCOS_POLY) {
        const double n = rint(q * 0.63661977236758134308);
        double r = fma(-n, 1.5707963267948966192, q);
        r = fma(-n, 6.123233995736766036e-17, r);
        sincos_poly((float)r, (int)n, s, c);
        return;
    }
    const double r = q * 0.15915494309189533577;
    const float f = (float)(r - rint(r));
    s = __builtin_amdgcn_sinf(f);
    c = __builtin_amdgcn_cosf(f);
}

// fp32 state (torch.sin of a float32 tensor): 1/2pi = C_HI + C_LO, the fractional
// revolution by two FMAs (the polynomial path: a two-constant Cody-Waite reduction by
// pi/2, the dropped tail 1.8e-15 * n).
__device__ __forceinline__ void sincos_joint(float q, float& s, float& c) {
    if (MPPI_SINCOS_POLY) {
        const float n = __builtin_rintf(q * 0.636619772367581343f);
        float r = fmaf(-n, 1.5707963705062866f, q);
        r = fmaf(-n, -4.371138828673793e-08f, r);
        sincos_poly(r, (int)n, s, c);
        return;
    }
    const float n = __builtin_rintf(q * 0.15915494309189535f);
    float f = fmaf(q, 0.15915494309189535f, -n);
    f = fmaf(q, 6.4206382e-09f, f);
    s = __builtin_amdgcn_sinf(f);
    c = __builtin_amdgcn_cosf(f);
}

// One Kinova joint: T <- T * [P | o] * Rz(q), P a signed permutation fixed at
// compile time (kKinova, mppi_dev.h): the rotation part is register renaming and
// negation (source modifiers), the translation only its nonzero components.
template <int J, typename QT>
__device__ __forceinline__ void kin_joint(Mat34& T, const float* O, QT q) {
    constexpr KinOrigin k = kKinova[J];
    Mat34 r;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        float tr = T.m[4 * i + 3];
        if (k.tmask & 1) tr = fmaf(T.m[4 * i + 0], O[3], tr);
        if (k.tmask & 2) tr = fmaf(T.m[4 * i + 1], O[7], tr);
        if (k.tmask & 4) tr = fmaf(T.m[4 * i + 2], O[11], tr);
#pragma unroll
        for (int j = 0; j < 3; ++j) r.m[4 * i + j] = (k.s[j] > 0) ? T.m[4 * i + k.p[j]] : -T.m[4 * i + k.p[j]];
        r.m[4 * i + 3] = tr;
    }
    float s, c;
    sincos_joint(q, s, c);
    // Rodrigues about z (transformation_matrix.py:68-93).  Its R22 = fl(c + fl(1 - c)) is
    // 1 or 1 - 2^-24 (a rounding tie of 1 - c for some c < -1/2); the fast path takes 1,
    // as it takes the origins' pi/2 rotations exactly (<= 6e-8 relative).
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float a0 = r.m[4 * i], a1 = r.m[4 * i + 1];
        T.m[4 * i] = a0 * c + a1 * s;
        T.m[4 * i + 1] = a1 * c - a0 * s;
        T.m[4 * i + 2] = r.m[4 * i + 2];   // R22 = fl(c + fl(1 - c)) taken as 1
        T.m[4 * i + 3] = r.m[4 * i + 3];
    }
}

// atan2 with octant reduction and a degree-8 odd minimax polynomial on [0,1]
// (SLEEF atanf coefficients): ~25 ops, <= 3.5 ulp (ocml atan2f: 45 ops).
__device__ __forceinline__ float atan2_fast(float y, float x) {
    const float ax = fabsf(x), ay = fabsf(y);
    const float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
    float rc = __builtin_amdgcn_rcpf(mx);
    rc = rc * fmaf(-mx, rc, 2.0f);
    const float a = (mx > 0.0f) ? mn * rc : 0.0f;
    const float t = a * a;
    float u = 0.00282363896258175373077393f;
    u = fmaf(u, t, -0.0159569028764963150024414f);
    u = fmaf(u, t, 0.0425049886107444763183594f);
    u = fmaf(u, t, -0.0748900920152664184570312f);
    u = fmaf(u, t, 0.106347933411598205566406f);
    u = fmaf(u, t, -0.142027363181114196777344f);
    u = fmaf(u, t, 0.199926957488059997558594f);
    u = fmaf(u, t, -0.333331018686294555664062f);
    float r = fmaf(a * t, u, a);
    if (ay > ax) r = 1.57079632679489661923f - r;
    if (__builtin_signbit(x)) r = 3.14159265358979323846f - r;
    return __builtin_copysignf(r, y);
}

// Pose cost of one (k,t): w_pos*||p - p*|| + w_ori*||eulerZYX(R^T R*)||
// (pose_cost.py:24-63; rotation_conversions.py:277-319; inv(R) of the
// orthonormal FK rotation taken as R^T).
__device__ __forceinline__ float pose_cost(const Mat34& T, const VehicleConst& vc, float wp, float wo) {
    const float dx = T.m[3] - vc.tpos[0], dy = T.m[7] - vc.tpos[1], dz = T.m[11] - vc.tpos[2];
    const float cp = __builtin_amdgcn_sqrtf(dx * dx + dy * dy + dz * dz);
    const float* tR = vc.tR;
    const float r00 = T.m[0] * tR[0] + T.m[4] * tR[3] + T.m[8] * tR[6];
    const float r10 = T.m[1] * tR[0] + T.m[5] * tR[3] + T.m[9] * tR[6];
    const float r20 = T.m[2] * tR[0] + T.m[6] * tR[3] + T.m[10] * tR[6];
    const float r21 = T.m[2] * tR[1] + T.m[6] * tR[4] + T.m[10] * tR[7];
    const float r22 = T.m[2] * tR[2] + T.m[6] * tR[5] + T.m[10] * tR[8];
    const float yaw = atan2_fast(r10, r00);
    const float pitch = asinf(fminf(fmaxf(-r20, -1.0f), 1.0f));
    const float roll = atan2_fast(r21, r22);
    const float co = __builtin_amdgcn_sqrtf(yaw * yaw + pitch * pitch + roll * roll);
    return wp * cp + wo * co;
}

}  // namespace

// =============================================================================
// k_rollout
// =============================================================================
// Diagnostic phase stamps (build with -DMPPI_STAMPS; see tools/stamps.md):
// s_memtime per wave between scheduling barriers.  Compiled out otherwise.
#if defined(MPPI_STAMPS) && !defined(MPPI_TIMELINE)
#define STAMP(i)                                                                                      \
    do {                                                                                              \
        __builtin_amdgcn_sched_barrier(0);                                                            \
        if (pk.stamps && lane == 0) {                                                                 \
            const size_t w_ = ((size_t)blockIdx.y * p.nb + blockIdx.x) * nw + wid;        \
            pk.stamps[w_ * kStamps + (i)] = __builtin_amdgcn_s_memtime();                             \
        }                                                                                             \
        __builtin_amdgcn_sched_barrier(0);                                                            \
    } while (0)
// STAMPW first drains this wave's outstanding memory operations, so the stamp
// after a load phase measures its latency (diagnostic builds perturb overlap).
#define STAMPW(i)                                                                  \
    do {                                                                           \
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                \
        STAMP(i);                                                                  \
    } while (0)
// STAMPRT: the 100 MHz real-time counter (s_memrealtime), slots 13/14 = wave start/end:
// wall-clock wave lifetimes, the shader clock (memtime / realtime) and the grid's timeline
#define STAMPRT(i)                                                                                    \
    do {                                                                                              \
        __builtin_amdgcn_sched_barrier(0);                                                            \
        if (pk.stamps && lane == 0) {                                                                 \
            const size_t w_ = ((size_t)blockIdx.y * p.nb + blockIdx.x) * nw + wid;        \
            pk.stamps[w_ * kStamps + (i)] = __builtin_amdgcn_s_memrealtime();                         \
            if ((i) == 13) /* where the wave ran: XCC_ID (hwreg 20) << 32 | HW_ID (hwreg 4) */        \
                pk.stamps[w_ * kStamps + 15] = ((unsigned long long)__builtin_amdgcn_s_getreg(0xF814) << 32) | \
                                               (unsigned)__builtin_amdgcn_s_getreg(0xF804);           \
        }                                                                                             \
        __builtin_amdgcn_sched_barrier(0);                                                            \
    } while (0)
#elif defined(MPPI_STAMPS)   // MPPI_TIMELINE: wall-clock time at wave start / end and at three phase
                             // boundaries (after the first group's Philox: slot 10, after the
                             // prologue's barrier: slot 1, after the rollout groups: slot 5), no
                             // waits: the kernel's own schedule; -DMPPI_TIMELINE_FINE=1 stamps every
                             // phase boundary (tools/probes.py timeline prints the per-phase medians)
#ifndef MPPI_TIMELINE_FINE
#define MPPI_TIMELINE_FINE 0
#endif
#define STAMP(i)                                                                                      \
    do {                                                                                              \
        if (((i) == 1 || (i) == 5 || (i) == 10 || MPPI_TIMELINE_FINE) && pk.stamps && lane == 0) {    \
            const size_t w_ = ((size_t)blockIdx.y * p.nb + blockIdx.x) * nw + wid;        \
            pk.stamps[w_ * kStamps + (i)] = __builtin_amdgcn_s_memrealtime();                         \
        }                                                                                             \
    } while (0)
#define STAMPW(i) STAMP(i)
#define STAMPRT(i)                                                                                    \
    do {                                                                                              \
        if (pk.stamps && lane == 0) {                                                                 \
            const size_t w_ = ((size_t)blockIdx.y * p.nb + blockIdx.x) * nw + wid;        \
            pk.stamps[w_ * kStamps + (i)] = __builtin_amdgcn_s_memrealtime();                         \
            if ((i) == 13)                                                                            \
                pk.stamps[w_ * kStamps + 15] = ((unsigned long long)__builtin_amdgcn_s_getreg(0xF814) << 32) | \
                                               (unsigned)__builtin_amdgcn_s_getreg(0xF804);           \
        }                                                                                             \
    } while (0)
#else
#define STAMP(i) do { } while (0)
#define STAMPW(i) do { } while (0)
#define STAMPRT(i) do { } while (0)
#endif

// Static instruction-mix sections (diagnostic builds, -DMPPI_SECTIONS; tools/isa_sections.py):
// a named comment in the listing with scheduling barriers on both sides, so no instruction moves
// across it.  Compiled out otherwise.
#ifdef MPPI_SECTIONS
#define SECTION(name)                                        \
    do {                                                     \
        __builtin_amdgcn_sched_barrier(0);                   \
        asm volatile("; MPPI_SECTION " name ::: "memory");   \
        __builtin_amdgcn_sched_barrier(0);                   \
    } while (0)
#else
#define SECTION(name) do { } while (0)
#endif

// Inclusive fp32 segment sum (cost reduction; order-insensitive at tolerance).
template <int L>
__device__ __forceinline__ float seg_scan_f32(float x) {
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x111, 0xF, 0xF, true));
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x112, 0xF, 0xF, true));
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x114, 0xF, 0xF, true));
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x118, 0xF, 0xF, true));
    if (L >= 32) x += dpp_f32<0x142, 0xA>(x);
    if (L >= 64) x += dpp_f32<0x143, 0xC>(x);
    return x;
}


// Trajectory stores (every wave store instruction writes 256 contiguous bytes).  The
// planes of one vehicle are one buffer resource (C*K*H*4 < 4 GiB, checked at create):
// the lane's byte offset sits in one VGPR and the plane offset in an SGPR, so a store
// costs no 64-bit address arithmetic (a v_lshl_add_u64 per store with flat addresses).
// MPPI_TRAJ_AUX is the stores' cache-policy field: sc1 (device scope: written through
// the XCD's L2) | nt (streaming).  With plain stores (0) the L2s hold up to 8 x 4 MB of
// dirty trajectory lines when the waves finish, and the kernel-end release writes them
// back serially: same-box A/B (profiles/r02/ab_store_policy.txt) whole-body K=8192 H=64
// rollout 16.4 -> 12.8 us, arm C3 7.1 -> 6.0 us, V=8 fleet 93.7 -> 81.2 us.
#ifndef MPPI_TRAJ_AUX
#define MPPI_TRAJ_AUX 18
#endif
__device__ __forceinline__ __amdgpu_buffer_rsrc_t traj_rsrc(float* planes_v, uint32_t plane_b, int C) {
    return __builtin_amdgcn_make_buffer_rsrc(planes_v, 0, (int)(plane_b * (uint32_t)C), 0x00020000);
}
__device__ __forceinline__ void traj_store(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff, float x) {
    if (MPPI_KO & 16) return;
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(x), rs, (int)voff, (int)soff, MPPI_TRAJ_AUX);
}
// Write-through stores for the record bodies the finalize reads (full 256 B t-runs): a raw
// buffer over a wave-uniform base, byte offsets < 4 GiB.  NOT for S: its one-lane 4 B
// stores become partial-line writes through to memory (whole-body K=8192 rollout
// 13.7 -> 19.0 us, profiles/r02/ab_store_policy.txt); in L2 they merge into full lines.
// Record bodies: sc1 (written through) without nt, so the lines stay allocated on their way
// to memory and the finalize's loads (other XCDs) come back sooner.  Order-balanced A/B vs
// sc1|nt (profiles/r02/ab_record_store_policy.txt): step pair arm C3 10.40 -> 10.08 us,
// whole-body K=8192 19.66 -> 18.96 us, quadrotor 12.25 -> 11.99 us.
#ifndef MPPI_REC_AUX
#define MPPI_REC_AUX 16
#endif
__device__ __forceinline__ void wt_store(float* base_uniform, uint32_t byte_off, float x) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base_uniform, 0, (int)0xFFFFFFFFu, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(x), rs, (int)byte_off, 0, MPPI_REC_AUX);
}
// the record header (rho, eta, eta2, nan) of one block, written through like the bodies
__device__ __forceinline__ void wt_store4(float* base_uniform, uint32_t byte_off, float4 x) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base_uniform, 0, (int)0xFFFFFFFFu, 0x00020000);
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = {__float_as_uint(x.x), __float_as_uint(x.y), __float_as_uint(x.z), __float_as_uint(x.w)};
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)byte_off, 0, MPPI_REC_AUX);
}
// The rollout's outputs the finalize reads (record bodies and headers, and the vehicle
// constants block 0 hands over) are written through at device scope; every wave waits for its
// stores before it ends.  So they are visible device-wide when the kernel completes, and the
// native dispatch's rollout packet needs no release fence (the end-of-kernel L2 writeback,
// ~0.8 us per step at C3; mppi_aql.cpp).
__device__ __forceinline__ void drain_stores() {
    if (!(MPPI_KO & 512)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// fp32 inclusive scans of NA independent dims inside L-lane segments, step-major
// (the DPP wait states of one dim are filled by the others).  Each step is one
// v_add_f32_dpp: x + dpp(x), where out-of-row sources read 0 (row_shr with
// bound_ctrl) or rows outside row_mask add 0 (row_bcast), so no zeroing moves.
template <int L, int NA>
__device__ __forceinline__ void seg_scan_f32_multi(float (&x)[NA]) {
    if (MPPI_KO & 1) return;
#define MPPI_SCAN_STEP(CTRL, RM, BC)                                                    \
    _Pragma("unroll") for (int a = 0; a < NA; ++a) x[a] += __int_as_float(             \
        __builtin_amdgcn_update_dpp(0, __float_as_int(x[a]), CTRL, RM, 0xF, BC));
    MPPI_SCAN_STEP(0x111, 0xF, true)
    MPPI_SCAN_STEP(0x112, 0xF, true)
    MPPI_SCAN_STEP(0x114, 0xF, true)
    MPPI_SCAN_STEP(0x118, 0xF, true)
#undef MPPI_SCAN_STEP
    // row_bcast steps as in-place v_add_f32_dpp: rows outside row_mask keep x (the
    // compiler's DPP combiner would zero a temporary and add instead).  s_nop 1 covers
    // the VALU-write -> DPP-read hazard the asm hides from the hazard recognizer.
    if (L >= 32) {
#pragma unroll
        for (int a = 0; a < NA; ++a)
            asm volatile("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf" : "+v"(x[a]));
    }
    if (L >= 64) {
#pragma unroll
        for (int a = 0; a < NA; ++a)
            asm volatile("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf" : "+v"(x[a]));
    }
}

// Value of segment s's lane l, as a wave-uniform (scalar) quantity.
template <int R>
__device__ __forceinline__ float seg_pick(float x, int sub, int l_in_seg, int L) {
    float r = read_lane_f32(x, l_in_seg);
#pragma unroll
    for (int s = 1; s < R; ++s) r = (sub == s) ? read_lane_f32(x, s * L + l_in_seg) : r;
    return r;
}

// ---------------------------------------------------------------------------
// Integrator in the transposed domain (NCH == 1).  The two cumsums of
// standard_normal_noise.py:41-48 as DPP scans cost 13 DPP ops per dim and lane
// (row_shr 1/2/4/8, row_bcast 15/31, wave_shr 1).  Instead the wave writes its
// controls to its LDS slot (row = lane = (segment, t), pitch P = NA rounded up to odd,
// so the transposed reads are bank-conflict free) and re-reads them with lane =
// (series = (segment, dim), chunk of CL consecutive t).  Each lane integrates its chunk
// sequentially (4 full-rate ops per element), the chunks of a series combine by an
// affine exclusive scan over CPS consecutive lanes (2 log2 CPS + 2 DPP moves), and the
// position increments go back through LDS to lane = t.  For a chunk starting at
// velocity V and position P (relative to q0, q0dot), element i:
//   dq(i) = P + lp(i) + (i + 1) dt V,   lp(i) = sum_{j <= i} (lv(j) dt + a_j dt^2 / 2),
//   lv(j) = sum_{m < j} a_m dt;   combine(L then R) : V = V_L + V_R,
//   P = P_L + P_R + n_R dt V_L  (n_R elements in R).
// q0dot enters as (t + 1) dt q0dot.  fp32 throughout (the old scans were fp32 too); the
// increments stay ~1e-10 from the reference's double-accumulated cumsums.
template <int L, int NA>
struct IntegGeom {
    static constexpr int R = 64 / L;
    static constexpr int S = R * NA;   // series per wave
    static constexpr int CPS = (S <= 4) ? 16 : (S <= 8) ? 8 : (S <= 16) ? 4 : (S <= 32) ? 2 : 1;
    static constexpr int CL = L / CPS;   // elements per chunk
    static constexpr int P = NA | 1;     // LDS row pitch (odd)
    static_assert(S * CPS <= 64 && CPS <= L, "integrator lane map");
};

// floats per wave slot in LDS: the block-combine deposit (4 + NCH*64*NA) and, for
// NCH == 1, the integrator's 64 x P transposition buffer
template <int NA, int NCH, int L>
constexpr int wave_slot_floats() {
    return (NCH == 1 && 64 * IntegGeom<L, NA>::P > 4 + NCH * 64 * NA) ? 64 * IntegGeom<L, NA>::P
                                                                     : 4 + NCH * 64 * NA;
}

template <int CTRL>
__device__ __forceinline__ float row_shr_f32(float x) {   // out-of-row sources read 0
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, true));
}

// inc[a] (lane = segment*L + t) = q(t) - q0 for the controls act[a] of this lane
template <int L, int NA>
__device__ __forceinline__ void integrate_lds(const float (&act)[NA], float* xw, const int lane, const float dt,
                                              const float dt2h, const float* vel0f, float (&inc)[NA]) {
    using G = IntegGeom<L, NA>;
    constexpr int P = G::P, CPS = G::CPS, CL = G::CL, S = G::S;
#pragma unroll
    for (int a = 0; a < NA; ++a) xw[lane * P + a] = act[a];
    wave_lds_handoff();
    const int sr = lane / CPS, ch = lane & (CPS - 1);
    const bool on = sr < S;
    const int seg = sr / NA, a = sr - seg * NA;
    const int rb = on ? (seg * L + ch * CL) * P + a : 0;
    float lv = 0.0f, lp = 0.0f, loc[CL];
#pragma unroll
    for (int i = 0; i < CL; ++i) {
        const float x = xw[rb + i * P];
        lp += fmaf(lv, dt, x * dt2h);
        lv = fmaf(x, dt, lv);
        loc[i] = lp;
    }
    // inclusive affine scan over the series' chunks (consecutive lanes of one DPP row)
    float V = lv, Q = lp;
#define MPPI_ISCAN(D, CTRL)                                                                if (CPS > D) {                                                                             const float vs = row_shr_f32<CTRL>(V), qs = row_shr_f32<CTRL>(Q);                       if (ch >= D) { Q = Q + fmaf((float)(D * CL) * dt, vs, qs); V = V + vs; }            }
    MPPI_ISCAN(1, 0x111)
    MPPI_ISCAN(2, 0x112)
    MPPI_ISCAN(4, 0x114)
    MPPI_ISCAN(8, 0x118)
#undef MPPI_ISCAN
    float Vx = row_shr_f32<0x111>(V), Qx = row_shr_f32<0x111>(Q);   // exclusive: previous chunk's
    if (ch == 0) { Vx = 0.0f; Qx = 0.0f; }
    const float v0 = on ? vel0f[a] : 0.0f;
    const float q0 = fmaf((float)(ch * CL) * dt, v0, Qx);   // chunk start incl. the q0dot drift
    const float vb = dt * (Vx + v0);
    wave_lds_handoff();
    if (on) {
#pragma unroll
        for (int i = 0; i < CL; ++i) xw[rb + i * P] = fmaf((float)(i + 1), vb, q0 + loc[i]);
    }
    wave_lds_handoff();
#pragma unroll
    for (int a2 = 0; a2 < NA; ++a2) inc[a2] = xw[lane * P + a2];
}

// The leading scalar arguments are preloaded into SGPRs at wave launch on gfx950
// (-mllvm -amdgpu-kernarg-preload-count, build.py): the first group's Philox
// draw and the u_prev / joint-table loads start without waiting for the
// kernel-argument segment (its first s_load costs ~1.5k cycles).
// ONEG: every wave runs exactly one rollout group (iters == 1).  Straight-line code with
// no loop-carried softmin state: the common whole-body kernel fits in 52 VGPRs, so it is
// budgeted for 8 waves per SIMD (the looping variant needs 87: 5 waves; the fp64-state
// arm kernel would spill at 64 and keeps the 4-wave budget -- C3 runs 2 waves per SIMD).  At the C4 shard
// (whole-body K=8192 H=64) that is 1024 blocks x 8 waves, all resident at once: twice the
// latency hiding of 512 blocks x 2 groups, and no wave left alone in the grid's tail.
template <int MODEL, int NA, int NCH, int LSEG, bool F64, bool VONE, bool XC, bool ONEG>
__global__ void __launch_bounds__(512, (ONEG && !F64) ? 8 : (NCH >= 4 ? 2 : NCH == 2 ? (XC ? MPPI_ROLL_OCC_NCH2_XC : MPPI_ROLL_OCC_NCH2) : (XC ? MPPI_ROLL_OCC_XC : MPPI_ROLL_OCC))) k_rollout(const uint32_t seed_lo, const uint32_t seed_hi,
                                                 const uint32_t step_arg, const uint32_t k_off,
                                                 const int32_t noise_arg, const int32_t H_arg,
                                                 const int32_t geo_arg,
                                                 const float* __restrict__ u_prev,
                                                 const JointDev* __restrict__ jtab, const DevParams pk) {
    constexpr int R = 64 / LSEG;
    constexpr int QOFF = (MODEL == MPPI_MODEL_WHOLEBODY) ? 3 : 0;
    constexpr int NQ = (MODEL == MPPI_MODEL_DRONE) ? 0 : NA - QOFF;
    constexpr int kJW = (int)(sizeof(JointDev) * kMaxJ / 4);   // joint table, dwords
    extern __shared__ __attribute__((aligned(16))) float smem[];
    // Scalars and (V == 1) the vehicle constants are read from the kernel
    // arguments with scalar loads (SGPR operands, no LDS latency in the hot
    // phases); the joint table and (V > 1) the vehicle block go to LDS.
    __shared__ JointDev jnt[kMaxJ];
    __shared__ VehicleConst vcv;
    const DevParams& p = pk;
    const int v = blockIdx.y;
    // block size and groups per block as one preloaded argument (threads | iters << 16): blockDim
    // would be an implicit-argument s_load, p.iters a kernel-argument one
    const int nthr = geo_arg & 0xFFFF, iters = ONEG ? 1 : (geo_arg >> 16);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, nw = nthr >> 6;
    const int sub = lane / LSEG, t0 = lane & (LSEG - 1);
    const int32_t noise_mode = noise_arg & 0xFF;
    const uint32_t step_ctr = step_of(step_arg, noise_arg);   // (native dispatch: from the dispatch id)
    // the vehicle's Philox key: its index in the whole fleet (mppi_config.vehicle_offset rides in the
    // noise argument's high half), so a fleet split over engines draws what one engine would
    const uint32_t vkey = (uint32_t)v + ((uint32_t)noise_arg >> 16);
    STAMPRT(13);
    STAMP(0);
    // issue the global loads first (addresses need only preloaded scalars and the
    // kernarg pointer), keep the values in registers across the Philox draw
    float* u_lds = smem;
    const int HA = H_arg * NA;
    const float* usrc = u_prev + (size_t)v * HA;
    float ur[4];
    int jr[2];
    // an overlapped batch (kNoiseOverlap): u_prev is read only after the finalize before this
    // rollout has written it (the wait below, after the first group's normals)
    const bool ovl = (noise_arg & kNoiseOverlap) != 0;
    auto load_u = [&]() __attribute__((always_inline)) {
        // through a buffer resource over this vehicle's u_prev: 32-bit offsets, and the rows past
        // H*A read 0 from the range check (no per-load branch, no 64-bit address math)
        const __amdgpu_buffer_rsrc_t urs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float*>(usrc), 0, (MPPI_KO & 128) ? 0 : HA * 4, 0x00020000);
#pragma unroll
        for (int j = 0; j < 4; ++j)
            ur[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(urs, (tid + j * nthr) * 4, 0, kAuxDev));
    };
    if (!ovl) load_u();
    if (MODEL != MPPI_MODEL_DRONE) {
        const int* js = (const int*)jtab;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int i = tid + j * nthr;
            jr[j] = (i < kJW) ? js[i] : 0;
        }
    }
    // vehicle constants -> LDS (uniform reads in the FK / cost; keeping ~60 of them
    // in SGPRs spills): V == 1 from the kernel arguments, else from vc[v]
    constexpr int kVCW = (int)(sizeof(VehicleConst) / 4);
    const int vcr = (tid < kVCW) ? (VONE ? ((const int*)&pk.vc0)[tid] : ((const int*)(pk.vc + v))[tid]) : 0;
    // touch every kernel-argument line the hot phases read (one s_load per 64 B): they
    // land in the scalar cache while the first group's Philox draw runs below
    // (an integer fold: uniform, so SALU -- a float sum took one VALU op per line)
    uint32_t kwarm = 0u;
    {
        const uint32_t* kp = (const uint32_t*)&pk;
#pragma unroll
        for (int o = 0; o < (int)(offsetof(DevParams, sigma) / 4); o += 16) kwarm ^= kp[o];
    }
    STAMPW(9);
    // the first group's standard normals overlap the loads above
    float z0[NCH][NA];
    SECTION("prologue_philox");
    if (noise_mode != MPPI_NOISE_INJECTED) {
        const uint32_t kg = k_off + (uint32_t)((blockIdx.x * nw + wid) * R + sub);
#pragma unroll
        for (int c = 0; c < NCH; ++c)
            draw_normals<NA>(z0[c], kg, (uint32_t)(t0 + 64 * c), vkey, step_ctr, seed_lo, seed_hi);
    }
    if (ovl) {   // wave 0 waits until every finalize block of the previous step has counted it (its
                 // slice of u_prev written and drained), then the block goes on together
        if (wid == 0) {
            const uint32_t* fl = pk.ovl + (size_t)v * pk.ovl_n;
            const int nfl = pk.ovl_n;
            for (;;) {
                bool ok = true;
                for (int i = lane; i < nfl; i += 64) ok &= (int32_t)(ld_dev(fl + i) - step_ctr) >= 0;
                if (__builtin_amdgcn_ballot_w64(!ok) == 0ull) break;
                __builtin_amdgcn_s_sleep(1);
            }
        }
        lds_barrier();
        load_u();
    }
    SECTION("prologue_staging");
    STAMP(10);
    asm volatile("" :: "s"(kwarm));
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int i = tid + j * nthr;
        if (i < HA) u_lds[i] = ur[j];
    }
    for (int i = tid + 4 * nthr; i < HA; i += nthr) u_lds[i] = usrc[i];   // H*A > 2048
    if (MODEL != MPPI_MODEL_DRONE) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int i = tid + j * nthr;
            if (i < kJW) ((int*)jnt)[i] = jr[j];
        }
        for (int i = tid + 2 * nthr; i < kJW; i += nthr) ((int*)jnt)[i] = ((const int*)jtab)[i];
    }
    if (tid < kVCW) {
        ((int*)&vcv)[tid] = vcr;
        if (VONE && blockIdx.x == 0)   // hand vc0 to the finalize (written through), with this
                                       // step's Philox counter in a spare word (the peer exchange's tag)
            __hip_atomic_store((int*)pk.vc + tid, tid == kVcStepWord ? (int)step_ctr : vcr, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    for (int i = tid + nthr; i < kVCW; i += nthr) {   // nthr < 124
        const int x = VONE ? ((const int*)&pk.vc0)[i] : ((const int*)(pk.vc + v))[i];
        ((int*)&vcv)[i] = x;
        if (VONE && blockIdx.x == 0)
            __hip_atomic_store((int*)pk.vc + i, i == kVcStepWord ? (int)step_ctr : x, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    STAMPW(8);
    if (!(MPPI_KO & 256)) lds_barrier();
    const VehicleConst& vc = vcv;
    const float* sdiag = pk.sdiag;
    const int H = H_arg, K = pk.K;
    constexpr int kWs = wave_slot_floats<NA, NCH, LSEG>();
    float* const xw = smem + ((HA + 3) & ~3) + wid * kWs;   // this wave's LDS slot
    // the block's costs, nw * R consecutive k per group, staged in LDS for write-through store runs
    // after the combine barrier (st_dev_run)
    float* const s_stage = smem + ((HA + 3) & ~3) + 8 * kWs;
    STAMP(1);

    // trajectory planes of vehicle v (from kernel arguments and blockIdx only, so the
    // descriptor stays in SGPRs)
    // rows padded to 64 B (hp = H rounded up to 16) and written whole, pad lanes included: the
    // write-through stores then never leave a partial 64 B sector for HBM to merge
    const int hp = pk.hp;
    const uint32_t plane_b = (uint32_t)K * (uint32_t)hp * 4u;
    const __amdgpu_buffer_rsrc_t trs = traj_rsrc(pk.traj + (size_t)v * pk.C * K * hp, plane_b, pk.C);

    float acc[NCH][NA];
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
        for (int a = 0; a < NA; ++a) acc[c][a] = 0.0f;
    float rho_w = INFINITY, eta_w = 0.0f, eta2_w = 0.0f;   // wave-uniform
    bool nan_w = false;

    // One group of R rollouts per wave.  Written as a lambda so the common
    // single-group launch (iters == 1, e.g. K=4096 H=32) is straight-line code:
    // no loop-invariant hoisting of address math / key schedules into SGPRs.
    auto group = [&](const int it) __attribute__((always_inline)) {   // (the NCH = 4 extended kernel called it out of line: a 1.7 KB stack frame)
        asm volatile("" ::: "memory");   // keep LDS constant reads inside the group
        SECTION("noise");
        // group it of block b: groups b, b + nb, ...  All blocks' groups of one iteration are
        // consecutive, so the grid's concurrent trajectory stores stay in one region of the planes
        // (consecutive groups per block scattered them: whole-body K=65536 85.5 -> 106-110 us)
        const int g = blockIdx.x + it * p.nb;
        const int k = (g * nw + wid) * R + sub;
        const bool kval = k < K;
        const int kc = kval ? k : K - 1;   // clamped: every load stays in bounds
        const uint32_t kg = k_off + (uint32_t)k;

        // ---- A1/A2: eps = z Sigma (device Philox) or injected; act = u_prev + eps
        float eps[NCH][NA], act[NCH][NA];
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const int t = t0 + 64 * c;
            const bool val = kval && t < H;
            const int tc = (t < H) ? t : H - 1;
            if (noise_mode == MPPI_NOISE_INJECTED) {
                const float* src = p.noise_in + (((size_t)v * K + kc) * H + tc) * NA;
#pragma unroll
                for (int a = 0; a < NA; ++a) eps[c][a] = src[a];
            } else {
                float z[NA];
                if (it == 0) {
#pragma unroll
                    for (int a = 0; a < NA; ++a) z[a] = z0[c][a];
                } else {
                    draw_normals<NA>(z, kg, (uint32_t)t, vkey, step_ctr, seed_lo, seed_hi);
                }
                if (!XC || p.sigma_diag) {   // a full Sigma runs in the extended (XC) kernel
#pragma unroll
                    for (int a = 0; a < NA; ++a) eps[c][a] = z[a] * sdiag[a];
                } else {
#pragma unroll
                    for (int b = 0; b < NA; ++b) {
                        float e = 0.0f;
#pragma unroll
                        for (int a = 0; a < NA; ++a) e += z[a] * p.sigma[a * NA + b];
                        eps[c][b] = e;
                    }
                }
            }
            // the warm-start row first, unconditionally (tc is clamped): inside the select the
            // compiler turned every LDS read into its own exec-masked branch and s_waitcnt,
            // NA serial LDS round trips per lane
            float ur[NA];
#pragma unroll
            for (int a = 0; a < NA; ++a) ur[a] = u_lds[tc * NA + a];
#pragma unroll
            for (int a = 0; a < NA; ++a) {
                eps[c][a] = val ? eps[c][a] : 0.0f;
                act[c][a] = val ? ur[a] + eps[c][a] : 0.0f;
            }
            if (p.store_noise && val) {   // (readback only: written through, st_dev)
                float* dst = p.noise_out + (((size_t)v * K + k) * H + t) * NA;
#pragma unroll
                for (int a = 0; a < NA; ++a) st_dev(dst + a, eps[c][a]);
            }
        }
        // extra CostManager terms on the controls (cost_manager.py:83,86): covar
        // u_t^T Sigma^-1 v_t (covar_cost.py:20-25) and action w*gamma^t*||v_t||^2
        // (action_cost.py:14-24); per lane, summed over t with the costs below
        float ecov = 0.0f, eact = 0.0f, gts[NCH];
#pragma unroll
        for (int c = 0; c < NCH; ++c) gts[c] = 0.0f;
        if (XC && p.cost_terms) {   // (the XC kernel also runs a full Sigma without extra terms:
                                    //  gamma_t / sinv exist only with cost_terms)
#pragma unroll
            for (int c = 0; c < NCH; ++c) {
                const int t = t0 + 64 * c;
                const bool val = kval && t < H;
                const int tc = (t < H) ? t : H - 1;
                gts[c] = val ? p.gamma_t[tc] : 0.0f;
                if (p.cost_terms & MPPI_COST_COVAR) {
                    float qd = 0.0f;
#pragma unroll
                    for (int a = 0; a < NA; ++a) {
                        float y = 0.0f;
                        if (p.sigma_diag) {
                            y = p.sinv[a * NA + a] * act[c][a];
                        } else {
#pragma unroll
                            for (int b = 0; b < NA; ++b) y = fmaf(p.sinv[a * NA + b], act[c][b], y);
                        }
                        qd = fmaf(u_lds[tc * NA + a], y, qd);
                    }
                    ecov += val ? qd : 0.0f;
                }
                if (p.cost_terms & MPPI_COST_ACTION) {
                    float s2 = 0.0f;
#pragma unroll
                    for (int a = 0; a < NA; ++a) s2 = fmaf(act[c][a], act[c][a], s2);
                    eact += val ? (p.w_act * s2) * gts[c] : 0.0f;
                }
            }
        }
        if (it == 0) STAMP(2);
        SECTION("integrator");

        // ---- A3: double integrator (standard_normal_noise.py:41-48).  Both cumsums
        //      are fp32 Kogge-Stone scans over DPP: they sum small increments
        //      (a*dt, v*dt + a*dt^2/2), so their rounding stays ~1e-10 absolute, far
        //      below one ulp of the positions; q0 is added in the state
        //      dtype (fp64 state -> fp64 positions, as update_joint's float64 arrays).
        float posf[NCH][NA];
        double posd[NCH][F64 ? NA : 1];
        if constexpr (NCH == 1 && !(MPPI_KO & 1)) {
            float inc[NA];
            integrate_lds<LSEG, NA>(act[0], xw, lane, p.dt, 0.5f * p.dt2, vc.vel0f, inc);
#pragma unroll
            for (int a = 0; a < NA; ++a) {
                if (!F64) {
                    posf[0][a] = inc[a] + vc.pos0f[a];
                } else {
                    posd[0][a] = (double)inc[a] + vc.pos0[a];
                    posf[0][a] = (float)posd[0][a];
                }
            }
        } else {
#pragma clang fp contract(off)
            float carry1[NA], carry2[NA], lastv[NA];
#pragma unroll
            for (int a = 0; a < NA; ++a) { carry1[a] = 0.0f; carry2[a] = 0.0f; lastv[a] = 0.0f; }
#pragma unroll
            for (int c = 0; c < NCH; ++c) {
                float c1[NA], c2[NA];
#pragma unroll
                for (int a = 0; a < NA; ++a) c1[a] = act[c][a] * p.dt;
                seg_scan_f32_multi<LSEG, NA>(c1);
#pragma unroll
                for (int a = 0; a < NA; ++a) {
                    if (NCH > 1) {
                        c1[a] += carry1[a];
                        carry1[a] = read_lane_f32(c1[a], 63);
                    }
                    // (0.5 a) dt^2 == a (0.5 dt^2) bit for bit: both are one rounding of the
                    // same product, the halvings being exact
                    const float h2 = act[c][a] * (0.5f * p.dt2);
                    const float velf = c1[a] + vc.vel0f[a];
                    float prev = dpp_f32<0x138, 0xF>(velf);     // wave_shr:1
                    if (t0 == 0) prev = (c == 0) ? vc.vel0f[a] : lastv[a];
                    if (NCH > 1) lastv[a] = read_lane_f32(velf, 63);
                    c2[a] = prev * p.dt + h2;
                }
                seg_scan_f32_multi<LSEG, NA>(c2);
#pragma unroll
                for (int a = 0; a < NA; ++a) {
                    if (NCH > 1) {
                        c2[a] += carry2[a];
                        carry2[a] = read_lane_f32(c2[a], 63);
                    }
                    if (!F64) {
                        posf[c][a] = c2[a] + vc.pos0f[a];
                    } else {
                        posd[c][a] = (double)c2[a] + vc.pos0[a];
                        posf[c][a] = (float)posd[c][a];
                    }
                }
            }
        }
        if (it == 0) STAMP(3);
        SECTION("fk_chain");
        if (ONEG && MPPI_PRIO) set_wave_prio(2);   // progress priority (single group): see below

        // eps is read again only by the softmin accumulate at the end of the group: park
        // it in this wave's LDS slot (the integrator is done with it; each lane its own
        // row, so no hand-off) across the FK and cost, the kernel's register peak.  The
        // compiler barriers stop it from forwarding the stored values in registers.
        constexpr bool kStash = MPPI_EPS_STASH && NA >= 7 && (XC || NCH > 1);
        constexpr int kESP = (NCH == 1) ? IntegGeom<LSEG, NA>::P : NA;   // row pitch (odd for NCH == 1)
        if constexpr (kStash) {
#pragma unroll
            for (int c = 0; c < NCH; ++c)
#pragma unroll
                for (int a = 0; a < NA; ++a) xw[(c * 64 + lane) * kESP + a] = eps[c][a];
            asm volatile("" ::: "memory");
        }

        // ---- A4-A10: FK + per-step cost, trajectory planes
        float xs[NCH];
        float ecen = 0.0f, ejt = 0.0f, elim = 0.0f;
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const int t = t0 + 64 * c;
            const bool val = kval && t < H;
            const bool term = (t == H - 1);
            float x;
            const uint32_t toff = ((uint32_t)k * (uint32_t)hp + (uint32_t)t) * 4u;   // byte offset in a plane
            const bool stv = p.store_traj && kval && t < hp;   // row incl. its pad (finite values)
            if (MODEL == MPPI_MODEL_DRONE) {
                const float dx = posf[c][0] - vc.tpos[0], dy = posf[c][1] - vc.tpos[1],
                            dz = posf[c][2] - vc.tpos[2];
                x = dx * dx + dy * dy + dz * dz;
                if (stv) {
#pragma unroll
                    for (int a = 0; a < 3; ++a) traj_store(trs, toff, (uint32_t)a * plane_b, posf[c][a]);
                }
            } else {
                // joint angle j in the state dtype (fp64 state -> fp64 sin/cos reduction)
                auto qang = [&](int cc_, int j) {
                    if constexpr (F64) return posd[cc_][QOFF + j]; else return posf[cc_][QOFF + j];
                };
                if (stv) {   // positions first: each dies after its joint's FK step
#pragma unroll
                    for (int a = 0; a < NA; ++a) traj_store(trs, toff, (uint32_t)a * plane_b, posf[c][a]);
                }
                Mat34 T;   // base (times the folded leading fixed joints)
#pragma unroll
                for (int i = 0; i < 12; ++i) T.m[i] = vc.base[i];
                if (MODEL == MPPI_MODEL_WHOLEBODY) {   // [R(rpy) | p_drone(k,t)] * M_fixed
                    T.m[3] += posf[c][0]; T.m[7] += posf[c][1]; T.m[11] += posf[c][2];
                }
                if (MPPI_KO & 4) {
                    T.m[3] += posf[c][QOFF]; T.m[7] += posf[c][QOFF + 1];
                } else if (NQ == 7 && (!XC || p.chain_fast == 2)) {   // Kinova: origin rotations are signed
                    // permutations (the common kernel runs only this chain; any other goes to XC)
                    kin_joint<0>(T, jnt[p.j0 + 0].O, qang(c, 0));
                    kin_joint<1>(T, jnt[p.j0 + 1].O, qang(c, 1));
                    kin_joint<2>(T, jnt[p.j0 + 2].O, qang(c, 2));
                    kin_joint<3>(T, jnt[p.j0 + 3].O, qang(c, 3));
                    kin_joint<4>(T, jnt[p.j0 + 4].O, qang(c, 4));
                    kin_joint<5>(T, jnt[p.j0 + 5].O, qang(c, 5));
                    kin_joint<6>(T, jnt[p.j0 + 6].O, qang(c, 6));
                } else if (!XC) {   // (unreachable: the common kernel is dispatched for Kinova chains only)
                } else if (p.chain_fast) {   // nq revolute-z joints, q_index = 0..nq-1 in order
#pragma unroll
                    for (int j = 0; j < NQ; ++j) {
                        const JointDev& J = jnt[p.j0 + j];
                        mul_affine(T, J.O);
                        float s, cc;
                        sincos_joint(qang(c, j), s, cc);
                        const float omc = 1.0f - cc, r22 = cc + omc;
#pragma unroll
                        for (int i = 0; i < 3; ++i) {
                            const float a0 = T.m[4 * i], a1 = T.m[4 * i + 1];
                            T.m[4 * i] = a0 * cc + a1 * s;
                            T.m[4 * i + 1] = a1 * cc - a0 * s;
                            T.m[4 * i + 2] = T.m[4 * i + 2] * r22;
                        }
                    }
                } else {
                    for (int jn = p.j0; jn < p.nj; ++jn) {
                        const JointDev& J = jnt[jn];
                        mul_affine(T, J.O);
                        if (J.type == MPPI_JOINT_FIXED) continue;
                        double qd = 0.0;
                        float qf = 0.0f;
#pragma unroll
                        for (int a = 0; a < NQ; ++a)
                            if (a == J.q_index) {
                                qd = F64 ? posd[c][QOFF + a] : 0.0;
                                qf = posf[c][QOFF + a];
                            }
                        if (J.type == MPPI_JOINT_REVOLUTE) {
                            float s, cc;
                            if constexpr (F64) sincos_joint(qd, s, cc); else sincos_joint(qf, s, cc);
                            mul_revolute(T, J, cc, s);
                        } else {
                            mul_prismatic(T, J, qf);
                        }
                    }
                }
                // the four weights as SGPR values: selecting between two kernel-argument
                // addresses per lane would otherwise become two vector loads in the FK
                const float wsp = uniform_f32(p.w_sp), wso = uniform_f32(p.w_so), wtp = uniform_f32(p.w_tp),
                            wto = uniform_f32(p.w_to);
                SECTION("pose_cost");
                x = (MPPI_KO & 8) ? T.m[3] + T.m[7] + T.m[11] + T.m[0] : pose_cost(T, vc, term ? wtp : wsp, term ? wto : wso);
                SECTION("traj_ee_stores");
                if (stv) {
#pragma unroll
                    for (int i = 0; i < 12; ++i) traj_store(trs, toff, (uint32_t)(NA + i) * plane_b, T.m[i]);
                }
            }
            xs[c] = val ? x : 0.0f;
            // extra joint-space terms (cost_manager.py:84,85,87; joint_space_cost.py)
            if (XC && (p.cost_terms & (MPPI_COST_CENTER | MPPI_COST_JOINT_TRACK | MPPI_COST_JOINT_LIMIT))) {
                const int tc = (t < H) ? t : H - 1;
                const float* jt = p.jtraj ? p.jtraj + ((size_t)v * H + tc) * NQ : nullptr;
                float sc = 0.0f, sj = 0.0f;
                bool out = false;
#pragma unroll
                for (int j = 0; j < NQ; ++j) {
                    const float qj = posf[c][QOFF + j];
                    const float dc = qj - vc.qc[j];
                    sc = fmaf(dc, dc, sc);
                    const float dj = qj - (jt ? jt[j] : 0.0f);
                    sj = fmaf(dj, dj, sj);
                    const double qd = F64 ? posd[c][QOFF + j] : (double)qj;   // limits in the state dtype
                    out |= (qd < (double)vc.qlo[j]) | (qd > (double)vc.qhi[j]);
                }
                if (val) {
                    if (p.cost_terms & MPPI_COST_CENTER) ecen += (p.w_cen * sc) * gts[c];
                    if (p.cost_terms & MPPI_COST_JOINT_TRACK) ejt += (p.w_jt * sj) * gts[c];
                    if ((p.cost_terms & MPPI_COST_JOINT_LIMIT) && out) elim += p.lim_pen * gts[c];
                }
            }
        }
        if (it == 0) STAMP(4);
        SECTION("cost_sum_softmin");
        if (ONEG && MPPI_PRIO) set_wave_prio(1);

        // ---- S_k = fl(ws * sum_{t<H-1} x_t) + fl(wt * x_{H-1}) per segment (wave-uniform picks)
        float st = 0.0f;
#pragma unroll
        for (int c = 0; c < NCH; ++c) st += (t0 + 64 * c < H - 1) ? xs[c] : 0.0f;
        st = seg_scan_f32<LSEG>(st);
        float xt = 0.0f;
#pragma unroll
        for (int c = 0; c < NCH; ++c)
            if (c == (H - 1) / 64) xt = xs[c];
        float S_seg[R];
#pragma unroll
        for (int s = 0; s < R; ++s) {
            const int ks = (g * nw + wid) * R + s;
            const float stage = read_lane_f32(st, s * LSEG + LSEG - 1);
            const float term = read_lane_f32(xt, s * LSEG + ((H - 1) & 63));
            float S = (MODEL == MPPI_MODEL_DRONE) ? (p.w_sp * stage) + (p.w_tp * term) : stage + term;
            S_seg[s] = (ks < K) ? S : INFINITY;
        }
        if (XC) {   // S += covar, center, jtraj, action, limit
            float tsum[5] = {ecov, ecen, ejt, eact, elim};
            const int bits[5] = {MPPI_COST_COVAR, MPPI_COST_CENTER, MPPI_COST_JOINT_TRACK, MPPI_COST_ACTION,
                                 MPPI_COST_JOINT_LIMIT};
#pragma unroll
            for (int i = 0; i < 5; ++i) {
                if (!(p.cost_terms & bits[i])) continue;
                const float ts = seg_scan_f32<LSEG>(tsum[i]);
#pragma unroll
                for (int s = 0; s < R; ++s) {
                    float add = read_lane_f32(ts, s * LSEG + LSEG - 1);
                    if (i == 0) add = p.w_cov * add;
                    S_seg[s] += add;
                }
            }
        }
        float S_mine = S_seg[0];
#pragma unroll
        for (int s = 1; s < R; ++s) S_mine = (sub == s) ? S_seg[s] : S_mine;
        if (MPPI_S_PLAIN) { if (kval && t0 == 0) p.S[(size_t)v * K + k] = S_mine; }   // (experiment: round 3's plain store)
        else if (kval && t0 == 0) s_stage[it * cost_run_stride(nw * R) + wid * R + sub] = S_mine;

        // ---- online softmin (mppi.py:184-188) over this wave's rollouts (scalar bookkeeping)
        float m = INFINITY;
#pragma unroll
        for (int s = 0; s < R; ++s) {
            const bool bad = S_seg[s] != S_seg[s];
            nan_w |= bad;
            if (!bad) m = fminf(m, S_seg[s]);
        }
        if (m < INFINITY) {
            const float rn = fminf(rho_w, m);
            const float f = (rho_w == INFINITY) ? 0.0f : __expf(p.coef * (rho_w - rn));
            float es = 0.0f, e2 = 0.0f;
#pragma unroll
            for (int s = 0; s < R; ++s) {
                const float e = (S_seg[s] < INFINITY) ? __expf(p.coef * (S_seg[s] - rn)) : 0.0f;
                es += e;
                e2 += e * e;
            }
            eta_w = eta_w * f + es;
            eta2_w = eta2_w * f * f + e2;
            const float e_mine = (kval && !(S_mine != S_mine)) ? __expf(p.coef * (S_mine - rn)) : 0.0f;
            if constexpr (kStash) {
                asm volatile("" ::: "memory");
#pragma unroll
                for (int c = 0; c < NCH; ++c)
#pragma unroll
                    for (int a = 0; a < NA; ++a) eps[c][a] = xw[(c * 64 + lane) * kESP + a];
            }
#pragma unroll
            for (int c = 0; c < NCH; ++c)
#pragma unroll
                for (int a = 0; a < NA; ++a) acc[c][a] = acc[c][a] * f + e_mine * eps[c][a];
            rho_w = rn;
        }
    };
    if (ONEG) {
        // Progress priority: 3 until the integrator is done, 2 through FK and cost, 1 for the
        // softmin, 0 in the block combine.  The waves of a SIMD start over ~2 us of launch
        // ramp; under the arbiter's oldest-first order the early ones would finish early and
        // leave the late ones to run alone -- here a wave that is ahead yields.
        if (MPPI_PRIO) set_wave_prio(3);
        group(0);
        if (MPPI_PRIO) set_wave_prio(0);
    } else if (iters == 1) {
        group(0);
    } else {
        // Wave priority by remaining groups: the SIMD arbiter otherwise favours the oldest
        // wave, so the waves of a SIMD finish their (equal) work one after another and the
        // last ones run alone, without latency hiding (the grid's tail).  A
        // wave that is ahead drops its priority, the laggards catch up.
        for (int it = 0; it < iters; ++it) {
            if (MPPI_PRIO) set_wave_prio(iters - 1 - it);
            group(it);
        }
        if (MPPI_PRIO) set_wave_prio(0);
    }
    STAMP(5);
    SECTION("block_combine_record");

    // ---- cross-wave combine in LDS -> one partial record per block, one barrier:
    //      after the barrier every record thread takes rho_b = min of the 8 wave slots'
    //      rho and rescales them itself (f_w = exp(-(rho_w - rho_b)/lambda)).
    //      LDS: [8][4 + NCH*64*NA]; every lane (all R segments) deposits acc
    float* wsh = smem + ((HA + 3) & ~3);           // always 8 wave slots (unrolled reads)
    const int wstride = kWs;   // >= 4 + NCH*64*NA (the integrator's buffer may be larger)
    float* mine = wsh + wid * wstride;
    if (lane == 0) {
        mine[0] = rho_w; mine[1] = eta_w; mine[2] = eta2_w; mine[3] = nan_w ? 1.0f : 0.0f;
    }
    for (int i = nw * wstride + tid; i < 8 * wstride; i += nthr)   // absent waves: rho = inf, acc = 0
        wsh[i] = ((i - nw * wstride) % wstride == 0) ? INFINITY : 0.0f;
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
        for (int a = 0; a < NA; ++a) mine[4 + (c * 64 + lane) * NA + a] = acc[c][a];
    STAMPW(11);
    lds_barrier();
    STAMP(6);
    if (!MPPI_S_PLAIN && wid == nw - 1) {
        // The block's costs: one write-through run per group (st_dev_run), nw * R consecutive
        // samples each -- one whole 64 B line per group at R = 2 (H <= 32: C2, C3).  Issued by
        // the block's last wave, which has the fewest record stores behind it: from wave 0 the
        // write-through made the drone C2 step 0.2-0.3 us slower, from the last wave it is
        // within the A/B noise of round 3's plain stores (profiles/r04/ab_cost_store_variants.txt)
        const int nS = nw * R, q = (nS + 3) >> 2;
        float* const Sv = uniform_ptr(p.S + (size_t)v * K);
        for (int i = lane; i < iters * q; i += 64) {
            const int it = i / q, k0 = (blockIdx.x + it * p.nb) * nS;
            st_dev_run(Sv, (uint32_t)k0, s_stage + it * cost_run_stride(nS), min(nS, K - k0), i - it * q);
        }
    }
    if (MPPI_COMB_EXIT && wid != 0 && wid * 64 >= HA) {
        drain_stores();
        return;
    }
    // rho_b = the min of the 8 wave slots, which every thread reads for f_w anyway (an LDS
    // atomicMin before the barrier cost a waterfall loop and a ds_min per wave)
    float rws[8], rho_b = INFINITY;
#pragma unroll
    for (int w = 0; w < 8; ++w) {
        rws[w] = wsh[w * wstride];
        rho_b = fminf(rho_b, rws[w]);
    }
    // f_w = exp(-(rho_w - rho_b)/lambda): lane w evaluates wave w's, every lane reads all 8 back
    // (one transcendental per lane instead of eight)
    float fw[8];
    {
        float mine = INFINITY;
#pragma unroll
        for (int w = 0; w < 8; ++w) mine = ((lane & 7) == w) ? rws[w] : mine;
        const float f = (mine < INFINITY) ? __expf(p.coef * (mine - rho_b)) : 0.0f;
#pragma unroll
        for (int w = 0; w < 8; ++w) fw[w] = read_lane_f32(f, w);
    }
    STAMP(12);
    if (tid == 0) {
        float eta = 0.0f, eta2 = 0.0f, nanf = 0.0f;
#pragma unroll
        for (int w = 0; w < 8; ++w) {
            eta += fw[w] * wsh[w * wstride + 1];
            eta2 += fw[w] * fw[w] * wsh[w * wstride + 2];
            nanf = fmaxf(nanf, wsh[w * wstride + 3]);
        }
        wt_store4(uniform_ptr(p.hdr), ((uint32_t)v * (uint32_t)p.nb + blockIdx.x) * 16u, make_float4(rho_b, eta, eta2, nanf));
    }
    // record body, dim-major: rdata[v][a][block][t] = sum_w f_w sum_segments acc_w[seg*L + t].
    // (a, t) of element i without an integer division (~25 VALU): a = trunc((i + 1/2) / H)
    // in fp32 is exact, the quotient's error (< 1e-5 for i < A*H <= 2560) being far below
    // the 1/(2H) margin; 32-bit record indices (V*A*nb*H < 2^31, checked at create).
    const float rH = __builtin_amdgcn_rcpf((float)H);   // (1 ulp: far inside the 1/(2H) margin)
    float* const rdata_v = uniform_ptr(p.rdata + (size_t)v * NA * p.nb * H);   // this vehicle's bodies (< 1 GiB)
    const uint32_t rbase = blockIdx.x * (uint32_t)H;
    const uint32_t rstride = (uint32_t)p.nb * (uint32_t)H;
    for (int i = tid; i < ((MPPI_KO & 64) ? 0 : HA); i += nthr) {
        const int a = (int)(((float)i + 0.5f) * rH), t = i - a * H;
        const int c = t >> 6, tl = t & 63;
        float s = 0.0f;
#pragma unroll
        for (int w = 0; w < 8; ++w) {
            float sw = wsh[w * wstride + 4 + (c * 64 + tl) * NA + a];
#pragma unroll
            for (int sg = 1; sg < R; ++sg) sw += wsh[w * wstride + 4 + (c * 64 + sg * LSEG + tl) * NA + a];
            s += fw[w] * sw;
        }
        wt_store(rdata_v, (rbase + (uint32_t)a * rstride + (uint32_t)t) * 4u, s);
    }
    STAMP(7);
    STAMPRT(14);
    drain_stores();
}

// =============================================================================
// launchers
// =============================================================================
// the instantiation's symbol (native dispatch looks it up in the code object)
template <int MODEL, int NA, int NCH, int LSEG, bool F64, bool VONE, bool XC, bool ONEG>
inline void rollout_symbol(char* buf, size_t n) {
    snprintf(buf, n, "_Z9k_rolloutILi%dELi%dELi%dELi%dELb%dELb%dELb%dELb%dEEvjjjjiiiPKfPKN4mppi8JointDevENS2_9DevParamsE",
             MODEL, NA, NCH, LSEG, (int)F64, (int)VONE, (int)XC, (int)ONEG);
}

template <int MODEL, int NA, int NCH, int LSEG, bool F64, bool XC, bool ONEG>
inline int launch_rollout_g(const DevParams& p, int threads, hipStream_t s) {
    const int iters = ONEG ? 1 : p.iters;
    // (LDS: warm start, 8 wave slots, the block's cost runs: iters of them, one per group, each
    // (threads / 64) * R floats padded to 16 B -- sized by the block's own waves, not by 8)
    const int s_run = iters * cost_run_stride((threads / 64) * (64 / LSEG));
    if (threads <= 0 || threads > 512 || iters < 1 || s_run > kMaxCostRun) return -1;
    const size_t lds = (size_t)(((p.H * NA + 3) & ~3) + 8 * wave_slot_floats<NA, NCH, LSEG>() + s_run) * sizeof(float);
    const int32_t geo = threads | (iters << 16);
    if (p.V == 1)
        return go(k_rollout<MODEL, NA, NCH, LSEG, F64, true, XC, ONEG>,
                  rollout_symbol<MODEL, NA, NCH, LSEG, F64, true, XC, ONEG>, dim3(p.nb, p.V), dim3(threads), lds, s,
                  p.seed_lo, p.seed_hi, p.step_ctr, (uint32_t)p.k_offset, p.noise_mode, p.H, geo, p.u_prev,
                  p.joints, p);
    return go(k_rollout<MODEL, NA, NCH, LSEG, F64, false, XC, ONEG>,
              rollout_symbol<MODEL, NA, NCH, LSEG, F64, false, XC, ONEG>, dim3(p.nb, p.V), dim3(threads), lds, s,
              p.seed_lo, p.seed_hi, p.step_ctr, (uint32_t)p.k_offset, p.noise_mode, p.H, geo, p.u_prev, p.joints,
              p);
}

// the single-group (ONEG) variant exists for the common kernel at NCH == 1
template <int MODEL, int NA, int NCH, int LSEG, bool F64, bool XC>
inline int launch_rollout_x(const DevParams& p, int threads, hipStream_t s) {
    if constexpr (!XC && NCH == 1)
        if (p.iters == 1) return launch_rollout_g<MODEL, NA, NCH, LSEG, F64, XC, true>(p, threads, s);
    return launch_rollout_g<MODEL, NA, NCH, LSEG, F64, XC, false>(p, threads, s);
}

// The extended (XC) instantiation carries the extra CostManager terms, a full
// (non-diagonal) Sigma and the generic FK chains: their registers would otherwise be
// reserved in the common kernel (the full zSigma product alone held the A*A Sigma in
// VGPRs; with the generic chain loops the whole-body kernel needed 98 VGPRs, without
// them 87).  The common kernel assumes a diagonal Sigma, no extra terms and the Kinova
// chain (or no chain: the drone).
template <int MODEL, int NA, int NCH, int LSEG, bool F64>
inline int launch_rollout_t(const DevParams& p, int threads, hipStream_t s) {
    const bool generic_chain = MODEL != MPPI_MODEL_DRONE && !(NA - (MODEL == MPPI_MODEL_WHOLEBODY ? 3 : 0) == 7 &&
                                                              p.chain_fast == 2);
    if (p.cost_terms || !p.sigma_diag || generic_chain)
        return launch_rollout_x<MODEL, NA, NCH, LSEG, F64, true>(p, threads, s);
    return launch_rollout_x<MODEL, NA, NCH, LSEG, F64, false>(p, threads, s);
}

template <int MODEL, int NA, bool F64>
inline int dispatch_geom(const DevParams& p, int threads, hipStream_t s) {
    if (p.nch == 1 && p.L == 32) return launch_rollout_t<MODEL, NA, 1, 32, F64>(p, threads, s);
    if (p.nch == 1 && p.L == 64) return launch_rollout_t<MODEL, NA, 1, 64, F64>(p, threads, s);
    if (p.nch == 2) return launch_rollout_t<MODEL, NA, 2, 64, F64>(p, threads, s);
    if (p.nch == 4) return launch_rollout_t<MODEL, NA, 4, 64, F64>(p, threads, s);
    return -1;
}


// mppi_finalize.hip -- gfx950 (CDNA4) finalize kernel of the MPPI control step:
// combine the rollout blocks' partial records, w_eps, SavGol (svg_filter.py:13-90),
// u += w_eps and the outputs (mppi.py:144-158, drone_mppi.py:157-169).  The same
// kernel in PACK mode folds a shard's records into its exchange slot.
#include "mppi_device.h"

using namespace mppi;

// =============================================================================
// k_finalize: grid (A*ts, V); block (a, slice) owns t in one slice of action
// dim a of vehicle v (plus the SavGol halo it reads).
//   1. rho = min_r rho_r                     (record headers)
//   2. f_r = exp(-(rho_r - rho)/lambda); eta = sum f_r eta_r   (fp64 sums)
//   3. N[t] = sum_r f_r N_r[a][t]            (all loads in flight, one pass)
//   PACK: write (rho, eta, eta2, nan | N) into the shard's exchange slot.
//   FINAL: w_eps = N/eta, SavGol (symmetric pad), u += w_eps, outputs written
//          straight into mapped pinned host memory (no D2H copy).
// =============================================================================
constexpr int kFinThreads = 256;
constexpr int kMaxRec = 4096;

// DPP wave reductions: the identity is fed to out-of-row / masked lanes, the
// result lands in lane 63 and is broadcast with readlane (no LDS round trips).
template <int CTRL, int RM>
__device__ __forceinline__ float dpp_id(float x, float id) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(id), __float_as_int(x), CTRL, RM, 0xF, false));
}
__device__ __forceinline__ float wave_min(float x) {
    x = fminf(x, dpp_id<0x111, 0xF>(x, INFINITY));
    x = fminf(x, dpp_id<0x112, 0xF>(x, INFINITY));
    x = fminf(x, dpp_id<0x114, 0xF>(x, INFINITY));
    x = fminf(x, dpp_id<0x118, 0xF>(x, INFINITY));
    x = fminf(x, dpp_id<0x142, 0xA>(x, INFINITY));
    x = fminf(x, dpp_id<0x143, 0xC>(x, INFINITY));
    return read_lane_f32(x, 63);
}
__device__ __forceinline__ float wave_max(float x) {
    x = fmaxf(x, dpp_id<0x111, 0xF>(x, -INFINITY));
    x = fmaxf(x, dpp_id<0x112, 0xF>(x, -INFINITY));
    x = fmaxf(x, dpp_id<0x114, 0xF>(x, -INFINITY));
    x = fmaxf(x, dpp_id<0x118, 0xF>(x, -INFINITY));
    x = fmaxf(x, dpp_id<0x142, 0xA>(x, -INFINITY));
    x = fmaxf(x, dpp_id<0x143, 0xC>(x, -INFINITY));
    return read_lane_f32(x, 63);
}
__device__ __forceinline__ double wave_sum_f64(double x) {
    x += shr_f64<0x111>(x);
    x += shr_f64<0x112>(x);
    x += shr_f64<0x114>(x);
    x += shr_f64<0x118>(x);
    x += dpp_f64<0x142, 0xA>(x);
    x += dpp_f64<0x143, 0xC>(x);
    return read_lane_f64(x, 63);
}

#ifdef MPPI_STAMPS
#define FSTAMP(i)                                                                    \
    do {                                                                             \
        __builtin_amdgcn_sched_barrier(0);                                           \
        if (pk.stamps && threadIdx.x == 0)                                           \
            pk.stamps[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * kStamps + (i)] = \
                __builtin_amdgcn_s_memtime();                                        \
        __builtin_amdgcn_sched_barrier(0);                                           \
    } while (0)
#else
#define FSTAMP(i) do { } while (0)
#endif

__global__ void __launch_bounds__(kFinThreads) k_finalize(const FinParams pk) {
    // grid (A * ts, V): block (a, slice) owns t in [t_lo, t_hi) of action dim a
    // and reads the records' columns for that slice plus the SavGol halo -- the
    // record reads are spread over A*ts CUs (a single CU streams ~10 B/clk).
    constexpr int NWV = kFinThreads / 64;
    constexpr int kNPT = 16;                 // records per thread in the one-pass path
    constexpr int kWin = 16 + 2 * 15;        // max slice + halo
    __shared__ float nsum[kFinThreads];
    __shared__ float wcol[kWin];
    __shared__ float shm[2 * NWV];
    __shared__ double shd[2 * NWV];
    const FinParams& p = pk;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int a = blockIdx.x / p.ts, sl = blockIdx.x - a * p.ts, v = blockIdx.y;
    FSTAMP(0);
    const int H = p.H, n = p.nrec, hf = p.half;
    const int t_lo = sl * p.tsz, t_hi = min(H, t_lo + p.tsz);
    const int w0 = max(0, t_lo - hf), w1 = min(H, t_hi + hf), W = w1 - w0;   // window [w0, w1)
    const float* hdr = p.hdr + (size_t)v * p.hdr_vs;
    const size_t hrs = (size_t)p.hdr_rs;
    const float* col = p.dat + (size_t)v * p.d_vs + (size_t)a * p.d_as + w0;
    const size_t drs = (size_t)p.d_rs;
    float* up = p.u_prev + (size_t)v * H * p.A;
    const float uold0 = (tid == 0 && sl == 0) ? up[a] : 0.0f;   // the old u_prev[0] (mppi.py:157)
    FSTAMP(7);

    // thread (g, q): window column q of records g, g + rows, ...
    const int rows = kFinThreads / W;
    const int g = tid / W, q = tid - g * W;
    const bool active = g < rows;
    float acc = 0.0f;
    double eta = 0.0, eta2 = 0.0;
    float rho, nanflag;
    auto block_minmax = [&](float m, float nf) {
        m = wave_min(m);
        nf = wave_max(nf);
        if (lane == 0) { shm[wv] = m; shm[NWV + wv] = nf; }
        lds_barrier();
        rho = shm[0]; nanflag = shm[NWV];
#pragma unroll
        for (int i = 1; i < NWV; ++i) { rho = fminf(rho, shm[i]); nanflag = fmaxf(nanflag, shm[NWV + i]); }
    };
    if (n <= rows * kNPT) {   // one pass: every load in flight before the reductions
        float4 hd[kNPT];
        float xv[kNPT];
#pragma unroll
        for (int i = 0; i < kNPT; ++i) {
            const int r = g + i * rows;
            const bool ok = active && r < n;
            const size_t rr = (size_t)(ok ? r : 0);
            hd[i] = *reinterpret_cast<const float4*>(hdr + rr * hrs);
            xv[i] = col[rr * drs + q];
            if (!ok) { hd[i] = make_float4(INFINITY, 0.f, 0.f, 0.f); xv[i] = 0.0f; }
        }
        FSTAMP(8);
        float m = INFINITY, nf = 0.0f;
#pragma unroll
        for (int i = 0; i < kNPT; ++i) { m = fminf(m, hd[i].x); nf = fmaxf(nf, hd[i].w); }
        block_minmax(m, nf);
        FSTAMP(1);
#pragma unroll
        for (int i = 0; i < kNPT; ++i) {
            const float f = (hd[i].x == INFINITY) ? 0.0f : __expf(p.coef * (hd[i].x - rho));
            acc = fmaf(f, xv[i], acc);
            if (q == 0) { eta += (double)f * hd[i].y; eta2 += (double)f * f * hd[i].z; }
        }
    } else {                  // two passes (many records)
        float m = INFINITY, nf = 0.0f;
        for (int r = tid; r < n; r += kFinThreads) {
            const float4 h4 = *reinterpret_cast<const float4*>(hdr + (size_t)r * hrs);
            m = fminf(m, h4.x);
            nf = fmaxf(nf, h4.w);
        }
        FSTAMP(8);
        block_minmax(m, nf);
        FSTAMP(1);
        if (active) {
#pragma unroll 8
            for (int r = g; r < n; r += rows) {
                const float4 h4 = *reinterpret_cast<const float4*>(hdr + (size_t)r * hrs);
                const float f = (h4.x == INFINITY) ? 0.0f : __expf(p.coef * (h4.x - rho));
                acc = fmaf(f, col[(size_t)r * drs + q], acc);
                if (q == 0) { eta += (double)f * h4.y; eta2 += (double)f * f * h4.z; }
            }
        }
    }
    FSTAMP(2);
    {
        const double e1 = wave_sum_f64(eta), e2 = wave_sum_f64(eta2);
        if (lane == 0) { shd[wv] = e1; shd[NWV + wv] = e2; }
    }
    nsum[tid] = active ? acc : 0.0f;
    lds_barrier();
    eta = shd[0]; eta2 = shd[NWV];
#pragma unroll
    for (int i = 1; i < NWV; ++i) { eta += shd[i]; eta2 += shd[NWV + i]; }
    FSTAMP(3);
    int span = 1;
    while (span < rows) span <<= 1;
    for (int s = span >> 1; s > 0; s >>= 1) {   // log-step tree over g
        if (active && g < s && g + s < rows) nsum[tid] += nsum[tid + s * W];
        lds_barrier();
    }
    if (tid < W) wcol[tid] = nsum[tid];
    lds_barrier();
    FSTAMP(4);

    if (p.mode == 1) {   // PACK raw sums into this shard's exchange slot
        float* dst = p.dst + (size_t)v * p.P;
        if (a == 0 && sl == 0 && tid == 0) {
            dst[0] = rho; dst[1] = (float)eta; dst[2] = (float)eta2; dst[3] = nanflag;
        }
        for (int t = t_lo + tid; t < t_hi; t += kFinThreads) dst[kHdr + a * H + t] = wcol[t - w0];
        return;
    }

    // FINAL: w_eps = N/eta over the window, SavGol with the reference's symmetric
    // pad (svg_filter.py:58: index -i-1 left of 0, 2H-1-i right of H-1), u += w_eps
    const float etaf = (nanflag > 0.0f) ? NAN : (float)eta;
    if (tid < W) {
        const float w = wcol[tid] / etaf;
        wcol[tid] = w;
        const int t = w0 + tid;
        if (p.wraw && t >= t_lo && t < t_hi) p.wraw[((size_t)v * H + t) * p.A + a] = w;
    }
    lds_barrier();
    float u0new = 0.0f;
    for (int t = t_lo + tid; t < t_hi; t += kFinThreads) {
        float sm = 0.0f;
        for (int j = 0; j < p.window; ++j) {
            int idx = t + j - hf;
            idx = idx < 0 ? -idx - 1 : (idx >= H ? 2 * H - 1 - idx : idx);
            sm += p.sg[j] * wcol[idx - w0];
        }
        if (p.wsmooth) p.wsmooth[((size_t)v * H + t) * p.A + a] = sm;
        const float un = up[t * p.A + a] + sm;
        up[t * p.A + a] = un;
        if (t == 0) u0new = un;
    }
    FSTAMP(5);
    if (sl == 0 && tid == 0) {
#pragma clang fp contract(off)
        const float u0 = u0new;
        p.u0[(size_t)v * p.A + a] = u0;
        const VehicleConst& vc = (p.V == 1) ? p.vc0 : p.vc[v];
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
            float* st = p.stats + (size_t)v * 4;
            st[0] = rho;
            st[1] = (float)eta;
            st[2] = (eta2 > 0.0) ? (float)(eta * eta / eta2) : 0.0f;
            st[3] = nanflag;
        }
    }
    FSTAMP(6);
}

// w_k = exp(-(S_k - rho)/lambda) / eta  (mppi.py:184-191) -- readback only
__global__ void k_weights(const float* S, const float* stats, float* w, int V, int K, float coef) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= V * K) return;
    const int v = i / K;
    const float rho = stats[v * 4], eta = stats[v * 4 + 1];
    w[i] = expf(coef * (S[i] - rho)) / eta;
}

extern "C" int mppi_launch_finalize(const FinParams* p, void* stream) {
    if (p->nrec > kMaxRec || p->H > MPPI_MAX_HORIZON || p->tsz + 2 * p->half > 16 + 2 * 15) return -1;
    hipLaunchKernelGGL(k_finalize, dim3(p->A * p->ts, p->V), dim3(kFinThreads), 0, (hipStream_t)stream, *p);
    return (int)hipGetLastError();
}

extern "C" int mppi_launch_weights(const float* S, const float* stats, float* w, int V, int K, float coef,
                                   void* stream) {
    const int n = V * K;
    hipLaunchKernelGGL(k_weights, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, S, stats, w, V,
                       K, coef);
    return (int)hipGetLastError();
}

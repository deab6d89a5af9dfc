// mppi_finalize.hip -- gfx950 (CDNA4) finalize kernel of the MPPI control step:
// combine the rollout blocks' partial records, w_eps, SavGol (svg_filter.py:13-90),
// u += w_eps and the outputs (mppi.py:144-158, drone_mppi.py:157-169).  The same
// kernel in PACK mode folds a shard's records into its exchange slot.
#include <algorithm>

#include "mppi_device.h"

using namespace mppi;

// =============================================================================
// k_finalize: grid (Ga*ts, V), Ga = A rounded up to 8; block (a, slice) owns t in one slice of action
// dim a of vehicle v (plus the SavGol halo it reads).
//   1. rho = min_r rho_r                     (record headers)
//   2. f_r = exp(-(rho_r - rho)/lambda); eta = sum f_r eta_r   (fp64 sums)
//   3. N[t] = sum_r f_r N_r[a][t]            (all loads in flight, one pass)
//   PACK: write (rho, eta, eta2, nan | N) into the shard's exchange slot.
//   FINAL: w_eps = N/eta, SavGol (symmetric pad), u += w_eps, outputs written
//          straight into mapped pinned host memory (no D2H copy).
// =============================================================================
// Block size NT (template): the smallest of 128 / 256 / 512 threads whose one chunk of
// loads covers every record (rows per chunk = NT * kNPT / CW), else 512.  Measured on
// MI355X (profiles/r01/finalize_threads_s3.txt): arm C3 (256 records) 5.91 -> 5.26 us at
// 256 threads, the V=8 fleet (128 records per vehicle) 10.58 -> 5.46 us at 128, whole-body
// K=8192 (512 records) best at 512.
constexpr int kFinThreads = 512;   // upper bound (LDS arrays are sized for 8 waves)
constexpr int kMaxRec = 4096;
// timing knockouts for tools/ experiments (results wrong): 2 skips the mapped-memory
// outputs, 8 exits after the wave fold, 16 exits at the start (the launch floor), 32 skips
// the u_prev update, 128 the final drain, 256 the plain output arrays (the tagged records
// stay).  (64, "tail parameters not loaded", was removed in round 6: since the tail moved to
// FinTail its pointers are the only ones the stores use, and that build stored through null.)
#ifndef MPPI_FIN_KO
#define MPPI_FIN_KO 0
#endif
// timing knockout for tools/ A/B experiments (results unsafe): 1 = no commit marks (peer exchange)
#ifndef MPPI_FIN_NOMARK
#define MPPI_FIN_NOMARK 0
#endif
// XCDs the finalize's blocks run on (8; 4 = the first four, see the block map in k_finalize)
#ifndef MPPI_FIN_XCDS
#define MPPI_FIN_XCDS 8
#endif

#if defined(MPPI_STAMPS) && !defined(MPPI_TIMELINE)
#define FSTAMP(i)                                                                    \
    do {                                                                             \
        __builtin_amdgcn_sched_barrier(0);                                           \
        if (pk.stamps && threadIdx.x == 0)                                           \
            pk.stamps[(((size_t)v * A + a) * ts + sl) * kStamps + (i)] =               \
                __builtin_amdgcn_s_memtime();                                        \
        __builtin_amdgcn_sched_barrier(0);                                           \
    } while (0)
#define FSTAMPRT(i) do { } while (0)
#elif defined(MPPI_STAMPS)   // MPPI_TIMELINE: block start / end (wave 0) in wall-clock time, the
                             // XCD in slot 15, the first chunk's loads issued + tail pinned (slot 7)
                             // and the wave fold's end (slot 1: records combined)
#define FSTAMPRT(i)                                                                  \
    do {                                                                             \
        if (pk.stamps && threadIdx.x == 0) {                                         \
            pk.stamps[(((size_t)v * A + a) * ts + sl) * kStamps + (i)] =               \
                __builtin_amdgcn_s_memrealtime();                                    \
            if ((i) == 13)                                                           \
                pk.stamps[(((size_t)v * A + a) * ts + sl) * kStamps + 15] =            \
                    (unsigned long long)__builtin_amdgcn_s_getreg(0xF814);           \
        }                                                                            \
    } while (0)
#define FSTAMP(i) do { if ((i) == 1 || (i) == 7) FSTAMPRT(i); } while (0)
#else
#define FSTAMP(i) do { } while (0)
#define FSTAMPRT(i) do { } while (0)
#endif

// Block = 8 waves.  Lane (g, q) of wave wv holds window column q (CW = 16/32/64
// columns) of the records gr, gr + TR, gr + 2 TR, ... where gr = wv*ROWS + g is
// its global row and TR = 8*ROWS the row count.  Records are consumed in chunks
// of TR*kNPT with every load of a chunk in flight; each lane keeps a running
// rho_t (online softmin, like the rollout).  Rows are folded inside each wave
// (xor shuffles, DPP), the 8 waves through LDS behind ONE barrier, and wave 0
// finishes alone: w_eps, SavGol by lane shuffles (WIN taps, template), u_prev,
// outputs.
// The leading scalar arguments (through the step's sequence number) are preloaded into
// SGPRs (build.py: 14 dwords); the tail's parameters come from the device-resident FinTail
// (L2-hot across steps), so a FINAL launch of one vehicle reads nothing else of its
// kernel-argument block.  pk carries the PACK-mode fields and the diagnostic stamps.
template <int CW, int WIN, int NT>
__global__ void __launch_bounds__(NT) k_finalize(const float* __restrict__ hdr_base,
                                                          const float* __restrict__ dat_base,
                                                          const FinTail* __restrict__ tail,
                                                          const uint32_t nrec_H, const uint32_t geo,
                                                          const int32_t hdr_rs, const int32_t d_rs,
                                                          const int32_t d_as, const int32_t hdr_vs,
                                                          const int32_t d_vs, const uint32_t seq_arg,
                                                          const FinParams pk) {
    constexpr int NWV = NT / 64;
    constexpr int ROWS = 64 / CW;          // rows per wave
    constexpr int TR = NWV * ROWS;         // rows per block
    constexpr int kNPT = 16;
    __shared__ float wcol[NWV][CW];
    __shared__ float wrho[NWV], wnan[NWV], weta[NWV], weta2[NWV];
    __shared__ float wsg[96];   // wave 0: w over the window + reflected pads (SavGol taps by LDS reads)
    const FinParams& p = pk;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int n = (int)(nrec_H & 0xFFFFu), H = (int)(nrec_H >> 16);
    const int tsz = (int)(geo & 0xFFu), hf = (int)((geo >> 8) & 0xFFu), ts = (int)((geo >> 16) & 0xFFu);
    const int A = (int)(geo >> 24);
    // XCD-aware block map: the dispatcher deals blocks round robin over the 8 XCDs (block b
    // on XCD b mod 8).  Dim a lives on XCD a mod X (X = MPPI_FIN_XCDS of them), every slice of
    // it too: the slices read the same record lines (one 128 B line holds 32 t of a row),
    // which one L2 then fetches once instead of once per slice.  Blocks b mod 8 >= X and
    // dims >= A exit at once.
    const int x8 = blockIdx.x & 7, j8 = blockIdx.x >> 3, na = (A + MPPI_FIN_XCDS - 1) / MPPI_FIN_XCDS;
    // (na is 1 for A <= 8 and 2 for the whole-body's 10 dims: the general scalar division is
    // ~30 dependent SALU ops at the head of every block)
    const int sl = (na == 1) ? j8 : (na == 2) ? (j8 >> 1) : j8 / na;
    const int a = x8 + MPPI_FIN_XCDS * (j8 - sl * na), v = blockIdx.y;
    if (x8 >= MPPI_FIN_XCDS || a >= A) return;
    if (MPPI_FIN_KO & 16) { if (tid == 0) p.u_prev[blockIdx.x] = 0.0f; return; }   // timing knockout: launch floor
    FSTAMPRT(13);
    FSTAMP(0);
    const int t_lo = sl * tsz, t_hi = min(H, t_lo + tsz);
    const int w0 = max(0, t_lo - hf), w1 = min(H, t_hi + hf), W = w1 - w0;   // window [w0, w1), W <= CW
    // (both bases and the header range kept in SGPRs: in a build where the compiler put one
    // in VGPRs, every record load became a waterfall loop over a "divergent" resource)
    const float* hdr = uniform_ptr(hdr_base + (size_t)v * (uint32_t)hdr_vs);
    const float* col = uniform_ptr(dat_base + (size_t)v * (uint32_t)d_vs + (size_t)a * d_as + w0);
    const FinTail& T = *tail;
    const int g = lane / CW, q = lane - g * CW, gr = wv * ROWS + g;
    const bool qv = q < W;
    // wave 0's u_prev over the window (lane q <-> t = w0 + q, incl. the OLD u_prev[0],
    // mppi.py:157) and the vehicle constants of the outputs (slice 0 of each dim, lane 0) are
    // loaded AFTER the first chunk of record loads is issued (pin_tail below): they need the
    // tail's pointers (an s_load round trip, then their own), and issued first they held the
    // record loads behind both -- the register allocator paired a pending u_prev/vc load with
    // the record offsets, and the whole wave waited for vmcnt(0) before its first record load
    float u_old = 0.0f, x0f = 0.0f, v0f = 0.0f;
    double x0d = 0.0, v0d = 0.0;
    float* up = nullptr;

    // The tail's parameters (FinTail), read into SGPRs while the record loads fly: left to
    // the compiler, each was an s_load waited for on the spot in wave 0's tail (15 serial
    // scalar round trips).  The empty asm makes every value opaque, so it is neither
    // re-loaded later nor sunk to its use.
    float coef = 0.0f, dt = 0.0f, dt2 = 0.0f;
    int32_t mode = 0, model = 0, qoff = 0, nq = 0, sf64 = 0, odim = 0;
    const uint32_t seq = seq_arg;
    // native control calls (mppi_aql.cpp): the step's sequence number travels with the vehicle
    // constants (VehicleConst::_pad[0], written by the host into the rollout's arguments, handed
    // over by the rollout's block 0), so the finalize's own argument block stays static
    uint32_t seqv = seq;
    float *wraw = nullptr, *wsmooth = nullptr, *u0p = nullptr, *stats = nullptr;
    double* outp = nullptr;
    uint32_t* flags = nullptr;
    const VehicleConst* vcb = nullptr;
    unsigned long long* const* xpeers = nullptr;   // peer exchange (null: off)
    unsigned long long xpl = 0ull;   // lane d < xn: rank d's region address (wave 0's stores read it by readlane)
    unsigned long long* xlocal = nullptr;
    uint32_t* xovl = nullptr;   // overlapped batches' step counters (null: off)
    uint32_t* xstall = nullptr;   // diagnostics (mppi_debug_peer_stall; null: off)
    unsigned long long* xdec = nullptr;   // the rank's two decision words (peer exchange)
    int32_t xn = 0, xme = 0;
    uint32_t xstep = 0u, xep = 0u;
    float sg[WIN > 0 ? WIN : 1];
    auto pin_tail = [&]() {
        // every load issues first, then two empty asms consume them (one wait): pinned one
        // by one, each load was followed by its own s_waitcnt, ~20 serial round trips
        coef = T.coef; dt = T.dt; dt2 = T.dt2;
        mode = T.mode; model = T.model; qoff = T.qoff; nq = T.nq; sf64 = T.state_f64; odim = T.out_dim;
        wraw = T.wraw; wsmooth = T.wsmooth; u0p = T.u0; stats = T.stats; outp = T.out; flags = T.flags;
        up = T.u_prev; vcb = T.vc;
        xpeers = T.xpeers; xlocal = T.xlocal; xn = T.xn; xme = T.xme; xovl = T.xovl; xstall = T.xstall; xdec = T.xdec;
        if constexpr (WIN > 0) {
#pragma unroll
            for (int j = 0; j < WIN; ++j) sg[j] = T.sg[j];
        }
        asm volatile("" : "+s"(coef), "+s"(dt), "+s"(dt2), "+s"(mode), "+s"(model), "+s"(qoff), "+s"(nq),
                          "+s"(sf64), "+s"(odim), "+s"(wraw), "+s"(wsmooth), "+s"(u0p), "+s"(stats),
                          "+s"(outp), "+s"(flags), "+s"(up), "+s"(vcb), "+s"(xpeers), "+s"(xlocal), "+s"(xn),
                          "+s"(xme), "+s"(xovl), "+s"(xstall), "+s"(xdec));
        if constexpr (WIN == 9)
            asm volatile("" : "+s"(sg[0]), "+s"(sg[1]), "+s"(sg[2]), "+s"(sg[3]), "+s"(sg[4]), "+s"(sg[5]),
                              "+s"(sg[6]), "+s"(sg[7]), "+s"(sg[8]));
        else if constexpr (WIN == 5)
            asm volatile("" : "+s"(sg[0]), "+s"(sg[1]), "+s"(sg[2]), "+s"(sg[3]), "+s"(sg[4]));
        // then the loads that need those pointers (global address space: a flat load also
        // counts in lgkmcnt, so every later scalar wait would wait for it too)
        up += (size_t)v * H * A;
        // (device-scope loads: the previous finalize's u_prev, the rollout's handed-over vc)
        if (wv == 0 && q < W && g == 0) u_old = ld_dev(up + (w0 + q) * A + a);
        if (tid == 0 && sl == 0) {
            const VehicleConst* vcp = vcb + v;
            x0f = ld_dev(vcp->pos0f + a); v0f = ld_dev(vcp->vel0f + a);
            x0d = ld_dev(vcp->pos0 + a); v0d = ld_dev(vcp->vel0 + a);
            if (seq == kSeqFromVc) seqv = ld_dev((const uint32_t*)vcp->_pad);   // (its bits)
        }
        if (tid == 0 && xpeers) {   // the exchange's tag: the step's counter and the exchange epoch
            xstep = ld_dev((const uint32_t*)(vcb + v) + kVcStepWord);
            xep = ld_dev((const uint32_t*)(vcb + v) + kVcEpochWord);
        }
        // every rank's region address, one per lane, loaded here so it lands during the record fold:
        // loaded per rank inside the store loop, each pointer load's wait also waited for the
        // previous rank's system-scope stores to complete (vmcnt counts stores): G - 1 serial
        // remote-store completions before the poll could even start
        if (wv == 0 && xpeers)
            xpl = ((const __attribute__((address_space(1))) unsigned long long*)xpeers)[lane < xn ? lane : 0];
    };
    // running softmin per lane.  The header terms (rho, eta, eta2, nan) are the same for every
    // column of a row group, so each lane carries them and the wave fold runs over row groups
    // only.  eta in fp32, like the reference's torch.sum of the fp32 exponentials
    // (mppi.py:184-188): <= 16 terms per lane, then 2 + 3 (8 waves) folds.
    float rho_t = INFINITY, acc = 0.0f, nanflag = 0.0f, eta = 0.0f, eta2 = 0.0f;
    // Record loads through buffer resources over this vehicle's headers and this (dim,
    // window)'s body columns: each load is one 32-bit VGPR offset (a full-rate add per row)
    // instead of a 64-bit address (v_mad_u64_u32 + v_lshl_add_u64, both quarter-rate: ~380
    // cycles of address math ahead of the first load).  Rows past n are masked at use (okm);
    // their offsets run past the resources' ranges, which read 0 instead of faulting.
    const uint32_t hrs_b = (uint32_t)hdr_rs * 4u, drs_b = (uint32_t)d_rs * 4u;
    const __amdgpu_buffer_rsrc_t hrsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(hdr), 0, __builtin_amdgcn_readfirstlane((int)((uint32_t)n * hrs_b)),
                                          0x00020000);
    // (the range is block-uniform, but its W reaches the compiler through VGPR math: without
    // readfirstlane every body load became a waterfall loop over a "divergent" resource)
    const __amdgpu_buffer_rsrc_t crsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(col), 0, __builtin_amdgcn_readfirstlane((int)((uint32_t)(n - 1) * drs_b + (uint32_t)W * 4u)),
        0x00020000);
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    for (int base = 0; base < n; base += TR * kNPT) {
        float4 hd[kNPT];
        float xv[kNPT];
        uint32_t okm = 0;   // rows past n are masked at use: a select on the loaded value
                            // here made the compiler wait for each load in turn
        const uint32_t r0 = (uint32_t)(base + gr);
        const uint32_t hoff = r0 * hrs_b, coff = r0 * drs_b + (uint32_t)(qv ? q : 0) * 4u;
#pragma unroll
        for (int i = 0; i < kNPT; ++i) {
            okm |= (uint32_t)(r0 + (uint32_t)(i * TR) < (uint32_t)n) << i;
            const u32x4 h = __builtin_amdgcn_raw_buffer_load_b128(hrsrc, (int)(hoff + (uint32_t)(i * TR) * hrs_b), 0, kAuxDev);
            hd[i] = make_float4(__uint_as_float(h.x), __uint_as_float(h.y), __uint_as_float(h.z), __uint_as_float(h.w));
            xv[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(crsrc, (int)(coff + (uint32_t)(i * TR) * drs_b), 0, kAuxDev));
        }
        if (base == 0) {
            __builtin_amdgcn_sched_barrier(0);   // the first chunk's record loads issue first
            pin_tail();
        }
#pragma unroll
        for (int i = 0; i < kNPT; ++i)
            if (!((okm >> i) & 1u)) hd[i].x = INFINITY;   // f = 0: y, z and xv drop out
        FSTAMP(7);
        float m = INFINITY;
#pragma unroll
        for (int i = 0; i < kNPT; ++i) { m = fminf(m, hd[i].x); nanflag = fmaxf(nanflag, hd[i].w); }
        // the body terms are accumulated outside the branch: used only inside it, the
        // compiler sank the body loads into it, behind a wait for every header load (two
        // memory round trips instead of one).  f = 0 adds exactly nothing (bodies are finite:
        // sums of weighted noise, 0 for a block without a finite cost).
        float fr[kNPT];
#pragma unroll
        for (int i = 0; i < kNPT; ++i) fr[i] = 0.0f;
        if (m < INFINITY) {
            const float rn = fminf(rho_t, m);
            if (rho_t < INFINITY) {   // rescale the running sums to the new reference
                const float sc = __expf(coef * (rho_t - rn));
                acc *= sc;
                eta *= sc;
                eta2 *= sc * sc;
            }
            rho_t = rn;
#pragma unroll
            for (int i = 0; i < kNPT; ++i) {
                const float f = (hd[i].x < INFINITY) ? __expf(coef * (hd[i].x - rn)) : 0.0f;
                fr[i] = f;
                eta = fmaf(f, hd[i].y, eta);
                eta2 = fmaf(f * f, hd[i].z, eta2);
            }
        }
#pragma unroll
        for (int i = 0; i < kNPT; ++i) acc = fmaf(fr[i], xv[i], acc);
        FSTAMP(8);
    }
    {   // fold the wave's row groups: rescale every lane to the wave's rho, sum the rows
        const float rw = fold_rows<CW>(rho_t, OpMin());
        const float sc = (rho_t < INFINITY) ? __expf(coef * (rho_t - rw)) : 0.0f;
        acc = fold_rows<CW>(acc * sc, OpAdd());
        const float e1 = fold_rows<CW>(eta * sc, OpAdd()), e2 = fold_rows<CW>(eta2 * (sc * sc), OpAdd());
        const float nf = fold_rows<CW>(nanflag, OpMax());
        if (lane < CW) wcol[wv][lane] = acc;
        if (lane == 0) { wrho[wv] = rw; wnan[wv] = nf; weta[wv] = e1; weta2[wv] = e2; }
    }
    FSTAMP(1);
    if (MPPI_FIN_KO & 8) { if (lane < CW) p.u_prev[lane] += acc + (float)eta; return; }   // timing knockout
    lds_barrier();
    if (wv != 0) return;
    FSTAMP(2);
    // wave 0: combine the 4 waves (lane q = column q)
    float rho = wrho[0], nanf = wnan[0];
#pragma unroll
    for (int w = 1; w < NWV; ++w) { rho = fminf(rho, wrho[w]); nanf = fmaxf(nanf, wnan[w]); }
    float N = 0.0f;
    eta = 0.0f; eta2 = 0.0f;
#pragma unroll
    for (int w = 0; w < NWV; ++w) {
        const float f = (wrho[w] < INFINITY) ? __expf(coef * (wrho[w] - rho)) : 0.0f;
        N = fmaf(f, (lane < CW) ? wcol[w][lane] : 0.0f, N);
        eta = fmaf(f, weta[w], eta);
        eta2 = fmaf(f * f, weta2[w], eta2);
    }
    FSTAMP(3);
    bool xlate = false;   // the peer exchange gave the step up: this step keeps the warm start (w_eps = 0)
    if (xpeers != nullptr && mode != 1) {
        // Peer exchange (sharded V == 1 engines, mppi_dev.h kXW): this block's partial goes to every
        // other rank's region (a FINAL only; READBACK re-reads the last step's), then the other
        // ranks' partials of this block come back from this rank's region, each 8 B word valid once
        // its tag is this step's, and all are combined in rank order (the same order on every rank:
        // every rank finalises bit-identically; one rank reproduces the unsharded step exactly,
        // f = exp(0) = 1).
        const uint32_t step = __builtin_amdgcn_readfirstlane(xstep);
        const uint32_t tag = peer_tag(step, __builtin_amdgcn_readfirstlane(xep));
        // (the grid from geo, not gridDim: that reads the hidden kernel arguments, which native
        // dispatch does not supply; V == 1 on a peer-exchange engine)
        const size_t nbk = (size_t)8 * na * ts, blk = blockIdx.x;
        const size_t par = step & 1u;
        const float hown = (lane == 0) ? rho : (lane == 1) ? eta : (lane == 2) ? eta2 : nanf;
        const size_t off = ((par * (size_t)xn + (size_t)xme) * nbk + blk) * kXW;   // this block's slot
        typedef __attribute__((address_space(1))) unsigned long long gst64;
        auto region = [&](int d) {   // rank d's region (uniform: d is)
            return (gst64*)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(xpl >> 32), d) << 32) |
                            (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)xpl, d));
        };
        typedef __attribute__((address_space(1))) unsigned long long gu64;
        gu64* const ctl = (gu64*)xlocal - kXCtl;   // the ranks' timeout reports, the decision words
        if (mode == 0) {   // (this rank's own partial stays in registers: no round trip through memory)
            if (uint32_t* xs = xstall) {   // diagnostics (mppi_debug_peer_stall): one block's stores late
                const uint32_t sv = ld_dev(xs);
                if (sv != 0u && (sv & 0xFFFFu) == (uint32_t)blk) {
                    const uint64_t t_s = __builtin_amdgcn_s_memrealtime(), ticks = (uint64_t)(sv >> 16) * 100000ull;
                    while (__builtin_amdgcn_s_memrealtime() - t_s < ticks) __builtin_amdgcn_s_sleep(127);
                    if (lane == 0) __hip_atomic_store(xs, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // once
                }
            }
            const unsigned long long wc = ((unsigned long long)tag << 32) | __float_as_uint(N);
            const unsigned long long wh = ((unsigned long long)tag << 32) | __float_as_uint(hown);
#pragma unroll
            for (int d = 0; d < kMaxPeers; ++d) {   // (uniform branches; no wait between the ranks' stores)
                if (d >= xn || d == xme) continue;
                gst64* dst = region(d) + off;
                if (lane < W) __hip_atomic_store(dst + kHdr + lane, wc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if (lane < kHdr) __hip_atomic_store(dst + lane, wh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
        float nv[kMaxPeers], hv[kMaxPeers];
#pragma unroll
        for (int r = 0; r < kMaxPeers; ++r) {
            nv[r] = (r == xme) ? N : 0.0f;
            hv[r] = (r == xme) ? hown : 0.0f;
        }
        // Poll: every pending rank's words are loaded in ONE batch per round (each lane its column
        // word and, lanes < 4, a header word; global, not flat, loads into separate registers), then
        // checked together, so a round costs one memory round trip whatever the rank count.  (With
        // the loads issued per rank behind divergent branches, the compiler waited for each load
        // before the next: 2 (G - 1) serial round trips per round, ~14 at G = 8.)  Which ranks are
        // still pending is wave-uniform: a rank is done when every lane that needs a word of it has
        // seen the step's tag (a ballot), and its words are taken from that round.  true: given up
        // (the bound passed or, heeding reports, some rank reported a timeout since the last reset).
        const bool needc = lane < W, needh = lane < kHdr;
        uint32_t pend = ((1u << xn) - 1u) & ~(1u << xme);   // (uniform)
        const unsigned long long* src = xlocal + (par * (size_t)xn * nbk + blk) * kXW;
        auto poll = [&](bool heed_reports) -> bool {
            const uint64_t t_in = __builtin_amdgcn_s_memrealtime();
            while (pend != 0u) {
                unsigned long long xc[kMaxPeers], xh[kMaxPeers];
#pragma unroll
                for (int r = 0; r < kMaxPeers; ++r) {
                    xc[r] = 0ull; xh[r] = 0ull;
                    if ((pend >> r) & 1u) {   // (uniform branch)
                        gu64* s = (gu64*)(src + (size_t)r * nbk * kXW);
                        // lane < 64 <= kXW - kHdr: every lane's word lies inside the rank's slot (the
                        // words past W are not written and not checked)
                        xc[r] = __hip_atomic_load(s + kHdr + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        xh[r] = __hip_atomic_load(s + (lane & (kHdr - 1)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    }
                }
                if (heed_reports) {   // (in the same batch of loads: lane r < xn reads rank r's report)
                    const unsigned long long xk = __hip_atomic_load(ctl + (lane < xn ? lane : 0), __ATOMIC_RELAXED,
                                                                    __HIP_MEMORY_SCOPE_SYSTEM);
                    if (__builtin_amdgcn_ballot_w64(lane < xn && xk != 0ull) != 0ull) return true;
                }
#pragma unroll
                for (int r = 0; r < kMaxPeers; ++r) {
                    if (!((pend >> r) & 1u)) continue;
                    const bool ok = (!needc || (uint32_t)(xc[r] >> 32) == tag) && (!needh || (uint32_t)(xh[r] >> 32) == tag);
                    if (__builtin_amdgcn_ballot_w64(!ok) == 0ull) {
                        nv[r] = needc ? __uint_as_float((uint32_t)xc[r]) : 0.0f;
                        hv[r] = needh ? __uint_as_float((uint32_t)xh[r]) : 0.0f;
                        pend &= ~(1u << r);
                    }
                }
                pend = __builtin_amdgcn_readfirstlane(pend);
                if (pend == 0u) break;
                if (__builtin_amdgcn_s_memrealtime() - t_in > kPeerWaitTicks) return true;   // (2 s)
                __builtin_amdgcn_s_sleep(1);
            }
            return false;
        };
        bool late = poll(true), torn = false;
        if (mode == 0) {
            // All or nothing within the rank (mppi_dev.h, "All or nothing within a rank").  A block whose words all arrived in
            // time with no report in sight marks the rank's decision word "commit" and goes on at
            // once: nothing on this, the common, path waits.  A late block first reports (every
            // region, this rank's own included: from then on no block of this rank can see its
            // final round clean), then waits out kDecGraceTicks -- any block of this rank that found
            // its words before the report arrived has marked its commit by then -- and reads the
            // word: committed, it keeps polling its peers (a second bound, reports no longer heeded:
            // the peers' words stay in place) and completes; otherwise the rank gives the step up.
            gu64* dw = (gu64*)xdec + par * nbk;   // this parity's marks, one word per block (no two blocks
                                                  // store to one word: 80 stores into one would serialise)
            if (!late) {
                if (lane == 0 && !MPPI_FIN_NOMARK)
                    __hip_atomic_store(dw + blk, ((unsigned long long)tag << 32) | kDecCommit, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            } else {
                const unsigned long long cw = ((unsigned long long)tag << 32) | 1ull;
#pragma unroll
                for (int d = 0; d < kMaxPeers; ++d) {
                    if (d >= xn) continue;
                    gst64* rg = region(d);
                    if (lane == 0) __hip_atomic_store(rg - kXCtl + xme, cw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
                const uint64_t t_rep = __builtin_amdgcn_s_memrealtime();
                while (__builtin_amdgcn_s_memrealtime() - t_rep < kDecGraceTicks) __builtin_amdgcn_s_sleep(8);
                bool marked = false;   // any block of this rank marked this step (the words carry the tag:
                                       // an earlier step's marks never match)
                for (size_t i = lane; i < nbk; i += 64) {
                    const unsigned long long w = __hip_atomic_load(dw + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    marked |= (uint32_t)(w >> 32) == tag && ((uint32_t)w & 3u) == kDecCommit;
                }
                if (__builtin_amdgcn_ballot_w64(marked) != 0ull) {   // another block of this rank updated its slice
                    late = poll(false);
                    torn = late;
                }
                uint32_t* xe = T.xerr;   // (read only here: the late path) the sticky word the host reads
                if (late && lane == 0 && xe) {   // (mppi_synchronize / mppi_read_outputs / mppi_peer_status)
                    __hip_atomic_store(xe, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    if (torn) __hip_atomic_store(xe + 1, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
            }
        }
        rho = INFINITY;
        nanf = late ? (torn ? 3.0f : 2.0f) : 0.0f;   // (the records' nan flag: 2 given up, 3 torn)
#pragma unroll
        for (int r = 0; r < kMaxPeers; ++r) {
            if (r < xn) {
                rho = fminf(rho, __int_as_float(__builtin_amdgcn_readlane(__float_as_int(hv[r]), 0)));
                nanf = fmaxf(nanf, __int_as_float(__builtin_amdgcn_readlane(__float_as_int(hv[r]), 3)));
            }
        }
        N = 0.0f; eta = 0.0f; eta2 = 0.0f;
#pragma unroll
        for (int r = 0; r < kMaxPeers; ++r) {
            if (r < xn) {
                const float rr = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(hv[r]), 0));
                const float er = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(hv[r]), 1));
                const float e2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(hv[r]), 2));
                const float f = (rr < INFINITY) ? __expf(coef * (rr - rho)) : 0.0f;
                N = fmaf(f, nv[r], N);
                eta = fmaf(f, er, eta);
                eta2 = fmaf(f * f, e2, eta2);
            }
        }
        if (late) { xlate = true; N = 0.0f; }
    }
    const int t = w0 + lane;              // this lane's time index (lanes < W)
    const bool own = lane < W && t >= t_lo && t < t_hi;
    if (mode == 1) {   // PACK raw sums into this shard's exchange slot
        // the slot fields in one scalar round trip (each was its own wait in the tail)
        float* dst = T.dst;
        float* xbase = T.xbase;
        int64_t xslot = T.xslot;
        int32_t nslots = T.nslots, myslot = T.myslot, P = T.P;
        asm volatile("" : "+s"(dst), "+s"(xbase), "+s"(xslot), "+s"(nslots), "+s"(myslot), "+s"(P));
        dst += (size_t)v * P;
        if (a == 0 && sl == 0 && lane == 0) {
            dst[0] = rho; dst[1] = eta; dst[2] = eta2; dst[3] = nanf;
        }
        if (own) dst[kHdr + a * H + t] = N;
        for (int s = 0; s < nslots; ++s) {   // zero the other shards' slots (x + 0 is exact)
            if (s == myslot) continue;
            float* z = xbase + (size_t)s * xslot + (size_t)v * P;
            if (a == 0 && sl == 0 && lane < kHdr) z[lane] = 0.0f;
            if (own) z[kHdr + a * H + t] = 0.0f;
        }
        FSTAMPRT(14);
        return;
    }

    // FINAL: w_eps = N/eta over the window, SavGol, u += w_eps
    const float etaf = xlate ? 1.0f : (nanf > 0.0f) ? NAN : eta;
    const float w = __fdividef(N, etaf);
    FSTAMP(4);
    // SavGol with the reference's symmetric pad (svg_filter.py:58: index -i-1 left of 0,
    // 2H-1-i right of H-1; one reflection suffices, create checks H > window/2): w goes to
    // LDS at kPad + (t - w0), and the lanes within hf of an edge of the horizon also write
    // their mirror position, so every owned lane reads its WIN taps at consecutive addresses
    // (immediate offsets, one wait) -- no per-tap index arithmetic, no ds_bpermute.
    constexpr int kPad = kMaxW / 2;   // >= hf for every window create accepts (<= MPPI_MAX_SAVGOL)
    static_assert(kPad + 64 + kMaxW / 2 <= (int)(sizeof(wsg) / sizeof(float)),
                  "wsg holds the widest window: kPad + W (<= 64) + hf");
    float sm = 0.0f;
    if (lane < W) {
        wsg[kPad + lane] = w;
        if (w0 == 0 && t < hf) wsg[kPad - 1 - t] = w;                      // left pad
        if (w1 == H && t >= H - hf) wsg[kPad + 2 * H - 1 - t - w0] = w;    // right pad
    }
    wave_lds_handoff();
    {
        const float* src = wsg + kPad + lane - hf;
        if constexpr (WIN > 0) {
#pragma unroll
            for (int j = 0; j < WIN; ++j) sm = fmaf(sg[j], src[j], sm);
        } else {
            for (int j = 0; j < T.window; ++j) sm = fmaf(T.sg[j], src[j], sm);
        }
    }
    FSTAMP(5);
    if (mode == 2) {   // READBACK (mppi_get_weighted_noise): w_eps and its SavGol, nothing else
        if (own) {
            wraw[((size_t)v * H + t) * A + a] = w;
            wsmooth[((size_t)v * H + t) * A + a] = sm;
        }
        return;
    }
    const float un = u_old + sm;
    if (own) {
        // written through at device scope (the next rollout reads it on every XCD), drained at
        // the end: the native dispatch's finalize packets then need no release (mppi_aql.cpp)
        if (!(MPPI_FIN_KO & 32))   // (32: timing knockout, u_prev not written)
            __hip_atomic_store(up + t * A + a, un, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (!(MPPI_FIN_KO & 2) && sl == 0 && lane == 0) {   // t = 0 lives in lane 0 of slice 0: outputs into mapped host memory
#pragma clang fp contract(off)
        const float u0 = un;
        const float uold0 = u_old;
        const bool plain = !(MPPI_FIN_KO & 256);   // (256: timing knockout, the plain host arrays not written)
        if (plain) u0p[(size_t)v * A + a] = u0;
        double* out = outp + (size_t)v * odim;
        const bool drone_dim = (model == MPPI_MODEL_DRONE) || (model == MPPI_MODEL_WHOLEBODY && a < 3);
        double o1 = 0.0, o2 = 0.0;   // this dim's two outputs (position, velocity)
        if (model == MPPI_MODEL_QUADROTOR) {
            // coupled dims (thrust rotated by R(rpy)): the host forms the outputs from u0
            // (mppi_engine.cpp quad_outputs)
        } else if (drone_dim) {   // drone_mppi.py:168-169
            const float x0 = x0f, v0 = v0f;
            const float xo = (x0 + v0 * dt) + (0.5f * u0) * dt2;
            const float vo = v0 + dt * u0;
            o1 = xo;
            o2 = vo;
            if (plain) {
                out[a] = o1;
                out[3 + a] = o2;
            }
        } else {           // mppi.py:157-158 (qdes uses the OLD u_prev[0])
            const int j = a - qoff;
            const int base = (model == MPPI_MODEL_WHOLEBODY) ? 6 : 0;
            const float t1 = uold0 * dt;
            const float t2 = ((0.5f * u0) * dt) * dt;
            const float t3 = u0 * dt;
            if (sf64 && model == MPPI_MODEL_ARM) {
                o1 = (x0d + (double)t1) + (double)t2;
                o2 = v0d + (double)t3;
            } else {
                o1 = (double)((x0f + t1) + t2);
                o2 = (double)(v0f + t3);
            }
            if (plain) {
                out[base + j] = o1;
                out[base + nq + j] = o2;
            }
        }
        const float ess = (eta2 > 0.0f) ? eta * (eta / eta2) : 0.0f;
        if (plain && a == 0) {
            float* st = stats + (size_t)v * 4;
            st[0] = rho;
            st[1] = eta;
            st[2] = ess;
            st[3] = nanf;
        }
        // Completion of a read step (seq != 0; mppi_run_steps' earlier steps have none): tagged
        // output records in mapped host memory, each ONE 16 B store carrying the step's sequence
        // number beside its values -- (o1, u0, seq) and (o2, nan flag, seq) per dim, (rho, eta,
        // ess, seq) per vehicle -- so the host takes the values from a record whose own tag it
        // checks (mppi_step.cpp wait_outputs / mppi_read_outputs) and nothing needs ordering
        // against anything else: no system-scope fence (an L2 writeback of ~1.5 us of kernel
        // time on the call's latency path) and no separate flag store.  The plain arrays above
        // stay for the native batches (completed by their packet's system-scope release).
        if (seqv != 0u) {
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            u32x4* rec = reinterpret_cast<u32x4*>(flags) + (size_t)v * (2 * A + 1);
            const uint64_t b1 = (uint64_t)__double_as_longlong(o1), b2 = (uint64_t)__double_as_longlong(o2);
            rec[2 * a] = u32x4{(uint32_t)b1, (uint32_t)(b1 >> 32), __float_as_uint(u0), seqv};
            rec[2 * a + 1] = u32x4{(uint32_t)b2, (uint32_t)(b2 >> 32), __float_as_uint(nanf), seqv};
            if (a == 0) rec[2 * A] = u32x4{__float_as_uint(rho), __float_as_uint(eta), __float_as_uint(ess), seqv};
        }
    }
    FSTAMP(6);
    FSTAMPRT(14);
    if (!(MPPI_FIN_KO & 128)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // this block's slice of u_prev is complete (the wait above): count the step for an overlapped
    // rollout waiting on it (mppi_device.h kNoiseOverlap)
    if (xovl != nullptr && mode == 0 && lane == 0)
        __hip_atomic_fetch_add(xovl + ((size_t)v * A + a) * ts + sl, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Native dispatch's check of its one assumption (mppi_aql.cpp step_create): the dispatch id the
// waves receive is the packet's index in the engine's queue.  A tool that intercepts the queue
// (a profiler's counter packets) would break it, and with it the rollout's step counter.
extern "C" __global__ void __launch_bounds__(64) k_dispatch_probe(unsigned long long* out) {
    if (threadIdx.x == 0) out[0] = mppi_dispatch_id();
}

// The peer exchange's connection check (mppi_peer_probe phase 2): the finalize's own store and
// poll instructions over the mapped regions.  Lane d < n stores this rank's tagged word into rank
// d's region (word 0 of this rank's slot, parity 0), then lane r polls its own region for rank r's
// word until the tag matches or `ticks` (100 MHz) pass; out[r] = the word seen.
extern "C" __global__ void __launch_bounds__(64) k_peer_probe(unsigned long long* const* peers,
                                                              unsigned long long* local, int n, int me,
                                                              unsigned long long slot_words, uint32_t tag,
                                                              unsigned long long ticks,
                                                              unsigned long long* out) {
    const int lane = threadIdx.x;
    const unsigned long long w = ((unsigned long long)(tag | (uint32_t)me) << 32) | 0x3F800000ull;
    if (lane < n) __hip_atomic_store(peers[lane] + (size_t)me * slot_words, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    unsigned long long got = 0ull;
    if (lane < n) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        for (;;) {
            got = __hip_atomic_load(local + (size_t)lane * slot_words, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if ((uint32_t)(got >> 32) == (tag | (uint32_t)lane)) break;
            if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) break;
            __builtin_amdgcn_s_sleep(2);
        }
        out[lane] = got;
    }
}

extern "C" int mppi_launch_peer_probe(unsigned long long* const* peers, unsigned long long* local, int n, int me,
                                      unsigned long long slot_words, uint32_t tag, unsigned long long ticks,
                                      unsigned long long* out, void* stream) {
    hipLaunchKernelGGL(k_peer_probe, dim3(1), dim3(64), 0, (hipStream_t)stream, peers, local, n, me, slot_words, tag,
                       ticks, out);
    return (int)hipGetLastError();
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
    const int W = std::min(p->H, p->tsz + 2 * p->half);
    if (p->nrec > kMaxRec || p->nrec <= 0 || p->H > MPPI_MAX_HORIZON || p->tsz > 255 || p->half > 255 ||
        p->ts > 255 || p->A > 255 || W > 64 || !p->tail || p->hdr_vs > 0x7fffffff || p->d_vs > 0x7fffffff)
        return -1;
    const uint32_t nh = (uint32_t)p->nrec | ((uint32_t)p->H << 16);
    const uint32_t geo = (uint32_t)p->tsz | ((uint32_t)p->half << 8) | ((uint32_t)p->ts << 16) | ((uint32_t)p->A << 24);
    const int cw = (W <= 16) ? 16 : (W <= 32) ? 32 : 64;
    int nt = 512;
    for (int c : {128, 256})
        if (c * 16 / cw >= p->nrec) { nt = c; break; }
    const dim3 grid(8 * ((p->A + MPPI_FIN_XCDS - 1) / MPPI_FIN_XCDS) * p->ts, p->V), block(nt);   // XCD-aware map (k_finalize)
    hipStream_t s = (hipStream_t)stream;
#define MPPI_FIN_GO(CWV, WINV, NTV)                                                                       \
    return go(k_finalize<CWV, WINV, NTV>,                                                                 \
              [](char* b, size_t n) {                                                                     \
                  snprintf(b, n, "_Z10k_finalizeILi%dELi%dELi%dEEvPKfS1_PKN4mppi7FinTailEjjiiiiijNS2_9FinParamsE", \
                           CWV, WINV, NTV);                                                               \
              },                                                                                          \
              grid, block, 0, s, p->hdr, p->dat, p->tail, nh, geo, (int32_t)p->hdr_rs, (int32_t)p->d_rs,   \
              (int32_t)p->d_as, (int32_t)p->hdr_vs, (int32_t)p->d_vs, p->seq, *p)
#define MPPI_FIN_LAUNCH(CWV, WINV)                                                                        \
    do {                                                                                                  \
        if (nt == 128) MPPI_FIN_GO(CWV, WINV, 128);                                                       \
        else if (nt == 256) MPPI_FIN_GO(CWV, WINV, 256);                                                  \
        else MPPI_FIN_GO(CWV, WINV, 512);                                                                 \
    } while (0)
#define MPPI_FIN_WIN(CWV)                                                                                 \
    do {                                                                                                  \
        if (p->window == 9) MPPI_FIN_LAUNCH(CWV, 9);                                                      \
        else if (p->window == 5) MPPI_FIN_LAUNCH(CWV, 5);                                                 \
        else MPPI_FIN_LAUNCH(CWV, 0);                                                                     \
    } while (0)
    if (W <= 16) MPPI_FIN_WIN(16);
    else if (W <= 32) MPPI_FIN_WIN(32);
    else MPPI_FIN_WIN(64);
#undef MPPI_FIN_WIN
#undef MPPI_FIN_LAUNCH
#undef MPPI_FIN_GO
    return -1;
}

#ifdef MPPI_PROBE
__global__ void __launch_bounds__(256) k_boundary(float* scratch) {
    if (blockIdx.x == 0 && threadIdx.x == 0) scratch[0] = 0.0f;
}
extern "C" int mppi_launch_boundary(float* scratch, int blocks, void* stream) {
    hipLaunchKernelGGL(k_boundary, dim3(blocks), dim3(256), 0, (hipStream_t)stream, scratch);
    return (int)hipGetLastError();
}
#endif

extern "C" int mppi_launch_weights(const float* S, const float* stats, float* w, int V, int K, float coef,
                                   void* stream) {
    const int n = V * K;
    hipLaunchKernelGGL(k_weights, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, S, stats, w, V,
                       K, coef);
    return (int)hipGetLastError();
}

// mppi_step.cpp -- the control step of libmppi_hip.so (include/mppi_hip.h): the rollout and
// finalize launches on the engine's stream, the tagged output records and their wait, mppi_step /
// mppi_run_steps, and the native dispatch of both (raw AQL packets, mppi_aql.cpp).  See
// mppi_engine.h for the file map and DESIGN.md §2 for the dispatch and completion protocols.
#include <emmintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "mppi_engine.h"

using namespace mppi;

namespace mppi_host {

// the rollout's per-block partial records (DevParams::hdr / rdata layout)
void block_records(const mppi_engine* e, FinParams& f) {
    const int64_t nb = e->dp.nb, H = e->H;
    f.nrec = (int32_t)nb;
    f.hdr = e->d_hdr; f.hdr_vs = nb * 4; f.hdr_rs = 4;
    f.dat = e->d_rdata; f.d_vs = (int64_t)e->A * nb * H; f.d_as = nb * H; f.d_rs = H;
}

// The finalize's record source: the rollout blocks' records, or the exchange slots of a shard.
void final_records(const mppi_engine* e, FinParams& f) {
    if (sharded(e)) {   // slots [shard][v][P]: header then N[a][t]
        const int64_t P = e->dp.P;
        f.nrec = e->cfg.shard_count;
        f.hdr = e->d_exchange; f.hdr_vs = P; f.hdr_rs = (int64_t)e->V * P;
        f.dat = e->d_exchange + kHdr; f.d_vs = P; f.d_as = e->H; f.d_rs = (int64_t)e->V * P;
    } else {
        block_records(e, f);
    }
}

}  // namespace mppi_host

using namespace mppi_host;

extern "C" {

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
constexpr int32_t kNoiseOverlap = 0x200;      // = mppi_device.h

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
    const bool ovl = e->overlap && n > 1;   // (experiment, MPPI_OVERLAP=1)
    if (ovl) p.noise_mode |= kNoiseOverlap;
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
    if (pr == 0 && ovl) {   // every finalize block's counter at the batch's first step (queue drained:
                            // step_prepare above waited for it or found it idle)
        HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)e->d_ovl, (int)e->step_ctr, (size_t)e->V * e->A * e->fin_ts,
                                  e->stream));
        HIP_TRY(hipStreamSynchronize(e->stream));
    }
    if (pr != 0 || mppi_aql::step_dispatch(e->aql, n, &err, ovl) != 0)
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

// Diagnostic (not part of the public header): mppi_aql step_touch on the engine's own queue
// (tools/probes.py rate_split).  Same thread as the control calls.
int32_t mppi_debug_queue_touch(mppi_engine* e) {
    if (!e || !e->aql) return MPPI_ERR_INVALID_ARG;
    std::string err;
    const int r = mppi_aql::step_touch(e->aql, false, &err);
    return r == 0 ? MPPI_OK : fail(MPPI_ERR_HIP, "queue touch: %s", err.c_str());
}


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

// Diagnostic: mppi_aql step_ring (the doorbell again, no packet).  Refused while the prewarm thread
// runs: step_ring must come from the thread that writes the packets (mppi_aql.h).
int32_t mppi_debug_queue_ring(mppi_engine* e) {
    if (!e || !e->aql) return MPPI_ERR_INVALID_ARG;
    if (e->pw_us.load()) return fail(MPPI_ERR_STATE, "mppi_debug_queue_ring: the prewarm thread also writes packets");
    mppi_aql::step_ring(e->aql);
    return MPPI_OK;
}

}  // extern "C"

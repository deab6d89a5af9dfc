// mppi_engine.cpp -- the engine object of libmppi_hip.so (include/mppi_hip.h): create / destroy
// (device buffers allocated once, no allocation in a step), the per-vehicle constants baked the way
// the reference builds its tensors, state / target / warm-start uploads, readbacks and kernel
// timing.  The control step itself is mppi_step.cpp; see mppi_engine.h for the file map and
// DESIGN.md for the data layout.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "mppi_engine.h"

using namespace mppi;

namespace mppi_host {

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
    t.xstall = f.xstall; t.xovl = f.xovl; t.xdec = f.xdec;
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
            base_from_xyzquat(s, c.state_f64 != 0, T16);
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

}  // namespace mppi_host

using namespace mppi_host;

extern "C" {

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
    // experiment (MPPI_OVERLAP=1): overlapped native batches; k_rollout only (k_rollout_quad does not wait)
    e->overlap = getenv("MPPI_OVERLAP") && atoi(getenv("MPPI_OVERLAP")) != 0 && c.model != MPPI_MODEL_QUADROTOR;
    if (e->overlap) {
        const size_t n = (size_t)e->V * e->A * e->fin_ts;
        if (hipMalloc(&e->d_ovl, n * sizeof(uint32_t)) != hipSuccess || hipMemset(e->d_ovl, 0, n * sizeof(uint32_t)) != hipSuccess) {
            fail(MPPI_ERR_HIP, "overlap counters");
            mppi_destroy(e);
            return MPPI_ERR_HIP;
        }
        f.xovl = e->d_ovl;
        p.ovl = e->d_ovl;
        p.ovl_n = e->A * e->fin_ts;
    }
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
    exchange_release(e);   // the communicator and the other ranks' mapped regions
    void* dev[] = {e->d_xregion, e->d_xpeers, e->d_sigma, e->d_joints, e->d_vc, e->d_u_prev, e->d_noise_in, e->d_traj, e->d_noise_out,
                   e->d_S, e->d_hdr, e->d_rdata, e->d_out, e->d_wraw, e->d_wsmooth, e->d_w,
                   e->d_sinv, e->d_gamma, e->d_jtraj, e->d_xown, e->d_tail, e->d_stamps, e->d_fstamps, e->d_xstall, e->d_ovl, e->d_xdec};
    for (void* p : dev) if (p) (void)hipFree(p);
    if (e->h_out) (void)hipHostFree(e->h_out);
    if (e->h_vc) (void)hipHostFree(e->h_vc);
    if (e->ev_vc) (void)hipEventDestroy(e->ev_vc);
    if (e->ev_out) (void)hipEventDestroy(e->ev_out);
    if (e->own_stream) (void)hipStreamDestroy(e->own_stream);
    delete e;
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

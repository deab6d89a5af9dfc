// mppi_dev.h -- structures shared by the host C-ABI (mppi_engine.h and its .cpp units) and the
// gfx950 kernels (mppi_kernels.hip).  Internal: not part of the public ABI.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "../../include/mppi_hip.h"

namespace mppi {

constexpr int kMaxA = MPPI_MAX_ACTION;
constexpr int kMaxJ = MPPI_MAX_JOINTS;
constexpr int kMaxW = MPPI_MAX_SAVGOL;
constexpr int kHdr = 4;  // partial record header: rho, eta, eta2, pad
// k_rollout stages a block's costs (iters x waves x rollouts per wave consecutive samples) in LDS
// for one write-through store run; create keeps the run within this many floats (16 KB)
constexpr int kMaxCostRun = 4096;
// one group's run of costs in that stage (nS = waves x rollouts per wave floats), padded to 16 B
// so every run starts 16 B aligned for st_dev_run's b128 LDS reads
constexpr inline int cost_run_stride(int nS) { return (nS + 3) & ~3; }

// One joint of the chain, pre-baked on the host exactly the way the reference
// builds its tensors (transformation_matrix.py:28-35, 58-95).
struct JointDev {
    int32_t type;      // mppi_joint_type
    int32_t q_index;   // -1 = not actuated
    int32_t axis_z;    // 1 if the unit axis is exactly (0,0,1): fast Rodrigues
    int32_t _pad;
    float O[12];       // origin transform rows 0..2 (3x4, row-major), fp32 as torch builds it
    float ax[3];       // unit axis (fp32, axis / ||axis||)
    float axx[9];      // fl(a_i * a_j) products as the reference evaluates vx*vx etc.
};

// Per-vehicle constants derived on the host from state + target (uploaded with
// every mppi_set_state; everything the rollout needs that is uniform per vehicle).
struct VehicleConst {
    double pos0[kMaxA];   // initial positions per action dim (drone xyz / joints / both)
    double vel0[kMaxA];   // initial velocities
    float pos0f[kMaxA];   // fp32 copies (f32 state mode)
    float vel0f[kMaxA];
    float base[12];       // ARM: fp32 base transform (urdf_fk.py:30-55) times the leading fixed
                          //      joints of the chain, rows 0..2
                          // WB : R(rpy(quat)) (transformation_matrix.py:148-187) times the leading
                          //      fixed joints; column 3 = R * (their translation), p(k,t) is added
    float tpos[3];        // target position
    float tR[9];          // target rotation (quaternion_to_matrix, xyzw)
    float _pad[4];        // [0]: a native control call's sequence number (bits; k_finalize, kSeqFromVc);
                          // [1]: the step's Philox counter (written by the rollout, kVcStepWord);
                          // [2]: the peer exchange's epoch (host-set, kVcEpochWord)
    float qc[kMaxJ];      // extra cost terms (mppi_config): centering target and joint limits
    float qlo[kMaxJ];     //   per arm joint (the same for every vehicle)
    float qhi[kMaxJ];     // sizeof = 688 (16-byte multiple: keeps the dynamic LDS base aligned)
};
static_assert(sizeof(VehicleConst) % 16 == 0, "VehicleConst must be a 16-byte multiple");

// Kinova j2s7s300 fast path (aerial_manipulator_gpu.urdf:100-365): every joint
// origin rotation of joints 1..7 is a signed permutation -- rpy in {0, +-pi/2, pi};
// the reference's float32 residuals (sin(pi) = -8.7e-8, cos(pi/2) = -4.4e-8) are
// dropped.  Column j of T*O is s[j] * column p[j] of T; tmask
// marks the nonzero translation components (1 x, 2 y, 4 z).  The host enables
// the path only when the baked chain matches this table exactly.
struct KinOrigin { int p[3]; int s[3]; int tmask; };
constexpr KinOrigin kKinova[7] = {
    {{0, 1, 2}, {-1, 1, -1}, 4},    // joint_1: rpy (0, pi, 0),       xyz (0, 0, .15675)
    {{0, 2, 1}, {-1, -1, -1}, 6},   // joint_2: rpy (-pi/2, 0, pi),   xyz (0, .0016, -.11875)
    {{0, 2, 1}, {1, -1, 1}, 2},     // joint_3: rpy (-pi/2, 0, 0),    xyz (0, -.205, 0)
    {{0, 2, 1}, {-1, 1, 1}, 4},     // joint_4: rpy (pi/2, 0, pi),    xyz (0, 0, -.205)
    {{0, 2, 1}, {-1, -1, -1}, 6},   // joint_5: rpy (-pi/2, 0, pi),   xyz (0, .2073, -.0114)
    {{0, 2, 1}, {-1, 1, 1}, 4},     // joint_6: rpy (pi/2, 0, pi),    xyz (0, 0, -.10375)
    {{0, 2, 1}, {-1, -1, -1}, 2},   // joint_7: rpy (-pi/2, 0, pi),   xyz (0, .10375, 0)
};

struct DevParams {
    int32_t model, V, K, H, A;
    int32_t L;          // lanes per rollout segment (pow2 >= H, <= 64)
    int32_t R;          // rollouts per wave = 64 / L
    int32_t nch;        // 64-lane chunks per rollout when H > 64 (else 1)
    int32_t nb;         // rollout blocks per vehicle
    int32_t iters;      // rollout groups per block
    int32_t nq;         // arm joints (0 for drone)
    int32_t qoff;       // first arm dim in the action vector (0 arm, 3 whole-body)
    int32_t nj;         // joints in the chain
    int32_t noise_mode, state_f64, store_traj, store_noise;
    int32_t sigma_diag;
    int32_t j0;         // first chain joint not folded into VehicleConst::base
    int32_t chain_fast; // 1: joints j0.. are nq revolute-z joints with q_index 0..nq-1 in order;
                        // 2: additionally the Kinova origin table kKinova
    int32_t P;          // floats per partial record (kHdr + A*H, rounded up to 4)
    int32_t C;          // stored trajectory channels (EE as 12)
    int32_t hp;         // trajectory row pitch in floats, 64 B rows: H rounded up to 16 (k_rollout),
                        // K rounded up to 16 (k_rollout_quad, t-major planes)
    uint32_t seed_lo, seed_hi;
    int64_t k_offset;   // global index of this shard's first sample
    float dt, dt2;      // fp32(dt), fp32(dt**2)
    double dt_d;        // dt as double (fp64-promoted path)
    float coef;         // fp32(-1/lambda)
    float w_sp, w_so, w_tp, w_to;
    float sdiag[kMaxA];      // diagonal of Sigma (sigma_diag)
    VehicleConst vc0;        // vehicle 0 constants by value (V == 1: no upload per step; block 0
                             // stores them to vc[0] for the finalize)
    // device pointers
    const JointDev* joints;  // (kMaxJ) chain table, written once at create (L2-resident)
    const float* sigma;      // (A,A) full Sigma
    const VehicleConst* vc;  // (V) when V > 1
    const float* u_prev;     // (V,H,A)
    const float* noise_in;   // (V,K,H,A) injected
    uint32_t step_ctr;       // control-step index: the Philox counter word (host-counted)
    float* traj;             // (V,C,K,hp) SoA planes (QUADROTOR: (V,C,H,hp))
    float* noise_out;        // (V,K,H,A)
    float* S;                // (V,K)
    float* hdr;              // (V,nb,4) partial record headers: rho, eta, eta2, nan
    float* rdata;            // (V,A,nb,H) partial record bodies, dim-major
    unsigned long long* stamps;   // diagnostic s_memtime stamps per wave (MPPI_STAMPS), else null
    // extra CostManager terms (mppi_config.cost_terms; cost_manager.py:83-87)
    int32_t cost_terms;
    float w_cov;                  // fp32(w_covar * lambda * (1 - alpha)) (covar_cost.py:24)
    float w_cen, w_jt, w_act, lim_pen;
    const float* sinv;            // (A,A) Sigma^-1, fp32
    const float* gamma_t;         // (H) fp32 gamma^t
    const float* jtraj;           // (V,H,nq) joint tracking target
    // QUADROTOR rigid body (mppi_config.quad_*): fp32 as the reference's tensors
    float q_inv_m;                // fp32(1 / mass) (the Python-float 1/self.m of drone_mppi.py:68)
    float q_iinv[3];              // fp32(1 / I_ii), diagonal inertia
    float q_kd;                   // linear drag
    float q_g;                    // gravity magnitude, g = (0, 0, -q_g)
    int32_t q_literal_jinv;       // t >= 1 applies inv(J) to the body rates, as the commented loop
                                  // (drone_mppi.py:73-76); 0 = J at every step
    // overlapped native batches (kNoiseOverlap, MPPI_OVERLAP=1): the finalize blocks' step counters,
    // (V, A, ts) words each incremented once per FINAL (FinTail::xovl), and their count per vehicle
    const uint32_t* ovl;
    int32_t ovl_n;
};
constexpr int kStamps = 16;

// The finalize tail's parameters, device-resident: written once at create (one copy per
// launch kind), read by k_finalize through a preloaded pointer.  Read from the kernel
// arguments they were cold s_loads every launch (the host writes a fresh kernel-argument
// block per launch): ~1.1 us of the C3 finalize (profiles/r02/ab_finalize_tail_params.txt).
struct FinTail {
    float coef, dt, dt2;
    int32_t mode, model, qoff, nq, state_f64, out_dim, window;
    float* u_prev;           // (V,H,A) in/out
    const VehicleConst* vc;  // (V)
    double* out;
    float* u0;
    float* stats;
    uint32_t* flags;
    float* wraw;
    float* wsmooth;
    float* dst;              // PACK: this shard's slot, the exchange base, slot stride, count, own slot
    float* xbase;
    int64_t xslot;
    int32_t nslots, myslot, P, pad_;
    unsigned long long* const* xpeers;   // peer exchange (mppi_peer_connect): every rank's region, null = off
    unsigned long long* xlocal;          //   this rank's region (the ranks' partials are gathered from it)
    int32_t xn, xme;                     //   rank count, this rank
    uint32_t* xerr;                      //   sticky timeout word, then the torn word (mapped host memory;
                                         //   read on the late path only)
    uint32_t* xstall;                    //   diagnostics (mppi_debug_peer_stall): a block's stall, null = none
    uint32_t* xovl;                      // (V, A, ts) step counters for overlapped batches (MPPI_OVERLAP), null = off
    unsigned long long* xdec;            // peer exchange: the rank's commit marks (2 parities x blocks)
    float sg[kMaxW];
};
// FINAL (the step's finalize), PACK (a shard's slot), SCRATCH (FINAL into device scratch outputs:
// timing, probes), READBACK (mppi_get_weighted_noise: w_eps and its SavGol of the records as they
// stand, nothing else written)
enum { kTailFinal = 0, kTailPack = 1, kTailScratch = 2, kTailReadback = 3, kTailSlots = 4 };

// Peer exchange of a sharded V == 1 engine (mppi_exchange.cpp mppi_peer_open / mppi_peer_connect):
// every k_finalize block pushes its partial -- header (rho, eta, eta2, nan) and its window's
// columns N[t] -- into every rank's exchange region, and gathers the ranks' partials of the same
// block from its own.  Each word is 8 B, (value bits, tag): one store carries its own validity,
// so nothing is ordered against anything else.  Region: [kXCtl control words] then [2 step
// parities][ranks][V*grid.x blocks][kXW words]; the ranks' region pointers (FinTail::xpeers,
// xlocal) point past the control words.  Control word r is rank r's timeout report: any of its
// finalize blocks that gives up a step stores (tag, 1) there in EVERY rank's region, and from then
// on every rank's blocks find it in their own region and keep the warm start at once ("broken"
// until the host resets the exchange, mppi_peer_reset): no rank goes on updating a warm start the
// others did not.
// The tag (peer_tag) is bit 31 | the exchange epoch (10 bits) | the step's Philox counter (low 20
// bits).  The rollout's block 0 hands the counter to the finalize in the vehicle constants (word
// kVcStepWord); the host puts the epoch there (kVcEpochWord; mppi_set_step_counter and
// mppi_peer_reset move it), so words a rank left in a region before its counter was rewound can
// never pass for a later step's.  A block that gives a step up leaves the peers' words where they
// are (a peer block on a rank that committed may still need them, below): the report alone tells
// a peer still polling that step to give it up too.
// All or nothing within a rank: the blocks of one step either all update their slices of u_prev
// or all keep them.  A block commits only when its peers' words all arrived within the bound AND
// its final poll round saw no timeout report; it then stores (tag << 32) | kDecCommit into its own
// commit mark for the step's parity (FinTail::xdec: 2 x blocks words of plain device memory, written
// and read at device scope like u_prev; one word per block, as 80 stores into one word serialise)
// and updates its slice without waiting for anything.  A
// late block (bound passed, or a report seen) reports first -- into every region, its own included,
// so no block of its rank can commit after the report lands -- waits kDecGraceTicks (by then any
// block whose final round came before the report has stored its mark: the store is issued right
// after that round and lands within microseconds), and reads the rank's marks: if one is this
// step's (marks carry the tag, so earlier steps' never match), the
// late block keeps polling its peers for a second bound (reports no longer heeded: the peers' words
// stay in place) and completes; if not, the step is given up (every block of the rank is late or
// holds).  Only if the second bound passes too is the rank's warm start torn (that slice kept, the
// others updated): the block writes the step's tag into the torn word next to the sticky word, and
// the resync takes its warm start from a rank that is not torn.
constexpr int kMaxPeers = 8;
constexpr int kXW = kHdr + 64;   // header + the widest window (CW <= 64)
constexpr int kXCtl = 16;        // control words at the head of a region (8 B each; kMaxPeers timeout reports)
constexpr uint32_t kDecCommit = 1u;
constexpr uint64_t kDecGraceTicks = 10000ull;   // 100 us (s_memrealtime, 100 MHz)
constexpr int kVcStepWord = (int)(offsetof(VehicleConst, _pad) / 4) + 1;
constexpr int kVcEpochWord = kVcStepWord + 1;
constexpr uint32_t kTagValid = 0x80000000u;
// (constexpr: usable from host and device code alike)
constexpr inline uint32_t peer_tag(uint32_t step, uint32_t epoch) {
    return kTagValid | ((epoch & 0x3FFu) << 20) | (step & 0xFFFFFu);
}
// a finalize block waits at most this long for its peers' partials (s_memrealtime, 100 MHz), then
// finalises with the nan flag set (2): a rank that stopped stepping cannot hang the others
constexpr uint64_t kPeerWaitTicks = 200000000ull;   // 2 s
// k_finalize's sequence argument: this value = take the step's sequence number from the vehicle
// constants (VehicleConst::_pad[0]; native control calls, mppi_aql.cpp).  HIP-path sequence
// numbers stay below 2^31, native ones have bit 31 set: the two never meet in the flags.
constexpr uint32_t kSeqFromVc = 0xFFFFFFFFu;

// A kernel launch as data (mppi_aql.cpp): while a LaunchDesc is installed for the calling
// thread (mppi_capture_target), the launchers fill it in instead of launching through HIP --
// the kernel's symbol, grid, block, dynamic LDS and its argument block laid out as the
// kernel-argument segment (each argument at its natural alignment, as the code object's
// metadata lists them).
struct LaunchDesc {
    char symbol[192];
    uint32_t grid[3];        // blocks per dimension
    uint32_t block[3];       // threads per block
    uint32_t lds;            // dynamic LDS bytes
    uint32_t arg_bytes;
    alignas(16) unsigned char args[2048];
};

// Finalize / pack kernel parameters.
struct FinParams {
    int32_t model, V, H, A, nq, qoff, state_f64;
    int32_t nrec;            // records to combine per vehicle
    int32_t ts, tsz;         // t-slices per action dim (grid.x = A*ts), slice length
    const float* hdr;        // record headers (rho, eta, eta2, nan) at hdr + v*hdr_vs + r*hdr_rs
    int64_t hdr_vs, hdr_rs;
    const float* dat;        // record bodies N[a][t] at dat + v*d_vs + a*d_as + r*d_rs + t
    int64_t d_vs, d_as, d_rs;
    int32_t P;
    int32_t mode;            // 0 = final, 1 = pack into dst slot
    int32_t window, half;
    float coef, dt, dt2;
    double dt_d;
    float sg[kMaxW];         // SavGol taps (already flipped for the correlation)
    float* dst;              // pack destination (slot base, vehicle stride P)
    float* xbase;            // pack: exchange buffer base; the other shards' slots are zeroed at
    int64_t xslot;           //   the same positions (slot stride xslot floats), so the SUM
    int32_t nslots, myslot;  //   all-reduce needs no memset first
    unsigned long long* const* xpeers;   // peer exchange (FinTail): the ranks' regions, this rank's,
    unsigned long long* xlocal;          //   rank count, this rank; xpeers null = off
    int32_t xn, xme;
    uint32_t* xerr;                      //   sticky timeout word, torn word (mapped host memory)
    uint32_t* xstall;                    //   diagnostics: a block's stall (mppi_debug_peer_stall), null = none
    uint32_t* xovl;                      // step counters for overlapped batches (FinTail::xovl), null = off
    unsigned long long* xdec;            // peer exchange: the rank's commit marks (FinTail::xdec)
    float* u_prev;           // (V,H,A) in/out
    const VehicleConst* vc;  // (V); for V == 1 written by the rollout from its kernel arguments
    double* out;             // (V, out_dim)   -- mapped pinned host memory (zero-copy)
    float* u0;               // (V, A)         -- "
    float* stats;            // (V, 4): rho, eta, ess, nonfinite -- "
    uint32_t* flags;         // (V, A) completion flags      -- " (seq stored after the outputs)
    uint32_t seq;            // this step's completion-flag value (never 0)
    float* wraw;             // (V,H,A) readback
    float* wsmooth;          // (V,H,A) readback
    int32_t out_dim;
    int32_t dbg;             // diagnostic phase-skip bits (MPPI_FIN_DEBUG), 0 in production
    unsigned long long* stamps;   // diagnostic s_memtime stamps (MPPI_STAMPS), else null
    const FinTail* tail;     // device copy of this launch kind's tail parameters
};

}  // namespace mppi

// launchers (mppi_kernels.hip)
extern "C" {
int mppi_launch_rollout(const mppi::DevParams* p, int block_threads, void* stream);
int mppi_launch_rollout_arm64(const mppi::DevParams* p, int block_threads, void* stream);
int mppi_launch_rollout_arm64_h32(const mppi::DevParams* p, int block_threads, void* stream);
int mppi_launch_rollout_arm32(const mppi::DevParams* p, int block_threads, void* stream);
int mppi_launch_rollout_wb(const mppi::DevParams* p, int block_threads, void* stream);
int mppi_launch_rollout_quad(const mppi::DevParams* p, int block_threads, void* stream);
int mppi_launch_finalize(const mppi::FinParams* p, void* stream);
int mppi_launch_peer_probe(unsigned long long* const* peers, unsigned long long* local, int n, int me,
                           unsigned long long slot_words, uint32_t tag, unsigned long long ticks,
                           unsigned long long* out, void* stream);
int mppi_launch_weights(const float* S, const float* stats, float* w, int V, int K, float coef,
                        void* stream);
int mppi_launch_philox(uint64_t seed, uint32_t step, int vehicle, int64_t k0, int K, int H, int A,
                       float* z, uint32_t* raw, void* stream);
// the calling thread's capture target (null: launch through HIP); mppi_aql.cpp
mppi::LaunchDesc* mppi_capture_target(void);
}

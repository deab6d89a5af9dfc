/*
 * mppi_hip.h -- C-ABI of the MI355X-native MPPI rollout engine (libmppi_hip.so).
 *
 * Drop-in boundary for the mav_mppi control step.  The
 * reference has no native FFI: its hot path is the Python methods below, and a
 * host binding (ctypes, quadrotor_manipulator_mppi_amd/_capi.py) replaces the
 * torch op sequence each entry point stands for:
 *
 *   mppi_create         <- MPPI.__init__            mppi_solver/mppi.py:28-93,
 *                                                   mppi_solver/drone_mppi.py:8-37
 *   mppi_set_state      <- MPPI.update_joint        mppi.py:196-200 (arm),
 *                          MPPI.set_state           drone_mppi.py:179-183 (drone)
 *   mppi_set_target     <- target_pose / target     mppi.py:70-72, drone_mppi.py:141
 *   mppi_rollout        <- sampling + rollout + FK + cost + softmin partials
 *                          mppi.py:129-143 / drone_mppi.py:142-156
 *                          (standard_normal_noise.py:22-50, urdf_fk.py:79-108,
 *                           urdfparser.py:122-163, pose_cost.py:24-63)
 *   mppi_finalize       <- weighted noise + SavGol + control update
 *                          mppi.py:144-158 / drone_mppi.py:157-169
 *                          (mppi.py:173-193, svg_filter.py:13-90)
 *   mppi_read_outputs   <- the (qdes, vdes) / (x, v) returned by
 *                          compute_control_input (mppi.py:161-169 incl. the
 *                          check_reach host FK at :95-120; drone_mppi.py:175)
 *   mppi_step           <- MPPI.compute_control_input as one call
 *   mppi_get_*          <- the reference's intermediate tensors (noise,
 *                          q_samples/trajectory, S, weights, w_eps, u_prev),
 *                          returned in the reference's own layouts
 *
 * Conventions: plain pointers and sizes, no torch types.  Host pointers unless
 * a name says d_ (device).  Every call returns mppi_status (0 = ok); on error
 * mppi_last_error() returns a thread-local message.  Calls on one engine must be
 * serialised by the caller (the Python wrapper holds a lock).
 */
#ifndef MPPI_HIP_H
#define MPPI_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPPI_ABI_VERSION 9
#define MPPI_COMM_ID_BYTES 128  /* ncclUniqueId */
#define MPPI_PEER_HANDLE_BYTES 64  /* hipIpcMemHandle_t */
#define MPPI_MAX_ACTION 16
#define MPPI_MAX_JOINTS 16
#define MPPI_MAX_HORIZON 256
#define MPPI_MAX_SAVGOL 31

typedef enum {
    MPPI_OK = 0,
    MPPI_ERR_INVALID_ARG = -1,
    MPPI_ERR_HIP = -2,
    MPPI_ERR_NONFINITE = -3,
    MPPI_ERR_STATE = -4,
    MPPI_ERR_COMM = -5,
    MPPI_ERR_PEER_TIMEOUT = -6  /* mppi_synchronize: a peer-exchange step was given up since the last
                                   mppi_peer_reset (the engine itself is fine; see mppi_peer_status) */
} mppi_status;

/* Rollout models.  A = action dimension. */
typedef enum {
    MPPI_MODEL_DRONE = 0,     /* xyz double integrator, squared position cost      (A=3)  drone_mppi.py   */
    MPPI_MODEL_ARM = 1,       /* joint double integrator + FK chain + pose cost    (A=nq) mppi.py         */
    MPPI_MODEL_WHOLEBODY = 2, /* drone xyz + arm joints, mobile-base FK, pose cost (A=3+nq) SURVEY A16    */
    MPPI_MODEL_QUADROTOR = 3  /* 6-DoF rigid-body quadrotor: thrust + body torques, Euler-angle attitude,
                               * squared position cost (A=4, H <= 64).  The model the reference ships
                               * commented out (drone_mppi.py:57-83, drone.py:114-154) */
} mppi_model;

typedef enum {
    MPPI_NOISE_PHILOX = 0,    /* device counter-based Philox4x32-10 + Box-Muller (production)          */
    MPPI_NOISE_INJECTED = 1   /* caller supplies eps (K,H,A) per step (parity: reference randn noise)  */
} mppi_noise_mode;

typedef enum {
    MPPI_JOINT_FIXED = 0,
    MPPI_JOINT_REVOLUTE = 1,
    MPPI_JOINT_PRISMATIC = 2,
    MPPI_JOINT_FLOATING = 3   /* free-flyer root of the dynamics model only (mppi_link)            */
} mppi_joint_type;

/* One entry of the active joint chain (urdfparser.py:133-161). xyz/rpy/axis as
 * the URDF floats (rounded to fp32 like torch.tensor(jt.origin.xyz)). */
typedef struct {
    int32_t type;       /* mppi_joint_type                                   */
    int32_t q_index;    /* index into the arm joint vector, -1 if not actuated */
    float xyz[3];
    float rpy[3];
    float axis[3];      /* raw URDF axis; normalised like transformation_matrix.py:63-66 */
    int32_t has_axis;   /* 0 -> (1,0,0) as urdfparser.py:140-143              */
} mppi_joint;

typedef struct {
    int32_t model;            /* mppi_model                                                     */
    int32_t n_vehicles;       /* V independent controllers batched in one launch (config C5)    */
    int32_t n_samples;        /* K samples owned by THIS engine (one shard)                      */
    int32_t n_horizon;        /* H                                                              */
    int32_t n_action;         /* A (3 drone, nq arm, 3+nq whole-body)                           */
    double dt;                /* 0.01 (mppi.py:42, drone_mppi.py:18); a Python float there       */
    double lambda_;           /* 0.1  (mppi.py:75, drone_mppi.py:33)                             */
    float sigma[MPPI_MAX_ACTION * MPPI_MAX_ACTION]; /* Sigma (A x A, row-major), eps = z^T Sigma */
    /* cost weights: pose (stage pos, stage ori, terminal pos, terminal ori) = 50,30,40,30
     * (cost_manager.py:25-28); drone uses w_stage_pos=100, w_term_pos=20 (drone_mppi.py:92,104) */
    float w_stage_pos, w_stage_ori, w_term_pos, w_term_ori;
    int32_t n_joints;
    mppi_joint joints[MPPI_MAX_JOINTS];
    int32_t savgol_window;    /* 5 drone, 9 arm (drone_mppi.py:160, mppi.py:149)                */
    int32_t savgol_order;     /* 2                                                              */
    int32_t noise_mode;       /* mppi_noise_mode                                                */
    uint64_t seed;            /* Philox key                                                     */
    int32_t device;           /* HIP device ordinal                                             */
    int32_t shard_rank;       /* sample sharding: this engine owns global samples               */
    int32_t shard_count;      /*   [rank*K, (rank+1)*K); partials exchanged by the caller       */
    int32_t state_f64;        /* reproduce the reference's fp64 promotion of an fp64 arm state  */
    int32_t store_trajectory; /* write the trajectory buffer (q / p and EE 3x4 per (k,t))       */
    int32_t store_noise;      /* write eps (K,H,A) (debug / parity readback)                    */
    int32_t check_reach;      /* host FK at qdes, L1 position error < reach_tol (mppi.py:95-120)*/
    float reach_tol;          /* 0.005                                                          */
    int32_t blocks_per_vehicle; /* rollout grid.x; 0 = auto                                     */
    int32_t block_threads;      /* rollout block size (multiple of 64); 0 = auto                */
    /* The CostManager terms the reference ships disabled (cost_manager.py:83-87), for the
     * ARM and WHOLEBODY models; summed after the pose terms in the reference's order
     * (covar, centering, joint tracking, action, joint limit).  Defaults = the reference's
     * weights (cost_manager.py:21-43, joint_space_cost.py:16,71-80). */
    int32_t cost_terms;         /* MPPI_COST_* bits; 0 = pose cost only, as the reference runs  */
    float w_covar;              /* covar_cost.py:20-25, scaled by lambda*(1-alpha)      (0.1)   */
    float cost_alpha;           /* cost_manager.py:22                                   (0.1)   */
    float cost_gamma;           /* per-step discount gamma^t of the joint/action terms  (0.98)  */
    float w_center;             /* joint_space_cost.py:19-27                            (1.0)   */
    float w_joint_track;        /* joint_space_cost.py:30-38 (target: mppi_set_joint_trajectory; zeros as mppi.py:134) */
    float w_action;             /* action_cost.py:14-24 on the perturbed controls v     (0.01)  */
    float joint_limit_penalty;  /* joint_space_cost.py:68-86                            (1e10)  */
    float q_center[MPPI_MAX_JOINTS];   /* centering target per arm joint                         */
    float q_lower[MPPI_MAX_JOINTS];    /* joint limits                                           */
    float q_upper[MPPI_MAX_JOINTS];
    /* MPPI_MODEL_QUADROTOR rigid body (drone.urdf:15-16; g and kd are undefined in the
     * commented reference loop, drone_mppi.py:64-79): */
    float quad_mass;            /* 14.7 kg                                                      */
    float quad_inertia[3];      /* diagonal body inertia 1.57, 3.93, 2.59                       */
    float quad_kd;              /* linear drag coefficient kd (0)                               */
    float quad_gravity;         /* g = (0, 0, -quad_gravity), 9.81                              */
    int32_t quad_literal_jinv;  /* 1: steps t >= 1 integrate rpy += dt inv(J(rpy)) omega exactly as
                                 * the commented loop (drone_mppi.py:73-76); 0 (default): J at
                                 * every step (J maps body rates to Euler rates, drone.py:114-124) */
    int32_t vehicle_offset;     /* fleet-wide index of this engine's vehicle 0 (vehicle sharding, config C5:
                                 * each GPU runs V of the fleet's vehicles).  The device noise is keyed by
                                 * the fleet-wide index, so an engine over vehicles [o, o+V) draws exactly
                                 * what one engine over the whole fleet draws for them.  0..32767-V */
} mppi_config;

typedef enum {
    MPPI_COST_COVAR = 1,
    MPPI_COST_CENTER = 2,
    MPPI_COST_JOINT_TRACK = 4,
    MPPI_COST_ACTION = 8,
    MPPI_COST_JOINT_LIMIT = 16
} mppi_cost_term;

/* Per-vehicle statistics of the last finalised step. */
typedef struct {
    float rho;          /* min_k S_k                                        */
    float eta;          /* sum_k exp(-(S_k - rho)/lambda)                   */
    float ess;          /* effective sample size 1 / sum_k w_k^2            */
    int32_t nonfinite;  /* 1 if rho/eta/u is not finite (reference propagates NaN); 2 if a
                           peer-exchange step gave up waiting for another rank (u_prev kept) */
    int32_t reach;      /* check_reach result (arm / whole-body)            */
    int32_t _pad;
} mppi_stats;

typedef struct mppi_engine mppi_engine;

int32_t mppi_abi_version(void);
const char* mppi_last_error(void);
/* sizeof(mppi_config), sizeof(mppi_joint), sizeof(mppi_stats): lets a binding check its layout. */
void mppi_struct_sizes(int32_t* config, int32_t* joint, int32_t* stats);

/* Reference defaults for a model (drone: K=1000 H=32 sigma=30I; arm: K=100 H=32
 * sigma=0.1I, Kinova chain must still be filled in by the caller). */
void mppi_config_default(mppi_config* cfg, int32_t model);

/* Sizes of the packed host-side state / output rows for a config. */
int32_t mppi_state_dim(const mppi_config* cfg);   /* doubles per vehicle  */
int32_t mppi_output_dim(const mppi_config* cfg);  /* doubles per vehicle  */
int32_t mppi_traj_channels(const mppi_config* cfg);

mppi_status mppi_create(const mppi_config* cfg, mppi_engine** out);
void mppi_destroy(mppi_engine* e);

/* Run on a caller stream (hipStream_t cast to void*); NULL = engine-owned stream. */
mppi_status mppi_set_stream(mppi_engine* e, void* hip_stream);

/* Joint-space tracking target of MPPI_COST_JOINT_TRACK per vehicle: (H, nq) fp32, the
 * joint_trajectories argument of CostManager.update_pose_cost (cost_manager.py:64-69;
 * the reference passes zeros, mppi.py:134).  NULL restores zeros. */
mppi_status mppi_set_joint_trajectory(mppi_engine* e, int32_t vehicle, const float* traj_h_nq);

/* Goal per vehicle: position (3) and orientation quaternion xyzw (4; ignored by DRONE). */
mppi_status mppi_set_target(mppi_engine* e, int32_t vehicle, const float* pos3, const float* quat_xyzw4);

/* Warm start (V,H,A) -- reference attribute u_prev (mppi.py:58, drone_mppi.py:29). */
mppi_status mppi_set_u_prev(mppi_engine* e, const float* u_prev);
mppi_status mppi_get_u_prev(mppi_engine* e, float* u_prev);

/* Measured state, packed per vehicle (doubles):
 *   DRONE:     x(3) v(3)
 *   ARM:       base xyz(3) quat xyzw(4) q(nq) qd(nq)        (q_full[:7]+q_full[7:], v_full[6:])
 *   WHOLEBODY: base xyz(3) quat xyzw(4) q(nq) base vel(3) qd(nq)
 *   QUADROTOR: xyz(3) rpy(3) (roll, pitch, yaw; R = Rz(yaw) Ry(pitch) Rx(roll), drone.py:126-154)
 *              v world(3) omega body(3)
 * Async host->device (pinned staging) on the engine stream. */
mppi_status mppi_set_state(mppi_engine* e, const double* state);

/* Step counter used as the Philox counter word (device resident).  On an engine connected by the
 * peer exchange it also moves the exchange epoch carried in the tags (every rank must call it the
 * same number of times, like the steps themselves): words left in the regions under the old
 * counter then never pass for a later step's. */
mppi_status mppi_set_step_counter(mppi_engine* e, uint32_t step);
mppi_status mppi_get_step_counter(mppi_engine* e, uint32_t* step);

/* Split-phase step (async, stream ordered).  d_noise: device eps (V,K,H,A) in
 * INJECTED mode, else NULL.  With shard_count > 1 either bind a zero-initialised
 * exchange buffer of shard_count*V*slot floats (mppi_rollout writes this shard's
 * slot and zeroes the others at the same positions); the caller sums it across
 * shards (one all-reduce), then calls mppi_finalize -- or let the engine own the
 * collective (mppi_comm_init below). */
mppi_status mppi_exchange_slot_floats(mppi_engine* e, int64_t* slot_floats);
mppi_status mppi_bind_exchange(mppi_engine* e, float* d_exchange);
mppi_status mppi_rollout(mppi_engine* e, const float* d_noise);
mppi_status mppi_finalize(mppi_engine* e);

/* Native collective: one process per GPU, one engine per process.
 * Every rank first checks mppi_comm_available (RCCL loadable, every entry point
 * present) and the ranks agree on the outcome before any of them enters the init.
 * Rank 0 makes an id, the caller broadcasts it (torch.distributed), and every rank
 * calls mppi_comm_init with it (collective); rank/world are the config's
 * shard_rank/shard_count.  The engine then owns an RCCL communicator over xGMI and
 * its zero-padded (shard_count, V, slot) exchange buffer, and mppi_step /
 * mppi_run_steps run rollout -> pack -> ONE all-reduce(SUM) -> finalize on the engine
 * stream with no host round trip.  mppi_exchange is that all-reduce alone (split
 * phases).  A one-rank communicator runs the same sharded path on one GPU.  The
 * reference has no distributed code (mppi.py:31 pins one device). */
mppi_status mppi_comm_available(void);
mppi_status mppi_comm_unique_id(uint8_t id[MPPI_COMM_ID_BYTES]);
/* The init is non-blocking with a deadline: the communicator (ncclCommInitRankConfig,
 * blocking = 0) is polled until it is ready or timeout_ms passes (<= 0: the
 * MPPI_COMM_INIT_TIMEOUT_MS environment value, default 60000); a communicator not
 * ready by then is aborted and the call returns MPPI_ERR_COMM, so a rank whose peers
 * never join returns instead of hanging.  mppi_comm_init = mppi_comm_init_ex(e, id, 0). */
mppi_status mppi_comm_init(mppi_engine* e, const uint8_t id[MPPI_COMM_ID_BYTES]);
mppi_status mppi_comm_init_ex(mppi_engine* e, const uint8_t id[MPPI_COMM_ID_BYTES], int32_t timeout_ms);
/* The communicator's own rank count and rank (ncclCommCount / ncclCommUserRank). */
mppi_status mppi_comm_info(mppi_engine* e, int32_t* nranks, int32_t* rank);
mppi_status mppi_exchange(mppi_engine* e);

/* Peer exchange: the sharded step without a collective (replaces the pack ->
 * all-reduce -> combine above for one-vehicle shards, at most 8 ranks).  Each rank's engine
 * opens an exchange region in its own GPU memory (uncached, 2 x ranks x finalize blocks x 68
 * words of 8 B: 5.6 MB at 8 ranks for the C4 shard) and exports it (mppi_peer_open -> an IPC
 * handle); the caller all-gathers the handles (torch.distributed) and every rank maps the
 * others' regions (mppi_peer_connect, the handles in rank order).  From then on each finalize
 * block stores its partial -- (rho, eta, eta2, nan) and its window of N[t], every 8 B word
 * tagged with the step -- into every other rank's region over xGMI, and combines the ranks'
 * partials (its own from registers, the others from its own region once all their tags are the
 * step's): a control step is the unsharded step's two kernels (native dispatch included), no
 * PACK launch, no host-enqueued collective.  Every rank finalises bit-identically, and one
 * rank reproduces the unsharded engine exactly.
 * Failure handling.  A block that waits 2 s for a peer proposes to give the step up; within a rank
 * the step is all or nothing (mppi_peer_info): the first block's proposal decides for every block
 * of the rank, so either every slice of u_prev is updated or every one is kept (w_eps = 0).  A rank
 * that gives the step up reports it twice -- into the control word of this rank in EVERY rank's
 * region (a peer still polling that step gives it up too) and into this engine's sticky word.  From
 * then on every rank's finalize blocks find the report in their own region and give every step up
 * at once (u_prev held on every rank, no 2 s waits) until the host resets the exchange, so no rank
 * keeps updating a warm start the others did not.  The host sees it as stats nonfinite = 2 from
 * mppi_read_outputs (this step's flag on any dim, or the sticky word: any block of any step of a
 * batch), as MPPI_ERR_PEER_TIMEOUT from mppi_synchronize, and through mppi_peer_status (this rank's
 * sticky word and every rank's report as stored in this rank's region).  Recovery is collective
 * (distributed.py ShardedEngine.resync): agree over the process group, take the warm start, step
 * counter and epoch of the lowest rank that is not torn (rank 0 normally), and call mppi_peer_reset
 * on every rank between two barriers.
 * Every rank must run the same sequence of steps with the same step counter (the tags are the
 * Philox counter): a rank that skips a step or rewinds its counter alone leaves the others
 * waiting out the 2 s bound.  mppi_get_weighted_noise gathers the last exchanged step's
 * partials (after mppi_kernel_timing, which exchanges nothing, it is undefined, as the
 * records it reads are then the timing launches').
 * Not combinable with mppi_comm_init / mppi_bind_exchange on the same engine. */
mppi_status mppi_peer_open(mppi_engine* e, uint8_t handle[MPPI_PEER_HANDLE_BYTES]);
mppi_status mppi_peer_connect(mppi_engine* e, const uint8_t* handles /* shard_count x MPPI_PEER_HANDLE_BYTES */);
/* The same connection for ranks inside ONE process (one process driving several engines: on one
 * GPU, or on several GPUs with peer access): mppi_peer_region returns this engine's region as a
 * device address after mppi_peer_open, and mppi_peer_connect_ptrs takes every rank's address in
 * rank order (this engine's own included) instead of IPC handles; across GPUs the caller enables
 * peer access first (hipDeviceEnablePeerAccess).  Every engine's steps must then be in flight
 * together (native dispatch: mppi_run_steps returns once the packets are queued). */
mppi_status mppi_peer_region(mppi_engine* e, uint64_t* device_address);
mppi_status mppi_peer_connect_ptrs(mppi_engine* e, const uint64_t* device_addresses /* shard_count */);
/* Connection check (collective, before the first step; a barrier between phases): phase 0 copies
 * a pattern word into this rank's slot of every rank's region; phase 1 checks that this rank's
 * region holds every rank's word (MPPI_OK, else MPPI_ERR_COMM) and clears it; phase 2 runs the
 * finalize's own tagged stores and polls over the regions in a one-wave kernel (every rank's word
 * within 2 s, else MPPI_ERR_COMM) and clears the region again. */
mppi_status mppi_peer_probe(mppi_engine* e, int32_t phase);
/* The exchange's failure state: sticky = this engine's timeout word (the given-up step's tag, 0 =
 * none; host memory, no device access); reports (kMaxPeers = 8 words, may be NULL) = the timeout
 * reports in this rank's region, word r from rank r (tag << 32 | 1, 0 = none; a device-to-host copy
 * after the engine's work); epoch (may be NULL) = the exchange epoch of the tags. */
mppi_status mppi_peer_status(mppi_engine* e, uint32_t* sticky, uint64_t* reports, uint32_t* epoch);
/* The connection and the warm start's integrity (ABI 9): connected = the ranks whose tagged word
 * reached this rank's region in mppi_peer_probe's kernel phase (phase 2; 0 before it), rank = this
 * engine's shard_rank, torn (may be NULL) = the step tag of a step this rank's warm start came out
 * of torn, 0 = none.  Within a rank a step is all or nothing: a finalize block updates its slice
 * of u_prev only if every peer word arrived in time with no timeout report in sight, and marks the
 * rank's decision word; a late block reports, waits 100 us for any such mark, and if its rank
 * committed keeps polling for a second 2 s bound instead of keeping its slice.  Only if that
 * passes too is the warm start torn (the resync then takes its u_prev from a rank that is not
 * torn). */
mppi_status mppi_peer_info(mppi_engine* e, int32_t* connected, int32_t* rank, uint32_t* torn);
/* Collective recovery after a timeout: with every rank's engine synchronised and a barrier passed
 * (no kernel writes into any region), clear this rank's region and sticky word and take the step
 * counter and epoch the ranks agreed on; a second barrier follows before any rank steps again. */
mppi_status mppi_peer_reset(mppi_engine* e, uint32_t step, uint32_t epoch);

/* Synchronise and copy the step's outputs: out (V, output_dim) doubles
 *   DRONE: x_des(3) v_des(3);  ARM: qdes(nq) vdes(nq);  WHOLEBODY: x(3) v(3) qdes(nq) vdes(nq)
 *   QUADROTOR: x_des = (xyz, rpy)(6), v_des = (v, omega)(6): the model's first step under u0
 * u0 (V, A) floats and stats (V) may be NULL. */
mppi_status mppi_read_outputs(mppi_engine* e, double* out, float* u0, mppi_stats* stats);

/* One whole control step: set_state, (upload host noise), rollout, finalize, read_outputs.
 * h_noise: host eps (V,K,H,A) in INJECTED mode, else NULL.  Single-shard, a shard connected
 * by the peer exchange, or a shard with an engine-owned communicator. */
mppi_status mppi_step(mppi_engine* e, const double* state, const float* h_noise, double* out,
                      float* u0, mppi_stats* stats);

/* n back-to-back asynchronous control steps (rollout + finalize each, device
 * noise, state and warm start resident on the GPU); single-shard engines, shards connected
 * by the peer exchange, or shards with an engine-owned communicator (rollout, PACK,
 * all-reduce, finalize).
 * No host synchronisation: pair with mppi_synchronize / mppi_read_outputs.
 * Single-shard and peer-exchange engines dispatch the steps natively: raw AQL packets on an
 * HSA queue the engine owns, the kernels from the library's code objects, their arguments
 * resident in device memory (MPPI_DISPATCH = auto (default) | aql (required) | hip). */
mppi_status mppi_run_steps(mppi_engine* e, int32_t n);

/* How the last mppi_run_steps and the last mppi_step were dispatched:
 * "<aql | hip: why not native>; calls: <aql (arguments in <where>) | hip>".  One-vehicle control
 * calls with device noise also go out as native packets: the state rides in the rollout's
 * arguments, which the host writes per call into a ring of blocks in host-writable device memory
 * (the GPU's CPU-visible kernarg or fine-grained pool, through the BAR, followed by an HDP
 * flush), or into pinned host memory when the device has no such pool or MPPI_AQL_CALL_HOSTMEM=1.
 * Native dispatch is refused (HIP launches instead, the reason here) when the engine's queue
 * fails its creation probe: dispatch ids that are not the queue's packet indices, as under a
 * tool that intercepts queues (rocprofv3 --pmc). */
mppi_status mppi_dispatch_info(mppi_engine* e, char* buf, int32_t len);

mppi_status mppi_synchronize(mppi_engine* e);

/* Prewarm for a controller that ticks with idle gaps (the arm node's rospy.Rate(100) loop,
 * kinova.py:101; no reference counterpart -- the reference's torch calls pay the same wake-up).
 * A call on a native queue left idle for more than ~50-100 us runs ~6-7 us longer than back to
 * back.  While window_us > 0 a host thread of the engine predicts the next mppi_step from the
 * median interval of the last calls' start times and, from window_us before that until the call
 * starts (at most window_us after it), puts a pair of one-wave packets on the engine's native
 * queue every 25 us; those write a scratch word only, so results are unchanged.  Calls back to back
 * (interval < 4 windows) or slower than 1 s get no touches; nor do calls that go out as HIP
 * launches (HIP dispatch, several vehicles, an RCCL or torch-collective shard; a peer-exchange
 * shard's calls are native).  Through each window the thread sleeps
 * between touches (MPPI_PREWARM_SPIN=1, a diagnostic: it spins).
 * window_us: 0 = off (the default), else 50 .. 5000.  mppi_destroy stops it.
 * mppi_get_prewarm: the window and the touches so far. */
mppi_status mppi_set_prewarm(mppi_engine* e, int32_t window_us);
mppi_status mppi_get_prewarm(mppi_engine* e, int32_t* window_us, int64_t* touches);

/* Readback in the reference's layouts (synchronous):
 *   costs    S (V,K)                         compute_all_cost()
 *   weights  w (V,K)                         compute_weights()
 *   noise    eps (V,K,H,A)                   sampling()            [store_noise]
 *   traj     (V,K,H,C) C = traj_channels    DRONE p(3) / ARM q(nq)+EE(16) / WB p(3)+q(nq)+EE(16)
 *                                            QUADROTOR xyz(3)+rpy(3) (drone_mppi.py:62 trajectory)
 *            EE as the 4x4 row-major matrix of urdf_fk.py:108       [store_trajectory]
 *   wnoise   w_eps before / after SavGol (V,H,A), recomputed from the records the last
 *            step combined (a k_finalize launch in READBACK mode): the step itself stores
 *            no readback copies                                      */
mppi_status mppi_get_costs(mppi_engine* e, float* S);
mppi_status mppi_get_weights(mppi_engine* e, float* w);
mppi_status mppi_get_noise(mppi_engine* e, float* eps);
mppi_status mppi_get_trajectory(mppi_engine* e, float* traj);
mppi_status mppi_get_weighted_noise(mppi_engine* e, float* raw, float* smoothed);

/* Kernel timing with HIP events on the engine stream (bench / roofline). */
mppi_status mppi_enable_timing(mppi_engine* e, int32_t enable);
mppi_status mppi_get_timing(mppi_engine* e, double* rollout_ms_total, double* finalize_ms_total,
                            int64_t* n_rollout, int64_t* n_finalize);
/* Average device time of the two kernels measured back to back: n rollout launches
 * bracketed by one event pair, then n finalize launches bracketed by another (the
 * per-launch pairs of mppi_enable_timing add ~2-3 us of event overhead each).  The
 * warm start and step counter are saved and restored, and the timing launches write
 * their outputs (out/u0/stats) to device scratch, so the controller state and a pending
 * mppi_read_outputs are unchanged (mppi_get_weighted_noise then reflects the timing launches'
 * records: read it before timing).  The
 * trajectory and cost buffers (mppi_get_trajectory / mppi_get_costs / mppi_get_weights)
 * DO hold the timing loop's last rollout afterwards.  Single-shard engines with device
 * noise. */
mppi_status mppi_kernel_timing(mppi_engine* e, int32_t n, double* rollout_us, double* finalize_us);

/* mppi_kernel_timing plus pair_us: the average of n (rollout, finalize) pairs launched as
 * a control step runs them (the rollout after a finalize, its inputs just written).  Also
 * on a shard: the finalize then combines the exchange slots as they stand (no collective).
 * pair_us may be NULL. */
mppi_status mppi_kernel_timing_ex(mppi_engine* e, int32_t n, double* rollout_us, double* finalize_us,
                                  double* pair_us);

/* Average time of the step's all-reduce (mppi_exchange) over n back-to-back calls on the
 * engine stream.  Collective: every rank of the communicator calls it with the same n.
 * The slots are summed in place, so run a step (which repacks them) before reading outputs. */
mppi_status mppi_exchange_timing(mppi_engine* e, int32_t n, double* allreduce_us);

/* Algorithmic HBM bytes one mppi_rollout launch moves. */
int64_t mppi_rollout_bytes(const mppi_config* cfg);

/* Host-side helpers (no GPU needed): the fp32 constants the engine bakes, exposed so
 * the CPU test-suite can pin them against the reference fixtures. */
void mppi_joint_origin(const mppi_joint* j, float* T16);                 /* transformation_matrix.py:28-35 */
void mppi_base_transform(const double* xyzquat, int32_t f64, float* T16); /* urdf_fk.py:30-55             */
void mppi_target_rotation(const float* quat_xyzw, float* R9);            /* rotation_conversions.py:45-75 */
int32_t mppi_savgol_coefficients(int32_t window, int32_t order, float* c); /* svg_filter.py:50-55        */
/* Host FK of one joint vector (check_reach, urdf_fk.py:60-75); base as xyzquat. */
mppi_status mppi_host_fk(const mppi_joint* joints, int32_t n_joints, const double* q, const double* xyzquat,
                         int32_t f64, float* T16);

/* Device RNG check: standard normals z (K,H,A) and the raw Philox words (K,H,W),
 * W = mppi_philox_words(A), exactly as the rollout kernel draws them for (seed, step,
 * vehicle, global k0..k0+K): A/8 Philox4x32-10 calls, then the A mod 8 remainder from one
 * Philox2x32-10 call (remainder <= 4) or one more Philox4x32-10 call.
 * A in {2, 3, 4, 7, 8, 10}. */
int32_t mppi_philox_words(int32_t A);
mppi_status mppi_philox_normals(uint64_t seed, uint32_t step, int32_t vehicle, int64_t k0, int32_t K,
                                int32_t H, int32_t A, int32_t device, float* z, uint32_t* raw);

/* ---------------------------------------------------------------------------------------
 * Host rigid-body dynamics of the arm node.  The reference node
 * calls pin.computeAllTerms(model, data, q, v) on the free-flyer model of
 * full_robot_floating2.urdf every tick (kinova.py:54-61, 126) and applies
 *     tau = M[6:,6:] (400 (qdes - q[7:]) - 40 v[6:]) + nle[6:]              (kinova.py:184)
 * These replace those Pinocchio calls (double precision, Pinocchio's conventions: q = base
 * xyz + quaternion xyzw + joints, v = base linear + angular velocity in the base frame +
 * joint rates, gravity (0,0,-g)).  Fixed-joint links are merged into their movable
 * ancestor.  K = 1 per tick: host code, no GPU. */
typedef struct {
    int32_t parent;        /* index of the parent link entry, -1 = the world                  */
    int32_t type;          /* joint attaching this link: MPPI_JOINT_FIXED / REVOLUTE /
                            * PRISMATIC / FLOATING (root only)                                 */
    double xyz[3], rpy[3]; /* joint origin in the parent link frame (URDF <origin>)           */
    double axis[3];        /* joint axis in the joint frame (URDF <axis>)                     */
    double mass;           /* URDF <inertial>: mass, COM in the link frame, inertia about the */
    double com[3];         /*   COM in the link frame (row-major 3x3; the <inertial> origin    */
    double inertia[9];     /*   rotation already applied)                                     */
} mppi_link;

typedef struct mppi_dyn mppi_dyn;

/* Build the model from links in topological order (robot/urdf_tree.py writes them). */
mppi_status mppi_dyn_create(const mppi_link* links, int32_t n_links, double gravity, mppi_dyn** out);
void mppi_dyn_destroy(mppi_dyn* d);
void mppi_dyn_dims(const mppi_dyn* d, int32_t* nq, int32_t* nv, int32_t* n_bodies);
/* Inverse dynamics tau = M(q) a + nle(q, v) (a NULL = 0), recursive Newton-Euler. */
mppi_status mppi_dyn_rnea(mppi_dyn* d, const double* q, const double* v, const double* a, double* tau);
/* pin.computeAllTerms' M (nv x nv, row-major) and nle = C(q,v) v + g(q) (nv); either may be NULL. */
mppi_status mppi_dyn_terms(mppi_dyn* d, const double* q, const double* v, double* M, double* nle);
/* kinova.py:184 for the trailing actuated joints (rows first_v..nv-1):
 * tau = M[first_v:, first_v:] (kp (qdes - q_act) - kd v_act) + nle[first_v:], as ONE RNEA
 * pass with a = (0, ades) (the base-acceleration columns of M are multiplied by 0). */
mppi_status mppi_computed_torque(mppi_dyn* d, const double* q, const double* v, const double* qdes, double kp,
                                 double kd, int32_t first_v, double* tau);

#ifdef __cplusplus
}
#endif
#endif /* MPPI_HIP_H */

// mppi_device.h -- device helpers shared by the gfx950 kernels (rollout, finalize).
// Internal: included only by mppi_rollout.hip / mppi_finalize.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <type_traits>

#include "mppi_dev.h"

using namespace mppi;

// The dispatch id of the running kernel: the AQL packet's index in its queue, handed to the
// waves in user SGPRs (no memory access).  The LLVM intrinsic by its name: clang has no
// builtin for it.
extern "C" __device__ uint64_t mppi_dispatch_id(void) __asm("llvm.amdgcn.dispatch.id");

namespace {

// noise-mode flag of native dispatch (mppi_aql.cpp): the rollout's step-counter argument is
// relative to the dispatch id -- step = arg + (dispatch id >> 1) -- so one argument block,
// written once, serves every (rollout, finalize) pair the engine's queue runs
constexpr int32_t kNoiseStepFromId = 0x100;
// noise-mode flag of an overlapped native batch (MPPI_OVERLAP=1, mppi_step.cpp run_steps_aql): the
// rollout is dispatched while the finalize before it still runs (no barrier bit), draws its first
// group's normals, then waits for that finalize's blocks (DevParams::ovl counters) before it reads
// u_prev or hands the vehicle constants on
constexpr int32_t kNoiseOverlap = 0x200;
__device__ __forceinline__ uint32_t step_of(uint32_t step_arg, int32_t noise_arg) {
    return (noise_arg & kNoiseStepFromId) ? step_arg + (uint32_t)(mppi_dispatch_id() >> 1) : step_arg;
}

// Loads of what one kernel of a step hands the next (record bodies and headers, u_prev, the
// handed-over vehicle constants): device scope (sc1), past this CU's L1.  The producers write
// these through at device scope and drain their stores (mppi_rollout.h drain_stores), so a
// native batch's packets after its first need no acquire fence (mppi_aql.cpp): nothing a
// kernel reads from its predecessor can come from a stale L1 line.
template <typename T>
__device__ __forceinline__ T ld_dev(const T* p) {
    return __hip_atomic_load((const __attribute__((address_space(1))) T*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
constexpr int kAuxDev = 16;   // the same for buffer loads (cache-policy operand: sc1)

// Stores of values read back only after a native batch (the costs S, the readback copies of
// w_eps, the stored noise): written through at device scope (sc1), so no XCD's L2 keeps a dirty
// copy.  Plain stores left such lines dirty across a batch's release-free packets, and which XCD
// runs a block is not fixed from step to step (MI355X_MICROARCH.md, "Workgroup dispatch, XCD
// placement"): two L2s could hold dirty copies of one line from different steps, and the order of
// their write-backs would decide what the host reads after the batch.
__device__ __forceinline__ void st_dev(float* p, float x) {
    __hip_atomic_store(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// A pointer the compiler keeps in SGPRs (its halves read from the first lane): built from
// kernel arguments through 64-bit VALU math it can land in VGPRs, and a buffer resource over
// it then becomes a waterfall loop around every load or store.
template <typename T>
__device__ __forceinline__ T* uniform_ptr(T* p) {
    const uint64_t a = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    return (T*)(((uint64_t)hi << 32) | lo);
}

// A run of n consecutive floats from LDS (src) to base[off .. off + n), base wave-uniform (off may
// vary per lane), written through: thread i stores elements 4i..4i+3 of the run as ONE 16 B sc1
// buffer store where all four exist and the address is 16 B aligned (a block's costs are whole
// 64 B lines at the common shapes: no partial-line writes, which HBM merges slowly), else one 4 B
// sc1 store per element.
__device__ __forceinline__ void st_dev_run(float* base_uniform, uint32_t off, const float* src, int n, int i) {
    const int e = 4 * i;
    if (e >= n) return;
    const uint32_t o = off + (uint32_t)e;
    if (e + 4 <= n && ((((uintptr_t)base_uniform) + 4u * o) & 15u) == 0u) {
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(base_uniform, 0, (int)0x7FFFFFFF, 0x00020000);
        const float4 x = *reinterpret_cast<const float4*>(src + e);
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 w = {__float_as_uint(x.x), __float_as_uint(x.y), __float_as_uint(x.z), __float_as_uint(x.w)};
        __builtin_amdgcn_raw_buffer_store_b128(w, rs, (int)(4u * o), 0, kAuxDev);
        return;
    }
    for (int j = 0; j < 4 && e + j < n; ++j) st_dev(base_uniform + o + j, src[e + j]);
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS traffic
// (lgkmcnt) but NOT for its outstanding global stores (vmcnt), which
// __syncthreads() would drain -- nothing in these kernels reads its own
// trajectory / record stores back, so the store round trip stays off the
// critical path.  The memory clobber keeps the compiler from moving LDS
// accesses across it.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Hand-off between lanes of one wave through LDS: a wave's LDS instructions execute in
// order, so no s_waitcnt is needed; the wavefront-scope fences order the accesses in the
// memory model and keep the compiler from moving them (rocPRIM's wave_barrier idiom).
__device__ __forceinline__ void wave_lds_handoff() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

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

__device__ __forceinline__ double read_lane_f64(double x, int lane) {
    int lo = __builtin_amdgcn_readlane(__double2loint(x), lane);
    int hi = __builtin_amdgcn_readlane(__double2hiint(x), lane);
    return __hiloint2double(hi, lo);
}

// DPP helpers with bound_ctrl (out-of-row sources read 0): no zeroing moves.
template <int CTRL>
__device__ __forceinline__ double shr_f64(double x) {
    const int lo = __builtin_amdgcn_update_dpp(__double2loint(x), __double2loint(x), CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_update_dpp(__double2hiint(x), __double2hiint(x), CTRL, 0xF, 0xF, true);
    return __hiloint2double(hi, lo);
}

__device__ __forceinline__ float read_lane_f32(float x, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), l));
}

// Folds over the row groups of a wave (lane = g * CW + q; ROWS = 64 / CW groups) with the
// gfx950 lane swaps: v_permlane16_swap exchanges odd rows of one operand with even rows of
// the other, v_permlane32_swap the halves.  With both operands = x, the two results hold
// the partner rows' values, so op(r0, r1) is the pairwise fold in every lane (bit-identical
// across the partners: op is commutative).  Two VALU ops per level instead of an LDS-pipe
// ds_bpermute / ds_swizzle round trip; every lane of column q ends with the fold of q.
template <int CW, typename Op>
__device__ __forceinline__ float fold_rows(float x, Op op) {
    if constexpr (CW <= 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
        x = op(__uint_as_float(r[0]), __uint_as_float(r[1]));
    }
    if constexpr (CW <= 32) {
        const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
        x = op(__uint_as_float(r[0]), __uint_as_float(r[1]));
    }
    return x;
}
struct OpAdd { __device__ float operator()(float a, float b) const { return a + b; } };
struct OpMin { __device__ float operator()(float a, float b) const { return fminf(a, b); } };
struct OpMax { __device__ float operator()(float a, float b) const { return fmaxf(a, b); } };

// The fold of a whole wave in every lane: quad_perm [1,0,3,2] and [2,3,0,1], row_half_mirror,
// row_mirror, then the row-group swaps.  Every level pairs lanes symmetrically, so all 64
// lanes end with the same bits (six VALU/DPP levels instead of six ds_bpermute round trips).
template <int CTRL>
__device__ __forceinline__ float dpp_all(float x) {   // CTRL with a valid source for every lane
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(x), __float_as_int(x), CTRL, 0xF, 0xF, false));
}
template <typename Op>
__device__ __forceinline__ float wave_fold_all(float x, Op op) {
    x = op(x, dpp_all<0xB1>(x));    // quad_perm [1,0,3,2]
    x = op(x, dpp_all<0x4E>(x));    // quad_perm [2,3,0,1]
    x = op(x, dpp_all<0x141>(x));   // row_half_mirror
    x = op(x, dpp_all<0x140>(x));   // row_mirror
    return fold_rows<16>(x, op);
}

// ------------------------------------------------------------------ launches
// Every launch of the control step goes through go(): through HIP, or -- while the calling
// thread has a capture target (mppi_aql.cpp, native dispatch) -- described into it: the
// symbol (namef fills it; the Itanium name of the instantiation, which the code object's
// symbol table holds), the geometry, and the arguments converted to the kernel's parameter
// types and laid out at their natural alignment, as the kernel-argument segment holds them.
template <typename T>
inline void pack_arg(unsigned char* buf, uint32_t& off, const T& v) {
    off = (off + (uint32_t)alignof(T) - 1u) & ~((uint32_t)alignof(T) - 1u);
    if (off + sizeof(T) <= sizeof(LaunchDesc::args)) memcpy(buf + off, &v, sizeof(T));
    off += (uint32_t)sizeof(T);
}
template <typename NameF, typename... P, typename... Arg>
inline int go(void (*k)(P...), NameF namef, dim3 grid, dim3 block, size_t lds, hipStream_t s, Arg... a) {
    static_assert(sizeof...(P) == sizeof...(Arg), "one value per kernel parameter");
    if (LaunchDesc* d = mppi_capture_target()) {
        namef(d->symbol, sizeof(d->symbol));
        d->grid[0] = grid.x; d->grid[1] = grid.y; d->grid[2] = grid.z;
        d->block[0] = block.x; d->block[1] = block.y; d->block[2] = block.z;
        d->lds = (uint32_t)lds;
        uint32_t off = 0;
        (pack_arg<std::decay_t<P>>(d->args, off, static_cast<std::decay_t<P>>(a)), ...);
        d->arg_bytes = off;
        return off <= sizeof(d->args) ? 0 : -1;
    }
    hipLaunchKernelGGL(k, grid, block, lds, s, a...);
    return (int)hipGetLastError();
}

}  // namespace

// mppi_device.h -- device helpers shared by the gfx950 kernels (rollout, finalize).
// Internal: included only by mppi_rollout.hip / mppi_finalize.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stddef.h>
#include <stdint.h>

#include "mppi_dev.h"

using namespace mppi;

namespace {

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

}  // namespace

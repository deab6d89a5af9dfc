// mppi_rollout_arm.hip -- arm rollout kernels, fp64 state (the ROS node feeds float64 arrays, mppi.py:196-200).
// H <= 32 (one 32-lane segment per rollout) lives in mppi_rollout_arm_h32.hip (its own scheduler).
#include "mppi_rollout.h"

extern "C" int mppi_launch_rollout_arm64(const DevParams* p, int threads, void* stream) {
    const hipStream_t s = (hipStream_t)stream;
    // (dispatch_geom's geometries, the H <= 32 one from its own unit)
    if (p->nch == 1 && p->L == 32) return mppi_launch_rollout_arm64_h32(p, threads, stream);
    if (p->nch == 1 && p->L == 64) return launch_rollout_t<MPPI_MODEL_ARM, 7, 1, 64, true>(*p, threads, s);
    if (p->nch == 2) return launch_rollout_t<MPPI_MODEL_ARM, 7, 2, 64, true>(*p, threads, s);
    if (p->nch == 4) return launch_rollout_t<MPPI_MODEL_ARM, 7, 4, 64, true>(*p, threads, s);
    return -1;
}

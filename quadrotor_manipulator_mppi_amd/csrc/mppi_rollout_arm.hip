// mppi_rollout_arm.hip -- arm rollout kernels, fp64 state (the ROS node feeds float64 arrays, mppi.py:196-200).
#include "mppi_rollout.h"

extern "C" int mppi_launch_rollout_arm64(const DevParams* p, int threads, void* stream) {
    return dispatch_geom<MPPI_MODEL_ARM, 7, true>(*p, threads, (hipStream_t)stream);
}

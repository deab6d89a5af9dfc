// mppi_rollout_arm32.hip -- arm rollout kernels, fp32 state.
#include "mppi_rollout.h"

extern "C" int mppi_launch_rollout_arm32(const DevParams* p, int threads, void* stream) {
    return dispatch_geom<MPPI_MODEL_ARM, 7, false>(*p, threads, (hipStream_t)stream);
}

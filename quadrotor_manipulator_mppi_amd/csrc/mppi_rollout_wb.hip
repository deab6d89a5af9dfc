// mppi_rollout_wb.hip -- whole-body rollout kernels.
#include "mppi_rollout.h"

extern "C" int mppi_launch_rollout_wb(const DevParams* p, int threads, void* stream) {
    return dispatch_geom<MPPI_MODEL_WHOLEBODY, 10, false>(*p, threads, (hipStream_t)stream);
}

// mppi_rollout_arm_h32.hip -- arm rollout kernels, fp64 state, H <= 32 (one 32-lane segment per
// rollout: config C3).  A unit of its own so that it builds with the max-ilp scheduler (build.py):
// the single-group C3 kernel is one wave's dependent chain, and max-ilp's interleaving took the C3
// step from 8.78 to 8.56 us (mean of both A/B orders, profiles/r05/sched_maxilp), where the other
// rollout units measured slower or mixed with it.
#include "mppi_rollout.h"

extern "C" int mppi_launch_rollout_arm64_h32(const DevParams* p, int threads, void* stream) {
    return launch_rollout_t<MPPI_MODEL_ARM, 7, 1, 32, true>(*p, threads, (hipStream_t)stream);
}

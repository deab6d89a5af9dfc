// mppi_rollout_drone.hip -- drone rollout kernels, the rollout dispatcher, and the Philox readback kernel.
#include "mppi_rollout.h"

// readback of the device noise: draw_normals for every (k, t) of one vehicle, with the
// raw Philox words in consumption order (philox_words(A) per (k, t))
template <int A>
__device__ __forceinline__ void philox_one(uint64_t seed, uint32_t step, int veh, uint32_t kg, uint32_t t,
                                           float* z, uint32_t* raw) {
    float zz[A];
    draw_normals<A>(zz, kg, t, (uint32_t)veh, step, (uint32_t)seed, (uint32_t)(seed >> 32));
    for (int a = 0; a < A; ++a) z[a] = zz[a];
    constexpr int J = A / 8, REM = A % 8, N4 = J + (REM >= 5 ? 1 : 0);
    for (int j = 0; j < N4; ++j) {
        uint32_t c0 = kg, c1 = t, c2 = ((uint32_t)veh << 8) | (uint32_t)j, c3 = step;
        philox10(c0, c1, c2, c3, (uint32_t)seed, (uint32_t)(seed >> 32));
        raw[4 * j] = c0; raw[4 * j + 1] = c1; raw[4 * j + 2] = c2; raw[4 * j + 3] = c3;
    }
    if constexpr (REM >= 1 && REM <= 4) {
        uint32_t c0 = kg, c1 = philox2_ctr1((uint32_t)veh, t, step);
        philox2x10(c0, c1, philox2_key((uint32_t)seed, (uint32_t)(seed >> 32), step));
        raw[4 * N4] = c0; raw[4 * N4 + 1] = c1;
    }
}

template <int A>
__global__ void k_philox(uint64_t seed, uint32_t step, int veh, int64_t k0, int K, int H, float* z, uint32_t* raw) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= K * H) return;
    const int k = i / H, t = i - k * H;
    philox_one<A>(seed, step, veh, (uint32_t)(k0 + k), (uint32_t)t, z + (size_t)i * A,
                  raw + (size_t)i * philox_words(A));
}

extern "C" int mppi_launch_rollout(const DevParams* p, int threads, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    switch (p->model) {
        case MPPI_MODEL_DRONE:
            if (p->A == 3) return dispatch_geom<MPPI_MODEL_DRONE, 3, false>(*p, threads, s);
            break;
        case MPPI_MODEL_ARM:
            if (p->A == 7) return p->state_f64 ? mppi_launch_rollout_arm64(p, threads, stream)
                                               : mppi_launch_rollout_arm32(p, threads, stream);
            break;
        case MPPI_MODEL_WHOLEBODY:
            if (p->A == 10) return mppi_launch_rollout_wb(p, threads, stream);
            break;
        case MPPI_MODEL_QUADROTOR:
            if (p->A == 4) return mppi_launch_rollout_quad(p, threads, stream);
            break;
    }
    return -1;
}

extern "C" int mppi_launch_philox(uint64_t seed, uint32_t step, int vehicle, int64_t k0, int K, int H, int A,
                                  float* z, uint32_t* raw, void* stream) {
    const int n = K * H;
    const dim3 g((n + 255) / 256), b(256);
    hipStream_t s = (hipStream_t)stream;
    switch (A) {   // the action dims the models draw (drone 3, quadrotor 4, arm 7, whole-body 10) + 2, 8
        case 2: hipLaunchKernelGGL(k_philox<2>, g, b, 0, s, seed, step, vehicle, k0, K, H, z, raw); break;
        case 3: hipLaunchKernelGGL(k_philox<3>, g, b, 0, s, seed, step, vehicle, k0, K, H, z, raw); break;
        case 4: hipLaunchKernelGGL(k_philox<4>, g, b, 0, s, seed, step, vehicle, k0, K, H, z, raw); break;
        case 7: hipLaunchKernelGGL(k_philox<7>, g, b, 0, s, seed, step, vehicle, k0, K, H, z, raw); break;
        case 8: hipLaunchKernelGGL(k_philox<8>, g, b, 0, s, seed, step, vehicle, k0, K, H, z, raw); break;
        case 10: hipLaunchKernelGGL(k_philox<10>, g, b, 0, s, seed, step, vehicle, k0, K, H, z, raw); break;
        default: return -1;
    }
    return (int)hipGetLastError();
}

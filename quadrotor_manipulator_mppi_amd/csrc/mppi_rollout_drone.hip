// mppi_rollout_drone.hip -- drone rollout kernels, the rollout dispatcher, and the Philox readback kernel.
#include "mppi_rollout.h"

__global__ void k_philox(uint64_t seed, uint32_t step, int veh, int64_t k0, int K, int H, int A,
                         float* z, uint32_t* raw) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= K * H) return;
    const int k = i / H, t = i - k * H;
    const int nj = (A + 7) / 8;   // one Philox call per 8 normals (box_muller32: one pair per word)
    for (int j = 0; j < nj; ++j) {
        uint32_t c0 = (uint32_t)(k0 + k), c1 = (uint32_t)t, c2 = ((uint32_t)veh << 8) | (uint32_t)j, c3 = step;
        philox10(c0, c1, c2, c3, (uint32_t)seed, (uint32_t)(seed >> 32));
        uint32_t* rw = raw + ((size_t)i * nj + j) * 4;
        rw[0] = c0; rw[1] = c1; rw[2] = c2; rw[3] = c3;
        const uint32_t wv[4] = {c0, c1, c2, c3};
        for (int q = 0; q < 4; ++q) {
            float n0, n1;
            box_muller32(wv[q], n0, n1);
            const int a = 8 * j + 2 * q;
            if (a < A) z[(size_t)i * A + a] = n0;
            if (a + 1 < A) z[(size_t)i * A + a + 1] = n1;
        }
    }
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
    hipLaunchKernelGGL(k_philox, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, seed, step,
                       vehicle, k0, K, H, A, z, raw);
    return (int)hipGetLastError();
}

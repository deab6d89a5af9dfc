// Accuracy of the hardware v_sin_f32 / v_cos_f32 (argument in revolutions) for joint
// angles, against double-precision sin/cos, next to the kernel's Cody-Waite + minimax
// sincos_joint (fp32 and fp64 reduction).  tools/ only:
//   hipcc --offload-arch=gfx950 -O3 -I include -o /tmp/mb7 tools/microbench7.hip && /tmp/mb7
#include <cmath>
#include <cstdio>
#include <vector>
#include "../quadrotor_manipulator_mppi_amd/csrc/mppi_rollout.h"

// candidate: reduce to f in [-1/2, 1/2] revolutions in the angle's own precision, then
// the hardware sin/cos of 2 pi f
__device__ __forceinline__ void sincos_hw(double q, float& s, float& c) {
    const double r = q * 0.15915494309189533577;
    const float f = (float)(r - rint(r));
    s = __builtin_amdgcn_sinf(f);
    c = __builtin_amdgcn_cosf(f);
}
__device__ __forceinline__ void sincos_hw(float q, float& s, float& c) {
    const float n = __builtin_rintf(q * 0.15915494309189535f);
    float f = fmaf(q, 0.15915494309189535f, -n);            // 1/2pi = C_HI + C_LO
    f = fmaf(q, 6.4206382e-09f, f);
    s = __builtin_amdgcn_sinf(f);
    c = __builtin_amdgcn_cosf(f);
}

__global__ void k_sc(const float* xf, const double* xd, int n, float* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float x = xf[i];
    float s, c;
    sincos_hw(x, s, c);
    out[8 * i + 0] = s; out[8 * i + 1] = c;
    sincos_hw(xd[i], s, c);
    out[8 * i + 2] = s; out[8 * i + 3] = c;
    sincos_joint(x, s, c);
    out[8 * i + 4] = s; out[8 * i + 5] = c;
    sincos_joint(xd[i], s, c);
    out[8 * i + 6] = s; out[8 * i + 7] = c;
}

int main() {
    const int n = 1 << 22;
    std::vector<float> xf(n);
    std::vector<double> xd(n);
    uint64_t st = 0x9E3779B97F4A7C15ull;
    for (int i = 0; i < n; ++i) {   // random joint angles in [-3 pi, 3 pi] (not a dyadic grid)
        st = st * 6364136223846793005ull + 1442695040888963407ull;
        const double u = (double)(st >> 11) * 0x1.0p-53;
        xd[i] = -3.0 * M_PI + 6.0 * M_PI * u;
        xf[i] = (float)xd[i];
    }
    float *dxf, *dout; double* dxd;
    hipMalloc(&dxf, n * 4); hipMalloc(&dxd, n * 8); hipMalloc(&dout, (size_t)n * 32);
    hipMemcpy(dxf, xf.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(dxd, xd.data(), n * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_sc, dim3(n / 256), dim3(256), 0, 0, dxf, dxd, n, dout);
    std::vector<float> out((size_t)n * 8);
    hipMemcpy(out.data(), dout, (size_t)n * 32, hipMemcpyDeviceToHost);
    const char* names[4] = {"hw-red(fp32 q)", "hw-red(fp64 q)", "poly(fp32 q)", "poly(fp64 q)"};
    for (int m = 0; m < 4; ++m) {
        double es = 0, ec = 0, us = 0, uc = 0;
        for (int i = 0; i < n; ++i) {
            const double x = (m == 0 || m == 2) ? (double)xf[i] : xd[i];
            const double s = std::sin(x), c = std::cos(x);
            const double ds = std::fabs(out[8 * (size_t)i + 2 * m] - s), dc = std::fabs(out[8 * (size_t)i + 2 * m + 1] - c);
            es = std::fmax(es, ds); ec = std::fmax(ec, dc);
            // error in units of the fp32 ulp of the exact value (floor 2^-24 near 0 -> absolute)
            const double ul_s = std::fmax(std::ldexp(1.0, std::ilogb(std::fabs(s)) - 23), std::ldexp(1.0, -24));
            const double ul_c = std::fmax(std::ldexp(1.0, std::ilogb(std::fabs(c)) - 23), std::ldexp(1.0, -24));
            us = std::fmax(us, ds / ul_s); uc = std::fmax(uc, dc / ul_c);
        }
        printf("%-14s max|dsin| %.3e (%.2f ulp*)  max|dcos| %.3e (%.2f ulp*)\n", names[m], es, us, ec, uc);
    }
    return 0;
}

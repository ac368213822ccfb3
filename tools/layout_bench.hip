// Edge-state layout probe: the fused kernel's streams (read theta, g_uprev and 7 z blocks; write 7 z
// blocks, g_alpha, g_u) with z block-major (7 streams 1 GiB apart, the current layout) against z in
// 64-cell chunks holding all 7 blocks (AoSoA: one z stream). Same bytes; 512^3 cells.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1); } } while (0)

template <bool AOS>
__global__ __launch_bounds__(256) void k_fusedlike(const double* __restrict__ th, const double* __restrict__ gp,
                                                  const double* __restrict__ zo, double* __restrict__ zn,
                                                  double* __restrict__ ga, double* __restrict__ gu, size_t n) {
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
        const double t = th[i], p = gp[i];
        double v[7];
        const size_t c = i >> 6, l = i & 63;
#pragma unroll
        for (int k = 0; k < 7; ++k) v[k] = AOS ? zo[(c * 7 + k) * 64 + l] : zo[k * n + i];
        double sa = 0.0, su = 0.0;
#pragma unroll
        for (int k = 0; k < 7; ++k) {
            const double z = v[k] * 0.999 + t;
            sa += z;
            su -= z * p;
            __builtin_nontemporal_store(z, AOS ? zn + (c * 7 + k) * 64 + l : zn + k * n + i);
        }
        __builtin_nontemporal_store(sa, ga + i);
        __builtin_nontemporal_store(su, gu + i);
    }
}

int main() {
    const size_t n = size_t(512) * 512 * 512;
    double *th, *gp, *z1, *z2, *ga, *gu;
    CK(hipMalloc(&th, n * 8)); CK(hipMalloc(&gp, n * 8)); CK(hipMalloc(&ga, n * 8)); CK(hipMalloc(&gu, n * 8));
    CK(hipMalloc(&z1, 7 * n * 8)); CK(hipMalloc(&z2, 7 * n * 8));
    for (double* p : {th, gp, ga, gu}) CK(hipMemset(p, 0, n * 8));
    CK(hipMemset(z1, 0, 7 * n * 8)); CK(hipMemset(z2, 0, 7 * n * 8));
    hipEvent_t t0, t1;
    CK(hipEventCreate(&t0)); CK(hipEventCreate(&t1));
    const double bytes = 8.0 * n * (2 + 7 + 7 + 2);
    for (int rep = 0; rep < 2; ++rep)
        for (int aos = 0; aos < 2; ++aos)
            for (int dir = 0; dir < 2; ++dir) {
                const double* src = dir ? z2 : z1;
                double* dst = dir ? z1 : z2;
                auto go = [&] {
                    if (aos) hipLaunchKernelGGL(k_fusedlike<true>, dim3(4096), dim3(256), 0, 0, th, gp, src, dst, ga, gu, n);
                    else hipLaunchKernelGGL(k_fusedlike<false>, dim3(4096), dim3(256), 0, 0, th, gp, src, dst, ga, gu, n);
                };
                go();
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(t0));
                for (int r = 0; r < 5; ++r) go();
                CK(hipEventRecord(t1));
                CK(hipEventSynchronize(t1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, t0, t1));
                printf("{\"layout\": \"%s\", \"dir\": %d, \"ms\": %.3f, \"GBps\": %.1f}\n", aos ? "aosoa64" : "block", dir,
                       ms / 5, bytes / (ms / 5 * 1e-3) / 1e9);
            }
    return 0;
}

// Channel / bank conflict probe: 7 blocks read and 7 blocks written at the same index (the fused
// edge kernel's pattern), with the block stride padded by PAD doubles, between two separate
// allocations in both directions (the ping-pong parity).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1); } } while (0)

__global__ void k_copy7(const double* __restrict__ a, double* __restrict__ b, size_t n, size_t stride) {
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
        double v[7];
#pragma unroll
        for (int k = 0; k < 7; ++k) v[k] = a[k * stride + i];
#pragma unroll
        for (int k = 0; k < 7; ++k) __builtin_nontemporal_store(v[k] * 1.0000001, b + k * stride + i);
    }
}

int main() {
    const size_t n = size_t(1) << 26;
    const size_t pads[] = {0, 8, 64, 512, 520, 4096 + 8, (size_t(1) << 18) + 8};
    const size_t maxpad = (size_t(1) << 18) + 8;
    double *A, *B;
    CK(hipMalloc(&A, 7 * (n + maxpad) * sizeof(double)));
    CK(hipMalloc(&B, 7 * (n + maxpad) * sizeof(double)));
    CK(hipMemset(A, 0, 7 * (n + maxpad) * sizeof(double)));
    CK(hipMemset(B, 0, 7 * (n + maxpad) * sizeof(double)));
    printf("{\"A\": \"%p\", \"B\": \"%p\"}\n", (void*)A, (void*)B);
    hipEvent_t t0, t1;
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    const int grid = 256 * 16, block = 256;
    for (size_t pad : pads) {
        for (int dir = 0; dir < 2; ++dir) {
            const double* src = dir ? B : A;
            double* dst = dir ? A : B;
            for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(k_copy7, dim3(grid), dim3(block), 0, 0, src, dst, n, n + pad);
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(t0));
            for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(k_copy7, dim3(grid), dim3(block), 0, 0, src, dst, n, n + pad);
            CK(hipEventRecord(t1));
            CK(hipEventSynchronize(t1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, t0, t1));
            const double per = ms / 10;
            printf("{\"pad\": %zu, \"dir\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n", pad, dir, per, 14.0 * 8 * n / (per * 1e-3) / 1e9);
        }
    }
    return 0;
}

// Calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths the mvtv
// kernels use: streams a known byte count with 8-byte and 16-byte per-lane loads and stores.
// Run under `rocprofv3 --pmc FETCH_SIZE` (and separately WRITE_SIZE); bytes / counter = factor.
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void copy8(const double* __restrict__ a, double* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) b[i] = a[i];
}
__global__ void copy16(const double2* __restrict__ a, double2* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) b[i] = a[i];
}

int main() {
    const size_t n = size_t(1) << 28;   // 2 GiB per array
    double *a, *b;
    if (hipMalloc(&a, n * 8) != hipSuccess || hipMalloc(&b, n * 8) != hipSuccess) return 1;
    (void)hipMemset(a, 0, n * 8);
    (void)hipMemset(b, 0, n * 8);
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(copy8, dim3(4096), dim3(256), 0, 0, a, b, n);
        hipLaunchKernelGGL(copy16, dim3(4096), dim3(256), 0, 0, reinterpret_cast<const double2*>(a),
                           reinterpret_cast<double2*>(b), n / 2);
    }
    (void)hipDeviceSynchronize();
    std::printf("bytes_read_per_launch %zu bytes_written_per_launch %zu\n", n * 8, n * 8);
    (void)hipFree(a);
    (void)hipFree(b);
    return 0;
}

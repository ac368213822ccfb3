// Achievable HBM bandwidth for the access mixes of the mvtv kernels (fp64, 512^3-sized arrays):
// read-only, copy (1R1W), and 3R3W (the fused PCG's x, r, p in / x, r', p' out).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/stream_bench tools/stream_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

__global__ void k_read(const double* __restrict__ a, size_t n, double* out) {
    double s = 0.0;
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
        s += a[i];
    if (s == 12345.678) out[0] = s;
}

__global__ void k_copy(const double* __restrict__ a, double* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
        b[i] = a[i] * 1.0000001;
}

__global__ void k_3r3w(const double* __restrict__ a, const double* __restrict__ b, const double* __restrict__ c,
                       double* __restrict__ d, double* __restrict__ e, double* __restrict__ f, size_t n) {
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
        const double x = a[i], y = b[i], z = c[i];
        d[i] = x + 0.5 * y;
        e[i] = y - 0.25 * z;
        f[i] = z + x;
    }
}

// 3R3W in z-marching form: a workgroup owns a 64 x 8 column and walks the planes, like k_cg3d
__global__ void k_3r3w_march(const double* __restrict__ a, const double* __restrict__ b, const double* __restrict__ c,
                             double* __restrict__ d, double* __restrict__ e, double* __restrict__ f, int m) {
    const int tx = blockIdx.x % (m / 64), ty = blockIdx.x / (m / 64);
    const int x = tx * 64 + (threadIdx.x & 63), y = ty * 8 + (threadIdx.x >> 6);
    const size_t pl = size_t(m) * m;
    for (int z = 0; z < m; ++z) {
        const size_t i = z * pl + size_t(y) * m + x;
        const double xa = a[i], ya = b[i], za = c[i];
        d[i] = xa + 0.5 * ya;
        e[i] = ya - 0.25 * za;
        f[i] = za + xa;
    }
}

typedef double dvec2 __attribute__((ext_vector_type(2)));

__global__ void k_copy16(const dvec2* __restrict__ a, dvec2* __restrict__ b, size_t n2) {
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n2; i += size_t(gridDim.x) * blockDim.x)
        b[i] = a[i] * 1.0000001;
}

__global__ void k_copy8_nt(const double* __restrict__ a, double* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
        __builtin_nontemporal_store(a[i] * 1.0000001, b + i);
}

__global__ void k_copy16_nt(const dvec2* __restrict__ a, dvec2* __restrict__ b, size_t n2) {
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n2; i += size_t(gridDim.x) * blockDim.x)
        __builtin_nontemporal_store(a[i] * 1.0000001, b + i);
}

__global__ void k_3r3w16(const dvec2* __restrict__ a, const dvec2* __restrict__ b, const dvec2* __restrict__ c,
                         dvec2* __restrict__ d, dvec2* __restrict__ e, dvec2* __restrict__ f, size_t n2) {
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n2; i += size_t(gridDim.x) * blockDim.x) {
        const dvec2 x = a[i], y = b[i], z = c[i];
        d[i] = x + 0.5 * y;
        e[i] = y - 0.25 * z;
        f[i] = z + x;
    }
}

// 8-B lanes, but a contiguous chunk per wave instead of grid-stride (each wave streams 8 KB runs)
__global__ void k_copy8_chunk(const double* __restrict__ a, double* __restrict__ b, size_t n) {
    const size_t per = 1024;
    const size_t nchunk = n / per;
    for (size_t c = blockIdx.x * size_t(blockDim.x / 64) + threadIdx.x / 64; c < nchunk; c += size_t(gridDim.x) * (blockDim.x / 64)) {
        const size_t base = c * per + (threadIdx.x & 63);
#pragma unroll
        for (int k = 0; k < 16; ++k) b[base + 64 * k] = a[base + 64 * k] * 1.0000001;
    }
}

int main() {
    const int m = 512;
    const size_t n = size_t(m) * m * m;
    double* buf[6];
    for (auto& p : buf) {
        CK(hipMalloc(&p, n * sizeof(double)));
        CK(hipMemset(p, 0, n * sizeof(double)));
    }
    double* out;
    CK(hipMalloc(&out, 64));
    hipEvent_t t0, t1;
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    const int grid = 256 * 16, block = 256;
    auto timeit = [&](const char* name, double bytes, auto launch) {
        for (int w = 0; w < 3; ++w) launch();
        CK(hipDeviceSynchronize());
        const int reps = 20;
        CK(hipEventRecord(t0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(t1));
        CK(hipEventSynchronize(t1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, t0, t1));
        const double per = ms / reps;
        printf("{\"kernel\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", name, per, bytes / (per * 1e-3) / 1e9);
    };
    timeit("read_1", 8.0 * n, [&] { hipLaunchKernelGGL(k_read, dim3(grid), dim3(block), 0, 0, buf[0], n, out); });
    timeit("copy_1r1w", 16.0 * n, [&] { hipLaunchKernelGGL(k_copy, dim3(grid), dim3(block), 0, 0, buf[0], buf[1], n); });
    timeit("copy16_1r1w", 16.0 * n, [&] {
        hipLaunchKernelGGL(k_copy16, dim3(grid), dim3(block), 0, 0, (const dvec2*)buf[0], (dvec2*)buf[1], n / 2);
    });
    timeit("copy8_nt", 16.0 * n, [&] { hipLaunchKernelGGL(k_copy8_nt, dim3(grid), dim3(block), 0, 0, buf[0], buf[1], n); });
    timeit("copy16_nt", 16.0 * n, [&] {
        hipLaunchKernelGGL(k_copy16_nt, dim3(grid), dim3(block), 0, 0, (const dvec2*)buf[0], (dvec2*)buf[1], n / 2);
    });
    timeit("copy8_chunk", 16.0 * n, [&] { hipLaunchKernelGGL(k_copy8_chunk, dim3(grid), dim3(block), 0, 0, buf[0], buf[1], n); });
    timeit("grid_3r3w16", 48.0 * n, [&] {
        hipLaunchKernelGGL(k_3r3w16, dim3(grid), dim3(block), 0, 0, (const dvec2*)buf[0], (const dvec2*)buf[1],
                           (const dvec2*)buf[2], (dvec2*)buf[3], (dvec2*)buf[4], (dvec2*)buf[5], n / 2);
    });
    timeit("grid_3r3w", 48.0 * n, [&] {
        hipLaunchKernelGGL(k_3r3w, dim3(grid), dim3(block), 0, 0, buf[0], buf[1], buf[2], buf[3], buf[4], buf[5], n);
    });
    timeit("march_3r3w", 48.0 * n, [&] {
        hipLaunchKernelGGL(k_3r3w_march, dim3((m / 64) * (m / 8)), dim3(512), 0, 0, buf[0], buf[1], buf[2], buf[3],
                           buf[4], buf[5], m);
    });
    return 0;
}

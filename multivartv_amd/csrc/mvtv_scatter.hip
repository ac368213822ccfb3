// Scattered-data setup on the device: the observation map O of
// create_cache_objects (rcpp-code/MultivarTV/src/solvers.cpp:36-44), which the reference builds with
// nearest_interp_matrix / nearest1 (rcpp…/utils.cpp:267-304: a brute-force scan of all N mesh rows
// per point, first minimum of sum((x - mesh_row)^2)), and the two products the ADMM loop needs from
// it, diag(O^T O) (points per mesh node) and O^T y.
//
// The mesh of create_mesh (rcpp…/utils.cpp:234-254) is a tensor product of sorted axes in column-major
// order, so the brute-force minimum lies among the 2^p corners of the cell that brackets the point:
// a binary search per axis finds the bracket, then the 2^p candidate distances are summed in the
// reference's order (dims 0..p-1, no fused multiply-add) and the first minimum in mesh-row order wins.
//
// O^T y: y is sorted by mesh index with a stable radix sort (rocPRIM), then each run of equal keys is
// summed left to right, so every node's sum adds the same values in the same order as the reference's
// sparse product (and numpy's bincount): bit-identical, and deterministic from run to run, which a
// scatter with floating-point atomics would not be.
#include <rocprim/device/device_radix_sort.hpp>

#include "mvtv/mvtv.h"
#include "mvtv_device.h"
#include "mvtv_internal.h"

namespace mvtv {

struct NearestArgs {
    const double* axes;     // sum_j m_j values, axis j at off[j], ascending
    const double* data;     // n x p column-major (arma::mat layout)
    int64_t n;
    int p;
    uint32_t m[MVTV_MAX_DIMS];
    uint32_t off[MVTV_MAX_DIMS];
    uint32_t stride[MVTV_MAX_DIMS];
    double inv_h[MVTV_MAX_DIMS];   // (m_j - 1) / (axis_j[last] - axis_j[0]): the first guess of the bracket
};

// P = p as a template parameter: the per-dim arrays stay in registers (fully unrolled loops)
template <int P>
__global__ __launch_bounds__(256) void k_nearest(const NearestArgs a, uint32_t* __restrict__ key,
                                                 int64_t* __restrict__ idx_out) {
#pragma clang fp contract(off)
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < a.n; i += int64_t(gridDim.x) * blockDim.x) {
        // per dim: the bracket [ax[b-1], ax[b]) of x (b = lower bound) and the squared distances to
        // its two ends (one end at the axis' edges)
        double t0[MVTV_MAX_DIMS], t1[MVTV_MAX_DIMS];
        uint32_t lo[MVTV_MAX_DIMS], two[MVTV_MAX_DIMS];
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const double x = a.data[i + int64_t(j) * a.n];
            const double* ax = a.axes + a.off[j];
            const uint32_t mj = a.m[j];
            // first guess as if the axis were uniform (create_mesh's linspace), checked against the
            // actual values; a binary search when it is off
            const double g = (x - ax[0]) * a.inv_h[j] + 1.0;
            uint32_t b = g <= 0.0 ? 0u : (g >= double(mj) ? mj : uint32_t(g));
            double vl = ax[(b > 0 ? b : 1) - 1], vh = ax[b < mj ? b : mj - 1];
            if (!((b == mj || !(vh < x)) && (b == 0 || vl < x))) {
                uint32_t e = mj;
                b = 0;
                while (b < e) {
                    const uint32_t h = (b + e) >> 1;
                    if (ax[h] < x) b = h + 1;
                    else e = h;
                }
                vl = ax[(b > 0 ? b : 1) - 1];
                vh = ax[b < mj ? b : mj - 1];
            }
            if (b == 0) {
                lo[j] = 0; two[j] = 0;
                t0[j] = (x - vh) * (x - vh);
            } else if (b == mj) {
                lo[j] = mj - 1; two[j] = 0;
                t0[j] = (x - vl) * (x - vl);
            } else {
                lo[j] = b - 1; two[j] = 1;
                t0[j] = (x - vl) * (x - vl);
            }
            t1[j] = (x - vh) * (x - vh);
        }
        // the 2^p corners: squared distance summed over dims 0..p-1 as the reference does (no fused
        // multiply-add); the first minimum in mesh-row (column-major) order wins
        double best = 0.0;
        uint32_t best_idx = 0;
        bool have = false;
#pragma unroll
        for (int s = 0; s < (1 << P); ++s) {
            uint32_t node = 0;
            bool ok = true;
            double d = 0.0;
#pragma unroll
            for (int j = 0; j < P; ++j) {
                const uint32_t bit = (s >> j) & 1;
                ok = ok && bit <= two[j];
                node += (lo[j] + bit) * a.stride[j];
                d = d + (bit ? t1[j] : t0[j]);
            }
            if (!ok) continue;
            if (!have || d < best || (d == best && node < best_idx)) {
                best = d;
                best_idx = node;
                have = true;
            }
        }
        key[i] = best_idx;
        if (idx_out) idx_out[i] = int64_t(best_idx);
    }
}

// runs of equal keys in the sorted order: the first element of each run sums it left to right
__global__ __launch_bounds__(256) void k_run_sums(const uint32_t* __restrict__ key, const double* __restrict__ y,
                                                  int64_t n, double* __restrict__ oty, double* __restrict__ wdiag,
                                                  unsigned long long* __restrict__ nruns) {
    unsigned runs = 0;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
        const uint32_t k = key[i];
        if (i > 0 && key[i - 1] == k) continue;
        double s = 0.0;
        int64_t j = i;
        for (; j < n && key[j] == k; ++j) s = s + y[j];
        oty[k] = s;
        wdiag[k] = double(j - i);
        ++runs;
    }
    for (int off = 32; off > 0; off >>= 1) runs += __shfl_down(runs, off, 64);
    __shared__ unsigned part[4];
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = runs;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(nruns, (unsigned long long)(part[0] + part[1] + part[2] + part[3]));
}

namespace {
unsigned grid_for(int64_t n) {
    const int64_t b = (n + 255) / 256;
    return unsigned(std::max<int64_t>(1, std::min<int64_t>(b, 65536)));
}
}  // namespace

hipError_t launch_nearest(hipStream_t s, int p, const uint32_t* m, const double* axes, const double* axes_host_span,
                          const double* data, int64_t n, uint32_t* key, int64_t* idx_out) {
    NearestArgs a{};
    a.axes = axes;
    a.data = data;
    a.n = n;
    a.p = p;
    uint32_t off = 0, stride = 1;
    for (int j = 0; j < p; ++j) {
        a.m[j] = m[j];
        a.off[j] = off;
        a.stride[j] = stride;
        const double span = axes_host_span ? axes_host_span[j] : 0.0;
        a.inv_h[j] = span > 0.0 ? double(m[j] - 1) / span : 0.0;
        off += m[j];
        stride *= m[j];
    }
    if (n > 0) {
        const dim3 grid(grid_for(n)), block(256);
        switch (p) {
            case 1: klaunch(k_nearest<1>, grid, block, 0, s, a, key, idx_out); break;
            case 2: klaunch(k_nearest<2>, grid, block, 0, s, a, key, idx_out); break;
            case 3: klaunch(k_nearest<3>, grid, block, 0, s, a, key, idx_out); break;
            default: klaunch(k_nearest<4>, grid, block, 0, s, a, key, idx_out); break;
        }
    }
    return hipGetLastError();
}

// keys (consumed) and y -> wdiag[N], oty[N] (zero where no point falls); *nruns = nodes hit
hipError_t launch_scatter_sums(hipStream_t s, uint32_t* key, const double* y, int64_t n, uint32_t N, double* oty,
                               double* wdiag, unsigned long long* nruns) {
    hipError_t e = hipMemsetAsync(oty, 0, size_t(N) * sizeof(double), s);
    if (e == hipSuccess) e = hipMemsetAsync(wdiag, 0, size_t(N) * sizeof(double), s);
    if (e == hipSuccess) e = hipMemsetAsync(nruns, 0, sizeof(unsigned long long), s);
    if (e != hipSuccess || n == 0) return e;
    unsigned end_bit = 1;
    while (end_bit < 32 && (uint64_t(1) << end_bit) < uint64_t(N)) ++end_bit;
    uint32_t* key2 = nullptr;
    double* y2 = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    e = rocprim::radix_sort_pairs(nullptr, tmp_bytes, key, key2, y, y2, size_t(n), 0u, end_bit, s);
    if (e == hipSuccess) e = hipMalloc(&tmp, std::max<size_t>(tmp_bytes, 1));
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&key2), size_t(n) * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&y2), size_t(n) * sizeof(double));
    if (e == hipSuccess) e = rocprim::radix_sort_pairs(tmp, tmp_bytes, key, key2, y, y2, size_t(n), 0u, end_bit, s);
    if (e == hipSuccess) {
        klaunch(k_run_sums, dim3(grid_for(n)), dim3(256), 0, s, static_cast<const uint32_t*>(key2),
                static_cast<const double*>(y2), n, oty, wdiag, nruns);
        e = hipGetLastError();
    }
    const hipError_t es = hipStreamSynchronize(s);
    if (e == hipSuccess) e = es;
    (void)hipFree(tmp);
    (void)hipFree(key2);
    (void)hipFree(y2);
    return e;
}

}  // namespace mvtv

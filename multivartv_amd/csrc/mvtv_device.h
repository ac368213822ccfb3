// mvtv_device.h — device helpers shared by the kernel translation units.
#pragma once
#include <type_traits>

#include "mvtv_internal.h"

namespace mvtv {

template <int K, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (K < N) {
        f(std::integral_constant<int, K>{});
        static_for<K + 1, N>(f);
    }
}

__device__ __forceinline__ double clampd(double z, double t) { return fmin(fmax(z, -t), t); }

// Workgroup barrier that orders LDS only: __syncthreads() also waits for every outstanding
// global load (s_waitcnt vmcnt(0)), which would drain a prefetch issued before the barrier.
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Wave (64-lane) shuffle reduction, then across the block's waves through LDS. The last NMAX
// slots are max-reductions, the others sums. Thread 0 writes this block's partials.
template <int NR, int NMAX, int NT = kThreads>
__device__ __forceinline__ void block_reduce_store(double (&v)[NR], double* __restrict__ partials) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
#pragma unroll
        for (int k = 0; k < NR; ++k) {
            double o = __shfl_down(v[k], off, 64);
            v[k] = (k < NR - NMAX) ? v[k] + o : fmax(v[k], o);
        }
    }
    __shared__ double sm[NT / 64][NR];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < NR; ++k) sm[wid][k] = v[k];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < NR; ++k) {
            double acc = sm[0][k];
            for (int w = 1; w < NT / 64; ++w) acc = (k < NR - NMAX) ? acc + sm[w][k] : fmax(acc, sm[w][k]);
            partials[blockIdx.x * NR + k] = acc;
        }
    }
}

}  // namespace mvtv

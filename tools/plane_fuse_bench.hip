// Probe: can the two in-plane transform passes of the spectral theta-solve (dim 0, then dim 1 of
// every 512 x 512 plane) become ONE pass over HBM, the plane handed between the workgroups of one
// XCD inside the launch?
//
// Stand-in work with the real access pattern, in place on a 512^3 fp64 mesh:
//   stage 1: a workgroup owns 16 contiguous dim-0 lines of a plane (64 KB), loads them, x -> 2x + 1
//   stage 2: a workgroup owns 16 adjacent dim-0 positions x all 512 dim-1 rows (512 128-B segments),
//            x -> x * 0.5 + row
// Variants:
//   sep      two launches over the mesh (what the solve does now)
//   fused/s  one launch, 1 workgroup per CU, groups = the workgroups of one XCD (by HW_REG_XCC_ID),
//            one plane per group at a time, stage-1 results handed over by sc1 stores + sc1 loads
//            (write-through, the guide's valid form), one counter barrier per plane
//   fused/p  the same with plain stage-1 stores (the line stays in the XCD's L2) and sc1 loads
//   +pf      stage-1 inputs of the next plane loaded into registers before the barrier wait
// Every spin is bounded; a timed-out barrier sets an error word that the host checks.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/plane_fuse_bench tools/plane_fuse_bench.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)

constexpr int M = 512;
constexpr int NT = 256;
constexpr int TQ = 16;
typedef double dvec2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct Ctl {
    unsigned int arrived;
    unsigned int err;
    unsigned int pad[14];
    unsigned int xcnt[8];        // workgroups per XCD (start census)
    unsigned int pad2[8];
    unsigned int bar[8 * 32];    // per-XCD plane barrier counters, one 128-B line each
};

__device__ __forceinline__ unsigned ld_acq(const unsigned* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ dvec2 ld_sc1(const double* base, uint32_t off_bytes) {
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7fffffff, 0x00020000);
    u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off_bytes, 0, 16);
    dvec2 d;
    __builtin_memcpy(&d, &v, 16);
    return d;
}
__device__ __forceinline__ void st_sc1(double* base, uint32_t off_bytes, dvec2 d) {
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7fffffff, 0x00020000);
    u32x4 v;
    __builtin_memcpy(&v, &d, 16);
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off_bytes, 0, 16);
}

// ---- separate passes ----------------------------------------------------------------------------
__global__ __launch_bounds__(NT) void k_rows(double* x) {
    // 16 contiguous lines = 64 KB: 16 loads of 16 B per thread
    double* t = x + size_t(blockIdx.x) * (TQ * M);
    dvec2 v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = __builtin_nontemporal_load((const dvec2*)(t + 2 * (threadIdx.x + NT * i)));
#pragma unroll
    for (int i = 0; i < 16; ++i) __builtin_nontemporal_store(v[i] * 2.0 + 1.0, (dvec2*)(t + 2 * (threadIdx.x + NT * i)));
}
__global__ __launch_bounds__(NT) void k_cols(double* x) {
    // plane e, columns c0..c0+15: 512 rows x 128 B; 8 threads per row segment, 32 rows per sweep
    const int e = blockIdx.x / (M / TQ), c0 = (blockIdx.x % (M / TQ)) * TQ;
    double* pl = x + size_t(e) * M * M;
    const int seg = threadIdx.x & 7, r0 = threadIdx.x >> 3;
    dvec2 v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = __builtin_nontemporal_load((const dvec2*)(pl + size_t(r0 + 32 * i) * M + c0 + 2 * seg));
#pragma unroll
    for (int i = 0; i < 16; ++i)
        __builtin_nontemporal_store(v[i] * 0.5 + double(r0 + 32 * i), (dvec2*)(pl + size_t(r0 + 32 * i) * M + c0 + 2 * seg));
}

// ---- fused, per-XCD groups --------------------------------------------------------------------------
template <bool SC1_STORE, bool PF>
__global__ __launch_bounds__(NT) void k_fused(double* x, Ctl* ctl, int nplanes) {
    extern __shared__ double pad_lds[];   // sized by the launch so one workgroup fits per CU
    __shared__ int s_info[4];
    const int t = threadIdx.x;
    if (t == 0) {
        unsigned xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11)) & 7u;   // HW_REG_XCC_ID[3:0]
        const unsigned rank = __hip_atomic_fetch_add(&ctl->xcnt[xcc], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(&ctl->arrived, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (ld_acq(&ctl->arrived) < gridDim.x) {
            __builtin_amdgcn_s_sleep(2);
            if (__builtin_amdgcn_s_memrealtime() - t0 > 50000000ull) {
                __hip_atomic_fetch_or(&ctl->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
        int ng = 0, gi = 0;
        for (unsigned q = 0; q < 8; ++q) {
            const unsigned c = ld_acq(&ctl->xcnt[q]);
            if (c) {
                if (q == xcc) gi = ng;
                ++ng;
            }
        }
        s_info[0] = int(xcc);
        s_info[1] = int(rank);
        s_info[2] = int(ld_acq(&ctl->xcnt[xcc]));
        s_info[3] = gi | (ng << 8);
    }
    __syncthreads();
    if (pad_lds[0] == 12345.0) pad_lds[1] = 0.0;   // keep the allocation
    const int xcc = s_info[0], rank = s_info[1], n = s_info[2], gi = s_info[3] & 255, ng = s_info[3] >> 8;
    unsigned* bar = &ctl->bar[32 * xcc];
    // rows of stage 1 / columns of stage 2 for this rank: M / TQ = 32 tiles per plane dealt over n ranks
    const int ntile = M / TQ;
    int step = 0;
    dvec2 nxt[16];
    auto load_rows = [&](int e, int tile, dvec2* v) {
        const double* tp = x + size_t(e) * M * M + size_t(tile) * TQ * M;
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = __builtin_nontemporal_load((const dvec2*)(tp + 2 * (t + NT * i)));
    };
    for (int e = gi; e < nplanes; e += ng, ++step) {
        double* pl = x + size_t(e) * M * M;
        // stage 1
        for (int tile = rank; tile < ntile; tile += n) {
            dvec2 v[16];
            if (PF && tile == rank && step > 0) {
#pragma unroll
                for (int i = 0; i < 16; ++i) v[i] = nxt[i];
            } else {
                load_rows(e, tile, v);
            }
            double* tp = pl + size_t(tile) * TQ * M;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const dvec2 w = v[i] * 2.0 + 1.0;
                const uint32_t off = uint32_t(size_t(tile) * TQ * M + 2 * (t + NT * i)) * 8u;
                if (SC1_STORE) st_sc1(pl, off, w);
                else *(dvec2*)(tp + 2 * (t + NT * i)) = w;
            }
        }
        // barrier: every storing wave drained, then one arrival per workgroup
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        const int en = e + ng;
        if (PF && en < nplanes && rank < ntile) load_rows(en, rank, nxt);
        if (t == 0) {
            __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned target = unsigned(n) * unsigned(step + 1);
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            while (ld_acq(bar) < target) {
                __builtin_amdgcn_s_sleep(1);
                if (__builtin_amdgcn_s_memrealtime() - t0 > 50000000ull) {
                    __hip_atomic_fetch_or(&ctl->err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
            }
        }
        __syncthreads();
        // stage 2: sc1 loads of the handed-over plane
        const int seg = t & 7, r0 = t >> 3;
        for (int tile = rank; tile < ntile; tile += n) {
            const int c0 = tile * TQ;
            dvec2 v[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) v[i] = ld_sc1(pl, uint32_t((size_t(r0 + 32 * i) * M + c0 + 2 * seg) * 8u));
#pragma unroll
            for (int i = 0; i < 16; ++i)
                __builtin_nontemporal_store(v[i] * 0.5 + double(r0 + 32 * i), (dvec2*)(pl + size_t(r0 + 32 * i) * M + c0 + 2 * seg));
        }
    }
}

// ---- fused, dynamic per-XCD queues ------------------------------------------------------------------
// Every XCD (by HW_REG_XCC_ID) has a queue of items: S1(0), then [S1(j+1), S2(j)] for j = 0, 1, ...; a
// block is T tiles of one stage of one queue-plane j, whose mesh plane is taken from a global counter by
// the claimant of S1(j)'s tile 0 and published in plane_of[x][j] (tagged with the launch generation).
// An S2 tile waits until all T S1 tiles of its plane are done (per-plane counter, cumulative over
// launches). A workgroup waits only on items claimed before its own by running workgroups that never
// wait after their claim except for the plane publication, so any residency makes progress.
struct DynQ {
    unsigned head[8 * 32];       // per-XCD item counters (one 128-B line each)
    unsigned gplane;             // global plane counter
    unsigned fin;                // workgroups finished
    unsigned gen;                // launch generation (starts at 1)
    unsigned err;
    unsigned diag[8];            // first timed-out wait: kind, xcc, i, j, e, value, gen, target
    unsigned pad[20];
};
__device__ __forceinline__ bool timed_out(unsigned long long t0) {
    return __builtin_amdgcn_s_memrealtime() - t0 > 50000000ull;   // 0.5 s at 100 MHz
}
__device__ __forceinline__ bool bail(const DynQ* q, unsigned long long t0) {
    return timed_out(t0) || __hip_atomic_load(&q->err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
}
__device__ void record(DynQ* q, unsigned kind, unsigned xcc, unsigned i, unsigned j, unsigned e, unsigned v, unsigned gen,
                       unsigned target) {
    if (__hip_atomic_fetch_or(&q->err, kind, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
        const unsigned d[8] = {kind, xcc, i, j, e, v, gen, target};
        for (int k = 0; k < 8; ++k) __hip_atomic_store(&q->diag[k], d[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
template <bool PLAIN, int NTD>
__global__ __launch_bounds__(NTD) void k_dyn(double* x, DynQ* q, unsigned long long* plane_of, unsigned* done1, int nplanes) {
    extern __shared__ double pad_lds[];
    __shared__ unsigned s_item, s_plane;
    const int t = threadIdx.x;
    constexpr int T = M / TQ;   // tiles per plane per stage
    const unsigned xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11)) & 7u;
    const unsigned gen = __hip_atomic_load(&q->gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (pad_lds[0] == 12345.0) pad_lds[1] = 0.0;
    unsigned long long* pof = plane_of + size_t(xcc) * nplanes;
    for (;;) {
        // wave 0 claims the next item; every branch and spin below is wave-uniform (values are read by all
        // 64 lanes from one address, or taken from lane 0 by readfirstlane), only the atomics are lane 0's
        if (t < 64) {
            unsigned i = 0;
            if (t == 0) i = __hip_atomic_fetch_add(&q->head[32 * xcc], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            i = __builtin_amdgcn_readfirstlane(i);
            const unsigned b = i / T, tile = i % T;
            // block b: 0 -> S1(0); b >= 1: c = b - 1, even c -> S1(c/2 + 1), odd c -> S2(c/2)
            const unsigned stage = b == 0 ? 1u : ((b - 1) % 2 == 0 ? 1u : 2u);
            const unsigned j = b == 0 ? 0u : (stage == 1 ? (b - 1) / 2 + 1 : (b - 1) / 2);
            unsigned e = 0xfffffu;
            if (j < unsigned(nplanes)) {
                if (stage == 1 && tile == 0) {
                    unsigned g = 0;
                    if (t == 0) g = __hip_atomic_fetch_add(&q->gplane, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    g = __builtin_amdgcn_readfirstlane(g);
                    e = g < unsigned(nplanes) ? g : 0xfffffu;
                    if (t == 0)
                        __hip_atomic_store(&pof[j], (static_cast<unsigned long long>(gen) << 32) | e, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                } else {
                    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                    for (;;) {
                        const unsigned long long v = __hip_atomic_load(&pof[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        const unsigned hi = __builtin_amdgcn_readfirstlane(unsigned(v >> 32));
                        const unsigned lo = __builtin_amdgcn_readfirstlane(unsigned(v));
                        if (hi == gen) {
                            e = lo;
                            break;
                        }
                        if (bail(q, t0)) {
                            if (t == 0) record(q, 1u, xcc, i, j, 0, hi, gen, 0);
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                }
            }
            if (stage == 2 && e < unsigned(nplanes)) {
                const unsigned target = unsigned(T) * gen;
                const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                for (;;) {
                    const unsigned v = __builtin_amdgcn_readfirstlane(
                        __hip_atomic_load(&done1[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                    if (v >= target) break;
                    if (bail(q, t0)) {
                        if (t == 0) record(q, 2u, xcc, i, j, e, v, gen, target);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            if (t == 0) {
                s_item = (stage << 30) | tile;
                s_plane = e;
            }
        }
        __syncthreads();
        const unsigned stage = s_item >> 30, tile = s_item & 0xffffu, e = s_plane;
        __syncthreads();
        if (e >= unsigned(nplanes)) {
            if (stage == 2) break;   // S2 of an unassigned plane: the queue has ended
            continue;
        }
        double* pl = x + size_t(e) * M * M;
        constexpr int NL = NTD / 16;   // 16-B slots per thread-row
        if (stage == 1) {
            // 16 lines = 4096 16-B slots
            constexpr int PER = 4096 / NTD;
            dvec2 v[PER];
#pragma unroll
            for (int i = 0; i < PER; ++i) v[i] = __builtin_nontemporal_load((const dvec2*)(pl + size_t(tile) * TQ * M + 2 * (t + NTD * i)));
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const dvec2 w = v[i] * 2.0 + 1.0;
                const uint32_t off = uint32_t(size_t(tile) * TQ * M + 2 * (t + NTD * i)) * 8u;
                if (PLAIN) *(dvec2*)(pl + size_t(tile) * TQ * M + 2 * (t + NTD * i)) = w;
                else st_sc1(pl, off, w);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (t == 0) __hip_atomic_fetch_add(&done1[e], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            constexpr int PER = 4096 / NTD;
            constexpr int RPS = NTD / 8;   // rows per sweep
            const int seg = t & 7, r0 = t >> 3;
            const int c0 = int(tile) * TQ;
            dvec2 v[PER];
#pragma unroll
            for (int i = 0; i < PER; ++i) v[i] = ld_sc1(pl, uint32_t((size_t(r0 + RPS * i) * M + c0 + 2 * seg) * 8u));
#pragma unroll
            for (int i = 0; i < PER; ++i)
                __builtin_nontemporal_store(v[i] * 0.5 + double(r0 + RPS * i), (dvec2*)(pl + size_t(r0 + RPS * i) * M + c0 + 2 * seg));
        }
        (void)NL;
    }
    // the last workgroup out resets the counters for the next launch and advances the generation
    if (t == 0) {
        const unsigned f = __hip_atomic_fetch_add(&q->fin, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (f == gridDim.x - 1) {
            for (int k = 0; k < 8; ++k) __hip_atomic_store(&q->head[32 * k], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&q->gplane, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&q->fin, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&q->gen, gen + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

int main(int argc, char** argv) {
    const size_t n = size_t(M) * M * M;
    double* x;
    CK(hipMalloc(&x, n * sizeof(double)));
    Ctl* ctl;
    CK(hipMalloc(&ctl, sizeof(Ctl)));
    std::vector<double> h(n), g(n);
    for (size_t i = 0; i < n; ++i) h[i] = double(i % 1000) * 0.001;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    printf("{\"cus\": %d}\n", cus);
    hipEvent_t t0, t1;
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    // expected result
    for (size_t i = 0; i < n; ++i) {
        const size_t r = (i / M) % M;
        g[i] = (h[i] * 2.0 + 1.0) * 0.5 + double(r);
    }
    const size_t lds = 96 * 1024;
    auto check = [&](const char* name) {
        std::vector<double> o(n);
        CK(hipMemcpy(o.data(), x, n * 8, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (size_t i = 0; i < n; ++i)
            if (o[i] != g[i]) ++bad;
        Ctl c;
        CK(hipMemcpy(&c, ctl, sizeof(Ctl), hipMemcpyDeviceToHost));
        printf("{\"check\": \"%s\", \"bad\": %zu, \"err\": %u, \"xcnt\": [%u,%u,%u,%u,%u,%u,%u,%u]}\n", name, bad, c.err,
               c.xcnt[0], c.xcnt[1], c.xcnt[2], c.xcnt[3], c.xcnt[4], c.xcnt[5], c.xcnt[6], c.xcnt[7]);
        fflush(stdout);
        return bad == 0 && c.err == 0;
    };
    auto run_sep = [&] {
        hipLaunchKernelGGL(k_rows, dim3(M * M / TQ), dim3(NT), 0, 0, x);
        hipLaunchKernelGGL(k_cols, dim3(M * M / TQ), dim3(NT), 0, 0, x);
    };
    auto fused = [&](int variant) {
        CK(hipMemsetAsync(ctl, 0, sizeof(Ctl), 0));
        switch (variant) {
            case 0: hipLaunchKernelGGL((k_fused<true, false>), dim3(cus), dim3(NT), lds, 0, x, ctl, M); break;
            case 1: hipLaunchKernelGGL((k_fused<false, false>), dim3(cus), dim3(NT), lds, 0, x, ctl, M); break;
            case 2: hipLaunchKernelGGL((k_fused<true, true>), dim3(cus), dim3(NT), lds, 0, x, ctl, M); break;
            case 3: hipLaunchKernelGGL((k_fused<false, true>), dim3(cus), dim3(NT), lds, 0, x, ctl, M); break;
        }
    };
    const char* names[4] = {"fused_sc1", "fused_plain", "fused_sc1_pf", "fused_plain_pf"};
    for (auto f : {(hipFuncAttribute)hipFuncAttributeMaxDynamicSharedMemorySize}) {
        CK(hipFuncSetAttribute((const void*)k_fused<true, false>, f, lds));
        CK(hipFuncSetAttribute((const void*)k_fused<false, false>, f, lds));
        CK(hipFuncSetAttribute((const void*)k_fused<true, true>, f, lds));
        CK(hipFuncSetAttribute((const void*)k_fused<false, true>, f, lds));
    }
    // correctness first (one run each from the same input)
    CK(hipMemcpy(x, h.data(), n * 8, hipMemcpyHostToDevice));
    run_sep();
    CK(hipDeviceSynchronize());
    bool ok = check("sep");
    for (int v = 0; v < 4 && ok; ++v) {
        CK(hipMemcpy(x, h.data(), n * 8, hipMemcpyHostToDevice));
        fused(v);
        CK(hipDeviceSynchronize());
        ok = check(names[v]);
    }
    if (!ok) return 2;
    auto timeit = [&](const char* name, auto launch) {
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
        printf("{\"kernel\": \"%s\", \"ms\": %.4f, \"GBps_2N\": %.1f}\n", name, per, 16.0 * n / (per * 1e-3) / 1e9);
        fflush(stdout);
    };
    // dynamic per-XCD queues
    DynQ* dq;
    unsigned long long* pof;
    unsigned* done1;
    CK(hipMalloc(&dq, sizeof(DynQ)));
    CK(hipMalloc(&pof, 8 * size_t(M) * sizeof(unsigned long long)));
    CK(hipMalloc(&done1, size_t(M) * sizeof(unsigned)));
    CK(hipMemset(dq, 0, sizeof(DynQ)));
    CK(hipMemset(pof, 0, 8 * size_t(M) * sizeof(unsigned long long)));
    CK(hipMemset(done1, 0, size_t(M) * sizeof(unsigned)));
    {
        unsigned one = 1;
        CK(hipMemcpy(&dq->gen, &one, 4, hipMemcpyHostToDevice));
    }
    for (auto f : {(const void*)k_dyn<true, 256>, (const void*)k_dyn<false, 256>, (const void*)k_dyn<true, 512>,
                   (const void*)k_dyn<false, 512>})
        CK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
    struct DV { const char* name; int plain, ntd, grid; size_t lds; };
    const DV dvs[] = {{"dyn_plain_256x1", 1, 256, cus, 96 * 1024}, {"dyn_plain_256x2", 1, 256, 2 * cus, 64 * 1024},
                      {"dyn_plain_256x4", 1, 256, 4 * cus, 32 * 1024}, {"dyn_plain_512x1", 1, 512, cus, 96 * 1024},
                      {"dyn_plain_512x2", 1, 512, 2 * cus, 64 * 1024}, {"dyn_sc1_256x2", 0, 256, 2 * cus, 64 * 1024},
                      {"dyn_sc1_256x4", 0, 256, 4 * cus, 32 * 1024}, {"dyn_plain_256x2_g300", 1, 256, 300, 64 * 1024}};
    auto dyn = [&](const DV& d) {
        if (d.ntd == 256) {
            if (d.plain) hipLaunchKernelGGL((k_dyn<true, 256>), dim3(d.grid), dim3(256), d.lds, 0, x, dq, pof, done1, M);
            else hipLaunchKernelGGL((k_dyn<false, 256>), dim3(d.grid), dim3(256), d.lds, 0, x, dq, pof, done1, M);
        } else {
            if (d.plain) hipLaunchKernelGGL((k_dyn<true, 512>), dim3(d.grid), dim3(512), d.lds, 0, x, dq, pof, done1, M);
            else hipLaunchKernelGGL((k_dyn<false, 512>), dim3(d.grid), dim3(512), d.lds, 0, x, dq, pof, done1, M);
        }
    };
    for (const DV& d : dvs) {
        CK(hipMemcpy(x, h.data(), n * 8, hipMemcpyHostToDevice));
        dyn(d);
        CK(hipDeviceSynchronize());
        std::vector<double> o(n);
        CK(hipMemcpy(o.data(), x, n * 8, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (size_t i = 0; i < n; ++i)
            if (o[i] != g[i]) ++bad;
        DynQ hq;
        CK(hipMemcpy(&hq, dq, sizeof(DynQ), hipMemcpyDeviceToHost));
        printf("{\"check\": \"%s\", \"bad\": %zu, \"err\": %u, \"gen\": %u, \"fin\": %u, \"gplane\": %u, \"diag\": [%u,%u,%u,%u,%u,%u,%u,%u]}\n",
               d.name, bad, hq.err, hq.gen, hq.fin, hq.gplane, hq.diag[0], hq.diag[1], hq.diag[2], hq.diag[3], hq.diag[4],
               hq.diag[5], hq.diag[6], hq.diag[7]);
        fflush(stdout);
        if (bad || hq.err) return 3;
    }
    timeit("rows", [&] { hipLaunchKernelGGL(k_rows, dim3(M * M / TQ), dim3(NT), 0, 0, x); });
    timeit("cols", [&] { hipLaunchKernelGGL(k_cols, dim3(M * M / TQ), dim3(NT), 0, 0, x); });
    timeit("sep", run_sep);
    for (int v = 0; v < 4; ++v) timeit(names[v], [&] { fused(v); });
    for (const DV& d : dvs) timeit(d.name, [&] { dyn(d); });
    {
        DynQ hq;
        CK(hipMemcpy(&hq, dq, sizeof(DynQ), hipMemcpyDeviceToHost));
        printf("{\"dyn_err\": %u, \"gen\": %u}\n", hq.err, hq.gen);
    }
    Ctl c;
    CK(hipMemcpy(&c, ctl, sizeof(Ctl), hipMemcpyDeviceToHost));
    printf("{\"final_err\": %u}\n", c.err);
    return 0;
}

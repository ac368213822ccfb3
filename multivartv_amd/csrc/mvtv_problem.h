// mvtv_problem.h — the mvtv_problem handle and host helpers shared by the C-ABI translation units
// (mvtv_capi.cpp: single-GPU ADMM, operators, setup; mvtv_slab.cpp: the slab-decomposed loop over RCCL).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>
#include <vector>

#include "mvtv/mvtv.h"
#include "mvtv_internal.h"

namespace mvtv {
extern thread_local std::string g_last_error;

inline mvtv_status fail(mvtv_status s, const std::string& msg) {
    g_last_error = msg;
    return s;
}
}  // namespace mvtv

#define HIP_TRY(expr)                                                                                 \
    do {                                                                                              \
        hipError_t _e = (expr);                                                                       \
        if (_e != hipSuccess)                                                                         \
            return mvtv::fail(_e == hipErrorOutOfMemory ? MVTV_OUT_OF_MEMORY : MVTV_HIP_ERROR,        \
                              std::string(#expr) + ": " + hipGetErrorString(_e));                     \
    } while (0)

#define MVTV_TRY(expr)                        \
    do {                                      \
        mvtv_status _s = (expr);              \
        if (_s != MVTV_OK) return _s;         \
    } while (0)

namespace mvtv {
constexpr int kPcgPoll = 8;   // PCG iterations enqueued between host polls of the done flag

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        (void)hipGetDevice(&prev);
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

inline mvtv_status alloc(double** ptr, size_t n) {
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(ptr), std::max<size_t>(n, 1) * sizeof(double)));
    return MVTV_OK;
}
}  // namespace mvtv

using namespace mvtv;   // the handle's members use the device-side types

struct mvtv_problem {
    int device = 0;
    hipStream_t stream = nullptr;
    Geom g{};
    int order = 0, weighted = 1, wmode = W_IDENTITY;
    double deltas[MVTV_MAX_DIMS] = {0, 0, 0, 0};
    int codes[kMaxBlocks] = {0};
    int sprime[kMaxBlocks] = {0};
    uint64_t blk_len[kMaxBlocks] = {0};
    int64_t E = 0;
    int grid = 1;
    bool fused3d = true;   // fused Chronopoulos-Gear PCG for p = 3 (MVTV_PCG=classic disables)
    int pcg_hint = 0;      // PCG iterations of the last theta-solve (poll schedule)

    double *oty = nullptr, *wdiag = nullptr;
    double *theta = nullptr, *edges = nullptr, *ga = nullptr, *gu = nullptr, *guprev = nullptr;
    double *r = nullptr, *p = nullptr, *q = nullptr, *thold = nullptr, *p2 = nullptr;
    double *partials = nullptr, *red = nullptr;
    PcgState* st = nullptr;
    double* stage = nullptr;
    size_t stage_n = 0;
    double* host_red = nullptr;   // pinned: reductions + PcgState mirror
    PcgState* host_st = nullptr;
    SpecPlan spec;                // spectral theta-solve tables (allocated when the mesh allows it)
    bool spec_mesh = false;       // every m_j <= 4096 a product of 2, 3, 5, 7 (spectral solve)
    bool spec_pow2 = false;       // ... and a power of two (k_dct8 / k_tri passes)
    bool spec_lead = false;       // dims 0..p-2 are (the slab loop: the last dimension may have any length)
    bool e3d = false;             // z-marching 3-D edge kernels
    bool f3d = false;             // fused 3-D edge update + gather (needs the second edge buffer)
    bool f4d = false;             // fused 4-D edge update + gather pass A (k_admm4a; second edge buffer, g4)
    double* edges2 = nullptr;     // ping-pong partner of edges for the fused kernel
    bool zpicked = false;         // the z ping-pong pair was chosen by timed probes (pick_zpair)
    double* edges3 = nullptr;     // third z buffer of the spectral loop (MVTV_EBUF3=1). On boxes where the fused
                                  // launches alternate fast / slow, the slow ones are those writing into
                                  // `edges` (measured 4.60 / 4.97 ms alternating -> 4.60 / 4.53 / 5.00);
                                  // +7.5 GB at 512^3
    double* pcg_b = nullptr;      // right-hand side of the spectrally preconditioned PCG
    double* g4 = nullptr;         // 4 N-arrays: the two-pass 4-D gather's partial sums
    double wmean = 1.0;           // mean(W): the preconditioner's identity weight
    double wstd = 0.0;            // std(W): chooses the diagonally scaled spectral preconditioner
    double wsum_own = 0.0, wsum2_own = 0.0;   // sum W, sum W^2 over the nodes [ibeg, iend) (slab: owned planes)
    double* pcg_s = nullptr;      // 1/s of the scaled spectral preconditioner
    double* pcg_t = nullptr;      // r / s, the preconditioner's input
    AdmmCtl* ctl = nullptr;       // device control block of the asynchronous ADMM loop
    AdmmCtl* host_ctl = nullptr;  // pinned mirror
    int admm_hint = 0;            // ADMM iterations of the last converged run (enqueue-ahead depth)
    // the asynchronous loop's two-iteration launch sequence captured as a HIP graph (mvtv_capi.cpp), valid while the
    // buffers and flags it was captured with (graph_key) are unchanged
    struct LoopGraph {
        std::vector<const void*> key;
        hipGraphExec_t exec = nullptr;   // nullptr: the capture failed, stream launches for this key
    };
    std::vector<LoopGraph> graphs;

    // slab decomposition (mvtv_problem_create_slab): this problem holds planes [zb, ze) of dim p-1
    // of a mesh with m_global planes, plus ghost planes below / above
    bool slab = false;
    int64_t m_global = 0, zb = 0, ze = 0;
    int g_lo = 0, g_hi = 0;
    double* slab_iface = nullptr;  // mvtv_slab_run: interface numbers of the distributed line solves (16 per line)
    hipStream_t comm_stream = nullptr;   // mvtv_slab_run: the collectives' stream (overlapped with `stream`)

    // resident ADMM state
    bool have_state = false;
    bool u_default = true;
    // the twin blocks (mvtv_internal.h twin_block) hold equal u: true for the variant defaults, checked on import
    bool twin_ok = true;
    bool twin_timed = false;   // the timed fused launches skipped the twin block (its bytes are not counted)
    int edge_mode = U_EXPLICIT;
    double t_z = 0.0, c_state = 1.0, rho = 0.0;

    // instrumentation
    bool timing = false;
    struct Pending {
        hipEvent_t a, b;
        int kid;
    };
    std::vector<Pending> pending;
    std::vector<hipEvent_t> ev_pool;
    double ms[MVTV_K_COUNT] = {0};
    int64_t launches[MVTV_K_COUNT] = {0};
    int64_t fold_fix = 0;   // timed folded first passes that also read g_u (a rho change before them)
    int64_t pcg_xmoves = 0;   // timed fused PCG iterations that also moved x (the odd ones)

    Launch L() const { return Launch{stream, grid}; }

    hipEvent_t get_event() {
        if (!ev_pool.empty()) {
            hipEvent_t e = ev_pool.back();
            ev_pool.pop_back();
            return e;
        }
        hipEvent_t e;
        (void)hipEventCreate(&e);
        return e;
    }
    int tstart(int kid) {
        if (!timing) return -1;
        Pending pd{get_event(), get_event(), kid};
        g_timed = TimedLaunch{pd.a, pd.b};   // stamped by the next kernel dispatch (klaunch)
        pending.push_back(pd);
        return int(pending.size()) - 1;
    }
    void tstop(int h) {
        if (h >= 0 && g_timed.start) pending[h].kid = -1;   // the launcher enqueued nothing
        g_timed = TimedLaunch{};
    }
    // second launch of a two-kernel launcher (armed in g_timed_b, moved to g_timed by the launcher)
    int tstart_b(int kid) {
        if (!timing) return -1;
        Pending pd{get_event(), get_event(), kid};
        g_timed_b = TimedLaunch{pd.a, pd.b};
        pending.push_back(pd);
        return int(pending.size()) - 1;
    }
    void tstop_b(int h) {
        if (h >= 0 && g_timed_b.start) pending[h].kid = -1;
        g_timed_b = TimedLaunch{};
    }
    void harvest() {  // call after a stream sync
        for (auto& pd : pending) {
            float t = 0.f;
            if (pd.kid >= 0 && hipEventElapsedTime(&t, pd.a, pd.b) == hipSuccess) {
                ms[pd.kid] += t;
                launches[pd.kid] += 1;
            }
            ev_pool.push_back(pd.a);
            ev_pool.push_back(pd.b);
        }
        pending.clear();
    }
    mvtv_status sync() {
        HIP_TRY(hipStreamSynchronize(stream));
        harvest();
        return MVTV_OK;
    }
};

// timed choice of the fused 3-D kernel's z ping-pong buffer pair, once per problem (mvtv_capi.cpp pick_zpair)
mvtv_status zpair_pick(mvtv_problem* P, bool track_theta, bool twin);

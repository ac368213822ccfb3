// mvtv_internal.h — device-side geometry, block tables and launcher declarations.
//
// The difference operator D of the reference (create_D, cpp-code/utils.cpp:245-269;
// rcpp-code/MultivarTV/src/utils.cpp:218-232; code/utils.py:138-149) is never
// materialised. It is described by the mesh shape plus, per row block k, its
// binary code b (MSB = dim 0), the effective difference set S'(b) (the
// dim-0-first mixed-partial quirk) and its weight w_k.
// D^T D is then the sum over subsets S of cS[S] * (tensor product of 1-D Neumann
// Laplacians over S), cS[S] = sum of w_k^2 over blocks with S'_k == S.
#pragma once
#include <stdint.h>

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdlib>

namespace mvtv {

// Experiment knobs (tile shapes, buffer placement probes, alternative kernels) are read from the
// environment only in a probe build (`make PROBES=1`, -DMVTV_PROBES); the release library always
// takes the defaults. The run-time options a user may set are MVTV_ZPICK=0 (keep the allocation-order
// z buffer pair), MVTV_ADMM_SYNC=1 (host-synchronous ADMM loop) and MVTV_PCG=classic (3-kernel PCG).
inline const char* probe_env(const char* name) {
#ifdef MVTV_PROBES
    return std::getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}

// a probe switch: set to a non-zero number (probe builds only)
inline bool probe_flag(const char* name) {
    const char* e = probe_env(name);
    return e && std::atoi(e) != 0;
}

// Unsigned 32-bit division by an invariant divisor (Granlund-Montgomery):
// q = (umulhi(n, mul) + n) >> shift, evaluated with a 64-bit add so it holds for every n < 2^32.
struct FastDiv {
    uint32_t d, mul, shift;
    __host__ __device__ FastDiv() : d(1), mul(0), shift(0) {}
    __host__ explicit FastDiv(uint32_t div) : d(div) {
        shift = 0;
        while ((uint64_t(1) << shift) < div) ++shift;
        mul = uint32_t(((uint64_t(1) << 32) * ((uint64_t(1) << shift) - div)) / div + 1);
        if (div == 1) { mul = 0; shift = 0; }
    }
    __host__ __device__ inline uint32_t div(uint32_t n) const {
#if defined(__HIP_DEVICE_COMPILE__)
        uint32_t hi = __umulhi(n, mul);
#else
        uint32_t hi = uint32_t((uint64_t(n) * mul) >> 32);
#endif
        return uint32_t((uint64_t(hi) + n) >> shift);
    }
};

constexpr int kMaxDims = 4;
constexpr int kMaxBlocks = 15;

// Effective difference set of binary code b in p dims, as a dim-bit mask (bit j = dim j).
__host__ __device__ constexpr int sprime_mask(int b, int p) {
    int S = 0, cnt = 0;
    for (int j = 0; j < p; ++j)
        if ((b >> (p - 1 - j)) & 1) { S |= 1 << j; ++cnt; }
    if (cnt <= 1 || (S & 1)) return S;
    int lo = 0;
    while (!((S >> lo) & 1)) ++lo;
    return (S & ~(1 << lo)) | 1;
}

// Binary code of row block k for a given order (0 = C++ create_D, 1 = Python create_D).
__host__ __device__ constexpr int block_code(int k, int p, int order) {
    return order == 0 ? (k == 0 ? (1 << p) - 1 : k) : k + 1;
}

// Twin blocks: under the S' map several codes can share one difference set (3-D: {1,2} -> {0,2}, the rows of {0,2};
// 4-D: {1,2} -> {0,2}, {1,3}, {2,3} -> {0,3}, {1,2,3} -> {0,2,3}); with equal weights and equal state their alpha, u
// and z are the same numbers. twin_of(k) is the first block of k's group (k itself for the first), twin_count(k) the
// size of k's group; twin_block / twin_canon name the first pair (-1: none).
__host__ __device__ constexpr int twin_of(int k, int p, int order) {
    for (int j = 0; j < k; ++j)
        if (sprime_mask(block_code(k, p, order), p) == sprime_mask(block_code(j, p, order), p)) return j;
    return k;
}
__host__ __device__ constexpr int twin_count(int k, int nb, int p, int order) {
    int n = 0;
    for (int j = 0; j < nb; ++j)
        if (sprime_mask(block_code(k, p, order), p) == sprime_mask(block_code(j, p, order), p)) ++n;
    return n;
}
__host__ __device__ constexpr int twin_block(int nb, int p, int order) {
    for (int k = 0; k < nb; ++k)
        if (twin_of(k, p, order) != k) return k;
    return -1;
}
__host__ __device__ constexpr int twin_canon(int nb, int p, int order) {
    const int k = twin_block(nb, p, order);
    return k < 0 ? -1 : twin_of(k, p, order);
}
struct Geom {
    int32_t p;
    int32_t nb;            // number of row blocks of D
    uint32_t N;            // nodes
    uint32_t m[kMaxDims];
    uint32_t stride[kMaxDims];
    FastDiv fd[kMaxDims - 1];  // division by m0, m1, m2
    double w[kMaxBlocks];      // block weights, in block order
    double cS[16];             // D^T D coefficient per subset mask S of dims
    uint32_t ibeg, iend;       // nodes the edge kernels update and reduce over (slab: owned planes)
    uint32_t eaos;             // edge layout: 0 block-major z[k][N]; 1 64-node chunks z[N/64][nb][64]
};

// Offset of block k's word at node i in the edge buffer. Block-major keeps each block a separate
// stream; the chunked layout (eaos, p = 3 fused problems) puts all blocks of 64 consecutive nodes in
// one 64 * nb-word run, so the fused kernel's z traffic is one stream instead of nb.
__host__ __device__ __forceinline__ uint64_t eix(const Geom& g, int k, uint32_t i) {
    return g.eaos ? (((uint64_t(i >> 6) * uint32_t(g.nb) + uint32_t(k)) << 6) | uint64_t(i & 63u))
                  : uint64_t(k) * g.N + i;
}

// every twin carries its group's first block's weight (bitwise): the twins may then share one state
inline bool twin_weights_equal(const Geom& g, int order) {
    for (int k = 0; k < g.nb; ++k)
        if (g.w[twin_of(k, g.p, order)] != g.w[k]) return false;
    return twin_block(g.nb, g.p, order) >= 0;
}

// Per-node multi-index decode (column-major, dim 0 fastest).
template <int P>
__device__ __forceinline__ void decode(const Geom& g, uint32_t i, uint32_t (&c)[kMaxDims]) {
    uint32_t rest = i;
#pragma unroll
    for (int j = 0; j < P - 1; ++j) {
        uint32_t q = g.fd[j].div(rest);
        c[j] = rest - q * g.m[j];
        rest = q;
    }
    c[P - 1] = rest;
}

// Reductions produced by each kernel family (indices into the reduction vector).
enum EdgeRed { ER_R2 = 0, ER_D2 = 1, ER_A2 = 2, ER_DTH = 3, ER_N = 4 };          // ER_DTH is a max
enum GatherRed { GR_GU2 = 0, GR_S2B = 1, GR_S2A = 2, GR_N = 3 };
enum PcgRed { PR_B2 = 0, PR_RZ = 1, PR_R2 = 2, PR_N = 3 };

struct PcgState {
    double gamma;    // r.z
    double alpha, beta;
    double alpha_prev;   // the alpha of the last iteration run (k_cg3d's deferred x update, k_cg_xflush)
    double rnorm2, bnorm2;
    double rtol2;
    int32_t iter, maxit;
    int32_t done;
    int32_t pad;
};

// Device-resident ADMM control (asynchronous loop, mvtv_capi.cpp): the scalars the kernels of one
// iteration consume, written by k_admm_control at the end of each iteration. Every kernel of the
// loop returns at once when `done` is set, so the host can enqueue iterations ahead of the decision.
struct AdmmCtl {
    int32_t done, status, it, counter;
    int32_t variant, fixed_iters, max_counter, pad;
    double lambda, tol, sqrtN, sqrtE;
    double rho, sigma, c_prev, t_z, t_next;   // t_z: threshold z was formed with; t_next = lambda / rho
    double r_norm, s_norm, eps_pri, eps_dual, dtheta, dual_norm, primal_norm;
    // folded right-hand side (variant B, fused 3-D kernel): the kernel of an iteration stores s = rho (g_alpha + g_u)
    // with the rho it ran at, beside g_u. b = oty + rho' g_alpha + rho' c g_u of the next solve is then
    // oty + fold_ka s + fold_kb g_u, fold_ka = rho' / rho, fold_kb = rho' (c - 1): oty + s unless the control step
    // changed rho (fix != 0, the first pass also reads g_u)
    double fold_ka, fold_kb;
    int32_t fix;
    int32_t nfix;   // iterations after which fix was set and the loop went on (folded first passes reading g_u)
};

enum UMode { U_EXPLICIT = 0, U_FROM_Z = 1 };
enum WMode { W_NONE = 0, W_IDENTITY = 1, W_DIAG = 2 };

constexpr int kThreads = 256;
constexpr int kMaxGrid = 2048;   // grid-stride cap for streaming kernels (8 workgroups per CU)
constexpr int kMaxRed = 8;
constexpr int kMaxCgBlocks = 8192;   // workgroups of the fused 3-D PCG (partials buffer rows)

// ------------------------------------------------------------------ launchers
struct Launch {
    hipStream_t stream;
    int grid;
};

// Kernel timing (mvtv_capi.cpp instrumentation). When a start/stop pair is armed, the next launch
// goes through hipExtLaunchKernelGGL, which stamps the events from the kernel's own dispatch packet
// (the begin/end rocprofv3 reports). Separate hipEventRecord markers around a launch would add a
// barrier packet plus a cache release/acquire each, inflating the measured duration.
struct TimedLaunch {
    hipEvent_t start = nullptr, stop = nullptr;
};
extern thread_local TimedLaunch g_timed;
extern thread_local TimedLaunch g_timed_b;   // a two-kernel launcher's second launch

template <typename F, typename... Args>
inline void klaunch(F kernel, dim3 grid, dim3 block, uint32_t shmem, hipStream_t s, Args... args) {
    if (g_timed.start) {
        const TimedLaunch t = g_timed;
        g_timed = TimedLaunch{};
        hipExtLaunchKernelGGL(kernel, grid, block, shmem, s, t.start, t.stop, 0u, args...);
    } else {
        hipLaunchKernelGGL(kernel, grid, block, shmem, s, args...);
    }
}

// ctl != nullptr: scalars come from the device control block (t_old = t_z, c_old = c_prev,
// t_new = t_next; gather t = t_next) and the launch is a no-op once ctl->done is set
hipError_t launch_edge_update(const Geom& g, int order, int umode, const Launch& L, const double* theta,
                              double* edges, double t_old, double c_old, double t_new, const double* theta_old,
                              double* partials, const AdmmCtl* ctl = nullptr);
hipError_t launch_gather(const Geom& g, int order, int umode, const Launch& L, const double* edges, double t,
                         double* g_alpha, double* g_u, const double* g_uprev, double c_prev, double* partials,
                         const AdmmCtl* ctl = nullptr);
// partials: x.q per workgroup, L.grid rows, or *nparts rows when nparts is given (then a whole 2-D / 3-D
// mesh takes the marching k_apply2d / k_apply3d)
hipError_t launch_apply_A(const Geom& g, const Launch& L, double sigma, int wmode, const double* wdiag,
                          const double* x, double* q, double* partials, const PcgState* st, int* nparts = nullptr);
hipError_t launch_pcg_init(const Geom& g, const Launch& L, double sigma, int wmode, const double* wdiag,
                           const double* oty, const double* ga, double ca, const double* gb, double cb,
                           const double* x, double* r, double* p, double* partials);
hipError_t launch_pcg_update(const Geom& g, const Launch& L, double sigma, int wmode, const double* wdiag,
                             double* x, double* r, const double* p, const double* q, const PcgState* st,
                             double* partials);
hipError_t launch_pcg_pupdate(const Geom& g, const Launch& L, double sigma, int wmode, const double* wdiag,
                              const double* r, double* p, const PcgState* st);
// op: 0 plain (sums; max in the last nmax slots, or in the slots of bitmask -nmax when nmax < 0), 1 pcg-init, 2 pcg-after-Ap, 3 pcg-after-update,
// 4 cg3d prologue, 5 cg3d iteration
// ctl_step: after writing `out`, take the asynchronous ADMM loop's control step (k_admm_control) on ctl_step
// from the reduction vector step_red in the same launch
hipError_t launch_finalize(hipStream_t s, const double* partials, int nparts, int nr, int nmax, int op, double* out,
                           PcgState* st, double rtol2 = 0.0, int maxit = 0, const AdmmCtl* ctl = nullptr,
                           AdmmCtl* ctl_step = nullptr, const double* step_red = nullptr);
// end of an asynchronous ADMM iteration: red = [|r|^2, |D theta|^2, |alpha|^2, max dtheta, |g_u|^2,
// |s_B|^2, |s_A|^2]; adapt_step, stopping test and the next iteration's scalars (mvtv_capi.cpp mirror)
hipError_t launch_admm_control(hipStream_t s, AdmmCtl* ctl, const double* red);
// fused 3-D Chronopoulos-Gear PCG (mvtv_cg3d.hip): mode 0 prologue, 1 first iteration, 2 iteration;
// partials get 4 values per workgroup (gamma, delta, |r|^2, |b|^2), *nblocks_out workgroups
// z-marching q = (W + sigma D^T D) x for p = 2, same contract as launch_apply3d
hipError_t launch_apply2d(const Geom& g, hipStream_t s, double sigma, int wmode, const double* wdiag,
                          const double* x, double* q, double* partials = nullptr, const PcgState* st = nullptr,
                          int* nparts = nullptr);
// partials (with st, nparts): x.q per workgroup (*nparts rows), a no-op once st->done
hipError_t launch_apply3d(const Geom& g, hipStream_t s, double sigma, int wmode, const double* wdiag,
                          const double* x, double* q, double* partials = nullptr, const PcgState* st = nullptr,
                          int* nparts = nullptr);
// w-marching q = (W + sigma D^T D) x for p = 4, same contract as launch_apply3d
hipError_t launch_apply4d(const Geom& g, hipStream_t s, double sigma, int wmode, const double* wdiag,
                          const double* x, double* q, double* partials = nullptr, const PcgState* st = nullptr,
                          int* nparts = nullptr);
hipError_t launch_cg3d(const Geom& g, hipStream_t s, int mode, double sigma, int wmode, const double* wdiag,
                       double* x, const double* r_in, const double* p_in, double* r_out, double* p_out,
                       const double* oty, const double* ga, double ca,
                       const double* gb, double cb, const PcgState* st, double* partials, int* nblocks_out);
hipError_t launch_cg_xflush(hipStream_t s, uint64_t n, double* x, const double* p, const PcgState* st);
hipError_t launch_maxabsdiff(const Geom& g, const Launch& L, const double* a, const double* b, double* partials);
hipError_t launch_fill(hipStream_t s, double* x, double v, uint64_t n);
// CG vector steps of lam_max_pinv (op 0 |x|^2 into partials, 1 x += c p & y -= c t, 2 x = p + c x, 3 y -= c t)
hipError_t launch_cg_vec(const Geom& g, const Launch& L, int op, double coef, double* x, double* y, const double* p,
                         const double* t, double* partials);
// vector steps of PCG with the (optionally diagonally scaled) spectral preconditioner (mvtv_kernels.hip
// k_pcgs_vec): op 0 b and r = b - q with t = r sinv; 1 x, r update with t = r sinv; 2 z *= sinv and
// (r.z, |r|^2 [, |b|^2]) in PR layout; 3 p = z + beta p. sinv / t may be nullptr (no scaling)
hipError_t launch_pcgs_vec(const Geom& g, const Launch& L, int op, const double* oty, const double* ga, double ca,
                           const double* gb, double cb, double* x, double* r, double* p, const double* q, double* z,
                           double* b, const double* sinv, double* t, const PcgState* st, double* partials,
                           int with_b2);
// sinv = sqrt(dbar / jacobi_diag) of W + sigma D^T D
hipError_t launch_pcgs_sinv(const Geom& g, const Launch& L, double sigma, int wmode, const double* wdiag, double dbar,
                            double* sinv);
// per-workgroup max |D x| (one max-partial per workgroup, L.grid rows)
hipError_t launch_dmaxabs(const Geom& g, int order, const Launch& L, const double* x, double* partials);
// compact <-> padded edge layouts for one block segment [e0, e0+cnt) of block k
hipError_t launch_edges_import(const Geom& g, int order, hipStream_t s, int k, uint64_t e0, uint64_t cnt,
                               const double* compact, double* padded);
hipError_t launch_edges_export(const Geom& g, int order, hipStream_t s, int k, uint64_t e0, uint64_t cnt,
                               const double* padded, double* compact, int umode, double t, double c);
hipError_t launch_edges_z_to_u(hipStream_t s, double* edges, uint64_t n, double t, double c);
// edges = value on every real edge, 0 on padding (variant u0 fills: B 0, A and C 1/lambda)
hipError_t launch_edges_fill_valid(const Geom& g, int order, const Launch& L, double* edges, double value);
hipError_t launch_apply_D_padded(const Geom& g, int order, const Launch& L, const double* theta, double* edges);
// Spectral theta-solve tables (mvtv_spectral.hip), device-resident, offsets in doubles.
struct SpecPlan {
    double* tw = nullptr;     // per dim: m_j complex FFT twiddles e^{-2 pi i k/m_j}
    double* twq = nullptr;    // per dim: m_j complex twiddles e^{-i pi k/(2 m_j)}
    double* lam = nullptr;    // per dim: m_j eigenvalues 4 sin^2(pi k/(2 m_j)) of the Neumann Laplacian
    uint32_t* perm = nullptr; // per dim (at lam_off): position of sample k in the mixed-radix FFT's input order
    uint32_t tw_off[kMaxDims] = {0, 0, 0, 0}, twq_off[kMaxDims] = {0, 0, 0, 0}, lam_off[kMaxDims] = {0, 0, 0, 0};
    // lengths without a 2-3-5-7 plan (Bluestein, k_dctb): per such dim, at blu_off (doubles), m complex chirp values
    // e^{-i pi n^2/m}, then M values each of the forward and inverse kernels' transforms / M, then M twiddles
    // e^{-2 pi i k/M}; blu_M[j] = M = 2^ceil(log2(2 m_j - 1)), 0 for a planned dim
    double* blu = nullptr;
    uint32_t blu_off[kMaxDims] = {0, 0, 0, 0}, blu_M[kMaxDims] = {0, 0, 0, 0};
};
// PCG vector work folded into the d = 0 passes of a preconditioner solve (spectrally preconditioned PCG,
// power-of-two m_0 >= 64): mode 1, first pass (`in` = r): r -= alpha q and x += alpha p on load (r, x
// written back, the transform taken of sinv * r); mode 2, last pass: out = sinv * transform, (r.z, |r|^2)
// per workgroup into `partials` (k_finalize op 3 layout, *nparts rows; a launch whose rows would exceed
// `cap` words is refused with hipErrorInvalidValue). sinv may be null.
struct PcgFuse {
    int32_t mode = 0;
    const PcgState* st = nullptr;
    double *x = nullptr, *r = nullptr;
    const double *p = nullptr, *q = nullptr, *sinv = nullptr;
    double* partials = nullptr;
    size_t cap = 0;
    int* nparts = nullptr;
};
// the two in-plane passes (dims 0 and 1) in one launch (k_plane8): m0 = m1 a power of two in [16, 128], p >= 3,
// >= 1024 planes
bool plane_pass_ok(const Geom& g);
// mode 0: forward along dims 0 then 1 (b = in + ca ga + cb gb formed on load when ga != nullptr; fold: from the
// control block's fold_ka / fold_kb); mode 1: inverse along dims 1 then 0. In place allowed.
hipError_t launch_plane_pass(const SpecPlan& sp, const Geom& g, hipStream_t s, int mode, const double* in,
                             const double* ga, double ca, const double* gb, double cb, double* out,
                             const AdmmCtl* ctl = nullptr, const int32_t* skip = nullptr, bool fold = false);
// 3-D meshes solved as dim-2 forward pass, k_march forward, k_march backward, dim-2 inverse pass (m0 a power of two in
// [256, 2048], m1 a multiple of the march step, 128 <= m2 <= 4096)
bool march_ok(const Geom& g);
// the marching passes over every dim-2 frequency plane of x, in place: forward (dim-0 DCT of the rows + Thomas
// forward elimination along dim 1) or backward (back substitution + inverse dim-0 DCT, scaled by m1 / N)
hipError_t launch_march(const SpecPlan& sp, const Geom& g, hipStream_t s, bool bwd, double* x, double sigma, double w0,
                        const AdmmCtl* ctl = nullptr, const int32_t* skip = nullptr);
// true when the d = 0 passes of this mesh run in k_dct8 with their partial rows within partial_words
bool dct_pcg_fusable(const Geom& g, size_t partial_words);
// radices (8, 4, 2, 3, 5, 7 in stage order) of a line length m = 2^a 3^b 5^c 7^d; false for any other m
bool dct_radix_plan(uint32_t m, int* rad, int* nrad);
// mode 0 forward DCT-II, 1 inverse (DCT-III, unnormalised), 2 forward + divide by mu * N + inverse;
// ga != nullptr forms the input as in + ca*ga + cb*gb. In place (in == out) is allowed.
hipError_t launch_dct_pass(const SpecPlan& sp, const Geom& g, hipStream_t s, int mode, int d, const double* in,
                           const double* ga, double ca, const double* gb, double cb, double* out, double sigma,
                           double w0, const AdmmCtl* ctl = nullptr, uint32_t q_off = 0, double inv_n = 0.0,
                           const int32_t* skip = nullptr, const PcgFuse* pf = nullptr, bool fold = false);
// Slab-decomposed last-dimension solve by substructuring (mvtv_spectral.hip, k_tris): og = the owned planes
// (m[p-1] = their count, stride[p-1] = plane lines). phase 1: per line the first / last rows of G, H, K of
// the local block into coef [chunk s][6][line in chunk]; phase 3: x = scale * (local solve with the
// neighbours' values lr [chunk s][2][line in chunk]) in place. lo_ext / hi_ext: the lines continue on the
// rank below / above. launch_tri_iface: the interface systems of one chunk's lines over the G ranks.
// sigma, w0: the operator c0 = w0 + ..., c1 (ignored when ctl gives sigma); skip: return at once when *skip
hipError_t launch_tri_slab(const SpecPlan& sp, const Geom& og, hipStream_t s, int phase, double* x, double* coef,
                           const double* lr, uint32_t chunk, int lo_ext, int hi_ext, double scale,
                           const AdmmCtl* ctl, double sigma = 1.0, double w0 = 1.0, const int32_t* skip = nullptr);
// a block of n planes splits into k_tris segments (<= 64 of <= 32 rows): false for e.g. a prime n > 64
bool tri_slab_ok(uint32_t n);
// The factorised form (k_trisr, the default; round 6): phase 1 writes 2 numbers per line [chunk s][2][line in chunk]
// (the block's F at its last row, B at its first), the interface gives every block its 2 carries, phase 3 reads them
// from lr; the Thomas form (k_tris, probe builds with MVTV_TRI_IIR=0) exchanges 6 and 2. tri_slab_ncoef(): the phase-1
// numbers per line (the first all-to-all's count). launch_tri_iface: og = the owned planes' geometry (its dims
// 0..p-2 and the line constants), rank = the chunk's owner, mg = the global plane count.
int tri_slab_ncoef();
hipError_t launch_tri_iface(const SpecPlan& sp, const Geom& og, hipStream_t s, double* coef_in, double* lr_out,
                            uint32_t chunk, int G, int rank, uint32_t mg, const AdmmCtl* ctl, double sigma = 1.0,
                            double w0 = 1.0, const int32_t* skip = nullptr);
// z-marching 3-D edge kernels (mvtv_admm3d.hip); same partials layout as launch_edge_update /
// launch_gather, *nparts workgroup rows
bool edge3d_ok(const Geom& g);
// fused edge update + D^T gather for p = 3 (one pass over the edge state, z ping-pong buffers);
// partials: 7 per workgroup in the order ER_* then GR_* (slot ER_DTH is a max)
bool fused3d_ok(const Geom& g);
hipError_t launch_admm3d(const Geom& g, int order, int umode, hipStream_t s, const double* theta, const double* z_old,
                         double* z_new, double t_old, double c_old, double t_new, double c_prev,
                         const double* theta_old, double* g_alpha, double* g_u, const double* g_uprev,
                         double* partials, int* nparts, const AdmmCtl* ctl = nullptr, bool fold = false,
                         bool twin = false);
hipError_t launch_edges_copy_block(const Geom& g, hipStream_t s, double* edges, int kdst, int ksrc, uint32_t i0 = 0,
                                   uint32_t i1 = 0xffffffffu);
hipError_t fill_twins(const Geom& g, int order, hipStream_t s, double* edges, uint32_t i0 = 0, uint32_t i1 = 0xffffffffu);
hipError_t launch_edge3d(const Geom& g, int order, int umode, hipStream_t s, const double* theta, double* edges,
                         double t_old, double c_old, double t_new, const double* theta_old, double* partials,
                         int* nparts, const AdmmCtl* ctl = nullptr);
// scratch4: 4 N-arrays for the two-pass 4-D gather (p = 4); nullptr selects the one-pass kernels
hipError_t launch_gather3d(const Geom& g, int order, int umode, hipStream_t s, const double* edges, double t,
                           double* g_alpha, double* g_u, const double* g_uprev, double c_prev, double* partials,
                           int* nparts, const AdmmCtl* ctl = nullptr, double* scratch4 = nullptr, bool fold = false);
bool gather4_ok(const Geom& g);
// fused 4-D edge update + the two-pass gather's pass A (k_admm4a, z ping-pong buffers), then pass B alone:
// ER partials from the first launch (*nparts rows), GR partials from the second
bool fused4_ok(const Geom& g);
hipError_t launch_admm4a(const Geom& g, int order, int umode, hipStream_t s, const double* theta, const double* z_old,
                         double* z_new, double t_old, double c_old, double t_new, const double* theta_old,
                         double* scratch4, double* partials, int* nparts, const AdmmCtl* ctl = nullptr, bool twin = false);
hipError_t launch_gather4b(const Geom& g, int umode, hipStream_t s, double* g_alpha, double* g_u, const double* g_uprev,
                           double c_prev, double* partials, int* nparts, const AdmmCtl* ctl, double* scratch4,
                           bool fold = false);
// a slab rank's pass A on its lower ghost plane (w = first owned - 1), after the z halo brought that plane's z_new
hipError_t launch_gather4a_ghost(const Geom& g, int order, hipStream_t s, const double* edges, double* scratch4,
                                 const AdmmCtl* ctl);
hipError_t launch_gather_index(hipStream_t s, const double* theta, const int64_t* idx, int64_t n, double* out);

// scattered-data setup (mvtv_scatter.hip)
// axes_host_span[j] = axis_j[last] - axis_j[0] (host values; only the first guess of the bracket)
hipError_t launch_nearest(hipStream_t s, int p, const uint32_t* m, const double* axes, const double* axes_host_span,
                          const double* data, int64_t n, uint32_t* key, int64_t* idx_out);
hipError_t launch_scatter_sums(hipStream_t s, uint32_t* key, const double* y, int64_t n, uint32_t N, double* oty,
                               double* wdiag, unsigned long long* nruns);

}  // namespace mvtv

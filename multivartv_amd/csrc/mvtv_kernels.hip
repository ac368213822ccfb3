// mvtv_kernels.hip — CDNA4 (gfx950) kernels of the mesh-TV ADMM hot path.
//
// Reference operations replaced (rcpp-code/MultivarTV/src/solvers.cpp):
//   D*theta, softthresh, alpha - D*theta, u += r   (:114-116)   -> k_edge_update
//   Dt*(alpha+u), Dt*(u-uold), Dt*u                  (:112,117,121) -> k_gather
//   spsolve(W + rho D^T D, b)  (SuperLU, :113)                  -> Jacobi-PCG: k_pcg_init,
//                                                                  k_apply_A, k_pcg_update, k_pcg_pupdate
//   norm(...) (:119-122)                                        -> fused block reductions + k_finalize
//
// Edge vectors live in a PADDED layout: block k occupies [k*N, (k+1)*N) indexed by the node at
// which the forward difference is anchored. Entries whose anchor sits on the upper face of a
// differenced dimension are padding and stay exactly 0: theta is read with upper-clamped indices,
// so their difference is 0, and the dual state there starts at 0. The dual state is kept as the
// single edge array z = D theta - u_old (one E-vector instead of alpha and u):
//   alpha = soft(z, t) = z - clamp(z, -t, t),   u = -c * clamp(z, -t, t)
// where t = lambda/rho at the time z was formed and c is the accumulated adapt_step scale.
#include "mvtv_device.h"

namespace mvtv {

thread_local TimedLaunch g_timed;
thread_local TimedLaunch g_timed_b;

// Jacobi diagonal of W + sigma * sum_S cS[S] (x)_{j in S} L_j at a node with multi-index c:
// the 1-D Neumann Laplacian's diagonal is (c > 0) + (c < m - 1).
template <int P, int WM>
__device__ __forceinline__ double jacobi_diag(const Geom& g, double sigma, const double* __restrict__ wdiag,
                                              uint32_t i, const uint32_t (&c)[kMaxDims]) {
    double l[P];
#pragma unroll
    for (int j = 0; j < P; ++j) l[j] = double(c[j] > 0) + double(c[j] + 1 < g.m[j]);
    double acc = 0.0;
#pragma unroll
    for (int S = 1; S < (1 << P); ++S) {
        double prod = g.cS[S];
#pragma unroll
        for (int j = 0; j < P; ++j)
            if ((S >> j) & 1) prod *= l[j];
        acc += prod;
    }
    double wv = (WM == W_DIAG) ? wdiag[i] : (WM == W_IDENTITY ? 1.0 : 0.0);
    return wv + sigma * acc;
}

// K-weighted 3^P-point stencil with per-dimension clamped neighbours: (D^T D x)_i.
template <int P>
__device__ __forceinline__ double stencil_DtD(const Geom& g, const double* __restrict__ x, uint32_t i,
                                              const uint32_t (&c)[kMaxDims], const double* __restrict__ K) {
    int32_t lo[P], hi[P];
#pragma unroll
    for (int j = 0; j < P; ++j) {
        lo[j] = c[j] > 0 ? -int32_t(g.stride[j]) : 0;
        hi[j] = c[j] + 1 < g.m[j] ? int32_t(g.stride[j]) : 0;
    }
    double acc = 0.0;
    constexpr int NT = (P == 1) ? 3 : (P == 2) ? 9 : (P == 3) ? 27 : 81;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        int32_t off = 0;
        int tt = t;
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const int o = tt % 3;
            tt /= 3;
            off += (o == 0) ? lo[j] : (o == 2 ? hi[j] : 0);
        }
        acc = fma(K[t], x[int64_t(i) + off], acc);
    }
    return acc;
}

// --------------------------------------------------------------------- edge update
// z_new = D theta - u_old; alpha = soft(z_new, t_new); r = alpha - D theta.
// Reductions: |r|^2, |D theta|^2, |alpha|^2 and (DTH) max |theta - theta_old|.
template <int P, int ORD, int UM, bool DTH>
__global__ __launch_bounds__(kThreads) void k_edge_update(Geom g, const double* __restrict__ theta,
                                                          double* __restrict__ edges, double t_old,
                                                          double c_old, double t_new,
                                                          const double* __restrict__ theta_old,
                                                          double* __restrict__ partials, const AdmmCtl* ctl) {
    constexpr int NC = 1 << P;
    if (ctl) {
        if (ctl->done) return;
        t_old = ctl->t_z;
        c_old = ctl->c_prev;
        t_new = ctl->t_next;
    }
    double red[ER_N] = {0.0, 0.0, 0.0, 0.0};
    for (uint32_t i = g.ibeg + blockIdx.x * kThreads + threadIdx.x; i < g.iend; i += gridDim.x * kThreads) {
        uint32_t c[kMaxDims];
        decode<P>(g, i, c);
        double a[NC];
#pragma unroll
        for (int T = 0; T < NC; ++T) {
            uint32_t idx = i;
#pragma unroll
            for (int j = 0; j < P; ++j)
                if ((T >> j) & 1) idx += (c[j] + 1 < g.m[j]) ? g.stride[j] : 0u;
            a[T] = theta[idx];
        }
        if constexpr (DTH) red[ER_DTH] = fmax(red[ER_DTH], fabs(a[0] - theta_old[i]));
        // forward-difference butterfly: afterwards a[S] = sum_{T subset S} (-1)^|T| theta(i + e_T)
#pragma unroll
        for (int j = 0; j < P; ++j) {
#pragma unroll
            for (int T = 0; T < NC; ++T)
                if (!((T >> j) & 1)) a[T | (1 << j)] = a[T] - a[T | (1 << j)];
        }
        static_for<0, NC - 1>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            constexpr int S = sprime_mask(block_code(k, P, ORD), P);
            if (k < g.nb) {
                const double d = g.w[k] * a[S];
                const uint64_t e = eix(g, k, i);
                const double stored = edges[e];
                const double uo = (UM == U_EXPLICIT) ? stored : -c_old * clampd(stored, t_old);
                const double z = d - uo;
                const double al = z - clampd(z, t_new);
                const double r = al - d;
                edges[e] = z;
                red[ER_R2] = fma(r, r, red[ER_R2]);
                red[ER_D2] = fma(d, d, red[ER_D2]);
                red[ER_A2] = fma(al, al, red[ER_A2]);
            }
        });
    }
    block_reduce_store<ER_N, 1>(red, partials);
}

// --------------------------------------------------------------------- D^T gather
// g_alpha = D^T alpha, g_u = D^T u (u unscaled: -clamp(z, t)); explicit mode: g_u = D^T v.
// Reductions: |g_u|^2, |g_u - c_prev g_uprev|^2 (B's dual residual), |g_alpha + c_prev g_uprev|^2 (A's).
template <int P, int ORD, int UM, bool PREV>
__global__ __launch_bounds__(kThreads) void k_gather(Geom g, const double* __restrict__ edges, double t,
                                                     double* __restrict__ g_alpha, double* __restrict__ g_u,
                                                     const double* __restrict__ g_uprev, double c_prev,
                                                     double* __restrict__ partials, const AdmmCtl* ctl) {
    constexpr int NC = 1 << P;
    if (ctl) {
        if (ctl->done) return;
        t = ctl->t_next;
        c_prev = ctl->c_prev;
    }
    double red[GR_N] = {0.0, 0.0, 0.0};
    for (uint32_t i = g.ibeg + blockIdx.x * kThreads + threadIdx.x; i < g.iend; i += gridDim.x * kThreads) {
        uint32_t c[kMaxDims];
        decode<P>(g, i, c);
        double ga = 0.0, gu = 0.0;
        static_for<0, NC - 1>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            constexpr int S = sprime_mask(block_code(k, P, ORD), P);
            if (k < g.nb) {
                double aa = 0.0, au = 0.0;
#pragma unroll
                for (int T = 0; T < NC; ++T) {
                    if ((T & ~S) != 0) continue;   // T subset of S
                    bool ok = true;
                    uint32_t idx = i;
#pragma unroll
                    for (int j = 0; j < P; ++j)
                        if ((T >> j) & 1) {
                            ok = ok && (c[j] > 0);
                            idx -= g.stride[j];
                        }
                    const double vv = edges[eix(g, k, ok ? idx : i)];
                    const double v = ok ? vv : 0.0;
                    const bool neg = __builtin_popcount(T) & 1;
                    if constexpr (UM == U_FROM_Z) {
                        const double cl = clampd(v, t);
                        const double al = v - cl;
                        aa = neg ? aa - al : aa + al;
                        au = neg ? au + cl : au - cl;   // u = -clamp
                    } else {
                        au = neg ? au - v : au + v;
                    }
                }
                ga = fma(g.w[k], aa, ga);
                gu = fma(g.w[k], au, gu);
            }
        });
        if constexpr (UM == U_FROM_Z) g_alpha[i] = ga;
        g_u[i] = gu;
        red[GR_GU2] = fma(gu, gu, red[GR_GU2]);
        if constexpr (PREV) {
            const double gp = c_prev * g_uprev[i];
            const double db = gu - gp, da = ga + gp;
            red[GR_S2B] = fma(db, db, red[GR_S2B]);
            red[GR_S2A] = fma(da, da, red[GR_S2A]);
        }
    }
    block_reduce_store<GR_N, 0>(red, partials);
}

// --------------------------------------------------------------------- D (padded output)
template <int P, int ORD>
__global__ __launch_bounds__(kThreads) void k_apply_D(Geom g, const double* __restrict__ theta,
                                                      double* __restrict__ edges) {
    constexpr int NC = 1 << P;
    for (uint32_t i = blockIdx.x * kThreads + threadIdx.x; i < g.N; i += gridDim.x * kThreads) {
        uint32_t c[kMaxDims];
        decode<P>(g, i, c);
        double a[NC];
#pragma unroll
        for (int T = 0; T < NC; ++T) {
            uint32_t idx = i;
#pragma unroll
            for (int j = 0; j < P; ++j)
                if ((T >> j) & 1) idx += (c[j] + 1 < g.m[j]) ? g.stride[j] : 0u;
            a[T] = theta[idx];
        }
#pragma unroll
        for (int j = 0; j < P; ++j) {
#pragma unroll
            for (int T = 0; T < NC; ++T)
                if (!((T >> j) & 1)) a[T | (1 << j)] = a[T] - a[T | (1 << j)];
        }
        static_for<0, NC - 1>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            constexpr int S = sprime_mask(block_code(k, P, ORD), P);
            if (k < g.nb) edges[eix(g, k, i)] = g.w[k] * a[S];
        });
    }
}

template <int P, int ORD>
__global__ __launch_bounds__(kThreads) void k_edges_fill_valid(Geom g, double* __restrict__ edges, double value) {
    constexpr int NC = 1 << P;
    for (uint32_t i = blockIdx.x * kThreads + threadIdx.x; i < g.N; i += gridDim.x * kThreads) {
        uint32_t c[kMaxDims];
        decode<P>(g, i, c);
        static_for<0, NC - 1>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            constexpr int S = sprime_mask(block_code(k, P, ORD), P);
            if (k < g.nb) {
                bool valid = true;
#pragma unroll
                for (int j = 0; j < P; ++j)
                    if ((S >> j) & 1) valid = valid && (c[j] + 1 < g.m[j]);
                edges[eix(g, k, i)] = valid ? value : 0.0;
            }
        });
    }
}

// --------------------------------------------------------------------- theta-solve (Jacobi-PCG)
struct StencilK {
    double K[81];
};

template <int P, int WM, bool DOT, bool CHECK>
__global__ __launch_bounds__(kThreads) void k_apply_A(Geom g, StencilK sk, double sigma,
                                                      const double* __restrict__ wdiag,
                                                      const double* __restrict__ x, double* __restrict__ q,
                                                      double* __restrict__ partials,
                                                      const PcgState* __restrict__ st) {
    if constexpr (CHECK) {
        if (st->done) return;
    }
    double red[1] = {0.0};
    // nodes [ibeg, iend): a slab rank's owned planes (its ghost planes are read as neighbours only)
    for (uint32_t i = g.ibeg + blockIdx.x * kThreads + threadIdx.x; i < g.iend; i += gridDim.x * kThreads) {
        uint32_t c[kMaxDims];
        decode<P>(g, i, c);
        const double xi = x[i];
        const double wv = (WM == W_DIAG) ? wdiag[i] : (WM == W_IDENTITY ? 1.0 : 0.0);
        const double qi = fma(sigma, stencil_DtD<P>(g, x, i, c, sk.K), wv * xi);
        q[i] = qi;
        if constexpr (DOT) red[0] = fma(xi, qi, red[0]);
    }
    if constexpr (DOT) block_reduce_store<1, 0>(red, partials);
}

// r = b - A x with b = oty + ca*ga + cb*gb; p = z = r / diag.  Reductions: |b|^2, r.z, |r|^2.
template <int P, int WM>
__global__ __launch_bounds__(kThreads) void k_pcg_init(Geom g, StencilK sk, double sigma,
                                                       const double* __restrict__ wdiag,
                                                       const double* __restrict__ oty,
                                                       const double* __restrict__ ga, double ca,
                                                       const double* __restrict__ gb, double cb,
                                                       const double* __restrict__ x, double* __restrict__ r,
                                                       double* __restrict__ p, double* __restrict__ partials) {
    double red[PR_N] = {0.0, 0.0, 0.0};
    for (uint32_t i = blockIdx.x * kThreads + threadIdx.x; i < g.N; i += gridDim.x * kThreads) {
        uint32_t c[kMaxDims];
        decode<P>(g, i, c);
        const double b = fma(cb, gb[i], fma(ca, ga[i], oty[i]));
        const double wv = (WM == W_DIAG) ? wdiag[i] : (WM == W_IDENTITY ? 1.0 : 0.0);
        const double ax = fma(sigma, stencil_DtD<P>(g, x, i, c, sk.K), wv * x[i]);
        const double rr = b - ax;
        const double z = rr / jacobi_diag<P, WM>(g, sigma, wdiag, i, c);
        r[i] = rr;
        p[i] = z;
        red[PR_B2] = fma(b, b, red[PR_B2]);
        red[PR_RZ] = fma(rr, z, red[PR_RZ]);
        red[PR_R2] = fma(rr, rr, red[PR_R2]);
    }
    block_reduce_store<PR_N, 0>(red, partials);
}

// x += alpha p; r -= alpha q; z = r / diag.  Reductions: r.z, |r|^2.
template <int P, int WM>
__global__ __launch_bounds__(kThreads) void k_pcg_update(Geom g, double sigma, const double* __restrict__ wdiag,
                                                         double* __restrict__ x, double* __restrict__ r,
                                                         const double* __restrict__ p,
                                                         const double* __restrict__ q,
                                                         const PcgState* __restrict__ st,
                                                         double* __restrict__ partials) {
    if (st->done) return;
    const double alpha = st->alpha;
    double red[2] = {0.0, 0.0};
    for (uint32_t i = blockIdx.x * kThreads + threadIdx.x; i < g.N; i += gridDim.x * kThreads) {
        uint32_t c[kMaxDims];
        decode<P>(g, i, c);
        const double pi = p[i];
        x[i] = fma(alpha, pi, x[i]);
        const double rn = fma(-alpha, q[i], r[i]);
        r[i] = rn;
        const double z = rn / jacobi_diag<P, WM>(g, sigma, wdiag, i, c);
        red[0] = fma(rn, z, red[0]);
        red[1] = fma(rn, rn, red[1]);
    }
    block_reduce_store<2, 0>(red, partials);
}

// p = z + beta p
template <int P, int WM>
__global__ __launch_bounds__(kThreads) void k_pcg_pupdate(Geom g, double sigma, const double* __restrict__ wdiag,
                                                          const double* __restrict__ r, double* __restrict__ p,
                                                          const PcgState* __restrict__ st) {
    if (st->done) return;
    const double beta = st->beta;
    for (uint32_t i = blockIdx.x * kThreads + threadIdx.x; i < g.N; i += gridDim.x * kThreads) {
        uint32_t c[kMaxDims];
        decode<P>(g, i, c);
        const double z = r[i] / jacobi_diag<P, WM>(g, sigma, wdiag, i, c);
        p[i] = fma(beta, p[i], z);
    }
}

// One thread: the host loop body of mvtv_admm_run after the reductions, verbatim (same operations
// in the same order, so decisions match the synchronous loop), then the next iteration's top test.
__device__ __forceinline__ void admm_control_step(AdmmCtl* __restrict__ c, const double* __restrict__ R) {
    const double* G = R + ER_N;
    const double r_norm = sqrt(R[ER_R2]);
    const double rho = c->rho;
    c->t_z = c->t_next;
    c->it += 1;
    c->counter += 1;
    double c_next = 1.0, rho_next = rho;
    int status = 0;
    const bool fixed = c->fixed_iters > 0;
    if (c->variant == 0) {   // B: rcpp-code/MultivarTV/src/solvers.cpp:117-125
        c->dual_norm = fabs(rho) * sqrt(G[GR_S2B]);
        c->primal_norm = r_norm;
        c->eps_dual = c->tol * (c->sqrtN + sqrt(G[GR_GU2]));
        c->eps_pri = c->tol * (c->sqrtE + fmax(sqrt(R[ER_D2]), sqrt(R[ER_A2])));
        const double tau = 2.0;
        if (c->primal_norm > 10 * c->dual_norm) {
            rho_next = tau * rho;
            c_next = 1.0 / tau;
        } else if (c->dual_norm > 10 * c->primal_norm) {
            rho_next = 1.0 / tau * rho;
            c_next = tau;
        }
        c->s_norm = c->dual_norm;
    } else if (c->variant == 1) {   // A: cpp-code/solvers.cpp:118-126
        const double s_norm = fabs(rho) * sqrt(G[GR_S2A]);
        c->dtheta = R[ER_DTH];
        c->s_norm = s_norm;
        if (!fixed && c->counter > c->max_counter) {
            status = 1;
            rho_next = rho;
        } else {
            if (r_norm > 20 * s_norm) {
                rho_next = 20 * rho;
                c_next = 0.05;
            } else if (s_norm > 20 * r_norm) {
                rho_next = 0.1 * rho;
                c_next = 10.0;
            }
            rho_next = double(int(rho_next));
        }
    } else {
        c->dtheta = R[ER_DTH];
    }
    c->r_norm = r_norm;
    // b_next = oty + rho_next D^T alpha + rho_next c_next D^T u from the folded s = rho (D^T alpha + D^T u) and D^T u
    c->fix = (rho_next != rho || c_next != 1.0) ? 1 : 0;
    c->fold_ka = c->fix ? rho_next / rho : 1.0;
    c->fold_kb = c->fix ? rho_next * (c_next - 1.0) : 0.0;
    c->c_prev = c_next;
    c->rho = rho_next;
    if (c->variant == 0) c->sigma = rho_next;
    c->t_next = rho_next != 0.0 ? c->lambda / rho_next : INFINITY;
    if (status) {
        c->status = 1;
        c->done = 1;
        return;
    }
    if (c->variant == 0 && !fixed && c->counter > c->max_counter) {
        c->status = 1;
        c->done = 1;
        return;
    }
    // loop-top test of the next iteration
    if (fixed) {
        if (c->it >= c->fixed_iters) c->done = 1;
    } else if (c->variant == 0) {
        if (!(c->dual_norm > c->eps_dual || c->primal_norm > c->eps_pri)) c->done = 1;
    } else {
        if (!(c->dtheta > c->tol)) {
            c->done = 1;
        } else if (c->variant == 2 && c->it >= c->max_counter) {
            c->status = 1;
            c->done = 1;
        }
    }
    if (!c->done) c->nfix += c->fix;   // the next folded first pass reads g_u too (bytes accounting)
}

// --------------------------------------------------------------------- reductions / scalars
// Sums the per-block partials in a fixed order (deterministic), then applies the PCG scalar step.
__global__ __launch_bounds__(1024) void k_finalize(const double* __restrict__ partials, int nparts, int nr,
                                                   int nmax, int op, double* __restrict__ out, PcgState* st,
                                                   double rtol2, int maxit, const AdmmCtl* ctl,
                                                   AdmmCtl* ctl_step, const double* step_red) {
    if ((op == 2 || op == 3 || op == 5) && st->done) return;
    if (ctl && ctl->done) return;
    // lane t sums rows t, t + 1024, ... in order for every slot k (rows loaded in batches of 4: 4 nr loads in flight
    // per lane), then a fixed shuffle tree within each wave and one over the 16 wave sums: one barrier instead of the
    // 10 of an LDS halving tree (1024^2: the launch 10.6 us, 15 % of an iteration, before)
    __shared__ double sm[kMaxRed][16];
    __shared__ double res[kMaxRed];
    double acc[kMaxRed];
#pragma unroll
    for (int k = 0; k < kMaxRed; ++k) acc[k] = 0.0;
    unsigned mxm = 0;   // bit k: slot k is a max
    for (int k = 0; k < nr; ++k)
        if (nmax >= 0 ? k >= nr - nmax : ((-nmax >> k) & 1) != 0) mxm |= 1u << k;
    for (int b0 = threadIdx.x; b0 < nparts; b0 += 4 * 1024) {
        double v[4][kMaxRed];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int k = 0; k < kMaxRed; ++k)
                v[u][k] = (k < nr && b0 + u * 1024 < nparts) ? partials[(b0 + u * 1024) * nr + k] : 0.0;
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int k = 0; k < kMaxRed; ++k)
                if (k < nr && b0 + u * 1024 < nparts) acc[k] = ((mxm >> k) & 1u) ? fmax(acc[k], v[u][k]) : acc[k] + v[u][k];
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1)
#pragma unroll
        for (int k = 0; k < kMaxRed; ++k)
            if (k < nr) {
                const double o = __shfl_down(acc[k], off, 64);
                acc[k] = ((mxm >> k) & 1u) ? fmax(acc[k], o) : acc[k] + o;
            }
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < kMaxRed; ++k)
            if (k < nr) sm[k][wv] = acc[k];
    __syncthreads();
    if (wv != 0) return;
#pragma unroll
    for (int k = 0; k < kMaxRed; ++k) acc[k] = (k < nr && lane < 16) ? sm[k][lane] : 0.0;
#pragma unroll
    for (int off = 8; off > 0; off >>= 1)
#pragma unroll
        for (int k = 0; k < kMaxRed; ++k)
            if (k < nr) {
                const double o = __shfl_down(acc[k], off, 64);
                acc[k] = ((mxm >> k) & 1u) ? fmax(acc[k], o) : acc[k] + o;
            }
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < kMaxRed; ++k)
            if (k < nr) res[k] = acc[k];
    if (threadIdx.x != 0) return;
    if (out)
        for (int k = 0; k < nr; ++k) out[k] = res[k];
    if (ctl_step) {   // asynchronous ADMM loop: the iteration's control step in the same launch
        admm_control_step(ctl_step, step_red);
        return;
    }
    if (op == 1) {
        st->bnorm2 = res[PR_B2];
        st->gamma = res[PR_RZ];
        st->rnorm2 = res[PR_R2];
        st->rtol2 = rtol2;
        st->maxit = maxit;
        st->iter = 0;
        st->alpha = st->beta = 0.0;
        st->done = (res[PR_R2] <= rtol2 * res[PR_B2]) || maxit <= 0;
    } else if (op == 2) {
        st->alpha = st->gamma / res[0];
    } else if (op == 3) {
        const double gnew = res[0];
        st->beta = gnew / st->gamma;
        st->gamma = gnew;
        st->rnorm2 = res[1];
        st->iter += 1;
        st->done = (res[1] <= st->rtol2 * st->bnorm2) || st->iter >= st->maxit;
    } else if (op == 4) {   // fused 3-D PCG prologue: gamma0, delta0, |r0|^2, |b|^2
        st->bnorm2 = res[3];
        st->gamma = res[0];
        st->rnorm2 = res[2];
        st->alpha = res[0] / res[1];
        st->alpha_prev = 0.0;
        st->beta = 0.0;
        st->rtol2 = rtol2;
        st->maxit = maxit;
        st->iter = 0;
        st->done = (res[2] <= rtol2 * res[3]) || maxit <= 0;
    } else if (op == 5) {   // Chronopoulos-Gear scalar recurrences
        const double gnew = res[0], dnew = res[1];
        const double beta = gnew / st->gamma;
        st->alpha_prev = st->alpha;
        st->alpha = gnew / (dnew - beta * gnew / st->alpha);
        st->beta = beta;
        st->gamma = gnew;
        st->rnorm2 = res[2];
        st->iter += 1;
        st->done = (res[2] <= st->rtol2 * st->bnorm2) || st->iter >= st->maxit;
    }
}

__global__ __launch_bounds__(kThreads) void k_maxabsdiff(uint32_t n, const double* __restrict__ a,
                                                         const double* __restrict__ b,
                                                         double* __restrict__ partials) {
    double red[1] = {0.0};
    for (uint32_t i = blockIdx.x * kThreads + threadIdx.x; i < n; i += gridDim.x * kThreads)
        red[0] = fmax(red[0], fabs(a[i] - b[i]));
    block_reduce_store<1, 1>(red, partials);
}

__global__ void k_fill(double* __restrict__ x, double v, uint64_t n) {
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x)
        x[i] = v;
}

// --------------------------------------------------------------------- lam_max_pinv support
// CG on (D^T D) with the reference's recurrences (rcpp-code/MultivarTV/src/utils.cpp:306-355):
// op 0: sum x*x;  op 1: x += alpha p, d -= alpha t;  op 2: p = r + beta p;  op 3: y -= coef t
__global__ __launch_bounds__(kThreads) void k_cg_vec(int op, uint32_t n, double coef, double* __restrict__ x,
                                                     double* __restrict__ y, const double* __restrict__ p,
                                                     const double* __restrict__ t, double* __restrict__ partials) {
    double red[1] = {0.0};
    for (uint32_t i = blockIdx.x * kThreads + threadIdx.x; i < n; i += gridDim.x * kThreads) {
        if (op == 0) {
            red[0] = fma(x[i], x[i], red[0]);
        } else if (op == 1) {
            x[i] = fma(coef, p[i], x[i]);
            y[i] = fma(-coef, t[i], y[i]);
        } else if (op == 2) {
            x[i] = fma(coef, x[i], p[i]);   // x = p (the new r) + beta x
        } else {
            y[i] = fma(-coef, t[i], y[i]);
        }
    }
    if (op == 0) block_reduce_store<1, 0>(red, partials);
}

// max over all blocks and anchors of |(D x)_e| (padding anchors give exactly 0)
template <int P, int ORD>
__global__ __launch_bounds__(kThreads) void k_dmaxabs(Geom g, const double* __restrict__ x,
                                                      double* __restrict__ partials) {
    constexpr int NC = 1 << P;
    double red[1] = {0.0};
    for (uint32_t i = blockIdx.x * kThreads + threadIdx.x; i < g.N; i += gridDim.x * kThreads) {
        uint32_t c[kMaxDims];
        decode<P>(g, i, c);
        double a[NC];
#pragma unroll
        for (int T = 0; T < NC; ++T) {
            uint32_t idx = i;
#pragma unroll
            for (int j = 0; j < P; ++j)
                if ((T >> j) & 1) idx += (c[j] + 1 < g.m[j]) ? g.stride[j] : 0u;
            a[T] = x[idx];
        }
#pragma unroll
        for (int j = 0; j < P; ++j)
#pragma unroll
            for (int T = 0; T < NC; ++T)
                if (!((T >> j) & 1)) a[T | (1 << j)] = a[T] - a[T | (1 << j)];
        static_for<0, NC - 1>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            constexpr int S = sprime_mask(block_code(k, P, ORD), P);
            if (k < g.nb) red[0] = fmax(red[0], fabs(g.w[k] * a[S]));
        });
    }
    block_reduce_store<1, 1>(red, partials);
}

// --------------------------------------------------------------------- PCG with the spectral preconditioner
// A = W + sigma D^T D, preconditioner M = S A0 S with A0 = w0 I + sigma D^T D (exact inverse by cosine
// transforms, mvtv_spectral.hip) and S = diag(s) (sinv = 1/s; sinv == nullptr: S = I, plain spectral).
// op 0: b = oty + ca ga + cb gb, r = b - q (q = A x); t = r sinv
// op 1: x += alpha p, r -= alpha q (alpha from the PCG state); t = r sinv
// op 2: z *= sinv (the solve's output, in place); partials, 3 per workgroup: (|b|^2, r.z, |r|^2) = k_finalize
//       op 1's layout when with_b2, else (r.z, |r|^2, 0) = op 3's
// op 3: p = z + beta p
// (t == nullptr: no scaled copy; the solve reads r itself)
__global__ __launch_bounds__(kThreads) void k_pcgs_vec(int op, uint32_t n, const double* __restrict__ oty,
                                                       const double* __restrict__ ga, double ca,
                                                       const double* __restrict__ gb, double cb,
                                                       double* __restrict__ x, double* __restrict__ r,
                                                       double* __restrict__ p, const double* __restrict__ q,
                                                       double* __restrict__ z, double* __restrict__ b,
                                                       const double* __restrict__ sinv, double* __restrict__ t,
                                                       const PcgState* __restrict__ st, double* __restrict__ partials,
                                                       int with_b2) {
    // op 0 and the init reduction (with_b2) run before k_finalize op 1 resets st->done
    if (op != 0 && !(op == 2 && with_b2) && st->done) return;
    double red[3] = {0.0, 0.0, 0.0};
    const double alpha = op == 1 ? st->alpha : 0.0, beta = op == 3 ? st->beta : 0.0;
    for (uint32_t i = blockIdx.x * kThreads + threadIdx.x; i < n; i += gridDim.x * kThreads) {
        if (op == 0) {
            const double bi = fma(cb, gb[i], fma(ca, ga[i], oty[i]));
            b[i] = bi;
            const double ri = bi - q[i];
            r[i] = ri;
            if (t) t[i] = ri * sinv[i];
        } else if (op == 1) {
            x[i] = fma(alpha, p[i], x[i]);
            const double ri = fma(-alpha, q[i], r[i]);
            r[i] = ri;
            if (t) t[i] = ri * sinv[i];
        } else if (op == 2) {
            const double ri = r[i];
            double zi = z[i];
            if (sinv) {
                zi *= sinv[i];
                z[i] = zi;
            }
            if (with_b2) {
                red[PR_B2] = fma(b[i], b[i], red[PR_B2]);
                red[PR_RZ] = fma(ri, zi, red[PR_RZ]);
                red[PR_R2] = fma(ri, ri, red[PR_R2]);
            } else {
                red[0] = fma(ri, zi, red[0]);
                red[1] = fma(ri, ri, red[1]);
            }
        } else {
            p[i] = fma(beta, p[i], z[i]);
        }
    }
    if (op == 2) block_reduce_store<3, 0>(red, partials);
}

// sinv = sqrt(dbar / d) with d the Jacobi diagonal of W + sigma D^T D: the diagonal scaling of the spectral
// preconditioner when W varies a lot against sigma D^T D's diagonal (M -> Jacobi as sigma -> 0)
template <int P, int WM>
__global__ __launch_bounds__(kThreads) void k_pcgs_sinv(Geom g, double sigma, const double* __restrict__ wdiag,
                                                        double dbar, double* __restrict__ sinv) {
    for (uint32_t i = blockIdx.x * kThreads + threadIdx.x; i < g.N; i += gridDim.x * kThreads) {
        uint32_t c[kMaxDims];
        decode<P>(g, i, c);
        sinv[i] = sqrt(dbar / jacobi_diag<P, WM>(g, sigma, wdiag, i, c));
    }
}

struct RedDims {
    uint64_t rd[kMaxDims];
    uint64_t stride[kMaxDims];
    int p;
    Geom g;   // edge layout (eix)
    int k;
};

__global__ void k_edges_import(RedDims rdd, uint64_t base, uint64_t e0, uint64_t cnt,
                               const double* __restrict__ compact, double* __restrict__ padded) {
    for (uint64_t t = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; t < cnt; t += uint64_t(gridDim.x) * blockDim.x) {
        uint64_t e = e0 + t, idx = 0;
        for (int j = 0; j < rdd.p; ++j) {
            const uint64_t q = e / rdd.rd[j];
            idx += (e - q * rdd.rd[j]) * rdd.stride[j];
            e = q;
        }
        padded[eix(rdd.g, rdd.k, uint32_t(idx))] = compact[t];
    }
}

__global__ void k_edges_export(RedDims rdd, uint64_t base, uint64_t e0, uint64_t cnt,
                               const double* __restrict__ padded, double* __restrict__ compact, int umode,
                               double t_, double c_) {
    for (uint64_t t = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; t < cnt; t += uint64_t(gridDim.x) * blockDim.x) {
        uint64_t e = e0 + t, idx = 0;
        for (int j = 0; j < rdd.p; ++j) {
            const uint64_t q = e / rdd.rd[j];
            idx += (e - q * rdd.rd[j]) * rdd.stride[j];
            e = q;
        }
        const double v = padded[eix(rdd.g, rdd.k, uint32_t(idx))];
        compact[t] = (umode == U_FROM_Z) ? -c_ * clampd(v, t_) : v;
    }
}

__global__ void k_edges_z_to_u(double* __restrict__ edges, uint64_t n, double t_, double c_) {
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x)
        edges[i] = -c_ * clampd(edges[i], t_);
}

__global__ void k_gather_index(const double* __restrict__ theta, const int64_t* __restrict__ idx, int64_t n,
                               double* __restrict__ out) {
    for (int64_t t = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; t < n; t += int64_t(gridDim.x) * blockDim.x)
        out[t] = theta[idx[t]];
}

// --------------------------------------------------------------------- host launchers
namespace {

StencilK make_stencil(const Geom& g) {
    // K(o) = sum_S cS[S] prod_j f_j, f_j = (j in S) ? (o_j == 0 ? 2 : -1) : (o_j == 0 ? 1 : 0);
    // offsets o_j in {-1, 0, +1} are encoded base-3 as (0 -> -1, 1 -> 0, 2 -> +1), dim 0 least significant.
    StencilK sk{};
    int nt = 1;
    for (int j = 0; j < g.p; ++j) nt *= 3;
    for (int t = 0; t < nt; ++t) {
        double acc = 0.0;
        for (int S = 1; S < (1 << g.p); ++S) {
            double prod = g.cS[S];
            int tt = t;
            for (int j = 0; j < g.p; ++j) {
                const int o = tt % 3;
                tt /= 3;
                const bool inS = (S >> j) & 1;
                prod *= inS ? (o == 1 ? 2.0 : -1.0) : (o == 1 ? 1.0 : 0.0);
            }
            acc += prod;
        }
        sk.K[t] = acc;
    }
    return sk;
}

template <class F>
hipError_t dispatch_p(int p, F&& f) {
    switch (p) {
        case 1: return f(std::integral_constant<int, 1>{});
        case 2: return f(std::integral_constant<int, 2>{});
        case 3: return f(std::integral_constant<int, 3>{});
        case 4: return f(std::integral_constant<int, 4>{});
        default: return hipErrorInvalidValue;
    }
}

template <class F>
hipError_t dispatch_w(int wmode, F&& f) {
    switch (wmode) {
        case W_NONE: return f(std::integral_constant<int, W_NONE>{});
        case W_IDENTITY: return f(std::integral_constant<int, W_IDENTITY>{});
        default: return f(std::integral_constant<int, W_DIAG>{});
    }
}

RedDims red_dims(const Geom& g, int order, int k) {
    RedDims r{};
    r.p = g.p;
    const int S = sprime_mask(block_code(k, g.p, order), g.p);
    for (int j = 0; j < g.p; ++j) {
        r.rd[j] = g.m[j] - ((S >> j) & 1);
        r.stride[j] = g.stride[j];
    }
    r.g = g;
    r.k = k;
    return r;
}

int elem_grid(uint64_t n) {
    uint64_t b = (n + 255) / 256;
    return int(b < 4096 ? (b ? b : 1) : 4096);
}

}  // namespace

hipError_t launch_edge_update(const Geom& g, int order, int umode, const Launch& L, const double* theta,
                              double* edges, double t_old, double c_old, double t_new, const double* theta_old,
                              double* partials, const AdmmCtl* ctl) {
    return dispatch_p(g.p, [&](auto pc) {
        constexpr int P = decltype(pc)::value;
        auto go = [&](auto kern) {
            klaunch(kern, dim3(L.grid), dim3(kThreads), 0, L.stream, g, theta, edges, t_old, c_old, t_new,
                               theta_old, partials, ctl);
            return hipGetLastError();
        };
        const bool dth = theta_old != nullptr;
        if (order == 0) {
            if (umode == U_EXPLICIT)
                return dth ? go(k_edge_update<P, 0, U_EXPLICIT, true>) : go(k_edge_update<P, 0, U_EXPLICIT, false>);
            return dth ? go(k_edge_update<P, 0, U_FROM_Z, true>) : go(k_edge_update<P, 0, U_FROM_Z, false>);
        }
        if (umode == U_EXPLICIT)
            return dth ? go(k_edge_update<P, 1, U_EXPLICIT, true>) : go(k_edge_update<P, 1, U_EXPLICIT, false>);
        return dth ? go(k_edge_update<P, 1, U_FROM_Z, true>) : go(k_edge_update<P, 1, U_FROM_Z, false>);
    });
}

hipError_t launch_gather(const Geom& g, int order, int umode, const Launch& L, const double* edges, double t,
                         double* g_alpha, double* g_u, const double* g_uprev, double c_prev, double* partials,
                         const AdmmCtl* ctl) {
    return dispatch_p(g.p, [&](auto pc) {
        constexpr int P = decltype(pc)::value;
        auto go = [&](auto kern) {
            klaunch(kern, dim3(L.grid), dim3(kThreads), 0, L.stream, g, edges, t, g_alpha, g_u, g_uprev,
                               c_prev, partials, ctl);
            return hipGetLastError();
        };
        const bool prev = g_uprev != nullptr;
        if (order == 0) {
            if (umode == U_EXPLICIT) return prev ? go(k_gather<P, 0, U_EXPLICIT, true>) : go(k_gather<P, 0, U_EXPLICIT, false>);
            return prev ? go(k_gather<P, 0, U_FROM_Z, true>) : go(k_gather<P, 0, U_FROM_Z, false>);
        }
        if (umode == U_EXPLICIT) return prev ? go(k_gather<P, 1, U_EXPLICIT, true>) : go(k_gather<P, 1, U_EXPLICIT, false>);
        return prev ? go(k_gather<P, 1, U_FROM_Z, true>) : go(k_gather<P, 1, U_FROM_Z, false>);
    });
}

hipError_t launch_apply_D_padded(const Geom& g, int order, const Launch& L, const double* theta, double* edges) {
    return dispatch_p(g.p, [&](auto pc) {
        constexpr int P = decltype(pc)::value;
        if (order == 0)
            klaunch((k_apply_D<P, 0>), dim3(L.grid), dim3(kThreads), 0, L.stream, g, theta, edges);
        else
            klaunch((k_apply_D<P, 1>), dim3(L.grid), dim3(kThreads), 0, L.stream, g, theta, edges);
        return hipGetLastError();
    });
}

hipError_t launch_edges_fill_valid(const Geom& g, int order, const Launch& L, double* edges, double value) {
    return dispatch_p(g.p, [&](auto pc) {
        constexpr int P = decltype(pc)::value;
        if (order == 0)
            klaunch((k_edges_fill_valid<P, 0>), dim3(L.grid), dim3(kThreads), 0, L.stream, g, edges, value);
        else
            klaunch((k_edges_fill_valid<P, 1>), dim3(L.grid), dim3(kThreads), 0, L.stream, g, edges, value);
        return hipGetLastError();
    });
}

hipError_t launch_apply_A(const Geom& g, const Launch& L, double sigma, int wmode, const double* wdiag,
                          const double* x, double* q, double* partials, const PcgState* st, int* nparts) {
    // plain operator application on a whole 3-D mesh: the z-marching kernel (MVTV_APPLY3D=0: generic)
    static const bool a3d = [] {
        const char* e = probe_env("MVTV_APPLY3D");
        return !e || std::atoi(e) != 0;
    }();
    if (a3d && g.p == 3 && !partials && g.ibeg == 0 && g.iend == g.N)
        return launch_apply3d(g, L.stream, sigma, wmode, wdiag, x, q);
    if (a3d && g.p == 3 && partials && st && nparts && g.ibeg == 0 && g.iend == g.N)
        return launch_apply3d(g, L.stream, sigma, wmode, wdiag, x, q, partials, st, nparts);
    if (a3d && g.p == 2 && g.ibeg == 0 && g.iend == g.N && (!partials || (st && nparts)))
        return launch_apply2d(g, L.stream, sigma, wmode, wdiag, x, q, partials, st, nparts);
    // 4-D: the w-marching kernel (128^4 run start 10.2 ms with the generic one); falls through when its grid would
    // overrun the partials rows
    if (a3d && g.p == 4 && g.ibeg == 0 && g.iend == g.N && (!partials || (st && nparts))) {
        const hipError_t e = launch_apply4d(g, L.stream, sigma, wmode, wdiag, x, q, partials, st, nparts);
        if (e != hipErrorInvalidValue) return e;
    }
    if (nparts) *nparts = L.grid;
    const StencilK sk = make_stencil(g);
    return dispatch_p(g.p, [&](auto pc) {
        constexpr int P = decltype(pc)::value;
        return dispatch_w(wmode, [&](auto wc) {
            constexpr int WM = decltype(wc)::value;
            if (partials && st)
                klaunch((k_apply_A<P, WM, true, true>), dim3(L.grid), dim3(kThreads), 0, L.stream, g, sk,
                                   sigma, wdiag, x, q, partials, st);
            else if (partials)
                klaunch((k_apply_A<P, WM, true, false>), dim3(L.grid), dim3(kThreads), 0, L.stream, g, sk,
                                   sigma, wdiag, x, q, partials, st);
            else
                klaunch((k_apply_A<P, WM, false, false>), dim3(L.grid), dim3(kThreads), 0, L.stream, g,
                                   sk, sigma, wdiag, x, q, partials, st);
            return hipGetLastError();
        });
    });
}

hipError_t launch_pcg_init(const Geom& g, const Launch& L, double sigma, int wmode, const double* wdiag,
                           const double* oty, const double* ga, double ca, const double* gb, double cb,
                           const double* x, double* r, double* p, double* partials) {
    const StencilK sk = make_stencil(g);
    return dispatch_p(g.p, [&](auto pc) {
        constexpr int P = decltype(pc)::value;
        return dispatch_w(wmode, [&](auto wc) {
            constexpr int WM = decltype(wc)::value;
            klaunch((k_pcg_init<P, WM>), dim3(L.grid), dim3(kThreads), 0, L.stream, g, sk, sigma, wdiag,
                               oty, ga, ca, gb, cb, x, r, p, partials);
            return hipGetLastError();
        });
    });
}

hipError_t launch_pcg_update(const Geom& g, const Launch& L, double sigma, int wmode, const double* wdiag,
                             double* x, double* r, const double* p, const double* q, const PcgState* st,
                             double* partials) {
    return dispatch_p(g.p, [&](auto pc) {
        constexpr int P = decltype(pc)::value;
        return dispatch_w(wmode, [&](auto wc) {
            constexpr int WM = decltype(wc)::value;
            klaunch((k_pcg_update<P, WM>), dim3(L.grid), dim3(kThreads), 0, L.stream, g, sigma, wdiag, x,
                               r, p, q, st, partials);
            return hipGetLastError();
        });
    });
}

hipError_t launch_pcg_pupdate(const Geom& g, const Launch& L, double sigma, int wmode, const double* wdiag,
                              const double* r, double* p, const PcgState* st) {
    return dispatch_p(g.p, [&](auto pc) {
        constexpr int P = decltype(pc)::value;
        return dispatch_w(wmode, [&](auto wc) {
            constexpr int WM = decltype(wc)::value;
            klaunch((k_pcg_pupdate<P, WM>), dim3(L.grid), dim3(kThreads), 0, L.stream, g, sigma, wdiag, r,
                               p, st);
            return hipGetLastError();
        });
    });
}

hipError_t launch_finalize(hipStream_t s, const double* partials, int nparts, int nr, int nmax, int op, double* out,
                           PcgState* st, double rtol2, int maxit, const AdmmCtl* ctl, AdmmCtl* ctl_step,
                           const double* step_red) {
    klaunch(k_finalize, dim3(1), dim3(1024), 0, s, partials, nparts, nr, nmax, op, out, st, rtol2, maxit, ctl, ctl_step,
            step_red);
    return hipGetLastError();
}

__global__ void k_admm_control(AdmmCtl* __restrict__ c, const double* __restrict__ R) {
    if (c->done) return;
    admm_control_step(c, R);
}

hipError_t launch_admm_control(hipStream_t s, AdmmCtl* ctl, const double* red) {
    klaunch(k_admm_control, dim3(1), dim3(1), 0, s, ctl, red);
    return hipGetLastError();
}

hipError_t launch_maxabsdiff(const Geom& g, const Launch& L, const double* a, const double* b, double* partials) {
    klaunch(k_maxabsdiff, dim3(L.grid), dim3(kThreads), 0, L.stream, g.N, a, b, partials);
    return hipGetLastError();
}

hipError_t launch_cg_vec(const Geom& g, const Launch& L, int op, double coef, double* x, double* y, const double* p,
                         const double* t, double* partials) {
    klaunch(k_cg_vec, dim3(L.grid), dim3(kThreads), 0, L.stream, op, g.N, coef, x, y, p, t, partials);
    return hipGetLastError();
}

hipError_t launch_dmaxabs(const Geom& g, int order, const Launch& L, const double* x, double* partials) {
    return dispatch_p(g.p, [&](auto pc) {
        constexpr int P = decltype(pc)::value;
        if (order == 0) klaunch(k_dmaxabs<P, 0>, dim3(L.grid), dim3(kThreads), 0, L.stream, g, x, partials);
        else klaunch(k_dmaxabs<P, 1>, dim3(L.grid), dim3(kThreads), 0, L.stream, g, x, partials);
        return hipGetLastError();
    });
}

hipError_t launch_pcgs_vec(const Geom& g, const Launch& L, int op, const double* oty, const double* ga, double ca,
                           const double* gb, double cb, double* x, double* r, double* p, const double* q, double* z,
                           double* b, const double* sinv, double* t, const PcgState* st, double* partials,
                           int with_b2) {
    klaunch(k_pcgs_vec, dim3(L.grid), dim3(kThreads), 0, L.stream, op, g.N, oty, ga, ca, gb, cb, x, r, p, q, z, b,
            sinv, t, st, partials, with_b2);
    return hipGetLastError();
}

hipError_t launch_pcgs_sinv(const Geom& g, const Launch& L, double sigma, int wmode, const double* wdiag, double dbar,
                            double* sinv) {
    return dispatch_p(g.p, [&](auto pc) {
        constexpr int P = decltype(pc)::value;
        return dispatch_w(wmode, [&](auto wc) {
            constexpr int WM = decltype(wc)::value;
            klaunch((k_pcgs_sinv<P, WM>), dim3(L.grid), dim3(kThreads), 0, L.stream, g, sigma, wdiag, dbar, sinv);
            return hipGetLastError();
        });
    });
}

hipError_t launch_fill(hipStream_t s, double* x, double v, uint64_t n) {
    klaunch(k_fill, dim3(elem_grid(n)), dim3(256), 0, s, x, v, n);
    return hipGetLastError();
}

hipError_t launch_edges_import(const Geom& g, int order, hipStream_t s, int k, uint64_t e0, uint64_t cnt,
                               const double* compact, double* padded) {
    klaunch(k_edges_import, dim3(elem_grid(cnt)), dim3(256), 0, s, red_dims(g, order, k),
                       uint64_t(k) * g.N, e0, cnt, compact, padded);
    return hipGetLastError();
}

hipError_t launch_edges_export(const Geom& g, int order, hipStream_t s, int k, uint64_t e0, uint64_t cnt,
                               const double* padded, double* compact, int umode, double t, double c) {
    klaunch(k_edges_export, dim3(elem_grid(cnt)), dim3(256), 0, s, red_dims(g, order, k),
                       uint64_t(k) * g.N, e0, cnt, padded, compact, umode, t, c);
    return hipGetLastError();
}

hipError_t launch_edges_z_to_u(hipStream_t s, double* edges, uint64_t n, double t, double c) {
    klaunch(k_edges_z_to_u, dim3(elem_grid(n)), dim3(256), 0, s, edges, n, t, c);
    return hipGetLastError();
}

hipError_t launch_gather_index(hipStream_t s, const double* theta, const int64_t* idx, int64_t n, double* out) {
    klaunch(k_gather_index, dim3(elem_grid(uint64_t(n))), dim3(256), 0, s, theta, idx, n, out);
    return hipGetLastError();
}

}  // namespace mvtv

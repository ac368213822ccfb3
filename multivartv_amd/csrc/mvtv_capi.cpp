// mvtv_capi.cpp — host driver of the ADMM hot path and the C ABI declared in include/mvtv/mvtv.h.
//
// One mvtv_problem = one GPU, one HIP stream, all vectors resident in HBM. The ADMM loop
// follows the reference variants line by line at the level of scalars (adapt_step, stopping
// tests, counters); every vector operation is a kernel from mvtv_kernels.hip:
//   B  rcpp-code/MultivarTV/src/solvers.cpp:96-136   (admm_update, adapt_step :77-94)
//   A  cpp-code/solvers.cpp:90-130                    (admm_update, adapt_step :70-88)
//   C  code/solvers.py:53-76                          (mbs_one's loop)
// Per ADMM iteration the host reads back 7 scalars (one stream sync); the PCG theta-solve
// keeps its scalars on the device and is polled every few iterations.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <complex>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "mvtv/mvtv.h"
#include "mvtv_internal.h"
#include "mvtv_problem.h"

using namespace mvtv;

namespace mvtv {
thread_local std::string g_last_error;
}  // namespace mvtv

namespace {

int popcount(int x) { return __builtin_popcount(unsigned(x)); }

// Placement-aware z ping-pong: the fused 3-D kernel's time depends on WHICH physical
// edge buffer it reads z from and writes to (profiles/r01/v12_zflip_probe.txt: up to 4.70 against
// 4.15 ms for the two directions of one pair). Once per problem, for 3-D meshes of >= 2^24 nodes, time
// every ordered pair of four candidate buffers (candidate 0 = edges2, 1..3 = new allocations; `edges`
// holds the state and is not a candidate) with side-effect-free launches of the steady-state kernel
// (zeroed z, scratch outputs, no control block), keep the pair with the lowest round-trip cost, move z into
// it and free the rest. Best effort: any failure (allocation, launch) leaves the allocation-order pair in
// place, frees everything the probe allocated and clears HIP's error state. MVTV_ZPICK=0 turns it off
// (MVTV_ZPICK=fail: allocate, then take the failure path; tests/test_gpu_zpick.py).
// The fused 3-D kernel may skip the twin block (mvtv_internal.h twin_block): one GPU, equal twin weights and state.
// MVTV_TWIN_OFF=1 (probe builds) keeps both.
bool twin_ready(const mvtv_problem* P) {
    if (P->slab || !P->twin_ok || probe_env("MVTV_TWIN_OFF")) return false;
    if (!((P->g.p == 3 && P->f3d) || (P->g.p == 4 && P->f4d))) return false;
    return twin_weights_equal(P->g, P->order);
}

// edge words the twins leave out (the twin blocks' lengths)
double twin_edges(const mvtv_problem* P) {
    double t = 0.0;
    for (int k = 0; k < P->g.nb; ++k)
        if (twin_of(k, P->g.p, P->order) != k) t += double(P->blk_len[k]);
    return t;
}

mvtv_status pick_zpair(mvtv_problem* P, bool track_theta, bool twin) {
    P->zpicked = true;
    const char* env = std::getenv("MVTV_ZPICK");
    if ((env && std::atoi(env) == 0) || P->g.p != 3 || P->g.N < (size_t(1) << 24) || !P->edges2) return MVTV_OK;
    const size_t ne = size_t(P->g.nb) * P->g.N, bytes = ne * sizeof(double);
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess || fr < 3 * bytes + (size_t(16) << 30)) {
        (void)hipGetLastError();
        return MVTV_OK;
    }
    constexpr int K = 4, R = 3;
    double* cand[K] = {P->edges2, nullptr, nullptr, nullptr};
    double* tmp[3] = {nullptr, nullptr, nullptr};   // the probes' g_alpha / g_u outputs and theta_old input
    hipEvent_t ev[2] = {nullptr, nullptr};
    bool ok = true;
    auto hip = [&](hipError_t e) {
        if (e != hipSuccess) ok = false;
        return ok;
    };
    for (int i = 1; i < K && ok; ++i) hip(hipMalloc(reinterpret_cast<void**>(&cand[i]), bytes));
    for (int i = 0; i < 3 && ok; ++i) hip(hipMalloc(reinterpret_cast<void**>(&tmp[i]), size_t(P->g.N) * sizeof(double)));
    for (int i = 0; i < K && ok; ++i) hip(hipMemsetAsync(cand[i], 0, bytes, P->stream));
    if (ok) hip(hipMemsetAsync(tmp[2], 0, size_t(P->g.N) * sizeof(double), P->stream));
    if (ok) hip(hipEventCreate(&ev[0]));
    if (ok) hip(hipEventCreate(&ev[1]));
    if (env && std::strcmp(env, "fail") == 0) ok = false;   // test hook: take the failure path after allocating
    double cost[K][K] = {};
    for (int rep = 0; rep <= R && ok; ++rep)   // rep 0 warms up
        for (int i = 0; i < K && ok; ++i)
            for (int j = 0; j < K && ok; ++j) {
                if (i == j) continue;
                int np = 0;
                float ms = 0.f;
                if (hip(hipEventRecord(ev[0], P->stream)) &&
                    hip(launch_admm3d(P->g, P->order, U_FROM_Z, P->stream, P->theta, cand[i], cand[j], 0.0, 1.0, 0.0,
                                      1.0, track_theta ? tmp[2] : nullptr, tmp[0], tmp[1], P->guprev, P->partials,
                                      &np, nullptr, false, twin)) &&
                    hip(hipEventRecord(ev[1], P->stream)) && hip(hipEventSynchronize(ev[1])) &&
                    hip(hipEventElapsedTime(&ms, ev[0], ev[1])) && rep > 0)
                    cost[i][j] += ms;
            }
    int a = 0, b = 1;
    if (ok) {
        for (int i = 0; i < K; ++i)
            for (int j = i + 1; j < K; ++j)
                if (cost[i][j] + cost[j][i] < cost[a][b] + cost[b][a]) a = i, b = j;
        // the probes wrote only the candidates, tmp and the partials (scratch until the next reduction)
        ok = hip(hipMemcpyAsync(cand[a], P->edges, bytes, hipMemcpyDeviceToDevice, P->stream)) &&
             hip(hipStreamSynchronize(P->stream));
    }
    (void)hipStreamSynchronize(P->stream);
    for (auto e : ev)
        if (e) (void)hipEventDestroy(e);
    for (auto t : tmp)
        if (t) (void)hipFree(t);
    if (!ok) {   // keep (edges, edges2); the candidates' contents were never used
        for (int i = 1; i < K; ++i)
            if (cand[i]) (void)hipFree(cand[i]);
        (void)hipGetLastError();
        return MVTV_OK;
    }
    (void)hipFree(P->edges);
    for (int i = 0; i < K; ++i)
        if (i != a && i != b) (void)hipFree(cand[i]);
    P->edges = cand[a];
    P->edges2 = cand[b];
    if (probe_env("MVTV_ZPICK_LOG"))
        std::fprintf(stderr, "[mvtv] z pair %d,%d: %.3f / %.3f ms (candidate 0 = edges2, 1-3 new; pair 0,1: %.3f / %.3f)\n",
                     a, b, cost[a][b] / R, cost[b][a] / R, cost[0][1] / R, cost[1][0] / R);
    return MVTV_OK;
}

void free_all(mvtv_problem* P) {
    double** bufs[] = {&P->oty, &P->wdiag, &P->theta, &P->edges, &P->ga, &P->gu, &P->guprev, &P->r,
                       &P->p, &P->q, &P->thold, &P->p2, &P->partials, &P->red, &P->stage, &P->slab_iface,
                       &P->edges2, &P->pcg_b, &P->g4, &P->edges3, &P->pcg_s, &P->pcg_t};
    for (double** b : bufs)
        if (*b) {
            (void)hipFree(*b);
            *b = nullptr;
        }
    if (P->st) (void)hipFree(P->st);
    if (P->ctl) (void)hipFree(P->ctl);
    if (P->host_ctl) (void)hipHostFree(P->host_ctl);
    for (double* t : {P->spec.tw, P->spec.twq, P->spec.lam, P->spec.blu})
        if (t) (void)hipFree(t);
    if (P->spec.perm) (void)hipFree(P->spec.perm);
    P->spec = SpecPlan{};
    if (P->host_red) (void)hipHostFree(P->host_red);
    for (auto& pd : P->pending) {
        (void)hipEventDestroy(pd.a);
        (void)hipEventDestroy(pd.b);
    }
    for (auto e : P->ev_pool) (void)hipEventDestroy(e);
    for (auto& lg : P->graphs)
        if (lg.exec) (void)hipGraphExecDestroy(lg.exec);
    P->graphs.clear();
    if (P->stream) (void)hipStreamDestroy(P->stream);
    if (P->comm_stream) (void)hipStreamDestroy(P->comm_stream);
}

double variant_tol(const mvtv_admm_opts& o) {
    if (o.tol > 0) return o.tol;
    return o.variant == MVTV_VARIANT_RCPP ? 1e-4 : 1e-3;
}
int variant_maxc(const mvtv_admm_opts& o) {
    if (o.max_counter > 0) return o.max_counter;
    return o.variant == MVTV_VARIANT_RCPP ? 3000 : (o.variant == MVTV_VARIANT_CPP ? 2000 : 1000000);
}

// Copy a compact [E] edge vector (reference block layout) into the padded device layout.
mvtv_status import_edges(mvtv_problem* P, const double* host_u, double* padded) {
    HIP_TRY(hipMemsetAsync(padded, 0, size_t(P->g.nb) * P->g.N * sizeof(double), P->stream));
    if (!P->stage) {
        P->stage_n = std::min<size_t>(size_t(P->E), size_t(1) << 24);
        MVTV_TRY(alloc(&P->stage, P->stage_n));
    }
    uint64_t off = 0;
    for (int k = 0; k < P->g.nb; ++k) {
        for (uint64_t e0 = 0; e0 < P->blk_len[k]; e0 += P->stage_n) {
            const uint64_t cnt = std::min<uint64_t>(P->stage_n, P->blk_len[k] - e0);
            HIP_TRY(hipMemcpyAsync(P->stage, host_u + off + e0, cnt * sizeof(double), hipMemcpyHostToDevice, P->stream));
            HIP_TRY(launch_edges_import(P->g, P->order, P->stream, k, e0, cnt, P->stage, padded));
        }
        off += P->blk_len[k];
    }
    HIP_TRY(hipStreamSynchronize(P->stream));
    return MVTV_OK;
}

mvtv_status export_edges(mvtv_problem* P, const double* padded, double* host_u, int umode, double t, double c) {
    if (!P->stage) {
        P->stage_n = std::min<size_t>(size_t(P->E), size_t(1) << 24);
        MVTV_TRY(alloc(&P->stage, P->stage_n));
    }
    uint64_t off = 0;
    for (int k = 0; k < P->g.nb; ++k) {
        for (uint64_t e0 = 0; e0 < P->blk_len[k]; e0 += P->stage_n) {
            const uint64_t cnt = std::min<uint64_t>(P->stage_n, P->blk_len[k] - e0);
            HIP_TRY(launch_edges_export(P->g, P->order, P->stream, k, e0, cnt, padded, P->stage, umode, t, c));
            HIP_TRY(hipMemcpyAsync(host_u + off + e0, P->stage, cnt * sizeof(double), hipMemcpyDeviceToHost, P->stream));
            HIP_TRY(hipStreamSynchronize(P->stream));
        }
        off += P->blk_len[k];
    }
    return MVTV_OK;
}

// PCG iterations enqueued before the first poll: the last solve's count plus this (probe: MVTV_PCG_AHEAD).
// Config 4's work item (2048^2 fold, one stream): -2 327, 0 335, +2 326, +4 325 ADMM it/s on one box
// (profiles/r03/v5_cv_tuning)
int pcg_ahead() {
    static const int v = [] {
        const char* e = probe_env("MVTV_PCG_AHEAD");
        return e ? std::atoi(e) : 0;
    }();
    return v;
}

// Solve (W + sigma D^T D) x = b, b = oty + ca*ga + cb*gb, by Jacobi-PCG warm-started at x.
mvtv_status pcg_solve(mvtv_problem* P, double sigma, const double* oty, const double* ga, double ca,
                      const double* gb, double cb, double* x, double rtol, int maxit, int* iters, double* relres) {
    const Launch L = P->L();
    const double* w = P->wdiag;
    const bool fused = P->g.p == 3 && P->fused3d && P->wmode != W_NONE;
    // fused 3-D: r and p ping-pong between two buffers (a launch reads neighbour halos of r_i and
    // p_{i-1} that their owning workgroups overwrite, so outputs must not alias inputs)
    if (fused && !P->p2) MVTV_TRY(alloc(&P->p2, P->g.N));
    double* rb[2] = {P->r, P->q};
    double* pb[2] = {P->p, P->p2};
    int nb = 0;
    int h = P->tstart(MVTV_K_PCG_INIT);
    if (fused)
        HIP_TRY(launch_cg3d(P->g, P->stream, 0, sigma, P->wmode, w, x, nullptr, nullptr, rb[0], nullptr, oty, ga, ca,
                            gb, cb, P->st, P->partials, &nb));
    else
        HIP_TRY(launch_pcg_init(P->g, L, sigma, P->wmode, w, oty, ga, ca, gb, cb, x, P->r, P->p, P->partials));
    P->tstop(h);
    h = P->tstart(MVTV_K_REDUCE);
    if (fused)
        HIP_TRY(launch_finalize(P->stream, P->partials, nb, 4, 0, 4, nullptr, P->st, rtol * rtol, maxit));
    else
        HIP_TRY(launch_finalize(P->stream, P->partials, L.grid, PR_N, 0, 1, nullptr, P->st, rtol * rtol, maxit));
    P->tstop(h);

    // one PCG iteration; kernels enqueued after convergence return at once (device done flag)
    auto enqueue = [&](int j) -> mvtv_status {
        if (fused) {
            int hh = P->tstart(MVTV_K_PCG_FUSED);
            // x moves in odd iterations only (both steps, k_cg3d); k_cg_xflush applies an even last one's
            HIP_TRY(launch_cg3d(P->g, P->stream, j == 0 ? 1 : ((j & 1) ? 3 : 2), sigma, P->wmode, w, x, rb[j & 1],
                                pb[j & 1], rb[(j + 1) & 1], pb[(j + 1) & 1], oty, ga, ca, gb, cb, P->st, P->partials,
                                &nb));
            P->tstop(hh);
            hh = P->tstart(MVTV_K_REDUCE);
            HIP_TRY(launch_finalize(P->stream, P->partials, nb, 4, 0, 5, nullptr, P->st));
            P->tstop(hh);
            return MVTV_OK;
        }
        int hh = P->tstart(MVTV_K_PCG_APPLY);
        HIP_TRY(launch_apply_A(P->g, L, sigma, P->wmode, w, P->p, P->q, P->partials, P->st));
        P->tstop(hh);
        hh = P->tstart(MVTV_K_REDUCE);
        HIP_TRY(launch_finalize(P->stream, P->partials, L.grid, 1, 0, 2, nullptr, P->st));
        P->tstop(hh);
        hh = P->tstart(MVTV_K_PCG_UPDATE);
        HIP_TRY(launch_pcg_update(P->g, L, sigma, P->wmode, w, x, P->r, P->p, P->q, P->st, P->partials));
        P->tstop(hh);
        hh = P->tstart(MVTV_K_REDUCE);
        HIP_TRY(launch_finalize(P->stream, P->partials, L.grid, 2, 0, 3, nullptr, P->st));
        P->tstop(hh);
        hh = P->tstart(MVTV_K_PCG_DIRECTION);
        HIP_TRY(launch_pcg_pupdate(P->g, L, sigma, P->wmode, w, P->r, P->p, P->st));
        P->tstop(hh);
        return MVTV_OK;
    };
    // Poll schedule: the previous solve's count predicts this one (warm starts change it slowly),
    // so the first poll comes just before it and later polls every 2 iterations.
    std::vector<size_t> mark;   // first timing entry of each enqueued iteration
    int enq = 0;
    int batch = P->pcg_hint > 0 ? std::max(2, P->pcg_hint + pcg_ahead()) : kPcgPoll;
    for (;;) {
        for (int b = 0; b < batch && enq < maxit; ++b, ++enq) {
            mark.push_back(P->pending.size());
            MVTV_TRY(enqueue(enq));
        }
        HIP_TRY(hipMemcpyAsync(P->host_st, P->st, sizeof(PcgState), hipMemcpyDeviceToHost, P->stream));
        HIP_TRY(hipStreamSynchronize(P->stream));
        const int done_iters = P->host_st->iter;
        if (P->timing && done_iters < int(mark.size()))   // launches past convergence did no work
            for (size_t e = mark[size_t(done_iters)]; e < P->pending.size(); ++e) P->pending[e].kid = -1;
        P->harvest();
        if (P->host_st->done || enq >= maxit) break;
        batch = 2;
    }
    if (fused) {   // an even last iteration's x step (p_i of an even i is in pb[1])
        h = P->tstart(MVTV_K_OTHER);
        HIP_TRY(launch_cg_xflush(P->stream, P->g.N, x, pb[1], P->st));
        P->tstop(h);
        if (P->timing) P->pcg_xmoves += P->host_st->iter / 2;
    }
    *iters = P->host_st->iter;
    P->pcg_hint = *iters;
    *relres = P->host_st->bnorm2 > 0 ? std::sqrt(P->host_st->rnorm2 / P->host_st->bnorm2) : 0.0;
    return MVTV_OK;
}

bool spectral_ok(const mvtv_problem* P) { return P->spec_mesh && P->wmode == W_IDENTITY; }

// Graph replay of the asynchronous loop: probe builds only (MVTV_ADMM_GRAPH=1). Measured slower than the stream
// launches it replaces, one process each, event-free (tools/launch_gap_probe.py, profiles/r04/v1_launch_gap):
// 1024^2 13510 against 14083 ADMM it/s, 2048^2 6088 against 6187. The ~37 us of "gaps" per 1024^2 iteration that
// the round-3 trace showed were the per-launch timing events (10105 it/s with them).
bool admm_graph_enabled() {
    static const bool on = [] {
        const char* e = probe_env("MVTV_ADMM_GRAPH");
        return e && std::atoi(e) != 0;
    }();
    return on;
}

// M = 2^ceil(log2(2m - 1)): the circular convolution length of Bluestein's identity for length m
uint32_t bluestein_length(uint32_t m) {
    uint32_t M = 1;
    while (M < 2 * m - 1) M <<= 1;
    return M;
}

// In-place radix-2 DFT (sign -1, unnormalised) in long double: the convolution kernels' transforms, once per
// problem (twiddles from exact angles 2 pi (k mod M) / M)
void fft_ld(std::vector<std::complex<long double>>& x) {
    const size_t M = x.size();
    const long double pi = 3.141592653589793238462643383279502884L;
    for (size_t i = 1, j = 0; i < M; ++i) {
        size_t bit = M >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) std::swap(x[i], x[j]);
    }
    for (size_t len = 2; len <= M; len <<= 1) {
        for (size_t i = 0; i < M; i += len)
            for (size_t k = 0; k < len / 2; ++k) {
                const long double ang = -2.0L * pi * (long double)(k * (M / len)) / (long double)M;
                const std::complex<long double> w(cosl(ang), sinl(ang));
                const std::complex<long double> u = x[i + k], v = x[i + k + len / 2] * w;
                x[i + k] = u + v;
                x[i + k + len / 2] = u - v;
            }
    }
}

// Bluestein tables of one dimension (SpecPlan::blu layout): chirp c[n] = e^{-i pi n^2/m} (n^2 mod 2m exactly), the
// transforms / M of the kernels b_f[j] = conj c[|j|] (forward DFT, s = -1) and b_i[j] = c[|j|] (inverse, s = +1)
// wrapped to length M, and the length-M twiddles e^{-2 pi i k/M}, k < M
void bluestein_tables(uint32_t m, uint32_t M, std::vector<double>& out) {
    const long double pi = 3.141592653589793238462643383279502884L;
    std::vector<std::complex<long double>> c(m), bf(M, 0.0L), bi(M, 0.0L);
    for (uint32_t n = 0; n < m; ++n) {
        const uint64_t r = (uint64_t(n) * n) % (2 * uint64_t(m));
        const long double ang = -pi * (long double)r / (long double)m;
        c[n] = std::complex<long double>(cosl(ang), sinl(ang));
    }
    for (uint32_t j = 0; j < m; ++j) {
        bf[j] = std::conj(c[j]);
        bi[j] = c[j];
        if (j > 0) {
            bf[M - j] = std::conj(c[j]);
            bi[M - j] = c[j];
        }
    }
    fft_ld(bf);
    fft_ld(bi);
    for (uint32_t n = 0; n < m; ++n) {
        out.push_back(double(c[n].real()));
        out.push_back(double(c[n].imag()));
    }
    for (auto* v : {&bf, &bi})
        for (uint32_t k = 0; k < M; ++k) {
            out.push_back(double((*v)[k].real() / (long double)M));
            out.push_back(double((*v)[k].imag() / (long double)M));
        }
    for (uint32_t k = 0; k < M; ++k) {   // (k_dctb reads k < M/2, k_dctb8's radix-8 stages k < M)
        const long double ang = -2.0L * pi * (long double)k / (long double)M;
        out.push_back(double(cosl(ang)));
        out.push_back(double(sinl(ang)));
    }
}

// Device tables of the spectral solve. Twiddles and eigenvalues are evaluated in long double.
mvtv_status spectral_plan(mvtv_problem* P) {
    std::vector<double> tw, twq, lam;
    std::vector<uint32_t> perm;
    SpecPlan& sp = P->spec;
    const long double pi = 3.141592653589793238462643383279502884L;
    for (int j = 0; j < P->g.p; ++j) {
        const uint32_t m = (P->slab && j == P->g.p - 1) ? uint32_t(P->m_global) : P->g.m[j];
        sp.tw_off[j] = uint32_t(tw.size());
        sp.twq_off[j] = uint32_t(twq.size());
        sp.lam_off[j] = uint32_t(lam.size());
        for (uint32_t k = 0; k < m; ++k) {
            const long double a = -2.0L * pi * k / m;
            tw.push_back(double(cosl(a)));
            tw.push_back(double(sinl(a)));
        }
        for (uint32_t k = 0; k < m; ++k) {
            const long double a = -pi * k / (2.0L * m);
            twq.push_back(double(cosl(a)));
            twq.push_back(double(sinl(a)));
            const long double sn = sinl(pi * k / (2.0L * m));
            lam.push_back(double(4.0L * sn * sn));
        }
        // k_dctg's input order: sample k goes to Makhoul position n (x[2n], x[2(m-1-n)+1]) at its
        // digit-reversed place for the radix plan (n = sum of digits d_s, most significant first in
        // stage order reversed; position = sum d_s prod_{u<s} rad[u])
        int rad[8], nrad = 0;
        const bool planned = dct_radix_plan(m, rad, &nrad);
        for (uint32_t k = 0; k < m; ++k) {
            uint32_t n = (k & 1u) ? m - 1u - (k >> 1) : (k >> 1), pos = 0;
            if (planned) {
                for (int st = nrad - 1; st >= 0; --st) {
                    uint32_t mul = 1;
                    for (int u = 0; u < st; ++u) mul *= uint32_t(rad[u]);
                    pos += (n % uint32_t(rad[st])) * mul;
                    n /= uint32_t(rad[st]);
                }
            }
            perm.push_back(pos);
        }
    }
    // Bluestein tables of the lengths without a 2-3-5-7 plan (k_dctb; mvtv_spectral.hip)
    std::vector<double> blu;
    for (int j = 0; j < P->g.p; ++j) {
        const uint32_t m = (P->slab && j == P->g.p - 1) ? uint32_t(P->m_global) : P->g.m[j];
        int rad[8], nrad = 0;
        sp.blu_M[j] = 0;
        if (m > 4096 || dct_radix_plan(m, rad, &nrad)) continue;
        const uint32_t M = bluestein_length(m);
        sp.blu_M[j] = M;
        sp.blu_off[j] = uint32_t(blu.size());
        bluestein_tables(m, M, blu);
    }
    auto up = [&](double** dst, const std::vector<double>& v) -> mvtv_status {
        MVTV_TRY(alloc(dst, v.size()));
        HIP_TRY(hipMemcpy(*dst, v.data(), v.size() * sizeof(double), hipMemcpyHostToDevice));
        return MVTV_OK;
    };
    if (!blu.empty()) MVTV_TRY(up(&sp.blu, blu));
    MVTV_TRY(up(&sp.tw, tw));
    MVTV_TRY(up(&sp.twq, twq));
    MVTV_TRY(up(&sp.lam, lam));
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(&sp.perm), perm.size() * sizeof(uint32_t)));
    HIP_TRY(hipMemcpy(sp.perm, perm.data(), perm.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    return MVTV_OK;
}

// Direct solve (I + sigma D^T D) x = oty + ca*ga + cb*gb: forward DCT along dims 0..p-2, the
// last dim's forward/divide/inverse in one pass, inverse DCT along dims p-2..0. All in place on x.
// fold: b = oty + fold_ka ga + fold_kb gb from the control block (ga = the fused kernel's folded
// s = rho (D^T alpha + D^T u), gb = D^T u)
mvtv_status spectral_solve(mvtv_problem* P, double sigma, const double* oty, const double* ga, double ca,
                           const double* gb, double cb, double* x, const AdmmCtl* ctl = nullptr, double w0 = 1.0,
                           const int32_t* skip = nullptr, bool fold = false) {
    // pass order: forward along dims order[0..p-2], forward/divide/inverse along order[p-1], inverse
    // back; the MID dimension defaults to p-1 (MVTV_DCT_MID selects another one for experiments)
    const int p = P->g.p;
    static const int mid_env = [] {
        const char* e = probe_env("MVTV_DCT_MID");
        return e ? std::atoi(e) : -1;
    }();
    const int mid = (mid_env >= 1 && mid_env < p) ? mid_env : p - 1;
    // 3-D: dim 2 forward (b formed on load), the two marching passes (dim-0 transforms + the dim-1 line solves),
    // dim 2 inverse: 9N words instead of 11N
    if (!P->slab && march_ok(P->g)) {
        int h = P->tstart(ga ? (fold ? MVTV_K_DCT_FOLD : MVTV_K_DCT_FIRST) : MVTV_K_DCT);
        if (ga && fold)
            HIP_TRY(launch_dct_pass(P->spec, P->g, P->stream, 0, 2, oty, ga, 1.0, gb, 0.0, x, sigma, w0, ctl, 0, 0.0, skip,
                                    nullptr, true));
        else if (ga)
            HIP_TRY(launch_dct_pass(P->spec, P->g, P->stream, 0, 2, oty, ga, ca, gb ? gb : ga, gb ? cb : 0.0, x, sigma, w0,
                                    ctl, 0, 0.0, skip));
        else
            HIP_TRY(launch_dct_pass(P->spec, P->g, P->stream, 0, 2, oty, nullptr, 0.0, nullptr, 0.0, x, sigma, w0, ctl, 0,
                                    0.0, skip));
        P->tstop(h);
        h = P->tstart(MVTV_K_DCT);
        HIP_TRY(launch_march(P->spec, P->g, P->stream, false, x, sigma, w0, ctl, skip));
        P->tstop(h);
        h = P->tstart(MVTV_K_DCT);
        HIP_TRY(launch_march(P->spec, P->g, P->stream, true, x, sigma, w0, ctl, skip));
        P->tstop(h);
        h = P->tstart(MVTV_K_DCT);
        HIP_TRY(launch_dct_pass(P->spec, P->g, P->stream, 1, 2, x, nullptr, 0.0, nullptr, 0.0, x, sigma, w0, ctl, 0, 0.0,
                                skip));
        P->tstop(h);
        return MVTV_OK;
    }
    // probe builds: MVTV_DCT_REV=1 takes the other dims in descending order (the first pass, b formed on load, and the
    // last inverse pass then run along dim p - 2 instead of the contiguous dim 0)
    static const bool rev = probe_env("MVTV_DCT_REV") != nullptr;
    int order[MVTV_MAX_DIMS], n = 0;
    for (int d = 0; d < p; ++d)
        if (d != mid) order[n++] = d;
    if (rev) std::reverse(order, order + n);
    order[n++] = mid;
    // m0 = m1 <= 128: dims 0 and 1 in one pass each way (k_plane8: the plane stays on chip between them)
    const bool plane = !rev && mid >= 2 && plane_pass_ok(P->g);
    if (plane) {
        const int h = P->tstart(ga ? (fold ? MVTV_K_DCT_FOLD : MVTV_K_DCT_FIRST) : MVTV_K_DCT);
        if (ga && fold)
            HIP_TRY(launch_plane_pass(P->spec, P->g, P->stream, 0, oty, ga, 1.0, gb, 0.0, x, ctl, skip, true));
        else if (ga)
            HIP_TRY(launch_plane_pass(P->spec, P->g, P->stream, 0, oty, ga, ca, gb, cb, x, ctl, skip));
        else
            HIP_TRY(launch_plane_pass(P->spec, P->g, P->stream, 0, oty, nullptr, 0.0, nullptr, 0.0, x, ctl, skip));
        P->tstop(h);
    }
    for (int t = plane ? 2 : 0; t < p; ++t) {
        const int d = order[t];
        const bool first = t == 0;
        const int mode = t == p - 1 ? 2 : 0;
        const int h = P->tstart(first ? (fold ? MVTV_K_DCT_FOLD : MVTV_K_DCT_FIRST) : MVTV_K_DCT);
        if (first && ga && fold)   // b = oty + fold_ka s + fold_kb g_u formed on load (g_u read after a rho change)
            HIP_TRY(launch_dct_pass(P->spec, P->g, P->stream, mode, d, oty, ga, 1.0, gb, 0.0, x, sigma, w0, ctl, 0, 0.0,
                                    skip, nullptr, true));
        else if (first && ga)   // b = oty + ca*ga + cb*gb formed on load
            HIP_TRY(launch_dct_pass(P->spec, P->g, P->stream, mode, d, oty, ga, ca, gb ? gb : ga, gb ? cb : 0.0, x,
                                    sigma, w0, ctl, 0, 0.0, skip));
        else
            HIP_TRY(launch_dct_pass(P->spec, P->g, P->stream, mode, d, first ? oty : x, nullptr, 0.0, nullptr, 0.0, x,
                                    sigma, w0, ctl, 0, 0.0, skip));
        P->tstop(h);
    }
    for (int t = p - 2; t >= (plane ? 2 : 0); --t) {
        const int h = P->tstart(MVTV_K_DCT);
        HIP_TRY(launch_dct_pass(P->spec, P->g, P->stream, 1, order[t], x, nullptr, 0.0, nullptr, 0.0, x, sigma, w0,
                                ctl, 0, 0.0, skip));
        P->tstop(h);
    }
    if (plane) {
        const int h = P->tstart(MVTV_K_DCT);
        HIP_TRY(launch_plane_pass(P->spec, P->g, P->stream, 1, x, nullptr, 0.0, nullptr, 0.0, x, ctl, skip));
        P->tstop(h);
    }
    return MVTV_OK;
}

// (W + sigma D^T D) x = oty + ca*ga + cb*gb by PCG with the spectral preconditioner M = S A0 S,
// A0 = mean(W) I + sigma D^T D applied exactly by the cosine-transform solve. S = I when W is nearly
// constant against sigma D^T D's diagonal d (std(W) < 0.1 mean(d)); otherwise S = diag(sqrt(d / mean d)),
// which turns M into the Jacobi preconditioner as sigma -> 0 and into A0 as sigma grows (PCG counts to
// rtol 1e-10 from zero, 128^2 / 256^2: CV-fold mask at sigma = 6: Jacobi 187-192, M 19; scattered counts
// at sigma = 0.04: Jacobi 115, scaled M 95, unscaled 297). Scalars stay on the device
// (PcgState, k_finalize ops 1-3); iterations enqueued after convergence return at once (st->done).
mvtv_status pcgs_solve(mvtv_problem* P, double sigma, const double* oty, const double* ga, double ca,
                       const double* gb, double cb, double* x, double rtol, int maxit, int* iters, double* relres) {
    const Launch L = P->L();
    if (!P->p2) MVTV_TRY(alloc(&P->p2, P->g.N));
    if (!P->pcg_b) MVTV_TRY(alloc(&P->pcg_b, P->g.N));
    double *r = P->r, *z = P->q, *p = P->p, *q = P->p2, *b = P->pcg_b;
    const double w0 = P->wmean > 0.0 ? P->wmean : 1.0;
    // mean over the mesh of D^T D's diagonal: sum_S cS[S] prod_{j in S} mean(l_j), l_j = 1 at the ends, 2 inside
    double cmean = 0.0;
    for (int S = 1; S < (1 << P->g.p); ++S) {
        double prod = P->g.cS[S];
        for (int j = 0; j < P->g.p; ++j)
            if ((S >> j) & 1) prod *= 2.0 * double(P->g.m[j] - 1) / double(P->g.m[j]);
        cmean += prod;
    }
    const double dbar = w0 + sigma * cmean;
    const bool scaled = P->wmode == W_DIAG && P->wstd >= 0.1 * dbar;
    double *sinv = nullptr, *t = nullptr;
    if (scaled) {
        if (!P->pcg_s) MVTV_TRY(alloc(&P->pcg_s, P->g.N));
        if (!P->pcg_t) MVTV_TRY(alloc(&P->pcg_t, P->g.N));
        sinv = P->pcg_s;
        t = P->pcg_t;
        HIP_TRY(launch_pcgs_sinv(P->g, L, sigma, P->wmode, P->wdiag, dbar, sinv));
    }
    const double* rin = scaled ? t : r;
    int h = P->tstart(MVTV_K_PCG_INIT);
    HIP_TRY(launch_apply_A(P->g, L, sigma, P->wmode, P->wdiag, x, q, nullptr, nullptr));
    P->tstop(h);
    HIP_TRY(launch_pcgs_vec(P->g, L, 0, oty, ga, ca, gb, cb, x, r, p, q, nullptr, b, sinv, t, P->st, nullptr, 0));
    MVTV_TRY(spectral_solve(P, sigma, rin, nullptr, 0.0, nullptr, 0.0, z, nullptr, w0, nullptr));
    HIP_TRY(launch_pcgs_vec(P->g, L, 2, nullptr, nullptr, 0.0, nullptr, 0.0, x, r, p, q, z, b, sinv, nullptr, P->st,
                            P->partials, 1));
    HIP_TRY(launch_finalize(P->stream, P->partials, L.grid, 3, 0, 1, nullptr, P->st, rtol * rtol, maxit));
    HIP_TRY(hipMemcpyAsync(p, z, size_t(P->g.N) * sizeof(double), hipMemcpyDeviceToDevice, P->stream));
    const int32_t* skip = &P->st->done;
    // power-of-two m_0 >= 64: the x / r update rides on the preconditioner's first (d = 0) pass and the
    // s^-1 scaling with r.z, |r|^2 on its last, seven launches per iteration instead of nine
    const size_t pwords = size_t(std::max(kMaxGrid, kMaxCgBlocks)) * kMaxRed;
    const bool fused7 = dct_pcg_fusable(P->g, pwords);
    auto enqueue7 = [&]() -> mvtv_status {
        const int pdim = P->g.p;
        int np_last = 0;
        for (int t = 0; t < 2 * pdim - 1; ++t) {
            const int d = t < pdim ? t : 2 * pdim - 2 - t;
            const int mode = t < pdim - 1 ? 0 : (t == pdim - 1 ? 2 : 1);
            PcgFuse f;
            if (t == 0 || t == 2 * pdim - 2) {
                f.mode = t == 0 ? 1 : 2;
                f.st = P->st;
                f.x = x;
                f.r = r;
                f.p = p;
                f.q = q;
                f.sinv = sinv;
                f.partials = P->partials;
                f.cap = pwords;
                f.nparts = &np_last;
            }
            const int hh = P->tstart(t == 0 ? MVTV_K_DCT_FIRST : MVTV_K_DCT);
            HIP_TRY(launch_dct_pass(P->spec, P->g, P->stream, mode, d, t == 0 ? r : z, nullptr, 0.0, nullptr, 0.0, z,
                                    sigma, w0, nullptr, 0, 0.0, skip, f.mode ? &f : nullptr));
            P->tstop(hh);
        }
        HIP_TRY(launch_finalize(P->stream, P->partials, np_last, 2, 0, 3, nullptr, P->st));        // beta, done
        return MVTV_OK;
    };
    auto enqueue = [&]() -> mvtv_status {
        int hh = P->tstart(MVTV_K_PCG_APPLY);
        int npa = L.grid;
        HIP_TRY(launch_apply_A(P->g, L, sigma, P->wmode, P->wdiag, p, q, P->partials, P->st, &npa));   // q = A p, p.q
        P->tstop(hh);
        HIP_TRY(launch_finalize(P->stream, P->partials, npa, 1, 0, 2, nullptr, P->st));              // alpha
        if (fused7) {
            MVTV_TRY(enqueue7());
            hh = P->tstart(MVTV_K_PCG_DIRECTION);
            HIP_TRY(launch_pcgs_vec(P->g, L, 3, nullptr, nullptr, 0.0, nullptr, 0.0, x, r, p, q, z, b, nullptr, nullptr,
                                    P->st, nullptr, 0));
            P->tstop(hh);
            return MVTV_OK;
        }
        hh = P->tstart(MVTV_K_PCG_UPDATE);
        HIP_TRY(launch_pcgs_vec(P->g, L, 1, nullptr, nullptr, 0.0, nullptr, 0.0, x, r, p, q, nullptr, b, sinv, t,
                                P->st, nullptr, 0));
        P->tstop(hh);
        MVTV_TRY(spectral_solve(P, sigma, rin, nullptr, 0.0, nullptr, 0.0, z, nullptr, w0, skip));   // z = M^-1 r
        HIP_TRY(launch_pcgs_vec(P->g, L, 2, nullptr, nullptr, 0.0, nullptr, 0.0, x, r, p, q, z, b, sinv, nullptr,
                                P->st, P->partials, 0));
        HIP_TRY(launch_finalize(P->stream, P->partials, L.grid, 3, 0, 3, nullptr, P->st));         // beta, done
        hh = P->tstart(MVTV_K_PCG_DIRECTION);
        HIP_TRY(launch_pcgs_vec(P->g, L, 3, nullptr, nullptr, 0.0, nullptr, 0.0, x, r, p, q, z, b, nullptr, nullptr,
                                P->st, nullptr, 0));
        P->tstop(hh);
        return MVTV_OK;
    };
    std::vector<size_t> mark;
    int enq = 0;
    int batch = P->pcg_hint > 0 ? std::max(2, P->pcg_hint + pcg_ahead()) : kPcgPoll;
    for (;;) {
        for (int bb = 0; bb < batch && enq < maxit; ++bb, ++enq) {
            mark.push_back(P->pending.size());
            MVTV_TRY(enqueue());
        }
        HIP_TRY(hipMemcpyAsync(P->host_st, P->st, sizeof(PcgState), hipMemcpyDeviceToHost, P->stream));
        HIP_TRY(hipStreamSynchronize(P->stream));
        const int done_iters = P->host_st->iter;
        if (P->timing && done_iters < int(mark.size()))
            for (size_t e = mark[size_t(done_iters)]; e < P->pending.size(); ++e) P->pending[e].kid = -1;
        P->harvest();
        if (P->host_st->done || enq >= maxit) break;
        batch = 2;
    }
    *iters = P->host_st->iter;
    P->pcg_hint = *iters;
    *relres = P->host_st->bnorm2 > 0 ? std::sqrt(P->host_st->rnorm2 / P->host_st->bnorm2) : 0.0;
    return MVTV_OK;
}

mvtv_status ensure_state(mvtv_problem* P) {
    if (!P->have_state) return fail(MVTV_BAD_ARG, "no ADMM state: call mvtv_state_set first");
    return MVTV_OK;
}

}  // namespace

// the slab loop's ranks pick their z ping-pong pair the same way (mvtv_slab.cpp)
mvtv_status zpair_pick(mvtv_problem* P, bool track_theta, bool twin) { return pick_zpair(P, track_theta, twin); }

// =================================================================================== C ABI
extern "C" {

const char* mvtv_version(void) { return "multivartv_amd 0.1.0 (gfx950)"; }

const char* mvtv_status_string(int32_t s) {
    switch (s) {
        case MVTV_OK: return "ok";
        case MVTV_MAXITER: return "maximum ADMM iterations reached";
        case MVTV_BAD_ARG: return "bad argument";
        case MVTV_DIM_MISMATCH: return "dimension mismatch (mixed-partial construction)";
        case MVTV_HIP_ERROR: return "HIP error";
        case MVTV_NO_DEVICE: return "no HIP device";
        case MVTV_OUT_OF_MEMORY: return "out of device memory";
        case MVTV_PCG_NOT_CONVERGED: return "PCG theta-solve did not converge";
        default: return "unknown status";
    }
}

const char* mvtv_last_error(void) { return g_last_error.c_str(); }

int32_t mvtv_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

void mvtv_default_opts(mvtv_admm_opts* o, int32_t variant) {
    std::memset(o, 0, sizeof(*o));
    o->variant = variant;
    o->sigma = std::nan("");
    o->ymean = 0.0;
}

}  // extern "C"

namespace {
mvtv_status problem_create_impl(const mvtv_problem_desc* d, const mvtv_slab_desc* sl, mvtv_problem** out) {
    if (!d || !out) return fail(MVTV_BAD_ARG, "null descriptor/output");
    *out = nullptr;
    if (d->p < 1 || d->p > MVTV_MAX_DIMS) return fail(MVTV_BAD_ARG, "p must be in 1..4");
    if (!d->oty) return fail(MVTV_BAD_ARG, "oty is required");
    if (d->block_order != MVTV_ORDER_CPP && d->block_order != MVTV_ORDER_PY) return fail(MVTV_BAD_ARG, "block_order");
    const int p = d->p;
    uint64_t N = 1;
    // slab: the mesh is validated (and D built) with the global extent of dim p-1
    int64_t mg[MVTV_MAX_DIMS];
    for (int j = 0; j < MVTV_MAX_DIMS; ++j) mg[j] = d->m[j];
    if (sl) {
        if (p < 2) return fail(MVTV_BAD_ARG, "slab decomposition needs p >= 2");
        if (sl->z_begin < 0 || sl->z_end <= sl->z_begin || sl->z_end > sl->m_global)
            return fail(MVTV_BAD_ARG, "slab plane range");
        if ((sl->ghost_lo != 0) != (sl->z_begin > 0) || (sl->ghost_hi != 0) != (sl->z_end < sl->m_global))
            return fail(MVTV_BAD_ARG, "slab ghosts: one plane below unless z_begin = 0, one above unless z_end = m");
        if (d->m[p - 1] != sl->z_end - sl->z_begin + (sl->ghost_lo ? 1 : 0) + (sl->ghost_hi ? 1 : 0))
            return fail(MVTV_BAD_ARG, "local m[p-1] must be owned planes + ghosts");
        mg[p - 1] = sl->m_global;
    }
    for (int j = 0; j < p; ++j) {
        if (d->m[j] < 2 && !(sl && j == p - 1)) return fail(MVTV_BAD_ARG, "every m_j must be >= 2");
        if (mg[j] < 2) return fail(MVTV_BAD_ARG, "every m_j must be >= 2");
        N *= uint64_t(d->m[j]);
    }
    if (N >= (uint64_t(1) << 31)) return fail(MVTV_BAD_ARG, "N >= 2^31 nodes on one GPU");
    const int full = (1 << p) - 1;
    int nb;
    if (d->block_order == MVTV_ORDER_CPP) nb = full;
    else nb = d->weighted ? full - 1 : full;
    if (nb <= 0) return fail(MVTV_BAD_ARG, "empty D (Python create_D with deltas at p = 1)");
    int ndev = mvtv_device_count();
    if (ndev <= 0) return fail(MVTV_NO_DEVICE, "no HIP device visible");
    if (d->device < 0 || d->device >= ndev) return fail(MVTV_BAD_ARG, "device ordinal out of range");

    auto* P = new mvtv_problem();
    P->device = d->device;
    P->order = d->block_order;
    P->weighted = d->weighted;
    Geom& g = P->g;
    g.p = p;
    g.nb = nb;
    g.N = uint32_t(N);
    uint32_t stride = 1;
    for (int j = 0; j < MVTV_MAX_DIMS; ++j) {
        g.m[j] = j < p ? uint32_t(d->m[j]) : 1u;
        g.stride[j] = stride;
        if (j < p) stride *= g.m[j];
        P->deltas[j] = j < p ? d->deltas[j] : 0.0;
    }
    for (int j = 0; j < MVTV_MAX_DIMS - 1; ++j) g.fd[j] = FastDiv(g.m[j]);
    for (int S = 0; S < 16; ++S) g.cS[S] = 0.0;
    P->E = 0;
    for (int k = 0; k < nb; ++k) {
        const int b = block_code(k, p, P->order);
        const int S = sprime_mask(b, p);
        // reference mixedpartial: a mixed block with min S > 0 multiplies incompatible
        // matrices unless m_0 == m_{min S} (code/utils.py:102-129)
        int nominal = 0;
        for (int j = 0; j < p; ++j)
            if ((b >> (p - 1 - j)) & 1) nominal |= 1 << j;
        if (popcount(nominal) >= 2 && !(nominal & 1)) {
            int lo = 0;
            while (!((nominal >> lo) & 1)) ++lo;
            if (mg[0] != mg[lo]) {
                delete P;
                return fail(MVTV_DIM_MISMATCH, "mixed partial of block " + std::to_string(b) +
                                                   ": m[0] != m[" + std::to_string(lo) + "]");
            }
        }
        double w = 1.0;
        if (d->weighted)
            for (int j = 0; j < p; ++j)
                if (!((b >> (p - 1 - j)) & 1)) w *= d->deltas[j];
        g.w[k] = w;
        g.cS[S] += w * w;
        P->codes[k] = b;
        P->sprime[k] = S;
        uint64_t len = 1;
        for (int j = 0; j < p; ++j) len *= uint64_t(g.m[j] - ((S >> j) & 1));
        P->blk_len[k] = len;
        P->E += int64_t(len);
    }
    for (int k = nb; k < kMaxBlocks; ++k) g.w[k] = 0.0;
    g.ibeg = 0;
    g.iend = uint32_t(N);
    if (sl) {
        const uint32_t plane = uint32_t(N / uint64_t(d->m[p - 1]));
        P->slab = true;
        P->m_global = sl->m_global;
        P->zb = sl->z_begin;
        P->ze = sl->z_end;
        P->g_lo = sl->ghost_lo ? 1 : 0;
        P->g_hi = sl->ghost_hi ? 1 : 0;
        g.ibeg = uint32_t(P->g_lo) * plane;
        g.iend = uint32_t(N) - uint32_t(P->g_hi) * plane;
    }
    P->grid = int(std::min<uint64_t>((N + kThreads - 1) / kThreads, kMaxGrid));
    if (const char* env = std::getenv("MVTV_PCG")) P->fused3d = std::strcmp(env, "classic") != 0;

    DeviceGuard dg(P->device);
    mvtv_status s = MVTV_OK;
    auto A = [&](double** ptr, size_t n) {
        if (s == MVTV_OK) s = alloc(ptr, n);
    };
    if (hipStreamCreateWithFlags(&P->stream, hipStreamNonBlocking) != hipSuccess) {
        delete P;
        return fail(MVTV_HIP_ERROR, "hipStreamCreate failed");
    }
    A(&P->oty, N);
    A(&P->theta, N);
    A(&P->edges, size_t(nb) * N);
    A(&P->ga, N);
    A(&P->gu, N);
    A(&P->guprev, N);
    A(&P->r, N);
    A(&P->p, N);
    A(&P->q, N);
    A(&P->partials, size_t(std::max(kMaxGrid, kMaxCgBlocks)) * kMaxRed);
    A(&P->red, 16);
    if (s == MVTV_OK && hipMalloc(reinterpret_cast<void**>(&P->st), sizeof(PcgState)) != hipSuccess)
        s = fail(MVTV_OUT_OF_MEMORY, "hipMalloc(PcgState)");
    if (s == MVTV_OK && hipHostMalloc(reinterpret_cast<void**>(&P->host_red), 16 * sizeof(double) + sizeof(PcgState)) != hipSuccess)
        s = fail(MVTV_OUT_OF_MEMORY, "hipHostMalloc");
    if (s == MVTV_OK && (hipMalloc(reinterpret_cast<void**>(&P->ctl), sizeof(AdmmCtl)) != hipSuccess ||
                         hipHostMalloc(reinterpret_cast<void**>(&P->host_ctl), sizeof(AdmmCtl)) != hipSuccess))
        s = fail(MVTV_OUT_OF_MEMORY, "control block");
    if (s != MVTV_OK) {
        free_all(P);
        delete P;
        return s;
    }
    P->host_st = reinterpret_cast<PcgState*>(P->host_red + 16);
    // cosine transforms of any length <= 4096: FFT plans for 2-3-5-7 lengths, Bluestein (k_dctb) for the rest
    P->spec_mesh = P->spec_pow2 = P->spec_lead = true;
    for (int j = 0; j < p; ++j) {
        const uint32_t mj = uint32_t(mg[j]);
        if (mj > 4096) {
            P->spec_mesh = false;
            if (j < p - 1) P->spec_lead = false;
        }
        if ((mj & (mj - 1)) != 0) P->spec_pow2 = false;
    }
    if (!P->spec_mesh) P->spec_pow2 = false;
    // a slab problem's last dimension is solved by the substructured line solves (any length): the tables
    // are needed for the transforms along dims 0..p-2 only
    if (P->spec_mesh || (P->slab && P->spec_lead && p >= 2)) s = spectral_plan(P);
    P->e3d = edge3d_ok(g);
    if (s == MVTV_OK && P->e3d && g.p == 4 && gather4_ok(g)) s = alloc(&P->g4, 4 * size_t(N));
    P->f3d = fused3d_ok(g);   // slab problems too: the fused pass runs on the owned planes (Geom.ibeg/iend)
    P->f4d = P->e3d && g.p == 4 && P->g4 != nullptr && fused4_ok(g);   // slab ranks: on the owned planes
    {   // chunked edge layout for the 3-D fused path (MVTV_EAOS=0 keeps block-major): the fused kernel's
        // launches 2-4 % shorter at 512^3 on the same box (4.21 -> 4.13 ms, 5.2-5.36 -> 5.13 ms)
        const char* e = probe_env("MVTV_EAOS");
        const bool want = e ? std::atoi(e) != 0 : true;
        // a slab rank decides from its plane size, which every rank shares (its N counts its own ghost
        // planes): the z halo moves whole planes, one contiguous run per plane only when planes are whole
        // 64-node chunks, so every rank must pick the same layout
        const uint64_t plane = g.N / g.m[g.p - 1];
        const bool chunks = P->slab ? plane % 64 == 0 : g.N % 64 == 0;
        g.eaos = (want && ((P->f3d && g.p == 3) || (P->e3d && g.p == 4)) && chunks) ? 1u : 0u;
    }
    if (s == MVTV_OK) s = mvtv_problem_set_data(P, d->oty, d->wdiag);
    if (s != MVTV_OK) {
        free_all(P);
        delete P;
        return s;
    }
    *out = P;
    return MVTV_OK;
}
}  // namespace

extern "C" {

mvtv_status mvtv_problem_create(const mvtv_problem_desc* d, mvtv_problem** out) {
    return problem_create_impl(d, nullptr, out);
}

mvtv_status mvtv_problem_create_slab(const mvtv_problem_desc* d, const mvtv_slab_desc* slab, mvtv_problem** out) {
    if (!slab) return fail(MVTV_BAD_ARG, "null slab descriptor");
    return problem_create_impl(d, slab, out);
}

void mvtv_problem_destroy(mvtv_problem* P) {
    if (!P) return;
    DeviceGuard dg(P->device);
    (void)hipStreamSynchronize(P->stream);
    free_all(P);
    delete P;
}

int64_t mvtv_problem_nodes(const mvtv_problem* P) { return P ? int64_t(P->g.N) : 0; }
int64_t mvtv_problem_edges(const mvtv_problem* P) { return P ? P->E : 0; }
int32_t mvtv_problem_blocks(const mvtv_problem* P) { return P ? P->g.nb : 0; }
int32_t mvtv_problem_spectral_ok(const mvtv_problem* P) { return P && spectral_ok(P) ? 1 : 0; }

mvtv_status mvtv_problem_block_info(const mvtv_problem* P, int32_t k, int32_t* code, int32_t* sprime, double* weight) {
    if (!P || k < 0 || k >= P->g.nb) return fail(MVTV_BAD_ARG, "block index");
    if (code) *code = P->codes[k];
    if (sprime) *sprime = P->sprime[k];
    if (weight) *weight = P->g.w[k];
    return MVTV_OK;
}

mvtv_status mvtv_problem_set_data(mvtv_problem* P, const double* oty, const double* wdiag) {
    if (!P || !oty) return fail(MVTV_BAD_ARG, "null problem/oty");
    DeviceGuard dg(P->device);
    const size_t bytes = size_t(P->g.N) * sizeof(double);
    HIP_TRY(hipMemcpyAsync(P->oty, oty, bytes, hipMemcpyHostToDevice, P->stream));
    if (wdiag) {
        if (!P->wdiag) MVTV_TRY(alloc(&P->wdiag, P->g.N));
        HIP_TRY(hipMemcpyAsync(P->wdiag, wdiag, bytes, hipMemcpyHostToDevice, P->stream));
        P->wmode = W_DIAG;
        double acc = 0.0, acc2 = 0.0;
        for (uint32_t i = 0; i < P->g.N; ++i) acc += wdiag[i];
        P->wmean = acc / double(P->g.N);
        for (uint32_t i = 0; i < P->g.N; ++i) acc2 += (wdiag[i] - P->wmean) * (wdiag[i] - P->wmean);
        P->wstd = std::sqrt(acc2 / double(P->g.N));
        // a slab rank's share of the global mean / spread (its owned planes), summed over the ranks by mvtv_slab_run
        P->wsum_own = P->wsum2_own = 0.0;
        for (uint32_t i = P->g.ibeg; i < P->g.iend; ++i) {
            P->wsum_own += wdiag[i];
            P->wsum2_own += wdiag[i] * wdiag[i];
        }
    } else {
        P->wmode = W_IDENTITY;
        P->wmean = 1.0;
        P->wstd = 0.0;
        P->wsum_own = P->wsum2_own = double(P->g.iend - P->g.ibeg);
    }
    HIP_TRY(hipStreamSynchronize(P->stream));
    return MVTV_OK;
}

mvtv_status mvtv_state_set(mvtv_problem* P, const double* theta, const double* u, double rho) {
    if (!P || !theta) return fail(MVTV_BAD_ARG, "null problem/theta");
    DeviceGuard dg(P->device);
    HIP_TRY(hipMemcpyAsync(P->theta, theta, size_t(P->g.N) * sizeof(double), hipMemcpyHostToDevice, P->stream));
    P->twin_ok = true;
    if (u) {
        MVTV_TRY(import_edges(P, u, P->edges));
        P->u_default = false;
        uint64_t off[kMaxBlocks + 1] = {0};   // the twin blocks of the caller's u (reference block layout)
        for (int k = 0; k < P->g.nb; ++k) off[k + 1] = off[k] + P->blk_len[k];
        for (int k = 0; k < P->g.nb && P->twin_ok; ++k) {
            const int c = twin_of(k, P->g.p, P->order);
            if (c != k)
                P->twin_ok = P->blk_len[k] == P->blk_len[c] &&
                             std::memcmp(u + off[k], u + off[c], size_t(P->blk_len[k]) * sizeof(double)) == 0;
        }
    } else {
        P->u_default = true;
    }
    HIP_TRY(hipStreamSynchronize(P->stream));
    P->edge_mode = U_EXPLICIT;
    P->t_z = 0.0;
    P->c_state = 1.0;
    P->rho = rho;
    P->have_state = true;
    return MVTV_OK;
}

mvtv_status mvtv_state_get(mvtv_problem* P, double* theta, double* u, double* rho) {
    if (!P) return fail(MVTV_BAD_ARG, "null problem");
    MVTV_TRY(ensure_state(P));
    DeviceGuard dg(P->device);
    if (theta) {
        HIP_TRY(hipMemcpyAsync(theta, P->theta, size_t(P->g.N) * sizeof(double), hipMemcpyDeviceToHost, P->stream));
        HIP_TRY(hipStreamSynchronize(P->stream));
    }
    if (u) {
        if (P->u_default) return fail(MVTV_BAD_ARG, "u is the variant default and has not been formed yet");
        MVTV_TRY(export_edges(P, P->edges, u, P->edge_mode, P->t_z, P->c_state));
    }
    if (rho) *rho = P->rho;
    return MVTV_OK;
}

mvtv_status mvtv_admm_run(mvtv_problem* P, const mvtv_admm_opts* opts_in, double lambda, mvtv_admm_stats* stats) {
    if (!P || !opts_in) return fail(MVTV_BAD_ARG, "null problem/opts");
    MVTV_TRY(ensure_state(P));
    if (!(lambda >= 0.0)) return fail(MVTV_BAD_ARG, "lambda must be >= 0");
    const auto t0 = std::chrono::steady_clock::now();
    DeviceGuard dg(P->device);
    const mvtv_admm_opts& o = *opts_in;
    const int variant = o.variant;
    if (variant < 0 || variant > 2) return fail(MVTV_BAD_ARG, "variant");
    const double tol = variant_tol(o);
    const int max_counter = variant_maxc(o);
    const double rtol = o.pcg_rtol > 0 ? o.pcg_rtol : 1e-10;
    const int pcg_maxit = o.pcg_max_iter > 0 ? o.pcg_max_iter : 20000;
    const Launch L = P->L();
    const double N = double(P->g.N), E = double(P->E);
    if (o.theta_solver < MVTV_SOLVER_AUTO || o.theta_solver > MVTV_SOLVER_PCG_SPECTRAL)
        return fail(MVTV_BAD_ARG, "theta_solver");
    if (o.theta_solver == MVTV_SOLVER_SPECTRAL && !spectral_ok(P))
        return fail(MVTV_BAD_ARG, "spectral theta-solve needs W = I and every m_j <= 4096");
    if (o.theta_solver == MVTV_SOLVER_PCG_SPECTRAL && (!P->spec_mesh || P->wmode == W_NONE))
        return fail(MVTV_BAD_ARG, "spectral preconditioner needs every m_j <= 4096");
    const bool spectral = o.theta_solver == MVTV_SOLVER_SPECTRAL ||
                          (o.theta_solver == MVTV_SOLVER_AUTO && spectral_ok(P));
    // AUTO with W != I on a spectral mesh: PCG with the spectral preconditioner (K an order of magnitude
    // below Jacobi's once sigma D^T D dominates); other meshes: Jacobi-PCG
    const bool pcg_spec = o.theta_solver == MVTV_SOLVER_PCG_SPECTRAL ||
                          (o.theta_solver == MVTV_SOLVER_AUTO && !spectral && P->spec_mesh && P->wmode != W_NONE &&
                           !P->slab);

    // ---- initial state: u explicit in the edge buffer, alpha_0 = D theta_0 ------------------
    double rho;
    if (variant == MVTV_VARIANT_RCPP) rho = P->rho;                      // rho_init (:100)
    else if (variant == MVTV_VARIANT_CPP) rho = double(int(lambda));     // int rho = lambda (:108)
    else rho = lambda;                                                   // rho = tune (py :55)
    double sigma = std::isnan(o.sigma) ? (variant == MVTV_VARIANT_RCPP ? rho : lambda) : o.sigma;
    double* gprev = P->guprev;
    double* gnew = P->gu;
    double c_prev = 1.0, t_z = 0.0;
    int mode = U_EXPLICIT;
    int h = -1;
    if (P->edge_mode == U_FROM_Z) {
        // resume from the resident state of the previous call: u0 = -c clamp(z, t_z) is read straight
        // from z by the first edge update, and P->guprev already holds D^T clamp-part of it (scale c)
        mode = U_FROM_Z;
        t_z = P->t_z;
        c_prev = P->c_state;
    } else {
        if (P->u_default) {
            const double u0 = variant == MVTV_VARIANT_RCPP ? 0.0 : 1.0 / lambda;   // A :101, C :62
            HIP_TRY(launch_edges_fill_valid(P->g, P->order, L, P->edges, u0));
            P->u_default = false;
        }
        // g_uprev = D^T u0
        h = P->tstart(MVTV_K_GATHER);
        int np0 = L.grid;
        if (P->e3d)
            HIP_TRY(launch_gather3d(P->g, P->order, U_EXPLICIT, P->stream, P->edges, 0.0, nullptr, gprev, nullptr, 1.0,
                                    P->partials, &np0, nullptr, P->g4));
        else
            HIP_TRY(launch_gather(P->g, P->order, U_EXPLICIT, L, P->edges, 0.0, nullptr, gprev, nullptr, 1.0,
                                  P->partials));
        P->tstop(h);
    }
    // g_alpha = D^T D theta0 (alpha0 = D theta0, rcpp…/solvers.cpp:101)  ->  b_1 = oty + rho D^T (alpha0 + u0)
    h = P->tstart(MVTV_K_OTHER);
    HIP_TRY(launch_apply_A(P->g, L, 1.0, W_NONE, nullptr, P->theta, P->ga, nullptr, nullptr));
    P->tstop(h);
    int np = L.grid;

    const bool track_theta = variant != MVTV_VARIANT_RCPP;
    const bool fused = P->f3d;
    const bool fused4 = P->f4d;   // 4-D: edge update + gather pass A fused, pass B separate
    const bool pingpong = fused || fused4;
    if (pingpong && !P->edges2) MVTV_TRY(alloc(&P->edges2, size_t(P->g.nb) * P->g.N));
    // MVTV_EBUF3=1: z rotates over three buffers (when the third fits with 16 GiB to spare). Opt-in:
    // over five boxes it is as often slower as faster than two (profiles/r01/v8_ebuf3_ab.txt)
    static const int rot3_env = [] {
        const char* e = probe_env("MVTV_EBUF3");
        return e ? std::atoi(e) : 0;
    }();
    if (fused && spectral && rot3_env != 0 && !P->edges3) {
        const size_t ne = size_t(P->g.nb) * P->g.N;
        size_t fr = 0, tot = 0;
        const bool fits = hipMemGetInfo(&fr, &tot) == hipSuccess && fr > ne * sizeof(double) + (size_t(16) << 30);
        if (rot3_env > 0 || fits) MVTV_TRY(alloc(&P->edges3, ne));
    }
    const int nbuf = (fused && P->edges3) ? 3 : 2;
    // MVTV_ZFLIP (probe only, tools/zflip_probe.py): move z to the other edge buffer before this run,
    // so the g_u ping-pong meets the z ping-pong in the other pairing of physical buffers
    if (fused && nbuf == 2 && probe_env("MVTV_ZFLIP")) {
        HIP_TRY(hipMemcpyAsync(P->edges2, P->edges, size_t(P->g.nb) * P->g.N * sizeof(double),
                               hipMemcpyDeviceToDevice, P->stream));
        std::swap(P->edges, P->edges2);
    }
    if (fused && probe_env("MVTV_GFLIP")) {   // probe only: the same for the g_u ping-pong
        HIP_TRY(hipMemcpyAsync(P->gu, P->guprev, size_t(P->g.N) * sizeof(double), hipMemcpyDeviceToDevice,
                               P->stream));
        std::swap(P->gu, P->guprev);
    }
    // the twin blocks are skipped by the fused kernels and filled from their group's first block when the run ends
    const bool twin = (fused || fused4) && twin_ready(P);
    // an early return (MVTV_TRY / HIP_TRY) after twin-skipping iterations must not leave a stale twin block behind
    // twin_ok: fill the twins of both edge buffers (whichever holds the state), best effort; the normal exits
    // fill them themselves and disarm
    struct TwinGuard {
        mvtv_problem* P;
        bool armed;
        ~TwinGuard() {
            if (!armed) return;
            (void)fill_twins(P->g, P->order, P->stream, P->edges);
            if (P->edges2) (void)fill_twins(P->g, P->order, P->stream, P->edges2);
            if (P->edges3) (void)fill_twins(P->g, P->order, P->stream, P->edges3);
            (void)hipStreamSynchronize(P->stream);
            (void)hipGetLastError();
        }
    } twin_guard{P, twin};
    if (P->timing && (fused || fused4)) P->twin_timed = twin;
    if (fused && spectral && nbuf == 2 && !P->zpicked) MVTV_TRY(pick_zpair(P, track_theta, twin));
    double dtheta = 0.0;
    if (track_theta) {
        if (!P->thold) MVTV_TRY(alloc(&P->thold, P->g.N));
        HIP_TRY(launch_fill(P->stream, P->thold, o.ymean - (variant == MVTV_VARIANT_CPP ? 0.1 : 1.0), P->g.N));
        HIP_TRY(launch_maxabsdiff(P->g, L, P->theta, P->thold, P->partials));
        HIP_TRY(launch_finalize(P->stream, P->partials, L.grid, 1, 1, 0, P->red, P->st));
        HIP_TRY(hipMemcpyAsync(P->host_red, P->red, sizeof(double), hipMemcpyDeviceToHost, P->stream));
        MVTV_TRY(P->sync());
        dtheta = P->host_red[0];
    }

    // ---- asynchronous loop (spectral theta-solve): the decisions of every iteration are taken on
    // the device by k_admm_control, the host enqueues iterations ahead and polls the done flag -------
    const bool first_runs = o.fixed_iters > 0 ? o.fixed_iters > 0
                                              : (variant == MVTV_VARIANT_RCPP ? true
                                                                              : (dtheta > tol && !(variant == MVTV_VARIANT_PY &&
                                                                                                   max_counter <= 0)));
    if (spectral && first_runs && !std::getenv("MVTV_ADMM_SYNC")) {
        AdmmCtl& c = *P->host_ctl;
        std::memset(&c, 0, sizeof(c));
        c.variant = variant;
        c.fixed_iters = o.fixed_iters > 0 ? o.fixed_iters : 0;
        c.max_counter = max_counter;
        c.lambda = lambda;
        c.tol = tol;
        c.sqrtN = std::sqrt(N);
        c.sqrtE = std::sqrt(E);
        c.rho = rho;
        c.sigma = sigma;
        c.c_prev = c_prev;
        c.t_z = t_z;
        c.t_next = rho != 0.0 ? lambda / rho : INFINITY;
        c.counter = 1;
        c.dtheta = dtheta;
        c.dual_norm = c.primal_norm = 1.0;
        c.eps_dual = c.eps_pri = tol;
        HIP_TRY(hipMemcpyAsync(P->ctl, &c, sizeof(AdmmCtl), hipMemcpyHostToDevice, P->stream));
        double* gbuf[2] = {P->guprev, P->gu};
        double* ebuf[3] = {P->edges, P->edges2, P->edges3};
        // FOLD (variant B): the fused 3-D kernel stores s = rho (D^T alpha + D^T u) in P->ga instead of D^T alpha, so
        // the next solve's first pass reads oty and s (2N words) instead of oty, D^T alpha and D^T u (3N); after a
        // control step that changed rho it forms oty + (rho'/rho) s + rho' (c - 1) D^T u (AdmmCtl::fold_ka / _kb)
        // (the first pass transforms dim 0, or dim 2 on k_march meshes)
        const uint32_t m0 = (!P->slab && march_ok(P->g)) ? P->g.m[2] : P->g.m[0];
        const bool fold_path = fused ? (P->g.p == 2 || P->g.p == 3)
                                     : (P->g.p == 4 && P->e3d && P->g4 != nullptr && gather4_ok(P->g));   // two-pass 4-D
        // on k_march meshes the folded first pass runs along dim 2 at stride m0 * m1, which must be a power of two too
        const uint64_t fold_stride = (!P->slab && march_ok(P->g)) ? uint64_t(P->g.m[0]) * P->g.m[1] : 1;
        const bool fold = fold_path && variant == MVTV_VARIANT_RCPP && m0 >= 8 && m0 <= 4096 &&
                          (m0 & (m0 - 1)) == 0 && (fold_stride & (fold_stride - 1)) == 0 &&
                          !probe_env("MVTV_FOLD_OFF") && !probe_env("MVTV_DCT_LDS") && !probe_env("MVTV_DCT_MID");
        auto enqueue = [&](int j) -> mvtv_status {
            double* gp = gbuf[j & 1];
            double* gn = gbuf[(j + 1) & 1];
            const int um = j == 0 ? mode : U_FROM_Z;
            if (track_theta)
                HIP_TRY(hipMemcpyAsync(P->thold, P->theta, size_t(P->g.N) * sizeof(double), hipMemcpyDeviceToDevice,
                                       P->stream));
            MVTV_TRY(spectral_solve(P, sigma, P->oty, P->ga, rho, gp, rho, P->theta, P->ctl, 1.0, nullptr,
                                    fold && j > 0));
            if (fused) {   // z ping-pongs between the two edge buffers
                int hh = P->tstart(MVTV_K_ADMM_FUSED);
                int npf = 0;
                HIP_TRY(launch_admm3d(P->g, P->order, um, P->stream, P->theta, ebuf[j % nbuf], ebuf[(j + 1) % nbuf], 0.0, 1.0,
                                      0.0, 1.0, track_theta ? P->thold : nullptr, P->ga, gn, gp, P->partials, &npf,
                                      P->ctl, fold, twin));
                P->tstop(hh);
                hh = P->tstart(MVTV_K_REDUCE);
                HIP_TRY(launch_finalize(P->stream, P->partials, npf, ER_N + GR_N, -(1 << ER_DTH), 0, P->red, P->st, 0.0,
                                        0, P->ctl, P->ctl, P->red));   // + the control step
                P->tstop(hh);
                return MVTV_OK;
            }
            if (fused4) {   // z ping-pongs as in the 3-D fused loop; pass B of the gather after the ER reduction
                int hh = P->tstart(MVTV_K_ADMM_FUSED4);
                int npe = 0;
                HIP_TRY(launch_admm4a(P->g, P->order, um, P->stream, P->theta, ebuf[j % nbuf], ebuf[(j + 1) % nbuf], 0.0,
                                      1.0, 0.0, track_theta ? P->thold : nullptr, P->g4, P->partials, &npe, P->ctl,
                                      twin));
                P->tstop(hh);
                hh = P->tstart(MVTV_K_REDUCE);
                HIP_TRY(launch_finalize(P->stream, P->partials, npe, ER_N, 1, 0, P->red, P->st, 0.0, 0, P->ctl));
                P->tstop(hh);
                hh = P->tstart(MVTV_K_GATHER4B);
                int npg = 0;
                HIP_TRY(launch_gather4b(P->g, U_FROM_Z, P->stream, P->ga, gn, gp, 1.0, P->partials, &npg, P->ctl, P->g4,
                                        fold));
                P->tstop(hh);
                hh = P->tstart(MVTV_K_REDUCE);
                HIP_TRY(launch_finalize(P->stream, P->partials, npg, GR_N, 0, 0, P->red + ER_N, P->st, 0.0, 0, P->ctl,
                                        P->ctl, P->red));   // + the control step
                P->tstop(hh);
                return MVTV_OK;
            }
            int hh = P->tstart(MVTV_K_EDGE_UPDATE);
            int npe = L.grid;
            if (P->e3d)
                HIP_TRY(launch_edge3d(P->g, P->order, um, P->stream, P->theta, P->edges, 0.0, 1.0, 0.0,
                                      track_theta ? P->thold : nullptr, P->partials, &npe, P->ctl));
            else
                HIP_TRY(launch_edge_update(P->g, P->order, um, L, P->theta, P->edges, 0.0, 1.0, 0.0,
                                           track_theta ? P->thold : nullptr, P->partials, P->ctl));
            P->tstop(hh);
            hh = P->tstart(MVTV_K_REDUCE);
            HIP_TRY(launch_finalize(P->stream, P->partials, npe, ER_N, 1, 0, P->red, P->st, 0.0, 0, P->ctl));
            P->tstop(hh);
            hh = P->tstart(MVTV_K_GATHER);
            const int hb = P->tstart_b(MVTV_K_GATHER4B);
            int npg = L.grid;
            if (P->e3d)
                HIP_TRY(launch_gather3d(P->g, P->order, U_FROM_Z, P->stream, P->edges, 0.0, P->ga, gn, gp, 1.0,
                                        P->partials, &npg, P->ctl, P->g4, fold));
            else
                HIP_TRY(launch_gather(P->g, P->order, U_FROM_Z, L, P->edges, 0.0, P->ga, gn, gp, 1.0, P->partials,
                                      P->ctl));
            P->tstop(hh);
            P->tstop_b(hb);
            hh = P->tstart(MVTV_K_REDUCE);
            HIP_TRY(launch_finalize(P->stream, P->partials, npg, GR_N, 0, 0, P->red + ER_N, P->st, 0.0, 0, P->ctl, P->ctl,
                                    P->red));   // + the control step
            P->tstop(hh);
            return MVTV_OK;
        };
        const int limit = o.fixed_iters > 0 ? o.fixed_iters
                                            : (variant == MVTV_VARIANT_PY ? max_counter : max_counter + 1);
        int target = o.fixed_iters > 0 ? o.fixed_iters : (P->admm_hint > 0 ? P->admm_hint : 16);
        // Iterations j >= 1 repeat with period 2 (the z and D^T u ping-pongs), so iterations (odd j, j + 1) can be
        // replayed as one captured HIP graph instead of ~10 stream launches: without per-launch events, for meshes
        // whose launches are short enough for the launch path to matter (< 2^24 nodes)
        hipGraphExec_t gexec = nullptr;
        if (!P->timing && nbuf == 2 && P->g.N < (uint32_t(1) << 24) && admm_graph_enabled()) {
            const std::vector<const void*> key = {P->theta, P->oty, P->ga, P->thold, gbuf[0], gbuf[1], ebuf[0], ebuf[1],
                                                  reinterpret_cast<const void*>(uintptr_t(fold)),
                                                  reinterpret_cast<const void*>(uintptr_t(track_theta)),
                                                  reinterpret_cast<const void*>(uintptr_t(fused)),
                                                  reinterpret_cast<const void*>(uintptr_t(twin))};
            auto it = std::find_if(P->graphs.begin(), P->graphs.end(), [&](const auto& lg) { return lg.key == key; });
            if (it == P->graphs.end()) {
                // capture iterations 1 and 2; any failure leaves stream launches for this key (best effort)
                mvtv_problem::LoopGraph lg;
                lg.key = key;
                hipGraph_t gr = nullptr;
                if (hipStreamBeginCapture(P->stream, hipStreamCaptureModeThreadLocal) == hipSuccess) {
                    const bool ok = enqueue(1) == MVTV_OK && enqueue(2) == MVTV_OK;
                    const bool ended = hipStreamEndCapture(P->stream, &gr) == hipSuccess;
                    if (ok && ended && gr && hipGraphInstantiate(&lg.exec, gr, nullptr, nullptr, 0) != hipSuccess)
                        lg.exec = nullptr;
                    if (gr) (void)hipGraphDestroy(gr);
                }
                (void)hipGetLastError();
                if (P->graphs.size() >= 4) {   // the two z / D^T u parities of a few buffer sets
                    if (P->graphs.front().exec) (void)hipGraphExecDestroy(P->graphs.front().exec);
                    P->graphs.erase(P->graphs.begin());
                }
                P->graphs.push_back(lg);
                it = P->graphs.end() - 1;
            }
            gexec = it->exec;
        }
        const bool use_graph = gexec != nullptr;
        std::vector<size_t> mark;   // first timing entry of each enqueued iteration
        int enq = 0;
        for (;;) {
            while (enq < target && enq < limit) {
                if (use_graph && (enq & 1) && enq + 2 <= std::min(target, limit)) {
                    HIP_TRY(hipGraphLaunch(gexec, P->stream));
                    enq += 2;
                    continue;
                }
                mark.push_back(P->pending.size());
                MVTV_TRY(enqueue(enq++));
            }
            HIP_TRY(hipMemcpyAsync(P->host_ctl, P->ctl, sizeof(AdmmCtl), hipMemcpyDeviceToHost, P->stream));
            HIP_TRY(hipStreamSynchronize(P->stream));
            if (c.done || enq >= limit) break;
            target = enq + std::max(4, enq / 4);
        }
        const int it_done = c.it;
        if (P->timing && it_done < int(mark.size()))   // iterations enqueued past the stop did no work
            for (size_t e = mark[size_t(it_done)]; e < P->pending.size(); ++e) P->pending[e].kid = -1;
        P->harvest();
        if (P->timing && fold) P->fold_fix += c.nfix;
        if (o.fixed_iters <= 0 && c.status == 0) P->admm_hint = it_done + 1;
        if (it_done & 1) std::swap(P->guprev, P->gu);   // P->guprev holds D^T u of the current state
        if (fused && nbuf == 3) {   // the state is in ebuf[it_done % 3]
            P->edges = ebuf[it_done % 3];
            P->edges2 = ebuf[(it_done + 1) % 3];
            P->edges3 = ebuf[(it_done + 2) % 3];
        } else if (pingpong && (it_done & 1)) {
            std::swap(P->edges, P->edges2);
        }
        twin_guard.armed = false;
        if (twin) HIP_TRY(fill_twins(P->g, P->order, P->stream, P->edges));
        if (it_done > 0) P->edge_mode = U_FROM_Z;
        if (it_done > 0) P->t_z = c.t_z;
        P->c_state = c.c_prev;
        P->rho = c.rho;
        mvtv_admm_stats S{};
        S.iters = it_done;
        S.rho = c.rho;
        S.r_norm = c.r_norm;
        S.s_norm = c.s_norm;
        if (variant == MVTV_VARIANT_RCPP) {
            S.eps_pri = c.eps_pri;
            S.eps_dual = c.eps_dual;
        }
        S.dtheta_max = c.dtheta;
        S.theta_solver = MVTV_SOLVER_SPECTRAL;
        mvtv_status status = c.status ? MVTV_MAXITER : MVTV_OK;
        if (status == MVTV_MAXITER) {
            if (variant == MVTV_VARIANT_CPP) fail(status, "Failed to converge!");
            else if (variant == MVTV_VARIANT_RCPP && o.verbose) std::printf("ADMM reached max_counter at lambda = %g\n", lambda);
        }
        if (o.verbose) std::printf("Lambda= %g, Counter = %d\n", lambda, c.counter);
        S.status = status;
        S.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (stats) *stats = S;
        return status;
    }

    mvtv_admm_stats S{};
    S.status = MVTV_OK;
    double dual_norm = 1.0, primal_norm = 1.0, eps_dual = tol, eps_primal = tol;
    int counter = 1, it = 0;
    mvtv_status status = MVTV_OK;
    for (;;) {
        // ---- loop condition, evaluated at the top as in the reference -----------------------
        if (o.fixed_iters > 0) {
            if (it >= o.fixed_iters) break;
        } else if (variant == MVTV_VARIANT_RCPP) {
            if (!(dual_norm > eps_dual || primal_norm > eps_primal)) break;   // :110
        } else {
            if (!(dtheta > tol)) break;   // any(|theta - thetaold| > TOL): A :113, C :69
            if (variant == MVTV_VARIANT_PY && it >= max_counter) {
                status = MVTV_MAXITER;
                break;
            }
        }
        if (track_theta) HIP_TRY(hipMemcpyAsync(P->thold, P->theta, size_t(P->g.N) * sizeof(double),
                                                hipMemcpyDeviceToDevice, P->stream));
        // ---- theta-update: (W + sigma D^T D) theta = oty + rho D^T (alpha + u) ----------------
        int pit = 0;
        double relres = 0.0;
        if (spectral)
            MVTV_TRY(spectral_solve(P, sigma, P->oty, P->ga, rho, gprev, rho * c_prev, P->theta));
        else if (pcg_spec)
            MVTV_TRY(pcgs_solve(P, sigma, P->oty, P->ga, rho, gprev, rho * c_prev, P->theta, rtol, pcg_maxit, &pit,
                                &relres));
        else
            MVTV_TRY(pcg_solve(P, sigma, P->oty, P->ga, rho, gprev, rho * c_prev, P->theta, rtol, pcg_maxit, &pit,
                               &relres));
        S.pcg_iters += pit;
        S.pcg_iters_max = std::max(S.pcg_iters_max, pit);
        if (!spectral && pit >= pcg_maxit && !(relres <= rtol)) {
            S.pcg_unconverged += 1;
            if (o.pcg_strict) {
                status = MVTV_PCG_NOT_CONVERGED;
                fail(status, "PCG hit pcg_max_iter");
                break;
            }
        }
        // ---- z-update (soft threshold) and dual update over all edges -----------------------
        const double t_new = rho != 0.0 ? lambda / rho : INFINITY;
        if (fused) {   // edge update + gather in one pass, z ping-pongs between the edge buffers
            h = P->tstart(MVTV_K_ADMM_FUSED);
            HIP_TRY(launch_admm3d(P->g, P->order, mode, P->stream, P->theta, P->edges, P->edges2, t_z, c_prev, t_new,
                                  c_prev, track_theta ? P->thold : nullptr, P->ga, gnew, gprev, P->partials, &np,
                                  nullptr, false, twin));
            P->tstop(h);
            std::swap(P->edges, P->edges2);
            h = P->tstart(MVTV_K_REDUCE);
            HIP_TRY(launch_finalize(P->stream, P->partials, np, ER_N + GR_N, -(1 << ER_DTH), 0, P->red, P->st));
            P->tstop(h);
            mode = U_FROM_Z;
            t_z = t_new;
        } else if (fused4) {   // 4-D: edge update + gather pass A in one pass (z ping-pong), then pass B
            h = P->tstart(MVTV_K_ADMM_FUSED4);
            HIP_TRY(launch_admm4a(P->g, P->order, mode, P->stream, P->theta, P->edges, P->edges2, t_z, c_prev, t_new,
                                  track_theta ? P->thold : nullptr, P->g4, P->partials, &np, nullptr, twin));
            P->tstop(h);
            std::swap(P->edges, P->edges2);
            h = P->tstart(MVTV_K_REDUCE);
            HIP_TRY(launch_finalize(P->stream, P->partials, np, ER_N, 1, 0, P->red, P->st));
            P->tstop(h);
            mode = U_FROM_Z;
            t_z = t_new;
            h = P->tstart(MVTV_K_GATHER4B);
            HIP_TRY(launch_gather4b(P->g, U_FROM_Z, P->stream, P->ga, gnew, gprev, c_prev, P->partials, &np, nullptr,
                                    P->g4));
            P->tstop(h);
            h = P->tstart(MVTV_K_REDUCE);
            HIP_TRY(launch_finalize(P->stream, P->partials, np, GR_N, 0, 0, P->red + ER_N, P->st));
            P->tstop(h);
        } else {
            h = P->tstart(MVTV_K_EDGE_UPDATE);
            np = L.grid;
            if (P->e3d)
                HIP_TRY(launch_edge3d(P->g, P->order, mode, P->stream, P->theta, P->edges, t_z, c_prev, t_new,
                                      track_theta ? P->thold : nullptr, P->partials, &np));
            else
                HIP_TRY(launch_edge_update(P->g, P->order, mode, L, P->theta, P->edges, t_z, c_prev, t_new,
                                           track_theta ? P->thold : nullptr, P->partials));
            P->tstop(h);
            h = P->tstart(MVTV_K_REDUCE);
            HIP_TRY(launch_finalize(P->stream, P->partials, np, ER_N, 1, 0, P->red, P->st));
            P->tstop(h);
            mode = U_FROM_Z;
            t_z = t_new;
            // ---- D^T alpha, D^T u and the dual residual norms ---------------------------------------
            h = P->tstart(MVTV_K_GATHER);
            const int hb = P->tstart_b(MVTV_K_GATHER4B);
            np = L.grid;
            if (P->e3d)
                HIP_TRY(launch_gather3d(P->g, P->order, U_FROM_Z, P->stream, P->edges, t_z, P->ga, gnew, gprev, c_prev,
                                        P->partials, &np, nullptr, P->g4));
            else
                HIP_TRY(launch_gather(P->g, P->order, U_FROM_Z, L, P->edges, t_z, P->ga, gnew, gprev, c_prev, P->partials));
            P->tstop(h);
            P->tstop_b(hb);
            h = P->tstart(MVTV_K_REDUCE);
            HIP_TRY(launch_finalize(P->stream, P->partials, np, GR_N, 0, 0, P->red + ER_N, P->st));
            P->tstop(h);
        }
        HIP_TRY(hipMemcpyAsync(P->host_red, P->red, (ER_N + GR_N) * sizeof(double), hipMemcpyDeviceToHost, P->stream));
        HIP_TRY(hipStreamSynchronize(P->stream));   // timing events are harvested after the loop
        const double* R = P->host_red;
        const double r_norm = std::sqrt(R[ER_R2]);
        it += 1;
        counter += 1;
        double c_next = 1.0, rho_next = rho;
        if (variant == MVTV_VARIANT_RCPP) {
            // :117-125
            dual_norm = std::fabs(rho) * std::sqrt(R[ER_N + GR_S2B]);
            primal_norm = r_norm;
            eps_dual = tol * (std::sqrt(N) + std::sqrt(R[ER_N + GR_GU2]));
            eps_primal = tol * (std::sqrt(E) + std::max(std::sqrt(R[ER_D2]), std::sqrt(R[ER_A2])));
            const double tau = 2.0;
            if (primal_norm > 10 * dual_norm) {
                rho_next = tau * rho;
                c_next = 1.0 / tau;
            } else if (dual_norm > 10 * primal_norm) {
                rho_next = 1.0 / tau * rho;
                c_next = tau;
            }
            S.s_norm = dual_norm;
            S.eps_pri = eps_primal;
            S.eps_dual = eps_dual;
        } else if (variant == MVTV_VARIANT_CPP) {
            // :118-126 — s uses the new alpha and the old u; rho is an int
            const double s_norm = std::fabs(rho) * std::sqrt(R[ER_N + GR_S2A]);
            dtheta = R[ER_DTH];
            S.s_norm = s_norm;
            if (o.fixed_iters <= 0 && counter > max_counter) {
                status = MVTV_MAXITER;
                fail(status, "Failed to converge!");
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
            dtheta = R[ER_DTH];
        }
        S.r_norm = r_norm;
        S.dtheta_max = dtheta;
        std::swap(gprev, gnew);
        c_prev = c_next;
        rho = rho_next;
        if (variant == MVTV_VARIANT_RCPP) sigma = rho;   // spcrosses = crossO + rho crossD (:126)
        if (status == MVTV_MAXITER) break;
        if (variant == MVTV_VARIANT_RCPP && o.fixed_iters <= 0 && counter > max_counter) {
            if (o.verbose) std::printf("ADMM reached max_counter at lambda = %g\n", lambda);
            status = MVTV_MAXITER;
            break;
        }
    }
    P->harvest();   // the stream is idle here (last iteration synchronised)
    twin_guard.armed = false;
    if (twin) {
        HIP_TRY(fill_twins(P->g, P->order, P->stream, P->edges));
        HIP_TRY(hipStreamSynchronize(P->stream));
    }
    if (o.verbose) std::printf("Lambda= %g, Counter = %d\n", lambda, counter);
    // keep the resident state consistent: g_uprev buffer is P->guprev
    if (gprev != P->guprev) std::swap(P->guprev, P->gu);
    P->edge_mode = mode;
    P->t_z = t_z;
    P->c_state = c_prev;
    P->rho = rho;
    S.iters = it;
    S.theta_solver = spectral ? MVTV_SOLVER_SPECTRAL : (pcg_spec ? MVTV_SOLVER_PCG_SPECTRAL : MVTV_SOLVER_PCG);
    S.rho = rho;
    S.status = status;
    S.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (stats) *stats = S;
    return status;
}

mvtv_status mvtv_admm(mvtv_problem* P, const mvtv_admm_opts* opts, double lambda, double* theta_inout,
                      double* u_inout, double* rho_inout, mvtv_admm_stats* stats) {
    if (!P || !opts || !theta_inout) return fail(MVTV_BAD_ARG, "null problem/opts/theta");
    const double rho0 = rho_inout ? *rho_inout : lambda / 5.0;
    MVTV_TRY(mvtv_state_set(P, theta_inout, u_inout, rho0));
    mvtv_status s = mvtv_admm_run(P, opts, lambda, stats);
    if (s != MVTV_OK && s != MVTV_MAXITER) return s;
    mvtv_status g = mvtv_state_get(P, theta_inout, u_inout, rho_inout);
    if (g != MVTV_OK) return g;
    return s;
}

mvtv_status mvtv_path(mvtv_problem* P, const mvtv_admm_opts* opts, const double* lambdas, int32_t n_lambda,
                      const double* theta_init, double rho_init, double* thetas_out, double* rhos_out,
                      mvtv_admm_stats* stats) {
    if (!P || !opts || !theta_init || n_lambda < 0 || (n_lambda > 0 && !lambdas))
        return fail(MVTV_BAD_ARG, "null argument");
    MVTV_TRY(mvtv_state_set(P, theta_init, nullptr, rho_init));
    mvtv_status worst = MVTV_OK;
    for (int32_t i = 0; i < n_lambda; ++i) {
        mvtv_admm_stats st{};
        const mvtv_status s = mvtv_admm_run(P, opts, lambdas[i], &st);
        if (s == MVTV_MAXITER) worst = MVTV_MAXITER;
        else if (s != MVTV_OK) return s;
        if (stats) stats[i] = st;
        if (thetas_out) MVTV_TRY(mvtv_state_get(P, thetas_out + size_t(i) * P->g.N, nullptr, nullptr));
        if (rhos_out) rhos_out[i] = P->rho;
    }
    return worst;
}

mvtv_status mvtv_fitted(mvtv_problem* P, const int64_t* mesh_index, int64_t n, double* fitted) {
    if (!P || (n > 0 && (!mesh_index || !fitted))) return fail(MVTV_BAD_ARG, "null argument");
    if (n == 0) return MVTV_OK;
    DeviceGuard dg(P->device);
    int64_t* didx = nullptr;
    double* dout = nullptr;
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(&didx), size_t(n) * sizeof(int64_t)));
    if (hipMalloc(reinterpret_cast<void**>(&dout), size_t(n) * sizeof(double)) != hipSuccess) {
        (void)hipFree(didx);
        return fail(MVTV_OUT_OF_MEMORY, "hipMalloc");
    }
    mvtv_status s = MVTV_OK;
    for (int64_t t = 0; t < n; ++t)
        if (mesh_index[t] < 0 || mesh_index[t] >= int64_t(P->g.N)) s = fail(MVTV_BAD_ARG, "mesh index out of range");
    if (s == MVTV_OK) {
        if (hipMemcpyAsync(didx, mesh_index, size_t(n) * sizeof(int64_t), hipMemcpyHostToDevice, P->stream) != hipSuccess ||
            launch_gather_index(P->stream, P->theta, didx, n, dout) != hipSuccess ||
            hipMemcpyAsync(fitted, dout, size_t(n) * sizeof(double), hipMemcpyDeviceToHost, P->stream) != hipSuccess ||
            hipStreamSynchronize(P->stream) != hipSuccess)
            s = fail(MVTV_HIP_ERROR, "fitted: HIP failure");
    }
    (void)hipFree(didx);
    (void)hipFree(dout);
    return s;
}

}  // extern "C"

namespace {
// device scratch freed on scope exit (setup paths, not the iteration loop)
struct TmpDev {
    void* p = nullptr;
    ~TmpDev() {
        if (p) (void)hipFree(p);
    }
    template <class T>
    T* get() const { return static_cast<T*>(p); }
};

// axes checked on the host (finite, ascending per dim), then axes and data copied over and the
// nearest node of every point computed into key (and idx when requested)
mvtv_status nearest_on_device(mvtv_problem* P, const double* axes, const double* data, int64_t n, TmpDev& key,
                              TmpDev& idx, bool want_idx) {
    if (P->slab) return fail(MVTV_BAD_ARG, "scattered data on a slab problem: set it up on the whole mesh");
    const int p = P->g.p;
    size_t na = 0;
    double span[MVTV_MAX_DIMS] = {0, 0, 0, 0};
    for (int j = 0; j < p; ++j) {
        const double* a = axes + na;
        span[j] = a[P->g.m[j] - 1] - a[0];
        for (uint32_t k = 0; k < P->g.m[j]; ++k)
            if (!std::isfinite(a[k]) || (k > 0 && !(a[k] > a[k - 1])))
                return fail(MVTV_BAD_ARG, "axes must be finite and strictly ascending per dimension");
        na += P->g.m[j];
    }
    for (int64_t i = 0; i < n * p; ++i)
        if (std::isnan(data[i])) return fail(MVTV_BAD_ARG, "NaN in data");
    TmpDev daxes, ddata;
    HIP_TRY(hipMalloc(&daxes.p, na * sizeof(double)));
    HIP_TRY(hipMalloc(&ddata.p, size_t(std::max<int64_t>(n * p, 1)) * sizeof(double)));
    HIP_TRY(hipMalloc(&key.p, size_t(std::max<int64_t>(n, 1)) * sizeof(uint32_t)));
    if (want_idx) HIP_TRY(hipMalloc(&idx.p, size_t(std::max<int64_t>(n, 1)) * sizeof(int64_t)));
    HIP_TRY(hipMemcpyAsync(daxes.p, axes, na * sizeof(double), hipMemcpyHostToDevice, P->stream));
    if (n > 0)
        HIP_TRY(hipMemcpyAsync(ddata.p, data, size_t(n * p) * sizeof(double), hipMemcpyHostToDevice, P->stream));
    uint32_t m[MVTV_MAX_DIMS];
    for (int j = 0; j < p; ++j) m[j] = P->g.m[j];
    HIP_TRY(launch_nearest(P->stream, p, m, daxes.get<double>(), span, ddata.get<double>(), n, key.get<uint32_t>(),
                           want_idx ? idx.get<int64_t>() : nullptr));
    HIP_TRY(hipStreamSynchronize(P->stream));   // the temporaries above go out of scope
    return MVTV_OK;
}
}  // namespace

extern "C" {

mvtv_status mvtv_nearest(mvtv_problem* P, const double* axes, const double* data, int64_t n, int64_t* mesh_index_out) {
    if (!P || !axes || n < 0 || (n > 0 && (!data || !mesh_index_out))) return fail(MVTV_BAD_ARG, "null argument");
    DeviceGuard dg(P->device);
    TmpDev key, idx;
    MVTV_TRY(nearest_on_device(P, axes, data, n, key, idx, true));
    if (n > 0) {
        HIP_TRY(hipMemcpyAsync(mesh_index_out, idx.p, size_t(n) * sizeof(int64_t), hipMemcpyDeviceToHost, P->stream));
        HIP_TRY(hipStreamSynchronize(P->stream));
    }
    return MVTV_OK;
}

mvtv_status mvtv_problem_set_scattered(mvtv_problem* P, const double* axes, const double* data, int64_t n,
                                       const double* y, int64_t* mesh_index_out) {
    if (!P || !axes || n < 0 || (n > 0 && (!data || !y))) return fail(MVTV_BAD_ARG, "null argument");
    DeviceGuard dg(P->device);
    TmpDev key, idx, dy, runs;
    MVTV_TRY(nearest_on_device(P, axes, data, n, key, idx, mesh_index_out != nullptr));
    if (mesh_index_out && n > 0)
        HIP_TRY(hipMemcpyAsync(mesh_index_out, idx.p, size_t(n) * sizeof(int64_t), hipMemcpyDeviceToHost, P->stream));
    HIP_TRY(hipMalloc(&dy.p, size_t(std::max<int64_t>(n, 1)) * sizeof(double)));
    HIP_TRY(hipMalloc(&runs.p, sizeof(unsigned long long)));
    if (n > 0) HIP_TRY(hipMemcpyAsync(dy.p, y, size_t(n) * sizeof(double), hipMemcpyHostToDevice, P->stream));
    if (!P->wdiag) MVTV_TRY(alloc(&P->wdiag, P->g.N));
    HIP_TRY(launch_scatter_sums(P->stream, key.get<uint32_t>(), dy.get<double>(), n, P->g.N, P->oty, P->wdiag,
                                runs.get<unsigned long long>()));
    unsigned long long hit = 0;
    HIP_TRY(hipMemcpy(&hit, runs.p, sizeof(hit), hipMemcpyDeviceToHost));
    // every node exactly one point <=> n == N and N nodes hit: W = I (the spectral solve applies)
    if (uint64_t(n) == uint64_t(P->g.N) && hit == uint64_t(P->g.N)) {
        P->wmode = W_IDENTITY;
        P->wmean = 1.0;
        P->wstd = 0.0;
    } else {
        P->wmode = W_DIAG;
        P->wmean = double(n) / double(P->g.N);
        std::vector<double> w(P->g.N);   // std(W) for the preconditioner choice (setup path)
        HIP_TRY(hipMemcpy(w.data(), P->wdiag, size_t(P->g.N) * sizeof(double), hipMemcpyDeviceToHost));
        double acc2 = 0.0;
        for (double v : w) acc2 += (v - P->wmean) * (v - P->wmean);
        P->wstd = std::sqrt(acc2 / double(P->g.N));
    }
    return MVTV_OK;
}

mvtv_status mvtv_predict(mvtv_problem* P, const double* axes, const double* data, int64_t n, double* fits) {
    if (!P || !axes || n < 0 || (n > 0 && (!data || !fits))) return fail(MVTV_BAD_ARG, "null argument");
    if (n == 0) return MVTV_OK;
    DeviceGuard dg(P->device);
    TmpDev key, idx, out;
    MVTV_TRY(nearest_on_device(P, axes, data, n, key, idx, true));
    HIP_TRY(hipMalloc(&out.p, size_t(n) * sizeof(double)));
    HIP_TRY(launch_gather_index(P->stream, P->theta, idx.get<int64_t>(), n, out.get<double>()));
    HIP_TRY(hipMemcpyAsync(fits, out.p, size_t(n) * sizeof(double), hipMemcpyDeviceToHost, P->stream));
    HIP_TRY(hipStreamSynchronize(P->stream));
    return MVTV_OK;
}

// ------------------------------------------------------------------------------ operators
mvtv_status mvtv_apply_D(mvtv_problem* P, const double* theta, double* d_out) {
    if (!P || !theta || !d_out) return fail(MVTV_BAD_ARG, "null argument");
    DeviceGuard dg(P->device);
    double *x = nullptr, *e = nullptr;
    MVTV_TRY(alloc(&x, P->g.N));
    mvtv_status s = alloc(&e, size_t(P->g.nb) * P->g.N);
    if (s == MVTV_OK) {
        if (hipMemcpyAsync(x, theta, size_t(P->g.N) * sizeof(double), hipMemcpyHostToDevice, P->stream) != hipSuccess ||
            launch_apply_D_padded(P->g, P->order, P->L(), x, e) != hipSuccess)
            s = fail(MVTV_HIP_ERROR, "apply_D");
        if (s == MVTV_OK) s = export_edges(P, e, d_out, U_EXPLICIT, 0.0, 1.0);
    }
    (void)hipFree(x);
    if (e) (void)hipFree(e);
    return s;
}

mvtv_status mvtv_apply_Dt(mvtv_problem* P, const double* v, double* g_out) {
    if (!P || !v || !g_out) return fail(MVTV_BAD_ARG, "null argument");
    DeviceGuard dg(P->device);
    double *gq = nullptr, *e = nullptr;
    MVTV_TRY(alloc(&gq, P->g.N));
    mvtv_status s = alloc(&e, size_t(P->g.nb) * P->g.N);
    if (s == MVTV_OK) s = import_edges(P, v, e);
    if (s == MVTV_OK) {
        if (launch_gather(P->g, P->order, U_EXPLICIT, P->L(), e, 0.0, nullptr, gq, nullptr, 1.0, P->partials) != hipSuccess ||
            hipMemcpyAsync(g_out, gq, size_t(P->g.N) * sizeof(double), hipMemcpyDeviceToHost, P->stream) != hipSuccess ||
            hipStreamSynchronize(P->stream) != hipSuccess)
            s = fail(MVTV_HIP_ERROR, "apply_Dt");
    }
    (void)hipFree(gq);
    if (e) (void)hipFree(e);
    return s;
}

mvtv_status mvtv_apply_A(mvtv_problem* P, double sigma, const double* x, double* q_out) {
    if (!P || !x || !q_out) return fail(MVTV_BAD_ARG, "null argument");
    DeviceGuard dg(P->device);
    double *dx = nullptr, *dq = nullptr;
    MVTV_TRY(alloc(&dx, P->g.N));
    mvtv_status s = alloc(&dq, P->g.N);
    if (s == MVTV_OK) {
        const size_t bytes = size_t(P->g.N) * sizeof(double);
        if (hipMemcpyAsync(dx, x, bytes, hipMemcpyHostToDevice, P->stream) != hipSuccess ||
            launch_apply_A(P->g, P->L(), sigma, P->wmode, P->wdiag, dx, dq, nullptr, nullptr) != hipSuccess ||
            hipMemcpyAsync(q_out, dq, bytes, hipMemcpyDeviceToHost, P->stream) != hipSuccess ||
            hipStreamSynchronize(P->stream) != hipSuccess)
            s = fail(MVTV_HIP_ERROR, "apply_A");
    }
    (void)hipFree(dx);
    if (dq) (void)hipFree(dq);
    return s;
}

mvtv_status mvtv_solve(mvtv_problem* P, double sigma, const double* b, double* x_inout, double rtol, int32_t max_iter,
                       int32_t* iters, double* relres) {
    if (!P || !b || !x_inout) return fail(MVTV_BAD_ARG, "null argument");
    DeviceGuard dg(P->device);
    double *db = nullptr, *dx = nullptr;
    MVTV_TRY(alloc(&db, P->g.N));
    mvtv_status s = alloc(&dx, P->g.N);
    int it = 0;
    double rr = 0.0;
    if (s == MVTV_OK) {
        const size_t bytes = size_t(P->g.N) * sizeof(double);
        if (hipMemcpyAsync(db, b, bytes, hipMemcpyHostToDevice, P->stream) != hipSuccess ||
            hipMemcpyAsync(dx, x_inout, bytes, hipMemcpyHostToDevice, P->stream) != hipSuccess)
            s = fail(MVTV_HIP_ERROR, "solve upload");
        if (s == MVTV_OK)
            s = pcg_solve(P, sigma, db, db, 0.0, db, 0.0, dx, rtol > 0 ? rtol : 1e-10, max_iter > 0 ? max_iter : 20000,
                          &it, &rr);
        if (s == MVTV_OK && (hipMemcpyAsync(x_inout, dx, bytes, hipMemcpyDeviceToHost, P->stream) != hipSuccess ||
                             hipStreamSynchronize(P->stream) != hipSuccess))
            s = fail(MVTV_HIP_ERROR, "solve download");
    }
    if (iters) *iters = it;
    if (relres) *relres = rr;
    (void)hipFree(db);
    if (dx) (void)hipFree(dx);
    return s;
}

mvtv_status mvtv_lambda_max(mvtv_problem* P, double* out, int32_t* iters) {
    if (!P || !out) return fail(MVTV_BAD_ARG, "null argument");
    DeviceGuard dg(P->device);
    const Launch L = P->L();
    const size_t bytes = size_t(P->g.N) * sizeof(double);
    // scratch: x, d, r, p, t (the PCG buffers; the ADMM state theta / edges is untouched)
    if (!P->p2) MVTV_TRY(alloc(&P->p2, P->g.N));
    if (!P->thold) MVTV_TRY(alloc(&P->thold, P->g.N));
    double *x = P->thold, *d = P->r, *r = P->q, *p = P->p, *t = P->p2;
    auto dot = [&](double* v, double* res) -> mvtv_status {
        HIP_TRY(launch_cg_vec(P->g, L, 0, 0.0, v, nullptr, nullptr, nullptr, P->partials));
        HIP_TRY(launch_finalize(P->stream, P->partials, L.grid, 1, 0, 0, P->red, P->st));
        HIP_TRY(hipMemcpyAsync(P->host_red, P->red, sizeof(double), hipMemcpyDeviceToHost, P->stream));
        HIP_TRY(hipStreamSynchronize(P->stream));
        *res = P->host_red[0];
        return MVTV_OK;
    };
    auto AtA = [&](const double* v, double* outv) -> mvtv_status {   // crossD * v (W = 0, sigma = 1)
        HIP_TRY(launch_apply_A(P->g, L, 1.0, W_NONE, nullptr, v, outv, nullptr, nullptr));
        return MVTV_OK;
    };
    // cg(ata, Oty) of rcpp…/utils.cpp:306-341, line by line
    HIP_TRY(hipMemsetAsync(x, 0, bytes, P->stream));
    HIP_TRY(hipMemcpyAsync(d, P->oty, bytes, hipMemcpyDeviceToDevice, P->stream));   // d = b - A x, x = 0
    MVTV_TRY(AtA(d, r));                                                             // r = A^T d
    HIP_TRY(hipMemcpyAsync(p, r, bytes, hipMemcpyDeviceToDevice, P->stream));
    double rr = 0.0;
    MVTV_TRY(dot(r, &rr));
    const double rsold0 = std::sqrt(rr);
    double rsold = std::pow(rsold0, 2), rsnew = rsold + 1.0;
    MVTV_TRY(AtA(p, t));
    int iter = 0;
    const int MAXIT = P->g.N < 2000 ? int(P->g.N) : 2000;
    while (std::sqrt(rsnew) >= 0.0001 * rsold0) {
        double tt = 0.0;
        MVTV_TRY(dot(t, &tt));
        const double alpha = rsold / std::pow(std::sqrt(tt), 2);
        HIP_TRY(launch_cg_vec(P->g, L, 1, alpha, x, d, p, t, nullptr));
        MVTV_TRY(AtA(d, r));
        MVTV_TRY(dot(r, &rr));
        rsnew = std::pow(std::sqrt(rr), 2);
        iter += 1;
        if (iter == MAXIT) break;
        HIP_TRY(launch_cg_vec(P->g, L, 2, rsnew / rsold, p, nullptr, r, nullptr, nullptr));   // p = r + beta p
        MVTV_TRY(AtA(p, t));
        rsold = rsnew;
    }
    // 5 * ||D x||_inf (lam_max_pinv, :351-355)
    HIP_TRY(launch_dmaxabs(P->g, P->order, L, x, P->partials));
    HIP_TRY(launch_finalize(P->stream, P->partials, L.grid, 1, 1, 0, P->red, P->st));
    HIP_TRY(hipMemcpyAsync(P->host_red, P->red, sizeof(double), hipMemcpyDeviceToHost, P->stream));
    HIP_TRY(hipStreamSynchronize(P->stream));
    *out = 5.0 * P->host_red[0];
    if (iters) *iters = iter;
    return MVTV_OK;
}

mvtv_status mvtv_lambda_max_cpp(mvtv_problem* P, double* out, int32_t* iters) {
    if (!P || !out) return fail(MVTV_BAD_ARG, "null argument");
    DeviceGuard dg(P->device);
    const Launch L = P->L();
    const size_t n = P->g.N, bytes = n * sizeof(double);
    if (!P->p2) MVTV_TRY(alloc(&P->p2, n));
    if (!P->thold) MVTV_TRY(alloc(&P->thold, n));
    double *x = P->thold, *r = P->r, *p = P->p, *ap = P->p2;
    auto reduce1 = [&](double* res) -> mvtv_status {   // the one partial sum in P->partials
        HIP_TRY(launch_finalize(P->stream, P->partials, L.grid, 1, 0, 0, P->red, P->st));
        HIP_TRY(hipMemcpyAsync(P->host_red, P->red, sizeof(double), hipMemcpyDeviceToHost, P->stream));
        HIP_TRY(hipStreamSynchronize(P->stream));
        *res = P->host_red[0];
        return MVTV_OK;
    };
    // cg(ata, Oty) of cpp-code/utils.cpp:354-386: x = mean(b), r = b - A x, p = r, absolute stop
    // ||r|| < 0.01, at most 500 iterations when N < 400 and 100 otherwise
    std::vector<double> hb(n);
    HIP_TRY(hipMemcpyAsync(hb.data(), P->oty, bytes, hipMemcpyDeviceToHost, P->stream));
    HIP_TRY(hipStreamSynchronize(P->stream));
    double sum = 0.0;
    for (double v : hb) sum += v;
    HIP_TRY(launch_fill(P->stream, x, sum / double(n), n));
    HIP_TRY(launch_apply_A(P->g, L, 1.0, W_NONE, nullptr, x, ap, nullptr, nullptr));   // A x
    HIP_TRY(hipMemcpyAsync(r, P->oty, bytes, hipMemcpyDeviceToDevice, P->stream));
    HIP_TRY(launch_cg_vec(P->g, L, 3, 1.0, nullptr, r, nullptr, ap, nullptr));          // r = b - A x
    HIP_TRY(hipMemcpyAsync(p, r, bytes, hipMemcpyDeviceToDevice, P->stream));
    double rsold = 0.0;
    HIP_TRY(launch_cg_vec(P->g, L, 0, 0.0, r, nullptr, nullptr, nullptr, P->partials));
    MVTV_TRY(reduce1(&rsold));
    double rsnew = rsold + 1.0;
    const int MAXIT = n < 400 ? 500 : 100;
    int iter = 0;
    while (std::sqrt(rsnew) >= 0.01) {
        double pap = 0.0;   // Ap = A p, p.Ap
        HIP_TRY(launch_apply_A(P->g, L, 1.0, W_NONE, nullptr, p, ap, P->partials, nullptr));
        MVTV_TRY(reduce1(&pap));
        const double alpha = rsold / pap;
        HIP_TRY(launch_cg_vec(P->g, L, 1, alpha, x, r, p, ap, nullptr));                // x += a p, r -= a Ap
        HIP_TRY(launch_cg_vec(P->g, L, 0, 0.0, r, nullptr, nullptr, nullptr, P->partials));
        MVTV_TRY(reduce1(&rsnew));
        iter += 1;
        if (iter == MAXIT) break;
        HIP_TRY(launch_cg_vec(P->g, L, 2, rsnew / rsold, p, nullptr, r, nullptr, nullptr));   // p = r + beta p
        rsold = rsnew;
    }
    // lam_max_pinv (:399-404): max |D x|, no factor
    HIP_TRY(launch_dmaxabs(P->g, P->order, L, x, P->partials));
    HIP_TRY(launch_finalize(P->stream, P->partials, L.grid, 1, 1, 0, P->red, P->st));
    HIP_TRY(hipMemcpyAsync(P->host_red, P->red, sizeof(double), hipMemcpyDeviceToHost, P->stream));
    HIP_TRY(hipStreamSynchronize(P->stream));
    *out = P->host_red[0];
    if (iters) *iters = iter;
    return MVTV_OK;
}

mvtv_status mvtv_solve_spectral(mvtv_problem* P, double sigma, const double* b, double* x_out) {
    if (!P || !b || !x_out) return fail(MVTV_BAD_ARG, "null argument");
    if (!spectral_ok(P)) return fail(MVTV_BAD_ARG, "spectral theta-solve needs W = I and every m_j <= 4096");
    DeviceGuard dg(P->device);
    double* dx = nullptr;
    MVTV_TRY(alloc(&dx, P->g.N));
    const size_t bytes = size_t(P->g.N) * sizeof(double);
    mvtv_status s = MVTV_OK;
    if (hipMemcpyAsync(dx, b, bytes, hipMemcpyHostToDevice, P->stream) != hipSuccess)
        s = fail(MVTV_HIP_ERROR, "solve upload");
    if (s == MVTV_OK) s = spectral_solve(P, sigma, dx, nullptr, 0.0, nullptr, 0.0, dx);
    if (s == MVTV_OK && (hipMemcpyAsync(x_out, dx, bytes, hipMemcpyDeviceToHost, P->stream) != hipSuccess ||
                         hipStreamSynchronize(P->stream) != hipSuccess))
        s = fail(MVTV_HIP_ERROR, "solve download");
    (void)hipFree(dx);
    return s;
}

mvtv_status mvtv_sync(mvtv_problem* P) {
    if (!P) return fail(MVTV_BAD_ARG, "null problem");
    DeviceGuard dg(P->device);
    return P->sync();
}

// ------------------------------------------------------------------------------ instrumentation
mvtv_status mvtv_timing_enable(mvtv_problem* P, int32_t on) {
    if (!P) return fail(MVTV_BAD_ARG, "null problem");
    DeviceGuard dg(P->device);
    MVTV_TRY(P->sync());
    P->timing = on != 0;
    for (int k = 0; k < MVTV_K_COUNT; ++k) {
        P->ms[k] = 0.0;
        P->launches[k] = 0;
    }
    P->fold_fix = 0;
    P->pcg_xmoves = 0;
    return MVTV_OK;
}

mvtv_status mvtv_timing_get(mvtv_problem* P, int32_t kid, double* total_ms, int64_t* launches, double* bytes) {
    if (!P || kid < 0 || kid >= MVTV_K_COUNT) return fail(MVTV_BAD_ARG, "kernel id");
    DeviceGuard dg(P->device);
    MVTV_TRY(P->sync());
    double N = double(P->g.N), E = double(P->E);
    const double w = P->wmode == W_DIAG ? 1.0 : 0.0;
    double own = 1.0;
    if (P->slab) {   // a slab rank's kernels work on its owned planes (ghost planes are read only as halos)
        own = double(P->ze - P->zb) / double(P->g.m[P->g.p - 1]);
        N *= own;
        E *= own;
    }
    // algorithmic bytes per launch (each array element read or written once)
    double b = 0.0;
    switch (kid) {
        case MVTV_K_EDGE_UPDATE: b = 8.0 * (N + 2.0 * E); break;        // theta in, z in/out
        case MVTV_K_GATHER:   // z in, g_uprev in, g_alpha/g_u out; 4-D two-pass: z in, 4 partial sums out
            b = P->g4 ? 8.0 * (E + 4.0 * N) : 8.0 * (E + 3.0 * N);
            break;
        case MVTV_K_GATHER4B: b = 8.0 * 7.0 * N; break;                // 4 partial sums, g_uprev in; g_alpha/g_u out
        case MVTV_K_PCG_INIT:   // classic: oty, ga, gb, x (+W) in, r, p out; fused 3-D: r out only
            b = 8.0 * (((P->g.p == 3 && P->fused3d) ? 5.0 : 6.0) + w) * N;
            break;
        case MVTV_K_PCG_APPLY: b = 8.0 * ((2.0 + w) * N); break;        // p (+W) in, q out
        case MVTV_K_PCG_UPDATE: b = 8.0 * ((6.0 + w) * N); break;       // x, r, p, q (+W) in, x, r out
        case MVTV_K_PCG_DIRECTION: b = 8.0 * ((3.0 + w) * N); break;    // r, p (+W) in, p out
        case MVTV_K_PCG_FUSED:   // r, p (+W) in, r, p out; + x in/out in the odd iterations (mean over the launches)
            b = 8.0 * N * (4.0 + w + (P->launches[kid] > 0 ? 2.0 * double(P->pcg_xmoves) / double(P->launches[kid]) : 0.0));
            break;
        case MVTV_K_DCT_FIRST: b = 8.0 * 4.0 * N; break;                 // oty, g_alpha, g_u in, x out
        case MVTV_K_DCT_FOLD:   // oty, s in, x out; + g_u in the launches after a rho change (mean over the launches)
            b = 8.0 * N * (3.0 + (P->launches[kid] > 0 ? double(P->fold_fix) / double(P->launches[kid]) : 0.0));
            break;
        case MVTV_K_DCT: b = 8.0 * 2.0 * N; break;                       // x in, x out
        case MVTV_K_ADMM_FUSED:   // theta, z, g_uprev in; z', g_alpha, g_u out (z without its twin blocks: twin_timed)
            b = 8.0 * (4.0 * N + 2.0 * (P->twin_timed ? E - twin_edges(P) * own : E));
            break;
        case MVTV_K_ADMM_FUSED4:   // theta, z in; z', 4 pass-A sums out (z without its twin blocks: twin_timed)
            b = 8.0 * (5.0 * N + 2.0 * (P->twin_timed ? E - twin_edges(P) * own : E));
            break;
        default: b = 0.0;
    }
    if (total_ms) *total_ms = P->ms[kid];
    if (launches) *launches = P->launches[kid];
    if (bytes) *bytes = b;
    return MVTV_OK;
}

const char* mvtv_kernel_name(int32_t kid) {
    static const char* names[MVTV_K_COUNT] = {"edge_update", "gather_Dt", "pcg_init", "pcg_apply_A",
                                               "pcg_update", "pcg_direction", "reduce", "other", "pcg_fused3d",
                                               "dct_first", "dct", "admm_fused", "gather4_b", "dct_first_fold",
                                               "admm_fused4"};
    return (kid >= 0 && kid < MVTV_K_COUNT) ? names[kid] : "?";
}

}  // extern "C"

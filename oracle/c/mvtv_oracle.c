/*
 * CPU ORACLE — TEST INFRASTRUCTURE ONLY (tests/, bench.py cpu_baseline).
 *
 * Plain-C restatement of the reference's variant-B ADMM loop
 * (rcpp-code/MultivarTV/src/solvers.cpp:96-136, adapt_step :77-94) on the
 * reference's own compact edge layout (blocks concatenated in C++ create_D
 * order, cpp-code/utils.cpp:245-269; each block a column-major reduced grid,
 * :103-134). D and D^T are applied matrix-free over the reduced grids; the
 * SuperLU theta-solve (:113) is replaced by Jacobi-PCG on the 3^p-point
 * operator W + sigma D^T D. OpenMP parallel loops, deterministic per thread
 * count. Pinned against oracle/mvtv_oracle.py (SuperLU) in
 * tests/test_oracle_c.py.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

#define MAXB 15

typedef struct {
    int p, nb;
    int64_t m[4], stride[4], N, E;
    int sp[MAXB];          /* effective difference set S' per block (bit j = dim j) */
    double w[MAXB];
    int64_t off[MAXB];     /* compact offset of each block */
    int64_t rd[MAXB][4];   /* reduced dims */
    double cS[16];
    double K[81];          /* 3^p stencil weights of D^T D with clamped neighbours */
} geom_t;

static int sprime(int b, int p) {
    int S = 0, cnt = 0;
    for (int j = 0; j < p; ++j)
        if ((b >> (p - 1 - j)) & 1) { S |= 1 << j; ++cnt; }
    if (cnt <= 1 || (S & 1)) return S;
    int lo = 0;
    while (!((S >> lo) & 1)) ++lo;
    return (S & ~(1 << lo)) | 1;
}

static int geom_init(geom_t* g, int p, const int64_t* m, int order, int weighted, const double* deltas) {
    memset(g, 0, sizeof(*g));
    g->p = p;
    g->N = 1;
    for (int j = 0; j < 4; ++j) {
        g->m[j] = j < p ? m[j] : 1;
        g->stride[j] = g->N;
        g->N *= g->m[j];
    }
    const int full = (1 << p) - 1;
    g->nb = order == 0 ? full : (weighted ? full - 1 : full);
    if (g->nb <= 0) return -1;
    for (int k = 0; k < g->nb; ++k) {
        const int b = order == 0 ? (k == 0 ? full : k) : k + 1;
        const int S = sprime(b, p);
        double w = 1.0;
        if (weighted)
            for (int j = 0; j < p; ++j)
                if (!((b >> (p - 1 - j)) & 1)) w *= deltas[j];
        g->sp[k] = S;
        g->w[k] = w;
        g->cS[S] += w * w;
        g->off[k] = g->E;
        int64_t len = 1;
        for (int j = 0; j < 4; ++j) {
            g->rd[k][j] = g->m[j] - ((S >> j) & 1);
            len *= g->rd[k][j];
        }
        g->E += len;
    }
    int nt = 1;
    for (int j = 0; j < p; ++j) nt *= 3;
    for (int t = 0; t < nt; ++t) {
        double acc = 0.0;
        for (int S = 1; S < (1 << p); ++S) {
            double prod = g->cS[S];
            int tt = t;
            for (int j = 0; j < p; ++j) {
                const int o = tt % 3;
                tt /= 3;
                const int in = (S >> j) & 1;
                prod *= in ? (o == 1 ? 2.0 : -1.0) : (o == 1 ? 1.0 : 0.0);
            }
            acc += prod;
        }
        g->K[t] = acc;
    }
    return 0;
}

static inline void decode(const geom_t* g, int64_t i, int64_t* c) {
    for (int j = 0; j < 4; ++j) {
        c[j] = i % g->m[j];
        i /= g->m[j];
    }
}

/* d = D theta (compact) */
static void apply_D(const geom_t* g, const double* th, double* d) {
    for (int k = 0; k < g->nb; ++k) {
        const int S = g->sp[k];
        const int64_t* rd = g->rd[k];
        const int64_t len = rd[0] * rd[1] * rd[2] * rd[3];
        double* dk = d + g->off[k];
#pragma omp parallel for schedule(static)
        for (int64_t e = 0; e < len; ++e) {
            int64_t c[4], r = e, base = 0;
            for (int j = 0; j < 4; ++j) {
                c[j] = r % rd[j];
                r /= rd[j];
                base += c[j] * g->stride[j];
            }
            double acc = 0.0;
            for (int T = 0; T < 16; ++T) {
                if (T & ~S) continue;
                int64_t idx = base;
                for (int j = 0; j < 4; ++j)
                    if ((T >> j) & 1) idx += g->stride[j];
                acc += (__builtin_popcount(T) & 1) ? -th[idx] : th[idx];
            }
            dk[e] = g->w[k] * acc;
        }
    }
}

/* out = D^T v (gather form, race-free) */
static void apply_Dt(const geom_t* g, const double* v, double* out) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < g->N; ++i) {
        int64_t c[4];
        decode(g, i, c);
        double acc = 0.0;
        for (int k = 0; k < g->nb; ++k) {
            const int S = g->sp[k];
            const int64_t* rd = g->rd[k];
            const double* vk = v + g->off[k];
            double a = 0.0;
            for (int T = 0; T < 16; ++T) {
                if (T & ~S) continue;
                int ok = 1;
                int64_t rl = 0, rs = 1;
                for (int j = 0; j < 4; ++j) {
                    int64_t cj = c[j] - ((T >> j) & 1);
                    if (cj < 0 || cj >= rd[j]) ok = 0;
                    rl += cj * rs;
                    rs *= rd[j];
                }
                if (!ok) continue;
                a += (__builtin_popcount(T) & 1) ? -vk[rl] : vk[rl];
            }
            acc += g->w[k] * a;
        }
        out[i] = acc;
    }
}

static inline double stencil(const geom_t* g, const double* x, int64_t i, const int64_t* c) {
    /* clamped neighbour offsets per dim (o = 0: -1, 1: 0, 2: +1), then the 3^p terms in t order
       (dim 0 fastest), the same summation order as the generic index walk */
    int64_t off[4][3];
    for (int j = 0; j < 4; ++j) {
        off[j][0] = (j < g->p && c[j] > 0) ? -g->stride[j] : 0;
        off[j][1] = 0;
        off[j][2] = (j < g->p && c[j] + 1 < g->m[j]) ? g->stride[j] : 0;
    }
    double acc = 0.0;
    const double* K = g->K;
    const double* xi = x + i;
    switch (g->p) {
        case 1:
            for (int a = 0; a < 3; ++a) acc += K[a] * xi[off[0][a]];
            break;
        case 2:
            for (int b = 0; b < 3; ++b)
                for (int a = 0; a < 3; ++a) acc += K[a + 3 * b] * xi[off[0][a] + off[1][b]];
            break;
        case 3:
            for (int d = 0; d < 3; ++d)
                for (int b = 0; b < 3; ++b)
                    for (int a = 0; a < 3; ++a) acc += K[a + 3 * b + 9 * d] * xi[off[0][a] + off[1][b] + off[2][d]];
            break;
        default:
            for (int e = 0; e < 3; ++e)
                for (int d = 0; d < 3; ++d)
                    for (int b = 0; b < 3; ++b)
                        for (int a = 0; a < 3; ++a)
                            acc += K[a + 3 * b + 9 * d + 27 * e] * xi[off[0][a] + off[1][b] + off[2][d] + off[3][e]];
    }
    return acc;
}

static inline double jdiag(const geom_t* g, const double* W, double sigma, int64_t i, const int64_t* c) {
    double acc = 0.0;
    for (int S = 1; S < (1 << g->p); ++S) {
        double prod = g->cS[S];
        for (int j = 0; j < g->p; ++j)
            if ((S >> j) & 1) prod *= (double)(c[j] > 0) + (double)(c[j] + 1 < g->m[j]);
        acc += prod;
    }
    return (W ? W[i] : 1.0) + sigma * acc;
}

/* Jacobi-PCG for (W + sigma D^T D) x = b, warm start x. fixed > 0: exactly that many iterations. */
static int pcg(const geom_t* g, const double* W, double sigma, const double* b, double* x, double* r, double* p,
               double* q, double rtol, int maxit, int fixed, double* relres) {
    const int64_t N = g->N;
    double bb = 0.0, rz = 0.0, rr = 0.0;
    double* dinv = (double*)malloc(sizeof(double) * N);   /* 1 / Jacobi diagonal, once per solve */
    if (!dinv) return -1;
#pragma omp parallel for schedule(static) reduction(+ : bb, rz, rr)
    for (int64_t i = 0; i < N; ++i) {
        int64_t c[4];
        decode(g, i, c);
        dinv[i] = 1.0 / jdiag(g, W, sigma, i, c);
        const double ax = (W ? W[i] : 1.0) * x[i] + sigma * stencil(g, x, i, c);
        const double ri = b[i] - ax;
        const double zi = ri * dinv[i];
        r[i] = ri;
        p[i] = zi;
        bb += b[i] * b[i];
        rz += ri * zi;
        rr += ri * ri;
    }
    int it = 0;
    const int lim = fixed > 0 ? fixed : maxit;
    while (it < lim && (fixed > 0 || rr > rtol * rtol * bb)) {
        double pq = 0.0;
#pragma omp parallel for schedule(static) reduction(+ : pq)
        for (int64_t i = 0; i < N; ++i) {
            int64_t c[4];
            decode(g, i, c);
            const double qi = (W ? W[i] : 1.0) * p[i] + sigma * stencil(g, p, i, c);
            q[i] = qi;
            pq += p[i] * qi;
        }
        const double alpha = rz / pq;
        double rz2 = 0.0;
        rr = 0.0;
#pragma omp parallel for schedule(static) reduction(+ : rz2, rr)
        for (int64_t i = 0; i < N; ++i) {
            x[i] += alpha * p[i];
            const double ri = r[i] - alpha * q[i];
            r[i] = ri;
            const double zi = ri * dinv[i];
            rz2 += ri * zi;
            rr += ri * ri;
        }
        const double beta = rz2 / rz;
        rz = rz2;
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < N; ++i) p[i] = r[i] * dinv[i] + beta * p[i];
        ++it;
    }
    free(dinv);
    *relres = bb > 0 ? sqrt(rr / bb) : 0.0;
    return it;
}

int mvtv_oracle_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* OpenMP threads of the following calls (CPU-baseline legs time 1 thread and all threads) */
void mvtv_oracle_set_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}

int64_t mvtv_oracle_edges(int p, const int64_t* m, int order, int weighted) {
    geom_t g;
    double d[4] = {1, 1, 1, 1};
    if (geom_init(&g, p, m, order, weighted, d)) return -1;
    return g.E;
}

/* stats[0] iters, [1] r_norm, [2] s_norm, [3] eps_pri, [4] eps_dual, [5] pcg iters total, [6] max pcg relres */
/* theta-solve callback: x = (I + sigma D^T D)^-1 b (the caller's direct solver, e.g. cosine transforms) */
typedef int (*theta_solve_fn)(double sigma, const double* b, double* x, void* ctx);

static int admm_rcpp_impl(int p, const int64_t* m, int order, int weighted, const double* deltas, const double* oty,
                          const double* W, double lambda, double* theta, double* u, double* rho_io, int fixed_iters,
                          double tol, int max_counter, double pcg_rtol, int pcg_fixed, int pcg_maxit, double* stats,
                          theta_solve_fn solve, void* ctx);

int mvtv_oracle_admm_rcpp(int p, const int64_t* m, int order, int weighted, const double* deltas,
                          const double* oty, const double* W, double lambda, double* theta, double* u, double* rho_io,
                          int fixed_iters, double tol, int max_counter, double pcg_rtol, int pcg_fixed,
                          int pcg_maxit, double* stats) {
    return admm_rcpp_impl(p, m, order, weighted, deltas, oty, W, lambda, theta, u, rho_io, fixed_iters, tol,
                          max_counter, pcg_rtol, pcg_fixed, pcg_maxit, stats, NULL, NULL);
}

/* the same loop with the theta-solve done by `solve` (W must be NULL: the direct solvers are for W = I) */
int mvtv_oracle_admm_rcpp_cb(int p, const int64_t* m, int order, int weighted, const double* deltas,
                             const double* oty, double lambda, double* theta, double* u, double* rho_io,
                             int fixed_iters, double tol, int max_counter, double* stats, theta_solve_fn solve,
                             void* ctx) {
    if (!solve) return -3;
    return admm_rcpp_impl(p, m, order, weighted, deltas, oty, NULL, lambda, theta, u, rho_io, fixed_iters, tol,
                          max_counter, 0.0, 0, 0, stats, solve, ctx);
}

/* d = D theta and out = D^T v on the compact edge layout (operator checks, CPU baselines) */
int mvtv_oracle_apply_D(int p, const int64_t* m, int order, int weighted, const double* deltas, const double* theta,
                        double* d) {
    geom_t g;
    if (geom_init(&g, p, m, order, weighted, deltas)) return -1;
    apply_D(&g, theta, d);
    return 0;
}
int mvtv_oracle_apply_Dt(int p, const int64_t* m, int order, int weighted, const double* deltas, const double* v,
                         double* out) {
    geom_t g;
    if (geom_init(&g, p, m, order, weighted, deltas)) return -1;
    apply_Dt(&g, v, out);
    return 0;
}

static int admm_rcpp_impl(int p, const int64_t* m, int order, int weighted, const double* deltas, const double* oty,
                          const double* W, double lambda, double* theta, double* u, double* rho_io, int fixed_iters,
                          double tol, int max_counter, double pcg_rtol, int pcg_fixed, int pcg_maxit, double* stats,
                          theta_solve_fn solve, void* ctx) {
    geom_t g;
    if (geom_init(&g, p, m, order, weighted, deltas)) return -1;
    const int64_t N = g.N, E = g.E;
    double* alpha = (double*)malloc(sizeof(double) * E);
    double* dth = (double*)malloc(sizeof(double) * E);
    double* uold = (double*)malloc(sizeof(double) * E);
    double* b = (double*)malloc(sizeof(double) * N);
    double* tmp = (double*)malloc(sizeof(double) * N);
    double* r = (double*)malloc(sizeof(double) * N);
    double* pv = (double*)malloc(sizeof(double) * N);
    double* q = (double*)malloc(sizeof(double) * N);
    if (!alpha || !dth || !uold || !b || !tmp || !r || !pv || !q) return -2;
    double rho = *rho_io;
    apply_D(&g, theta, alpha); /* alpha = D theta (:101) */
    int counter = 1, it = 0;
    double dual_norm = 1, primal_norm = 1, eps_dual = tol, eps_primal = tol, pcg_total = 0, relmax = 0;
    for (;;) {
        if (fixed_iters > 0) {
            if (it >= fixed_iters) break;
        } else if (!(dual_norm > eps_dual || primal_norm > eps_primal)) {
            break;
        }
        memcpy(uold, u, sizeof(double) * E);
#pragma omp parallel for schedule(static)
        for (int64_t e = 0; e < E; ++e) dth[e] = alpha[e] + u[e];
        apply_Dt(&g, dth, tmp);
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < N; ++i) b[i] = oty[i] + rho * tmp[i];
        double rel = 0.0;
        if (solve) {
            if (solve(rho, b, theta, ctx) != 0) return -4;
        } else {
            pcg_total += pcg(&g, W, rho, b, theta, r, pv, q, pcg_rtol, pcg_maxit, pcg_fixed, &rel);
        }
        if (rel > relmax) relmax = rel;
        apply_D(&g, theta, dth);
        const double t = lambda / rho;
        double r2 = 0, d2 = 0, a2 = 0;
#pragma omp parallel for schedule(static) reduction(+ : r2, d2, a2)
        for (int64_t e = 0; e < E; ++e) {
            const double z = dth[e] - u[e];
            const double az = fabs(z) - t;
            const double a = (z > 0 ? 1.0 : (z < 0 ? -1.0 : 0.0)) * (az > 0 ? az : 0.0);
            const double pr = a - dth[e];
            alpha[e] = a;
            u[e] += pr;
            uold[e] = u[e] - uold[e];
            r2 += pr * pr;
            d2 += dth[e] * dth[e];
            a2 += a * a;
        }
        apply_Dt(&g, uold, tmp);
        double s2 = 0;
#pragma omp parallel for schedule(static) reduction(+ : s2)
        for (int64_t i = 0; i < N; ++i) s2 += tmp[i] * tmp[i];
        apply_Dt(&g, u, tmp);
        double gu2 = 0;
#pragma omp parallel for schedule(static) reduction(+ : gu2)
        for (int64_t i = 0; i < N; ++i) gu2 += tmp[i] * tmp[i];
        dual_norm = fabs(rho) * sqrt(s2);
        primal_norm = sqrt(r2);
        eps_dual = tol * (sqrt((double)N) + sqrt(gu2));
        eps_primal = tol * (sqrt((double)E) + fmax(sqrt(d2), sqrt(a2)));
        double c = 1.0;
        if (primal_norm > 10 * dual_norm) {
            rho *= 2.0;
            c = 0.5;
        } else if (dual_norm > 10 * primal_norm) {
            rho *= 0.5;
            c = 2.0;
        }
        if (c != 1.0) {
#pragma omp parallel for schedule(static)
            for (int64_t e = 0; e < E; ++e) u[e] *= c;
        }
        ++counter;
        ++it;
        if (fixed_iters <= 0 && counter > max_counter) break;
    }
    *rho_io = rho;
    if (stats) {
        stats[0] = it;
        stats[1] = primal_norm;
        stats[2] = dual_norm;
        stats[3] = eps_primal;
        stats[4] = eps_dual;
        stats[5] = pcg_total;
        stats[6] = relmax;
    }
    free(alpha); free(dth); free(uold); free(b); free(tmp); free(r); free(pv); free(q);
    return 0;
}

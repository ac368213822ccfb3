// solvers.cpp — the reference's solver entry points (include/mvtv/solvers.hpp) over the C ABI.
//
// Host bookkeeping only; every vector operation of the ADMM loop is a HIP kernel behind
// mvtv_admm / mvtv_admm_run. Citations are to rcpp-code/MultivarTV/src (variant B) and
// cpp-code (variant A).
#include "mvtv/solvers.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <limits>

namespace mvtv {

namespace {

void check(int status) {
    if (status != MVTV_OK) throw mvtv_error(status, mvtv_last_error());
}

double mean(const vec& y) {
    double s = 0.0;
    for (double v : y) s += v;
    return y.empty() ? 0.0 : s / double(y.size());
}

// Armadillo linspace: start + i * delta, the last element set to `end` exactly.
vec linspace(double a, double b, int64_t n) {
    vec out(size_t(std::max<int64_t>(n, 0)));
    if (n == 1) {
        out[0] = b;
        return out;
    }
    const double d = (b - a) / double(n - 1);
    for (int64_t i = 0; i + 1 < n; ++i) out[size_t(i)] = a + double(i) * d;
    if (n > 0) out[size_t(n - 1)] = b;
    return out;
}

// Per-dimension axis values if `mesh` is a column-major tensor grid of shape m, else empty.
std::vector<vec> tensor_axes(const mat& mesh, const std::vector<int64_t>& m) {
    const int p = int(m.size());
    std::vector<vec> axes(static_cast<size_t>(p));
    int64_t stride = 1;
    for (int j = 0; j < p; ++j) {
        axes[size_t(j)].resize(size_t(m[size_t(j)]));
        for (int64_t k = 0; k < m[size_t(j)]; ++k) axes[size_t(j)][size_t(k)] = mesh(k * stride, j);
        stride *= m[size_t(j)];
    }
    for (int64_t i = 0; i < mesh.n_rows; ++i) {
        int64_t r = i;
        for (int j = 0; j < p; ++j) {
            const int64_t c = r % m[size_t(j)];
            r /= m[size_t(j)];
            if (mesh(i, j) != axes[size_t(j)][size_t(c)]) return {};
        }
    }
    return axes;
}

std::vector<int64_t> mesh_dims(const vec& m) {
    std::vector<int64_t> out;
    for (double v : m) out.push_back(int64_t(std::llround(v)));
    return out;
}

}  // namespace

mbs_cache::~mbs_cache() {
    if (prob) mvtv_problem_destroy(prob);
}

vec create_deltas(const mat& data, const vec& m, double eps) {
    vec d(size_t(data.n_cols));
    for (int64_t j = 0; j < data.n_cols; ++j) {
        double lo = std::numeric_limits<double>::infinity(), hi = -lo;
        for (int64_t i = 0; i < data.n_rows; ++i) {
            lo = std::min(lo, data(i, j));
            hi = std::max(hi, data(i, j));
        }
        d[size_t(j)] = (hi - lo + 2 * eps) / m[size_t(j)];
    }
    return d;
}

mat create_mesh(const mat& data, const vec& m, double eps) {
    const auto dims = mesh_dims(m);
    const int p = int(data.n_cols);
    int64_t N = 1;
    for (auto v : dims) N *= v;
    std::vector<vec> axes(static_cast<size_t>(p));
    for (int j = 0; j < p; ++j) {
        double lo = std::numeric_limits<double>::infinity(), hi = -lo;
        for (int64_t i = 0; i < data.n_rows; ++i) {
            lo = std::min(lo, data(i, j));
            hi = std::max(hi, data(i, j));
        }
        axes[size_t(j)] = linspace(lo - eps, hi + eps, dims[size_t(j)]);
    }
    mat mesh(N, p);
    for (int64_t i = 0; i < N; ++i) {   // vector2tensor (utils.cpp:59-73), in exact integer arithmetic
        int64_t r = i;
        for (int j = 0; j < p; ++j) {
            mesh(i, j) = axes[size_t(j)][size_t(r % dims[size_t(j)])];
            r /= dims[size_t(j)];
        }
    }
    return mesh;
}

std::vector<int64_t> nearest_index(const mat& data, const mat& mesh) {
    // The reference scans every mesh point (nearest1_unit, utils.cpp:267-278) and keeps the first
    // minimum. On a tensor grid the squared distance separates by dimension, so the per-dimension
    // nearest coordinate (first on ties) gives the same index in O(n p log m).
    std::vector<int64_t> out(size_t(data.n_rows));
    const int p = int(mesh.n_cols);
    std::vector<int64_t> dims;
    {
        // infer the grid shape from runs of the column-major coordinates
        int64_t stride = 1;
        for (int j = 0; j < p; ++j) {
            int64_t k = 1;
            while (k * stride < mesh.n_rows && mesh(k * stride, j) != mesh(0, j)) ++k;
            dims.push_back(k);
            stride *= k;
        }
        if (stride != mesh.n_rows) dims.clear();
    }
    const auto axes = dims.empty() ? std::vector<vec>{} : tensor_axes(mesh, dims);
    for (int64_t i = 0; i < data.n_rows; ++i) {
        if (!axes.empty()) {
            int64_t idx = 0, stride = 1;
            for (int j = 0; j < p; ++j) {
                const vec& ax = axes[size_t(j)];
                int64_t best = 0;
                double bd = std::numeric_limits<double>::infinity();
                for (int64_t k = 0; k < int64_t(ax.size()); ++k) {
                    const double d = (data(i, j) - ax[size_t(k)]) * (data(i, j) - ax[size_t(k)]);
                    if (d < bd) {
                        bd = d;
                        best = k;
                    }
                }
                idx += best * stride;
                stride *= int64_t(ax.size());
            }
            out[size_t(i)] = idx;
        } else {
            int64_t best = 0;
            double bd = std::numeric_limits<double>::infinity();
            for (int64_t k = 0; k < mesh.n_rows; ++k) {
                double d = 0.0;
                for (int j = 0; j < p; ++j) d += (data(i, j) - mesh(k, j)) * (data(i, j) - mesh(k, j));
                if (d < bd) {
                    bd = d;
                    best = k;
                }
            }
            out[size_t(i)] = best;
        }
    }
    return out;
}

vec softthresh(const vec& z, double lam) {
    vec out(z.size());
    for (size_t i = 0; i < z.size(); ++i) {
        const double a = std::fabs(z[i]) - lam;
        out[i] = (z[i] > 0 ? 1.0 : (z[i] < 0 ? -1.0 : 0.0)) * (a > 0 ? a : 0.0);
    }
    return out;
}

namespace {
// create_cache_objects of either variant: O as nearest-mesh indices, D's weights from `deltas` (empty: all 1,
// variant A's mbs_one without cache), W = O^T O and O^T y installed on the (re-used when possible) problem
void build_cache(const mat& data, const vec& y, const mat& mesh, const vec& m, const vec& deltas, mbs_cache& cache,
                 int device) {
    const auto dims = mesh_dims(m);
    if (dims.empty() || dims.size() > MVTV_MAX_DIMS) throw std::invalid_argument("mesh must have 1..4 dimensions");
    int64_t N = 1;
    for (auto v : dims) N *= v;
    if (mesh.n_rows != N) throw std::invalid_argument("mesh rows != prod(m)");
    if (data.n_cols != int64_t(dims.size()) || int64_t(y.size()) != data.n_rows)
        throw std::invalid_argument("data must be n x p and y of length n");
    if (!deltas.empty() && deltas.size() != dims.size()) throw std::invalid_argument("deltas must have p values");
    const auto axes = tensor_axes(mesh, dims);
    // the same mesh and D (CV folds): new data only
    const bool reuse = cache.prob && cache.ntheta == N && cache.deltas == deltas;
    if (!reuse) {
        if (cache.prob) mvtv_problem_destroy(cache.prob);
        cache.prob = nullptr;
        mvtv_problem_desc d{};
        d.p = int32_t(dims.size());
        for (size_t j = 0; j < dims.size(); ++j) {
            d.m[j] = dims[j];
            d.deltas[j] = deltas.empty() ? 1.0 : deltas[j];
        }
        d.block_order = MVTV_ORDER_CPP;
        d.weighted = deltas.empty() ? 0 : 1;
        const vec zeros(size_t(N), 0.0);
        d.oty = zeros.data();
        d.device = device;
        check(mvtv_problem_create(&d, &cache.prob));
        cache.ntheta = N;
        cache.rowsD = mvtv_problem_edges(cache.prob);
        cache.deltas = deltas;
    }
    cache.oidx.assign(size_t(data.n_rows), 0);
    if (!axes.empty()) {
        // tensor mesh (create_mesh): O, O^T O and O^T y built on the GPU (mvtv_problem_set_scattered)
        vec flat;
        for (const auto& a : axes) flat.insert(flat.end(), a.begin(), a.end());
        cache.oty.clear();
        cache.w.clear();
        check(mvtv_problem_set_scattered(cache.prob, flat.data(), data.v.data(), data.n_rows, y.data(),
                                         cache.oidx.data()));
        return;
    }
    cache.oidx = nearest_index(data, mesh);
    cache.oty.assign(size_t(N), 0.0);
    cache.w.assign(size_t(N), 0.0);
    for (size_t i = 0; i < cache.oidx.size(); ++i) {   // O^T y and diag(O^T O)
        cache.oty[size_t(cache.oidx[i])] += y[i];
        cache.w[size_t(cache.oidx[i])] += 1.0;
    }
    check(mvtv_problem_set_data(cache.prob, cache.oty.data(), cache.w.data()));
}
}  // namespace

void create_cache_objects(const mat& data, const vec& y, const mat& mesh, const vec& m, const vec& deltas,
                          mbs_cache& cache, int device) {
    if (deltas.empty()) throw std::invalid_argument("deltas must have p values");
    build_cache(data, y, mesh, m, deltas, cache, device);
}

void admm_update(const vec& /*y*/, mbs_cache& inits, vec& theta_init, double lambda, bool verbose, vec& u_init,
                 double& rho_init, admm_out& out) {
    mvtv_admm_opts o;
    mvtv_default_opts(&o, MVTV_VARIANT_RCPP);
    o.verbose = verbose;
    o.sigma = inits.sp_sigma;   // spcrosses = inits.sp_crosses for the first solve (:107, :113); NaN: rho
    out.theta = theta_init;
    out.u = u_init.empty() ? vec(size_t(inits.rowsD), 0.0) : u_init;
    out.rho = rho_init;
    const int s = mvtv_admm(inits.prob, &o, lambda, out.theta.data(), out.u.data(), &out.rho, &out.stats);
    if (s != MVTV_OK && s != MVTV_MAXITER) check(s);   // B breaks at max_counter (:129-132)
}

vec admm_update_cpp(const vec& y, mbs_cache& inits, const vec* theta_init, double lambda) {
    mvtv_admm_opts o;
    mvtv_default_opts(&o, MVTV_VARIANT_CPP);
    o.ymean = mean(y);
    vec theta = theta_init ? *theta_init : vec(size_t(inits.ntheta), o.ymean);
    double rho = lambda;
    mvtv_admm_stats st;
    const int s = mvtv_admm(inits.prob, &o, lambda, theta.data(), nullptr, &rho, &st);
    if (s == MVTV_MAXITER) throw std::invalid_argument("Failed to converge!");
    check(s);
    return theta;
}

void mbs_one(const mat& data, const vec& y, const vec& m, mbs_one_object& output, const mat& mesh, vec& u,
             double& rho, vec& theta_init, double lambda, mbs_cache& cache, bool verbose) {
    admm_out out;
    admm_update(y, cache, theta_init, lambda, verbose, u, rho, out);
    // fill_output_mbs_one (rcpp…/solvers.cpp:71-75)
    output.mesh = mesh;
    output.theta_hat = out.theta;
    output.uhat = out.u;
    output.rhohat = out.rho;
    output.fitted.resize(cache.oidx.size());
    for (size_t i = 0; i < cache.oidx.size(); ++i) output.fitted[i] = out.theta[size_t(cache.oidx[i])];
    output.data = data;
    output.y = y;
    output.m = m;
}

vec mbs_predict(const mbs_one_object& model, const mat& data) {
    const auto idx = nearest_index(data, model.mesh);
    vec fits(idx.size());
    for (size_t i = 0; i < idx.size(); ++i) fits[i] = model.theta_hat[size_t(idx[i])];
    return fits;
}

double mse(const vec& fits, const vec& y) {
    double s = 0.0;
    for (size_t i = 0; i < y.size(); ++i) s += (fits[i] - y[i]) * (fits[i] - y[i]);
    return s / double(y.size());
}

double mbs_mse(const mbs_one_object& model, const vec& y) { return mse(model.fitted, y); }

void mbs_path(const mat& data, const vec& y, const vec& m, const mat& mesh, const vec& lambdas, const vec& ftrue,
              mbs_object& output, mbs_cache& cache, bool verbose) {
    // theta, u, rho are carried from one lambda to the next (rcpp…/solvers.cpp:207-219); the state
    // stays resident on the GPU between lambdas and is read back once per lambda for the model.
    const size_t n_lambda = lambdas.size();
    vec theta(size_t(cache.ntheta), mean(y));
    double rho_in = lambdas.empty() ? 0.0 : lambdas[0] / 5.0;   // rho_init (:209)
    check(mvtv_state_set(cache.prob, theta.data(), nullptr, rho_in));
    mvtv_admm_opts o;
    mvtv_default_opts(&o, MVTV_VARIANT_RCPP);
    o.verbose = verbose;
    output.models.clear();
    output.mses.assign(n_lambda, 0.0);
    for (size_t i = 0; i < n_lambda; ++i) {
        cache.sp_sigma = rho_in;   // cache->sp_crosses = crossO + rho_init crossD (:213); o.sigma NaN = the same
        mvtv_admm_stats st;
        const int s = mvtv_admm_run(cache.prob, &o, lambdas[i], &st);
        if (s != MVTV_OK && s != MVTV_MAXITER) check(s);
        mbs_one_object model;
        model.theta_hat.resize(size_t(cache.ntheta));
        model.uhat.resize(size_t(cache.rowsD));
        check(mvtv_state_get(cache.prob, model.theta_hat.data(), model.uhat.data(), &model.rhohat));
        model.mesh = mesh;
        model.fitted.resize(cache.oidx.size());
        for (size_t k = 0; k < cache.oidx.size(); ++k) model.fitted[k] = model.theta_hat[size_t(cache.oidx[k])];
        model.data = data;
        model.y = y;
        model.m = m;
        output.mses[i] = mbs_mse(model, ftrue);
        rho_in = model.rhohat;   // :218 (the cache keeps the previous lambda's matrix after the loop)
        output.models.push_back(std::move(model));
    }
    // fill_output_mbs (:177-184): first minimum
    size_t best = 0;
    for (size_t i = 1; i < n_lambda; ++i)
        if (output.mses[i] < output.mses[best]) best = i;
    if (n_lambda) {
        output.minmse_model = output.models[best];
        output.minmse = output.mses[best];
        output.minmse_lambda = lambdas[best];
    }
}

std::vector<int> kfoldinds(int64_t n, int k, uint64_t seed) {
    std::vector<uint64_t> key(size_t(std::max<int64_t>(n, 0)));
    for (int64_t i = 0; i < n; ++i) {
        uint64_t z = seed * 0xD1B54A32D192ED03ull + uint64_t(i) + 0x9E3779B97F4A7C15ull;   // splitmix64
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        key[size_t(i)] = z ^ (z >> 31);
    }
    std::vector<int64_t> perm(key.size());
    for (size_t i = 0; i < perm.size(); ++i) perm[i] = int64_t(i);
    std::stable_sort(perm.begin(), perm.end(), [&](int64_t a, int64_t b) { return key[size_t(a)] < key[size_t(b)]; });
    std::vector<int> out(perm.size());
    for (size_t i = 0; i < perm.size(); ++i) out[i] = int(perm[i] % k);
    return out;
}

vec create_lambdas(int n_lambda, mbs_cache& inits, const vec* lambdas, bool verbose) {
    if (lambdas) return *lambdas;
    double lmax = 0.0;
    int32_t it = 0;
    check(mvtv_lambda_max(inits.prob, &lmax, &it));
    vec grid = linspace(std::log(lmax * 0.0001), std::log(lmax), n_lambda);
    vec out(grid.size());
    for (size_t i = 0; i < grid.size(); ++i) out[grid.size() - 1 - i] = std::exp(grid[i]);   // flipud
    if (verbose) std::printf("Lambda_max = %g\n", lmax);
    return out;
}

vec test_mse(const mat& data, const vec& y, const mbs_object& path, int n_lambda) {
    vec mses(size_t(std::max(n_lambda, 0)), 0.0);
    if (path.models.empty()) return mses;
    // every model of a path shares the mesh: one nearest-node map for all predictions
    const auto idx = nearest_index(data, path.models[0].mesh);
    for (int i = 0; i < n_lambda && size_t(i) < path.models.size(); ++i) {
        vec fits(idx.size());
        for (size_t k = 0; k < idx.size(); ++k) fits[k] = path.models[size_t(i)].theta_hat[size_t(idx[k])];
        mses[size_t(i)] = mse(fits, y);
    }
    return mses;
}

void mbs_fit_optimal(const mat& data, const vec& y, const vec& m, mbs_one_object& best_model, const mat& mesh,
                     const vec& lambdas, const mat& mse_mat, mbs_cache& cache, bool verbose) {
    size_t best = 0;
    double bestv = std::numeric_limits<double>::infinity();
    for (int64_t i = 0; i < mse_mat.n_rows; ++i) {   // rowmean, first minimum
        double s = 0.0;
        for (int64_t j = 0; j < mse_mat.n_cols; ++j) s += mse_mat(i, j);
        s /= double(mse_mat.n_cols);
        if (s < bestv) {
            bestv = s;
            best = size_t(i);
        }
    }
    // :266-268. mbs_one uses the cache (:273 -> use_cache :47), so admm_update's first solve takes
    // cache.sp_sigma, the rho the preceding mbs_path carried into its last lambda (:213), not rho_init.
    vec theta(size_t(cache.ntheta), mean(y));
    vec u(size_t(cache.rowsD), 0.0);
    double rho = lambdas[0] / 5.0;
    if (verbose) std::printf("Best lambda = %g\n", lambdas[best]);
    mbs_one(data, y, m, best_model, mesh, u, rho, theta, lambdas[best], cache, verbose);
}

mbs_impl_result mbs_impl(const mat& data, const vec& y, const vec& m, const mat* mesh, int n_lambda,
                         const vec* ftrue, const vec* lambdas, int folds, bool verbose, uint64_t seed, int device) {
    mbs_impl_result R;
    const mat MESH = mesh ? *mesh : create_mesh(data, m);
    const vec deltas = create_deltas(data, m);
    mbs_cache cache;
    create_cache_objects(data, y, MESH, m, deltas, cache, device);
    R.lambdas = create_lambdas(n_lambda, cache, lambdas, verbose);
    const int nl = int(R.lambdas.size());
    const vec FTRUE = ftrue ? *ftrue : y;
    mat mse_mat(nl, std::max(folds, 1));
    if (folds <= 1) {
        mbs_path(data, y, m, MESH, R.lambdas, FTRUE, R.final_path, cache, verbose);
        const vec t = test_mse(data, y, R.final_path, nl);
        for (int i = 0; i < nl; ++i) mse_mat(i, 0) = t[size_t(i)];
        mbs_fit_optimal(data, y, m, R.best, MESH, R.lambdas, mse_mat, cache, verbose);
        R.cv_mses = t;
    } else {
        const auto fi = kfoldinds(data.n_rows, folds, seed);
        for (int f = 0; f < folds; ++f) {
            int64_t ntr = 0, nte = 0;
            for (int v : fi) (v == f ? nte : ntr) += 1;
            mat trx(ntr, data.n_cols), tex(nte, data.n_cols);
            vec tr_y, te_y;
            for (int64_t i = 0, a = 0, b = 0; i < data.n_rows; ++i) {
                if (fi[size_t(i)] != f) {
                    for (int64_t j = 0; j < data.n_cols; ++j) trx(a, j) = data(i, j);
                    tr_y.push_back(y[size_t(i)]);
                    ++a;
                } else {
                    for (int64_t j = 0; j < data.n_cols; ++j) tex(b, j) = data(i, j);
                    te_y.push_back(y[size_t(i)]);
                    ++b;
                }
            }
            create_cache_objects(trx, tr_y, MESH, m, deltas, cache, device);
            mbs_object path;
            mbs_path(trx, tr_y, m, MESH, R.lambdas, tr_y, path, cache, verbose);
            if (verbose) std::printf("Fold Complete: %d\n", f);
            const vec t = test_mse(tex, te_y, path, nl);
            for (int i = 0; i < nl; ++i) mse_mat(i, f) = t[size_t(i)];
        }
        create_cache_objects(data, y, MESH, m, deltas, cache, device);
        mbs_path(data, y, m, MESH, R.lambdas, y, R.final_path, cache, verbose);
        R.cv_mses.assign(size_t(nl), 0.0);
        for (int i = 0; i < nl; ++i) {
            double s = 0.0;
            for (int f = 0; f < folds; ++f) s += mse_mat(i, f);
            R.cv_mses[size_t(i)] = s / double(folds);
        }
    }
    size_t best = 0;
    for (size_t i = 1; i < R.cv_mses.size(); ++i)
        if (R.cv_mses[i] < R.cv_mses[best]) best = i;
    R.lambda_minmse_ind = int64_t(best) + 1;
    if (folds > 1) R.best = R.final_path.models[best];
    R.residuals.resize(y.size());
    for (size_t i = 0; i < y.size(); ++i) R.residuals[i] = y[i] - R.best.fitted[i];
    return R;
}

// =============================================================================== variant A (cpp-code)
vec create_deltas_cpp(const mat& data, const vec& m) { return create_deltas(data, m, 0.01); }

mat create_mesh_cpp(const mat& data, const vec& m) {
    const auto dims = mesh_dims(m);
    const int p = int(data.n_cols);
    int64_t N = 1;
    for (auto v : dims) N *= v;
    std::vector<vec> axes(static_cast<size_t>(p));
    for (int j = 0; j < p; ++j) {
        double lo = std::numeric_limits<double>::infinity(), hi = -lo;
        for (int64_t i = 0; i < data.n_rows; ++i) {
            lo = std::min(lo, data(i, j));
            hi = std::max(hi, data(i, j));
        }
        axes[size_t(j)] = linspace(lo + 0.01, hi + 0.01, dims[size_t(j)]);   // EPS added to both ends (:281)
        for (double& v : axes[size_t(j)]) v = double(float(v));               // MAT = fmat (solvers.hpp:12)
    }
    mat mesh(N, p);
    for (int64_t i = 0; i < N; ++i) {
        int64_t r = i;
        for (int j = 0; j < p; ++j) {
            mesh(i, j) = axes[size_t(j)][size_t(r % dims[size_t(j)])];
            r /= dims[size_t(j)];
        }
    }
    return mesh;
}

void create_cache_objects_cpp(const mat& data, const vec& y, const mat& mesh, const vec& m, const vec& deltas,
                              mbs_cache& cache, int device) {
    build_cache(data, y, mesh, m, deltas, cache, device);
}

vec create_lambdas_cpp(int n_lambda, mbs_cache& inits, const vec* lambdas, double* lambda_max) {
    if (lambdas) return *lambdas;
    double lmax = 0.0;
    int32_t it = 0;
    check(mvtv_lambda_max_cpp(inits.prob, &lmax, &it));
    if (lambda_max) *lambda_max = lmax;
    const vec grid = linspace(std::log(lmax * 0.00001), std::log(lmax), n_lambda);
    vec out(grid.size());
    for (size_t i = 0; i < grid.size(); ++i) out[grid.size() - 1 - i] = std::exp(grid[i]);   // flipud
    return out;
}

vec admm_update(const vec& y, mbs_cache& inits, const vec* theta_init, double lambda) {
    mvtv_admm_opts o;
    mvtv_default_opts(&o, MVTV_VARIANT_CPP);
    o.ymean = mean(y);
    o.sigma = inits.sp_sigma;
    vec theta = theta_init ? *theta_init : vec(size_t(inits.ntheta), o.ymean);
    double rho = lambda;
    mvtv_admm_stats st;
    const int s = mvtv_admm(inits.prob, &o, lambda, theta.data(), nullptr, &rho, &st);
    if (s == MVTV_MAXITER) throw std::invalid_argument("Failed to converge!");
    check(s);
    return theta;
}

namespace {
// fill_output_mbs_one (cpp-code/solvers.cpp:64-68): fitted = O theta with the O the solve used
void fill_output_cpp(mbs_one_object& out, const mat& data, const vec& y, const mat& mesh, const vec& theta,
                     const mbs_cache& inits, const vec& m) {
    out.mesh = mesh;
    out.theta_hat = theta;
    out.fitted.resize(inits.oidx.size());
    for (size_t i = 0; i < inits.oidx.size(); ++i) out.fitted[i] = theta[size_t(inits.oidx[i])];
    out.data = data;
    out.y = y;
    out.m = m;
}
}  // namespace

void mbs_one(const mat& data, const vec& y, const vec& m, mbs_one_object& output, const mat& mesh,
             const vec* theta_init, double lambda, mbs_cache* cache, int device) {
    if (!cache) {   // :141-145: create_cache_objects with inits.deltas never set -> unit weights
        mbs_cache local;
        create_cache_objects_cpp(data, y, mesh, m, vec{}, local, device);
        local.sp_sigma = lambda;
        const vec theta = admm_update(y, local, theta_init, lambda);
        fill_output_cpp(output, data, y, mesh, theta, local, m);
        return;
    }
    const vec theta = admm_update(y, *cache, theta_init, lambda);
    fill_output_cpp(output, data, y, mesh, theta, *cache, m);
}

std::vector<int64_t> kfold_perm(int64_t n, uint64_t seed) {
    std::vector<uint64_t> key(size_t(std::max<int64_t>(n, 0)));
    for (int64_t i = 0; i < n; ++i) {
        uint64_t z = seed * 0xD1B54A32D192ED03ull + uint64_t(i) + 0x9E3779B97F4A7C15ull;   // splitmix64
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        key[size_t(i)] = z ^ (z >> 31);
    }
    std::vector<int64_t> perm(key.size());
    for (size_t i = 0; i < perm.size(); ++i) perm[i] = int64_t(i);
    std::stable_sort(perm.begin(), perm.end(), [&](int64_t a, int64_t b) { return key[size_t(a)] < key[size_t(b)]; });
    return perm;
}

void mbs(const mat& data, const vec& y, const vec& m, mbs_one_object& output, const mat* mesh, int n_lambda,
         const vec* ftrue, const vec* lambdas, int folds, const mbs_cpp_options& opts, mbs_cpp_report* report) {
    if (folds < 1) throw std::invalid_argument("folds must be >= 1");
    const vec deltas = create_deltas_cpp(data, m);                  // :281
    const mat MESH = mesh ? *mesh : create_mesh_cpp(data, m);       // :282
    mbs_cache cache;                                                // :286-289, full data
    create_cache_objects_cpp(data, y, MESH, m, deltas, cache, opts.device);
    double lmax = 0.0;
    const vec LAMBDAS = create_lambdas_cpp(n_lambda, cache, lambdas, &lmax);   // :292
    const int nl = int(LAMBDAS.size());
    (void)ftrue;   // FTRUE (:293) only feeds the path models' own MSEs, which mbs never reads
    // kfold (cpp-code/utils.cpp:417-436) over the permuted rows
    const int64_t n = data.n_rows, ntest = n / folds, p = data.n_cols;
    const auto perm = kfold_perm(n, opts.seed);
    mat mse_mat(nl, folds);
    std::vector<vec> path0;   // fold 0's path models (what test_mse and the refit read in reference mode)
    for (int f = 0; f < folds; ++f) {
        const int64_t first = int64_t(f) * ntest, last = first + ntest;   // test rows [first, last)
        mat trx(n - ntest, p), tex(ntest, p);
        vec tr_y, te_y;
        for (int64_t r = 0, a = 0, b = 0; r < n; ++r) {
            const int64_t i = perm[size_t(r)];
            const bool test = r >= first && r < last;
            for (int64_t j = 0; j < p; ++j) (test ? tex(b, j) : trx(a, j)) = data(i, j);
            (test ? te_y : tr_y).push_back(y[size_t(i)]);
            test ? ++b : ++a;
        }
        // mbs_path (:196-217): warm-started theta, rho = lambda, matrix crossO + lambda crossD
        mbs_cache fold_cache;
        mbs_cache& pc = opts.reference_cv ? cache : fold_cache;
        if (!opts.reference_cv) create_cache_objects_cpp(trx, tr_y, MESH, m, deltas, fold_cache, opts.device);
        vec theta(size_t(cache.ntheta), mean(tr_y));
        std::vector<vec> models;
        for (int i = 0; i < nl; ++i) {
            pc.sp_sigma = LAMBDAS[size_t(i)];
            theta = admm_update(tr_y, pc, &theta, LAMBDAS[size_t(i)]);
            models.push_back(theta);
        }
        if (f == 0) path0 = models;
        // test_mse (:264-273): reference mode reads the first n_lambda models of the accumulated path = fold 0's
        const std::vector<vec>& use = opts.reference_cv ? path0 : models;
        const auto idx = nearest_index(tex, MESH);
        for (int i = 0; i < nl; ++i) {
            vec fits(idx.size());
            for (size_t k = 0; k < idx.size(); ++k) fits[k] = use[size_t(i)][size_t(idx[k])];
            mse_mat(i, f) = mse(fits, te_y);
        }
        if (opts.reference_cv) cache.sp_sigma = LAMBDAS[size_t(nl - 1)];   // what the last path leaves (:209)
    }
    // mbs_fit_optimal (:248-260): rowmean, first minimum
    int64_t best = 0;
    double bestv = std::numeric_limits<double>::infinity();
    for (int i = 0; i < nl; ++i) {
        double s = 0.0;
        for (int f = 0; f < folds; ++f) s += mse_mat(i, f);
        s /= double(folds);
        if (s < bestv) {
            bestv = s;
            best = i;
        }
    }
    if (opts.reference_cv) {
        mbs_one(data, y, m, output, MESH, &path0[size_t(best)], LAMBDAS[size_t(best)], &cache);
    } else {
        cache.sp_sigma = LAMBDAS[size_t(best)];
        mbs_one(data, y, m, output, MESH, nullptr, LAMBDAS[size_t(best)], &cache);
    }
    if (report) {
        report->lambdas = LAMBDAS;
        report->lambda_max = lmax;
        report->mse_mat = mse_mat;
        report->best = best;
    }
}

}  // namespace mvtv

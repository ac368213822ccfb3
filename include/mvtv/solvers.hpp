// solvers.hpp — C++ host API with the reference's solver entry points, over the mvtv C ABI.
//
// Mirrors rcpp-code/MultivarTV/src/solvers.hpp (variant B, the released package) and
// cpp-code/solvers.hpp (variant A) with Armadillo types replaced by std::vector and a small
// column-major matrix. Every numerical step of the ADMM loop runs in libmvtv.so on the GPU;
// this layer only does the reference's host bookkeeping (mesh, nearest-mesh index O,
// warm-started lambda path, MSE bookkeeping).
#pragma once
#include <cstdint>
#include <limits>
#include <stdexcept>
#include <string>
#include <vector>

#include "mvtv/mvtv.h"

namespace mvtv {

using vec = std::vector<double>;

// Column-major matrix (Armadillo's layout): element (i, j) at v[i + j * n_rows].
struct mat {
    int64_t n_rows = 0, n_cols = 0;
    std::vector<double> v;
    mat() = default;
    mat(int64_t r, int64_t c) : n_rows(r), n_cols(c), v(size_t(r * c), 0.0) {}
    double& operator()(int64_t i, int64_t j) { return v[size_t(i + j * n_rows)]; }
    double operator()(int64_t i, int64_t j) const { return v[size_t(i + j * n_rows)]; }
};

class mvtv_error : public std::runtime_error {
   public:
    mvtv_error(int status, const std::string& what) : std::runtime_error(what), status(status) {}
    int status;
};

// ---- setup: rcpp-code/MultivarTV/src/utils.cpp -------------------------------------------
vec create_deltas(const mat& data, const vec& m, double eps = 1e-4);          // :256-263
mat create_mesh(const mat& data, const vec& m, double eps = 1e-4);            // :234-254
// nearest1 (:280-287) as an index map: row i of O has its 1 in column oidx[i]
std::vector<int64_t> nearest_index(const mat& data, const mat& mesh);
vec softthresh(const vec& z, double lam);                                     // solvers.cpp:29-34

// ---- cache: replaces mbs_cache / mbs_one_inits (rcpp…/solvers.hpp:30-50) -------------------
struct mbs_cache {
    mvtv_problem* prob = nullptr;   // GPU-resident D (as a stencil), W = O^T O, O^T y
    std::vector<int64_t> oidx;      // O as nearest-mesh indices
    vec oty, w;
    int64_t ntheta = 0, rowsD = 0;
    vec deltas;                     // block weights of D (empty: every weight 1, cpp-code mbs_one without cache)
    // the solve matrix the cache holds, sp_crosses = crossO + sp_sigma * crossD (rcpp…/solvers.hpp:46,
    // cpp-code/solvers.hpp:26); admm_update's FIRST theta-solve uses it (rcpp…/solvers.cpp:107,113;
    // cpp-code/solvers.cpp:116). NaN: not set (B: rho_init, A: lambda). mbs_path (B) leaves the rho carried
    // INTO its last lambda here (:213), which mbs_fit_optimal's refit then solves with (:273, :47).
    double sp_sigma = std::numeric_limits<double>::quiet_NaN();
    mbs_cache() = default;
    mbs_cache(const mbs_cache&) = delete;
    mbs_cache& operator=(const mbs_cache&) = delete;
    ~mbs_cache();
};

// create_cache_objects (rcpp…/solvers.cpp:36-44): O, D, D^T D, O^T O, O^T y for (data, y, mesh)
void create_cache_objects(const mat& data, const vec& y, const mat& mesh, const vec& m, const vec& deltas,
                          mbs_cache& cache, int device = 0);

struct admm_out {
    double rho = 0.0;
    vec theta, u;
    mvtv_admm_stats stats{};
};

// B: rcpp…/solvers.hpp:100 (y is unused by the loop, kept for signature parity). The first theta-solve uses
// the cache's matrix (inits.sp_sigma; NaN: rho_init), every later one crossO + rho crossD (:126).
void admm_update(const vec& y, mbs_cache& inits, vec& theta_init, double lambda, bool verbose, vec& u_init,
                 double& rho_init, admm_out& out);
// A: cpp-code/solvers.hpp:85 — throws std::invalid_argument("Failed to converge!") past 2000 iterations;
// the solve matrix is crossO + lambda crossD (mbs_one's, :144). See also the variant-A overload below.
vec admm_update_cpp(const vec& y, mbs_cache& inits, const vec* theta_init, double lambda);

struct mbs_one_object {   // rcpp…/solvers.hpp:52-61
    mat mesh;
    vec theta_hat, fitted;
    mat data;
    vec y, m;
    double rhohat = 0.0;
    vec uhat;
};

struct mbs_object {       // rcpp…/solvers.hpp:65-72
    mbs_one_object minmse_model;
    std::vector<mbs_one_object> models;
    double minmse = 0.0, minmse_lambda = 0.0;
    vec mses;
};

// rcpp…/solvers.cpp:140-159 (cache path)
void mbs_one(const mat& data, const vec& y, const vec& m, mbs_one_object& output, const mat& mesh, vec& u,
             double& rho, vec& theta_init, double lambda, mbs_cache& cache, bool verbose = false);
vec mbs_predict(const mbs_one_object& model, const mat& data);   // :161-165
double mse(const vec& fits, const vec& y);                       // :167-170
double mbs_mse(const mbs_one_object& model, const vec& y);       // :172-175
// rcpp…/solvers.cpp:204-222: warm-started path over lambdas (theta, u, rho carried)
void mbs_path(const mat& data, const vec& y, const vec& m, const mat& mesh, const vec& lambdas, const vec& ftrue,
              mbs_object& output, mbs_cache& cache, bool verbose = false);

// ---- cross-validation driver: rcpp…/solvers.cpp:186-376 ----------------------------------------
// kfoldinds (rcpp…/utils.cpp:367-376): the labels i % k, permuted. The reference shuffles with R's
// RNG (arma::shuffle), which cannot be reproduced outside R; here the permutation sorts a seeded
// splitmix64 key per position, exactly as multivartv_amd.cv.kfoldinds does.
std::vector<int> kfoldinds(int64_t n, int k, uint64_t seed = 0);
// create_lambdas (:186-200): flipud(exp(linspace(log(1e-4 lmax), log(lmax), n))), lmax = lam_max_pinv
// on the GPU (mvtv_lambda_max); `lambdas` (may be null) is returned as given
vec create_lambdas(int n_lambda, mbs_cache& inits, const vec* lambdas, bool verbose = false);
// test_mse (:278-288): MSE of each path model's predictions at (data, y)
vec test_mse(const mat& data, const vec& y, const mbs_object& path, int n_lambda);
// mbs_fit_optimal (:261-274): cold refit (theta = mean y, u = 0, rho = lambdas[0] / 5) at the lambda of the
// smallest row mean of mse_mat, whose first theta-solve uses the matrix the preceding mbs_path left in the
// cache (crossO + rho_in(last lambda) crossD, :213 -> :273 -> use_cache :47 -> :107, :113)
void mbs_fit_optimal(const mat& data, const vec& y, const vec& m, mbs_one_object& best_model, const mat& mesh,
                     const vec& lambdas, const mat& mse_mat, mbs_cache& cache, bool verbose = false);

// mbs_impl's result list (:368-373); models = listPATH(final_path, lambdas) (:292-302)
struct mbs_impl_result {
    mbs_one_object best;          // data, fitted, m, mesh, theta_hat, y of the chosen model
    vec residuals;                // y - fitted
    vec lambdas;                  // the grid (models[i].lambda)
    mbs_object final_path;        // models[i].theta_hat / fitted, mses[i] = models[i].mse
    int64_t lambda_minmse_ind = 0;   // 1-based, as R
    vec cv_mses;                  // "cv.mses"
};
// mbs_impl (:305-376). mesh, ftrue, lambdas may be null (R's NULL). seed: kfoldinds.
mbs_impl_result mbs_impl(const mat& data, const vec& y, const vec& m, const mat* mesh, int n_lambda,
                         const vec* ftrue, const vec* lambdas, int folds, bool verbose = false, uint64_t seed = 0,
                         int device = 0);

// ---- variant A: the research code's API, cpp-code/solvers.hpp ------------------------------------
// Its own setup constants: EPS = 0.01 (cpp-code/solvers.hpp:13, utils.hpp), TOL = 1e-3.
// create_deltas (cpp-code/utils.cpp:300-307): (max - min + 2 EPS) / m_j
vec create_deltas_cpp(const mat& data, const vec& m);
// create_mesh (cpp-code/utils.cpp:271-298): axis j = linspace(min + EPS, max + EPS, m_j) (both ends shifted
// up), stored in a float matrix (typedef fmat MAT): every mesh value is rounded to float
mat create_mesh_cpp(const mat& data, const vec& m);
// create_cache_objects (cpp-code/solvers.cpp:31-41): O, D (weights from `deltas`; empty: all 1), O^T O, O^T y
void create_cache_objects_cpp(const mat& data, const vec& y, const mat& mesh, const vec& m, const vec& deltas,
                              mbs_cache& cache, int device = 0);
// create_lambdas (cpp-code/solvers.cpp:179-192): flipud(exp(linspace(log(1e-5 lmax), log(lmax), n))) with
// lmax = lam_max_pinv (cpp-code/utils.cpp:354-404, GPU: mvtv_lambda_max_cpp)
vec create_lambdas_cpp(int n_lambda, mbs_cache& inits, const vec* lambdas, double* lambda_max = nullptr);
// admm_update (cpp-code/solvers.hpp:85) on inits.sp_sigma's matrix; y gives mean(y) for theta_old
vec admm_update(const vec& y, mbs_cache& inits, const vec* theta_init, double lambda);
// mbs_one (cpp-code/solvers.hpp:89, solvers.cpp:134-152). cache == nullptr: O and D are built here with EMPTY
// deltas, so every block weight is 1, and the matrix is crossO + lambda crossD; otherwise the
// cache's D and its sp_sigma matrix are used. Throws std::invalid_argument("Failed to converge!") past 2000
// iterations (:122-124).
void mbs_one(const mat& data, const vec& y, const vec& m, mbs_one_object& output, const mat& mesh,
             const vec* theta_init = nullptr, double lambda = 1.0, mbs_cache* cache = nullptr, int device = 0);

// mbs (cpp-code/solvers.hpp:129, solvers.cpp:277-310): k-fold CV over a lambda path, refit at the best lambda.
// The reference's CV differs from a textbook CV in three ways, all reproduced when reference_cv is set
// (the default):
//   1. the cache (O, O^T y, O^T O) is built once on the FULL data and never rebuilt per fold (:288-301): each
//      fold's path fits all n points and differs from the others only through mean(y_train) (theta_0 and
//      theta_old, :199, :103);
//   2. the path object accumulates models over folds and test_mse reads models[0 .. n_lambda-1] (:264-273),
//      so every fold's test MSE is computed with fold 0's path;
//   3. the refit (:248-260) starts from fold 0's model at the best lambda and solves with the matrix the
//      last path left in the cache, crossO + lambdas[n_lambda-1] crossD (:209).
// reference_cv = false: each fold's path runs on its own training cache, test MSEs use that fold's models,
// and the refit solves with crossO + best_lambda crossD from mean(y).
// Fold assignment is NOT the reference's (parity unpinned): kfold (cpp-code/utils.cpp:417-436) calls
// shuffle(join_horiz(data, y), 1), and Armadillo's shuffle(X, dim = 1) permutes the COLUMNS of X (per its
// documentation; no Armadillo source is in this image), so the reference's folds are unshuffled contiguous
// row blocks of a matrix whose p + 1 predictor / response columns were randomly reordered by Armadillo's RNG.
// Neither that RNG nor the column scramble is reproduced: here rows are permuted by the seeded
// kfold_perm(n, seed), fold i tests rows [i n/k, (i+1) n/k) of that order and trains on the rest.
struct mbs_cpp_options {
    uint64_t seed = 0;
    bool reference_cv = true;
    int device = 0;
};
struct mbs_cpp_report {        // what mbs computed on the way (the reference keeps these local)
    vec lambdas;
    double lambda_max = 0.0;
    mat mse_mat;               // n_lambda x folds (:296, :303)
    int64_t best = 0;          // 0-based row of the smallest row mean (:249-251)
};
std::vector<int64_t> kfold_perm(int64_t n, uint64_t seed);
void mbs(const mat& data, const vec& y, const vec& m, mbs_one_object& output, const mat* mesh = nullptr,
         int n_lambda = 100, const vec* ftrue = nullptr, const vec* lambdas = nullptr, int folds = 5,
         const mbs_cpp_options& opts = mbs_cpp_options(), mbs_cpp_report* report = nullptr);

}  // namespace mvtv

// R shim: the released package's three .Call entry points, with the names and
// argument order of rcpp-code/MultivarTV/src/init.c:15-20 and RcppExports.cpp, over the C++ host API
// (include/mvtv/solvers.hpp) and so over the C ABI of libmvtv.so. R's own C API only (no Rcpp, no
// Armadillo): arma::mat / arma::vec are R's column-major REALSXP storage either way.
//
//   _MultivarTV_mbs(data, y, m, mesh, n_lambda, ftrue, lambdas, folds, verbose)   MultivarTV.cpp:39-42
//   _MultivarTV_mbspredict(mvtvobject, data, mesh)                                MultivarTV.cpp:55-66
//   _MultivarTV_gen_mesh(data, m, mesh)                                           solvers.cpp:234-244
//
// Build (where R exists): R CMD INSTALL with src/Makevars from rshim/src/Makevars. R is not in this
// image, so this file is not compiled by `make` here.
#include <R.h>
#include <R_ext/Rdynload.h>
#include <Rinternals.h>

#include <cstring>
#include <exception>
#include <string>

#include "mvtv/solvers.hpp"

namespace {

// R errors longjmp: never raise one while a C++ object with a destructor is live in this frame.
char g_err[512];

mvtv::mat as_mat(SEXP x) {
    SEXP d = PROTECT(Rf_coerceVector(x, REALSXP));
    SEXP dim = Rf_getAttrib(x, R_DimSymbol);
    const int64_t nr = Rf_isNull(dim) ? XLENGTH(d) : INTEGER(dim)[0];
    const int64_t nc = Rf_isNull(dim) ? 1 : INTEGER(dim)[1];
    mvtv::mat out(nr, nc);
    std::memcpy(out.v.data(), REAL(d), sizeof(double) * size_t(nr * nc));
    UNPROTECT(1);
    return out;
}

mvtv::vec as_vec(SEXP x) {
    SEXP d = PROTECT(Rf_coerceVector(x, REALSXP));
    mvtv::vec out(REAL(d), REAL(d) + XLENGTH(d));
    UNPROTECT(1);
    return out;
}

SEXP vec_sexp(const mvtv::vec& v) {
    SEXP out = PROTECT(Rf_allocVector(REALSXP, R_xlen_t(v.size())));
    if (!v.empty()) std::memcpy(REAL(out), v.data(), sizeof(double) * v.size());
    UNPROTECT(1);
    return out;
}

SEXP mat_sexp(const mvtv::mat& m) {
    SEXP out = PROTECT(Rf_allocMatrix(REALSXP, int(m.n_rows), int(m.n_cols)));
    if (!m.v.empty()) std::memcpy(REAL(out), m.v.data(), sizeof(double) * m.v.size());
    UNPROTECT(1);
    return out;
}

SEXP list_get(SEXP list, const char* name) {
    SEXP names = Rf_getAttrib(list, R_NamesSymbol);
    for (R_xlen_t i = 0; i < XLENGTH(list); ++i)
        if (std::strcmp(CHAR(STRING_ELT(names, i)), name) == 0) return VECTOR_ELT(list, i);
    return R_NilValue;
}

// mbs_impl's result list (rcpp…/solvers.cpp:368-373)
SEXP result_list(const mvtv::mbs_impl_result& R) {
    const char* top[] = {"data", "fitted", "m", "mesh", "theta_hat", "y", "residuals", "models",
                         "lambda_minmse_ind", "cv.mses", ""};
    SEXP out = PROTECT(Rf_mkNamed(VECSXP, top));
    SET_VECTOR_ELT(out, 0, mat_sexp(R.best.data));
    SET_VECTOR_ELT(out, 1, vec_sexp(R.best.fitted));
    SET_VECTOR_ELT(out, 2, vec_sexp(R.best.m));
    SET_VECTOR_ELT(out, 3, mat_sexp(R.best.mesh));
    SET_VECTOR_ELT(out, 4, vec_sexp(R.best.theta_hat));
    SET_VECTOR_ELT(out, 5, vec_sexp(R.best.y));
    SET_VECTOR_ELT(out, 6, vec_sexp(R.residuals));
    // listPATH (:292-302)
    const R_xlen_t nl = R_xlen_t(R.lambdas.size());
    SEXP models = PROTECT(Rf_allocVector(VECSXP, nl));
    const char* mn[] = {"lambda", "mse", "theta_hat", "fitted", ""};
    for (R_xlen_t i = 0; i < nl; ++i) {
        SEXP mi = PROTECT(Rf_mkNamed(VECSXP, mn));
        SET_VECTOR_ELT(mi, 0, Rf_ScalarReal(R.lambdas[size_t(i)]));
        SET_VECTOR_ELT(mi, 1, Rf_ScalarReal(R.final_path.mses[size_t(i)]));
        SET_VECTOR_ELT(mi, 2, vec_sexp(R.final_path.models[size_t(i)].theta_hat));
        SET_VECTOR_ELT(mi, 3, vec_sexp(R.final_path.models[size_t(i)].fitted));
        SET_VECTOR_ELT(models, i, mi);
        UNPROTECT(1);
    }
    SET_VECTOR_ELT(out, 7, models);
    SET_VECTOR_ELT(out, 8, Rf_ScalarReal(double(R.lambda_minmse_ind)));
    SET_VECTOR_ELT(out, 9, vec_sexp(R.cv_mses));
    UNPROTECT(2);
    return out;
}

}  // namespace

extern "C" {

SEXP _MultivarTV_mbs(SEXP data, SEXP y, SEXP m, SEXP mesh, SEXP n_lambda, SEXP ftrue, SEXP lambdas, SEXP folds,
                     SEXP verbose) {
    SEXP out = R_NilValue;
    bool failed = false;
    {
        try {
            const mvtv::mat D = as_mat(data), M = Rf_isNull(mesh) ? mvtv::mat() : as_mat(mesh);
            const mvtv::vec Y = as_vec(y), Mv = as_vec(m);
            const mvtv::vec F = Rf_isNull(ftrue) ? mvtv::vec() : as_vec(ftrue);
            const mvtv::vec L = Rf_isNull(lambdas) ? mvtv::vec() : as_vec(lambdas);
            const auto R = mvtv::mbs_impl(D, Y, Mv, Rf_isNull(mesh) ? nullptr : &M, Rf_asInteger(n_lambda),
                                          Rf_isNull(ftrue) ? nullptr : &F, Rf_isNull(lambdas) ? nullptr : &L,
                                          Rf_asInteger(folds), Rf_asLogical(verbose) == TRUE);
            out = PROTECT(result_list(R));
        } catch (const std::exception& e) {
            std::strncpy(g_err, e.what(), sizeof(g_err) - 1);
            failed = true;
        }
    }
    if (failed) Rf_error("%s", g_err);   // Rcpp::stop equivalent (RcppExports.cpp BEGIN/END_RCPP)
    UNPROTECT(1);
    return out;
}

SEXP _MultivarTV_mbspredict(SEXP obj, SEXP data, SEXP mesh) {
    if (Rf_isNull(data)) return list_get(obj, "fitted");
    SEXP out = R_NilValue;
    bool failed = false;
    {
        try {
            const mvtv::mat D = as_mat(data);
            const mvtv::mat M = as_mat(Rf_isNull(mesh) ? list_get(obj, "mesh") : mesh);
            const mvtv::vec th = as_vec(list_get(obj, "theta_hat"));
            const auto idx = mvtv::nearest_index(D, M);   // nearest_interp_matrix (utils.cpp:289-304)
            mvtv::vec fits(idx.size());
            for (size_t i = 0; i < idx.size(); ++i) fits[i] = th[size_t(idx[i])];
            out = PROTECT(vec_sexp(fits));
        } catch (const std::exception& e) {
            std::strncpy(g_err, e.what(), sizeof(g_err) - 1);
            failed = true;
        }
    }
    if (failed) Rf_error("%s", g_err);
    UNPROTECT(1);
    return out;
}

SEXP _MultivarTV_gen_mesh(SEXP data, SEXP m, SEXP mesh) {
    if (!Rf_isNull(mesh)) return mesh;
    SEXP out = R_NilValue;
    bool failed = false;
    {
        try {
            out = PROTECT(mat_sexp(mvtv::create_mesh(as_mat(data), as_vec(m))));
        } catch (const std::exception& e) {
            std::strncpy(g_err, e.what(), sizeof(g_err) - 1);
            failed = true;
        }
    }
    if (failed) Rf_error("%s", g_err);
    UNPROTECT(1);
    return out;
}

static const R_CallMethodDef CallEntries[] = {
    {"_MultivarTV_gen_mesh", (DL_FUNC)&_MultivarTV_gen_mesh, 3},
    {"_MultivarTV_mbs", (DL_FUNC)&_MultivarTV_mbs, 9},
    {"_MultivarTV_mbspredict", (DL_FUNC)&_MultivarTV_mbspredict, 3},
    {NULL, NULL, 0}};

void R_init_MultivarTV(DllInfo* dll) {
    R_registerRoutines(dll, NULL, CallEntries, NULL, NULL);
    R_useDynamicSymbols(dll, FALSE);
}

}  // extern "C"

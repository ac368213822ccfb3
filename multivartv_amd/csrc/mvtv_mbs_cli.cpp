// mvtv_mbs — command-line front end of the C++ host API's mbs_impl (include/mvtv/solvers.hpp), the
// released package's mvtv_default (rcpp-code/MultivarTV/src/MultivarTV.cpp:39-42 -> mbs_impl,
// solvers.cpp:305-376). Used by the parity tests (tests/test_gpu_cxx_mbs.py) and as a minimal
// example of a non-Python host.
//
// Input file (little-endian, all int64 then float64):
//   n, p, n_lambda, folds, seed, given_lambdas (0/1), device
//   m[p], data[n*p] column-major, y[n], lambdas[n_lambda] if given_lambdas
// Output file:
//   n_lambda, lambda_minmse_ind, N, n   (int64)
//   lambdas[n_lambda], cv_mses[n_lambda], model_mses[n_lambda], theta_hat[N], fitted[n], residuals[n]
//
// `mvtv_mbs --cpp <input> <output>`: variant A's mbs (cpp-code/solvers.cpp:277-310) instead. Same input
// (hdr[6] = 1 selects the corrected CV, 0 the reference's); output:
//   n_lambda, best (0-based), N, n   (int64)
//   lambda_max, lambdas[n_lambda], mse_mat[n_lambda x folds] column-major, theta_hat[N], fitted[n]
// `mvtv_mbs --cpp-one <input> <output>`: variant A's mbs_one without cache (cpp-code/solvers.cpp:134-152) on
// create_mesh_cpp's mesh; input n, p, 0, 0, 0, 1, 0, m, data, y, lambda[1]; output N, n, theta_hat, fitted.
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "mvtv/solvers.hpp"

namespace {
template <class T>
bool rd(std::FILE* f, T* v, size_t n) { return std::fread(v, sizeof(T), n, f) == n; }
template <class T>
void wr(std::FILE* f, const T* v, size_t n) { std::fwrite(v, sizeof(T), n, f); }
}  // namespace

int main(int argc, char** argv) {
    int mode = 0;   // 0 mbs_impl (B), 1 mbs (A), 2 mbs_one without cache (A)
    if (argc == 4 && std::string(argv[1]) == "--cpp") mode = 1;
    if (argc == 4 && std::string(argv[1]) == "--cpp-one") mode = 2;
    if (mode) {
        ++argv;
        --argc;
    }
    if (argc != 3) {
        std::fprintf(stderr, "usage: %s [--cpp | --cpp-one] <input> <output>\n", argv[0]);
        return 2;
    }
    std::FILE* in = std::fopen(argv[1], "rb");
    if (!in) {
        std::perror(argv[1]);
        return 2;
    }
    int64_t hdr[7];
    if (!rd(in, hdr, 7)) return 2;
    const int64_t n = hdr[0], p = hdr[1], nl = hdr[2], folds = hdr[3], seed = hdr[4], given = hdr[5], dev = hdr[6];
    mvtv::vec m(static_cast<size_t>(p)), y(static_cast<size_t>(n)), lambdas(static_cast<size_t>(given ? nl : 0));
    mvtv::mat data(n, p);
    if (!rd(in, m.data(), m.size()) || !rd(in, data.v.data(), data.v.size()) || !rd(in, y.data(), y.size()) ||
        !rd(in, lambdas.data(), lambdas.size()))
        return 2;
    std::fclose(in);
    if (mode) {
        try {
            std::FILE* out = std::fopen(argv[2], "wb");
            if (!out) {
                std::perror(argv[2]);
                return 2;
            }
            const mvtv::mat mesh = mvtv::create_mesh_cpp(data, m);
            if (mode == 2) {
                mvtv::mbs_one_object o;
                mvtv::mbs_one(data, y, m, o, mesh, nullptr, lambdas.at(0));
                const int64_t oh[2] = {int64_t(o.theta_hat.size()), n};
                wr(out, oh, 2);
                wr(out, o.theta_hat.data(), o.theta_hat.size());
                wr(out, o.fitted.data(), o.fitted.size());
            } else {
                mvtv::mbs_one_object o;
                mvtv::mbs_cpp_options opt;
                opt.seed = uint64_t(seed);
                opt.reference_cv = dev == 0;
                mvtv::mbs_cpp_report rep;
                mvtv::mbs(data, y, m, o, &mesh, int(nl), nullptr, given ? &lambdas : nullptr, int(folds), opt, &rep);
                const int64_t oh[4] = {int64_t(rep.lambdas.size()), rep.best, int64_t(o.theta_hat.size()), n};
                wr(out, oh, 4);
                wr(out, &rep.lambda_max, 1);
                wr(out, rep.lambdas.data(), rep.lambdas.size());
                wr(out, rep.mse_mat.v.data(), rep.mse_mat.v.size());
                wr(out, o.theta_hat.data(), o.theta_hat.size());
                wr(out, o.fitted.data(), o.fitted.size());
            }
            std::fclose(out);
        } catch (const std::exception& e) {
            std::fprintf(stderr, "mbs: %s\n", e.what());
            return 1;
        }
        return 0;
    }
    try {
        const auto R = mvtv::mbs_impl(data, y, m, nullptr, int(nl), nullptr, given ? &lambdas : nullptr, int(folds),
                                      false, uint64_t(seed), int(dev));
        std::FILE* out = std::fopen(argv[2], "wb");
        if (!out) {
            std::perror(argv[2]);
            return 2;
        }
        const int64_t N = int64_t(R.best.theta_hat.size());
        const int64_t oh[4] = {int64_t(R.lambdas.size()), R.lambda_minmse_ind, N, n};
        wr(out, oh, 4);
        wr(out, R.lambdas.data(), R.lambdas.size());
        wr(out, R.cv_mses.data(), R.cv_mses.size());
        wr(out, R.final_path.mses.data(), R.final_path.mses.size());
        wr(out, R.best.theta_hat.data(), R.best.theta_hat.size());
        wr(out, R.best.fitted.data(), R.best.fitted.size());
        wr(out, R.residuals.data(), R.residuals.size());
        std::fclose(out);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "mbs_impl: %s\n", e.what());
        return 1;
    }
    return 0;
}

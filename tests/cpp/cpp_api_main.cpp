// Exercises the C++ host API (include/mvtv/solvers.hpp) end to end on the GPU.
#include <cmath>
#include <cstdio>

#include "mvtv/solvers.hpp"

int main() {
    const int n = 800;
    mvtv::mat data(n, 2);
    mvtv::vec y(n);
    unsigned s = 12345;
    auto rnd = [&]() { s = s * 1664525u + 1013904223u; return (s >> 8) / double(1 << 24); };
    for (int i = 0; i < n; ++i) {
        data(i, 0) = rnd();
        data(i, 1) = rnd();
        y[i] = (data(i, 0) > 0.5 && data(i, 1) > 0.5 ? 1.0 : 0.0) + 0.3 * (rnd() - 0.5);
    }
    mvtv::vec m = {12, 12};
    mvtv::mat mesh = mvtv::create_mesh(data, m);
    mvtv::vec deltas = mvtv::create_deltas(data, m);
    mvtv::mbs_cache cache;
    mvtv::create_cache_objects(data, y, mesh, m, deltas, cache);
    mvtv::mbs_object path;
    mvtv::mbs_path(data, y, m, mesh, {1.0, 0.3, 0.1}, y, path, cache);
    // fitted must equal theta at the nearest mesh point
    auto idx = mvtv::nearest_index(data, mesh);
    bool ok = true;
    for (int i = 0; i < n; ++i)
        ok = ok && path.minmse_model.fitted[i] == path.minmse_model.theta_hat[idx[i]];
    size_t best = 0;
    for (size_t i = 0; i < path.mses.size(); ++i)
        if (path.mses[i] == path.minmse) best = i;
    std::printf("n_models %zu best %zu minmse %.17g fitted_ok %d\n", path.models.size(), best, path.minmse, ok ? 1 : 0);
    return 0;
}

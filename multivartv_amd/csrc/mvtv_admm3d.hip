// mvtv_admm3d.hip — z-marching edge kernels for 3-D meshes (the BASELINE 512^3 path).
//
// Same arithmetic as k_edge_update / k_gather in mvtv_kernels.hip (the reference's
// alpha = soft(D theta - u), u += alpha - D theta and D^T alpha, D^T u;
// rcpp-code/MultivarTV/src/solvers.cpp:112-121), but each thread owns one (x, y) column of
// the mesh and walks dim 2, so the dim-2 neighbours every difference needs come from
// registers instead of a second trip to HBM:
//   k_edge3d:   D theta at anchor (x,y,e) reads theta at (x+a, y+b, e+c); the c = 1 plane
//               loaded at step e is the c = 0 plane of step e+1.
//   k_gather3d: D^T v at (x,y,e) is a sum over the backward corners (x-a, y-b, e-c); the
//               in-plane part Q_k(e) of every block whose difference set contains dim 2 is
//               carried to step e+1, which subtracts it (the c = 1 corners).
// The (x+1, y+1) / (x-1, y-1) in-plane neighbours are other lanes' and other waves' own
// cells of the same step, so they are L1/L2 hits. A workgroup is a 64 x 4 column tile over a
// chunk of dim-2 planes; tiles are dealt to XCDs in contiguous runs so a tile's neighbour rows
// sit in the same L2.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "mvtv_device.h"

namespace mvtv {

namespace e3d {
constexpr int TX = 64;
}

struct Edge3dArgs {
    Geom g;
    const double* theta;
    double* edges;
    const double* theta_old;
    double* g_alpha;
    double* g_u;
    const double* g_uprev;
    double* partials;
    double t_old, c_old, t_new;   // edge3d
    double t, c_prev;             // gather3d
    const AdmmCtl* ctl;           // device scalars (asynchronous loop) or nullptr
    int tiles_x, tiles_y, zchunk, nblocks;
    int ty;                       // rows per tile (= waves per workgroup)
    int zlo, zhi;                 // planes processed (g.ibeg / plane .. g.iend / plane)
};

// tile of this workgroup (XCD-aware: XCD b%8 gets a contiguous run of tiles)
struct Tile3 {
    int x, y, z0, z1;
    bool valid;
};
__device__ __forceinline__ Tile3 tile3(const Edge3dArgs& a) {
    Tile3 t{};
    const int bid = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
    t.valid = bid < a.nblocks;
    if (!t.valid) return t;
    const int nt = a.tiles_x * a.tiles_y;
    const int tz = bid / nt, rem = bid - tz * nt;
    const int ty = rem / a.tiles_x, tx = rem - ty * a.tiles_x;
    t.x = tx * e3d::TX + int(threadIdx.x & 63);
    t.y = ty * a.ty + int(threadIdx.x >> 6);
    t.z0 = a.zlo + tz * a.zchunk;
    t.z1 = min(a.zhi, t.z0 + a.zchunk);
    return t;
}

// --------------------------------------------------------------------- edge update
// z_new = D theta - u_old; alpha = soft(z_new, t_new); r = alpha - D theta.
// Reductions: |r|^2, |D theta|^2, |alpha|^2 and (DTH) max |theta - theta_old|.
// NB (blocks of D: 7, or 6 for Python's weighted create_D) is a template parameter so the block
// loop has no branches and every block's loads of a step issue together.
template <int ORD, int UM, bool DTH, int NT, int NB>
__global__ __launch_bounds__(NT) void k_edge3d(const Edge3dArgs a) {
    constexpr int P = 3, NC = 8;
    const Geom& g = a.g;
    double t_old = a.t_old, c_old = a.c_old, t_new = a.t_new;
    if (a.ctl) {
        if (a.ctl->done) return;
        t_old = a.ctl->t_z;
        c_old = a.ctl->c_prev;
        t_new = a.ctl->t_next;
    }
    double red[ER_N] = {0.0, 0.0, 0.0, 0.0};
    const Tile3 T = tile3(a);
    if (T.valid && T.x < int(g.m[0]) && T.y < int(g.m[1])) {
        const uint32_t m0 = g.m[0], pl = g.m[0] * g.m[1];
        const uint32_t xo[2] = {uint32_t(T.x), uint32_t(min(T.x + 1, int(g.m[0]) - 1))};
        const uint32_t yo[2] = {uint32_t(T.y) * m0, uint32_t(min(T.y + 1, int(g.m[1]) - 1)) * m0};
        double th0[4], th1[4];
        auto load_plane = [&](double (&th)[4], int e) {
            const uint32_t zo = uint32_t(e) * pl;
#pragma unroll
            for (int q = 0; q < 4; ++q) th[q] = a.theta[zo + yo[q >> 1] + xo[q & 1]];
        };
        load_plane(th0, T.z0);
        for (int e = T.z0; e < T.z1; ++e) {
            load_plane(th1, min(e + 1, int(g.m[2]) - 1));
            const uint32_t i = uint32_t(e) * pl + yo[0] + xo[0];
            double v[NC];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                v[q] = th0[q];       // corner T = q in dims 0, 1; dim 2 not set
                v[q | 4] = th1[q];   // dim 2 set
            }
            if constexpr (DTH) red[ER_DTH] = fmax(red[ER_DTH], fabs(v[0] - a.theta_old[i]));
            // forward-difference butterfly: v[S] = sum_{T subset S} (-1)^|T| theta(i + e_T)
#pragma unroll
            for (int j = 0; j < P; ++j)
#pragma unroll
                for (int q = 0; q < NC; ++q)
                    if (!((q >> j) & 1)) v[q | (1 << j)] = v[q] - v[q | (1 << j)];
            static_for<0, NB>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                constexpr int S = sprime_mask(block_code(k, P, ORD), P);
                {
                    const double d = g.w[k] * v[S];
                    double* ep = a.edges + eix(g, k, i);
                    const double stored = __builtin_nontemporal_load(ep);
                    const double uo = (UM == U_EXPLICIT) ? stored : -c_old * clampd(stored, t_old);
                    const double z = d - uo;
                    const double al = z - clampd(z, t_new);
                    const double r = al - d;
                    __builtin_nontemporal_store(z, ep);
                    red[ER_R2] = fma(r, r, red[ER_R2]);
                    red[ER_D2] = fma(d, d, red[ER_D2]);
                    red[ER_A2] = fma(al, al, red[ER_A2]);
                }
            });
#pragma unroll
            for (int q = 0; q < 4; ++q) th0[q] = th1[q];
        }
    }
    if (!T.valid)
        for (int k = 0; k < ER_N; ++k) red[k] = 0.0;
    block_reduce_store<ER_N, 1, NT>(red, a.partials);
}

// --------------------------------------------------------------------- D^T gather
// g_alpha = D^T alpha, g_u = D^T u (u unscaled: -clamp(z, t)); explicit mode: g_u = D^T v.
// Reductions: |g_u|^2, |g_u - c_prev g_uprev|^2 (B's dual residual), |g_alpha + c_prev g_uprev|^2 (A's).
template <int ORD, int UM, bool PREV, int NT, int NB>
__global__ __launch_bounds__(NT) void k_gather3d(const Edge3dArgs a) {
    constexpr int P = 3;
    const Geom& g = a.g;
    double tt = a.t, c_prev = a.c_prev;
    if (a.ctl) {
        if (a.ctl->done) return;
        tt = a.ctl->t_next;
        c_prev = a.ctl->c_prev;
    }
    double red[GR_N] = {0.0, 0.0, 0.0};
    const Tile3 T = tile3(a);
    if (T.valid && T.x < int(g.m[0]) && T.y < int(g.m[1])) {
        const uint32_t m0 = g.m[0], pl = g.m[0] * g.m[1];
        const bool okx = T.x > 0, oky = T.y > 0;
        const uint32_t base_xy = uint32_t(T.y) * m0 + uint32_t(T.x);
        // in-plane backward corner q (bit 0: x-1, bit 1: y-1) offset, and whether it exists
        const uint32_t qoff[4] = {0u, okx ? 1u : 0u, oky ? m0 : 0u, (okx ? 1u : 0u) + (oky ? m0 : 0u)};
        const bool qok[4] = {true, okx, oky, okx && oky};
        double qa_prev[7], qu_prev[7];   // Q_k(e-1) of blocks whose S' contains dim 2
#pragma unroll
        for (int k = 0; k < 7; ++k) qa_prev[k] = qu_prev[k] = 0.0;

        // in-plane sums Q_k(e) for alpha and u of block k at plane e
        auto plane_q = [&](auto kc, int e, double& qa, double& qu) {
            constexpr int k = decltype(kc)::value;
            constexpr int S = sprime_mask(block_code(k, P, ORD), P);
            constexpr int SI = S & 3;   // in-plane part of the difference set
            const uint32_t ic = uint32_t(e) * pl + base_xy;
            qa = 0.0;
            qu = 0.0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if ((q & ~SI) != 0) continue;   // corner q subset of S
                const double vv = a.edges[eix(g, k, ic - qoff[q])];
                const double v = qok[q] ? vv : 0.0;
                const bool neg = __builtin_popcount(q) & 1;
                if constexpr (UM == U_FROM_Z) {
                    const double cl = clampd(v, tt);
                    const double al = v - cl;
                    qa = neg ? qa - al : qa + al;
                    qu = neg ? qu + cl : qu - cl;   // u = -clamp
                } else {
                    qu = neg ? qu - v : qu + v;
                }
            }
        };
        if (T.z0 > 0) {   // carried sums of plane z0 - 1
            static_for<0, NB>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                constexpr int S = sprime_mask(block_code(k, P, ORD), P);
                if constexpr ((S & 4) != 0) plane_q(kc, T.z0 - 1, qa_prev[k], qu_prev[k]);
            });
        }
        for (int e = T.z0; e < T.z1; ++e) {
            double ga = 0.0, gu = 0.0;
            static_for<0, NB>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                constexpr int S = sprime_mask(block_code(k, P, ORD), P);
                {
                    double qa, qu;
                    plane_q(kc, e, qa, qu);
                    double ca = qa, cu = qu;
                    if constexpr ((S & 4) != 0) {
                        ca -= qa_prev[k];   // zero at e = 0 (no plane -1)
                        cu -= qu_prev[k];
                        qa_prev[k] = qa;
                        qu_prev[k] = qu;
                    }
                    ga = fma(g.w[k], ca, ga);
                    gu = fma(g.w[k], cu, gu);
                }
            });
            const uint32_t i = uint32_t(e) * pl + base_xy;
            if constexpr (UM == U_FROM_Z) __builtin_nontemporal_store(ga, a.g_alpha + i);
            __builtin_nontemporal_store(gu, a.g_u + i);
            red[GR_GU2] = fma(gu, gu, red[GR_GU2]);
            if constexpr (PREV) {
                const double gp = c_prev * __builtin_nontemporal_load(a.g_uprev + i);
                const double db = gu - gp, da = ga + gp;
                red[GR_S2B] = fma(db, db, red[GR_S2B]);
                red[GR_S2A] = fma(da, da, red[GR_S2A]);
            }
        }
    }
    if (!T.valid)
        for (int k = 0; k < GR_N; ++k) red[k] = 0.0;
    block_reduce_store<GR_N, 0, NT>(red, a.partials);
}

// ------------------------------------------------------------------------------------ launchers
namespace {
int e3d_rows() {
    static const int ty = [] {
        const char* e = probe_env("MVTV_E3D_TY");
        const int v = e ? std::atoi(e) : 4;
        return v == 8 ? 8 : 4;
    }();
    return ty;
}
Edge3dArgs e3d_args(const Geom& g) {
    Edge3dArgs a{};
    a.g = g;
    a.ty = e3d_rows();
    a.zlo = int(g.ibeg / (g.m[0] * g.m[1]));
    a.zhi = int(g.iend / (g.m[0] * g.m[1]));
    a.tiles_x = int((g.m[0] + e3d::TX - 1) / e3d::TX);
    a.tiles_y = int((g.m[1] + a.ty - 1) / a.ty);
    const int tiles = a.tiles_x * a.tiles_y;
    // dim-2 chunks: enough workgroups to fill 256 CUs several times over, long enough marches
    // that the carried plane (gather) and the extra theta plane (edge) are amortised
    static const int want = [] {
        const char* e = probe_env("MVTV_E3D_WG");
        return e ? std::atoi(e) : 8192;
    }();
    const int nzp = std::max(1, a.zhi - a.zlo);
    int nz = std::max(1, std::min(nzp, want / std::max(1, tiles)));
    while (nz > 1 && ((nz * tiles + 7) / 8 * 8) > kMaxCgBlocks) --nz;
    a.zchunk = (nzp + nz - 1) / nz;
    nz = (nzp + a.zchunk - 1) / a.zchunk;
    a.nblocks = tiles * nz;
    return a;
}
}  // namespace

bool edge4d_ok(const Geom& g);
hipError_t launch_edge4d(const Geom& g, int order, int umode, hipStream_t s, const double* theta, double* edges,
                         double t_old, double c_old, double t_new, const double* theta_old, double* partials,
                         int* nparts, const AdmmCtl* ctl);
hipError_t launch_gather4d(const Geom& g, int order, int umode, hipStream_t s, const double* edges, double t,
                           double* g_alpha, double* g_u, const double* g_uprev, double c_prev, double* partials,
                           int* nparts, const AdmmCtl* ctl);
bool gather4_ok(const Geom& g);
hipError_t launch_gather4(const Geom& g, int order, int umode, hipStream_t s, const double* edges, double t,
                          double* g_alpha, double* g_u, const double* g_uprev, double c_prev, double* partials,
                          int* nparts, const AdmmCtl* ctl, double* scratch, bool fold, int passes = 3);

bool edge3d_ok(const Geom& g) {
    if (g.p == 4) return edge4d_ok(g);
    if (g.p != 3 || probe_env("MVTV_E3D_OFF")) return false;
    const Edge3dArgs a = e3d_args(g);
    return (a.nblocks + 7) / 8 * 8 <= kMaxCgBlocks;
}

hipError_t launch_edge3d(const Geom& g, int order, int umode, hipStream_t s, const double* theta, double* edges,
                         double t_old, double c_old, double t_new, const double* theta_old, double* partials,
                         int* nparts, const AdmmCtl* ctl) {
    if (g.p == 4)
        return launch_edge4d(g, order, umode, s, theta, edges, t_old, c_old, t_new, theta_old, partials, nparts, ctl);
    Edge3dArgs a = e3d_args(g);
    a.ctl = ctl;
    a.theta = theta;
    a.edges = edges;
    a.theta_old = theta_old;
    a.partials = partials;
    a.t_old = t_old;
    a.c_old = c_old;
    a.t_new = t_new;
    const int grid = (a.nblocks + 7) / 8 * 8;
    *nparts = grid;
    const bool dth = theta_old != nullptr;
    auto pick = [&](auto ntc) {
        constexpr int NT = decltype(ntc)::value;
        auto go = [&](auto kern) {
            klaunch(kern, dim3(grid), dim3(NT), 0, s, a);
            return hipGetLastError();
        };
        if (order == 0) {
            if (umode == U_EXPLICIT)
                return dth ? go(k_edge3d<0, U_EXPLICIT, true, NT, 7>) : go(k_edge3d<0, U_EXPLICIT, false, NT, 7>);
            return dth ? go(k_edge3d<0, U_FROM_Z, true, NT, 7>) : go(k_edge3d<0, U_FROM_Z, false, NT, 7>);
        }
        if (g.nb == 6) {
            if (umode == U_EXPLICIT)
                return dth ? go(k_edge3d<1, U_EXPLICIT, true, NT, 6>) : go(k_edge3d<1, U_EXPLICIT, false, NT, 6>);
            return dth ? go(k_edge3d<1, U_FROM_Z, true, NT, 6>) : go(k_edge3d<1, U_FROM_Z, false, NT, 6>);
        }
        if (umode == U_EXPLICIT)
            return dth ? go(k_edge3d<1, U_EXPLICIT, true, NT, 7>) : go(k_edge3d<1, U_EXPLICIT, false, NT, 7>);
        return dth ? go(k_edge3d<1, U_FROM_Z, true, NT, 7>) : go(k_edge3d<1, U_FROM_Z, false, NT, 7>);
    };
    if (a.ty == 8) return pick(std::integral_constant<int, 512>{});
    return pick(std::integral_constant<int, 256>{});
}

hipError_t launch_gather3d(const Geom& g, int order, int umode, hipStream_t s, const double* edges, double t,
                           double* g_alpha, double* g_u, const double* g_uprev, double c_prev, double* partials,
                           int* nparts, const AdmmCtl* ctl, double* scratch4, bool fold) {
    if (fold && !(g.p == 4 && scratch4 && ctl && gather4_ok(g))) return hipErrorInvalidValue;   // two-pass 4-D only
    if (g.p == 4) {
        if (scratch4 && gather4_ok(g))
            return launch_gather4(g, order, umode, s, edges, t, g_alpha, g_u, g_uprev, c_prev, partials, nparts, ctl,
                                  scratch4, fold);
        // 4-D: the marching gather (k_gather4d) reads ~65 neighbour words per cell through L1/L2 and
        // measured slower at 128^4 (20.8 vs 18.4 ms) than the grid-stride kernel; opt-in only
        static const bool marching = probe_env("MVTV_G4D") != nullptr;
        if (marching)
            return launch_gather4d(g, order, umode, s, edges, t, g_alpha, g_u, g_uprev, c_prev, partials, nparts, ctl);
        const int grid = int(std::min<uint64_t>((uint64_t(g.N) + kThreads - 1) / kThreads, kMaxGrid));
        *nparts = grid;
        return launch_gather(g, order, umode, Launch{s, grid}, edges, t, g_alpha, g_u, g_uprev, c_prev, partials, ctl);
    }
    Edge3dArgs a = e3d_args(g);
    a.ctl = ctl;
    a.edges = const_cast<double*>(edges);   // read only in k_gather3d
    a.g_alpha = g_alpha;
    a.g_u = g_u;
    a.g_uprev = g_uprev;
    a.partials = partials;
    a.t = t;
    a.c_prev = c_prev;
    const int grid = (a.nblocks + 7) / 8 * 8;
    *nparts = grid;
    const bool prev = g_uprev != nullptr;
    auto pick = [&](auto ntc) {
        constexpr int NT = decltype(ntc)::value;
        auto go = [&](auto kern) {
            klaunch(kern, dim3(grid), dim3(NT), 0, s, a);
            return hipGetLastError();
        };
        if (order == 0) {
            if (umode == U_EXPLICIT)
                return prev ? go(k_gather3d<0, U_EXPLICIT, true, NT, 7>) : go(k_gather3d<0, U_EXPLICIT, false, NT, 7>);
            return prev ? go(k_gather3d<0, U_FROM_Z, true, NT, 7>) : go(k_gather3d<0, U_FROM_Z, false, NT, 7>);
        }
        if (g.nb == 6) {
            if (umode == U_EXPLICIT)
                return prev ? go(k_gather3d<1, U_EXPLICIT, true, NT, 6>) : go(k_gather3d<1, U_EXPLICIT, false, NT, 6>);
            return prev ? go(k_gather3d<1, U_FROM_Z, true, NT, 6>) : go(k_gather3d<1, U_FROM_Z, false, NT, 6>);
        }
        if (umode == U_EXPLICIT)
            return prev ? go(k_gather3d<1, U_EXPLICIT, true, NT, 7>) : go(k_gather3d<1, U_EXPLICIT, false, NT, 7>);
        return prev ? go(k_gather3d<1, U_FROM_Z, true, NT, 7>) : go(k_gather3d<1, U_FROM_Z, false, NT, 7>);
    };
    if (a.ty == 8) return pick(std::integral_constant<int, 512>{});
    return pick(std::integral_constant<int, 256>{});
}

// =============================================================================================
// Fused 3-D pass (k_admm3a below): edge update and D^T gather in ONE pass over the edge state (z read
// once, written once to the ping-pong partner buffer). The gather at (x,y,e) needs z_new at the
// in-plane backward neighbours (x-1, y), (x, y-1), (x-1, y-1) of plane e, which other threads produce
// in the same step, so a workgroup stages z_new of one plane in LDS; halo cells recompute the
// neighbouring tiles' z_new from the previous iterate (never stored), and the dim-2 backward corners
// come from in-plane sums carried from the previous plane, so no plane is ever re-read.
struct Fused3dArgs {
    Geom g;
    const double* theta;
    const double* z_old;
    double* z_new;
    const double* theta_old;
    double* g_alpha;
    double* g_u;
    const double* g_uprev;
    double* partials;
    double t_old, c_old, t_new, c_prev;
    const AdmmCtl* ctl;
    int tiles_x, tiles_y, zchunk, nblocks, zlo, zhi;
    int tpz;          // tiles per z chunk
    int xcd;          // contiguous tile runs per XCD (MVTV_F3D_XCD=0 in a probe build: blockIdx order)
    int fold;         // g_alpha receives s = rho (D^T alpha + D^T u), rho = ctl->rho (the next solve's b = oty + s)
};

// ---------------------------------------------------------------------------------------------
// k_admm3a: tiles aligned to the 64-node chunks of the edge layout (Geom.eaos) and of every N-vector
// row: a tile owns x in [64 t, 64 t + 63], so each wave's z_new, g_alpha and g_u stores are whole
// 512-B runs (four full 128-B lines). (The round-1 kernel owned 63 columns with lane 0 as the x - 1
// halo: its 63-word stores straddled two chunks, 10.3 GB written per launch at 512^3 against 9.66
// here, 3.90 -> 3.49 ms on one box, profiles/r02/v3_*.) The x - 1 column the gather of lane 0 needs is computed by a 16th wave (lanes
// 0..14 = image rows) that recomputes z_new at x = 64 t - 1 (never stored); waves 0..14 hold image
// rows 0..14, row 0 being the y - 1 halo (recomputed, never stored) and rows 1..14 the owned rows.
// The LDS image is 65 columns wide (column 0 = the halo column) and holds only the blocks whose
// difference set has dim 0 or dim 1 (the block with S' = {2} is read by its own cell only, from a
// register).
namespace f3a {
constexpr int IW = 65, IH = 15, TY = IH - 1, NT = 1024;
}

template <int NB, int ORD>
__host__ __device__ constexpr int f3a_nimg() {
    int n = 0;
    for (int k = 0; k < NB; ++k)
        if ((sprime_mask(block_code(k, 3, ORD), 3) & 3) != 0) ++n;
    return n;
}
template <int NB, int ORD>
__host__ __device__ constexpr int f3a_slot(int k) {   // image slot of block k (-1: not in the image)
    int n = 0;
    for (int j = 0; j < k; ++j)
        if ((sprime_mask(block_code(j, 3, ORD), 3) & 3) != 0) ++n;
    return (sprime_mask(block_code(k, 3, ORD), 3) & 3) != 0 ? n : -1;
}

// TW (twin blocks, mvtv_internal.h twin_block): block KD carries the same numbers as block KC (same S', equal weight,
// equal state; the host checks), so it is neither read nor written nor staged: KC's reductions count twice and its
// gather terms enter with weight 2 w. The state's KD region is filled from KC once the run ends.
template <int ORD, int UM, bool DTH, int NB, bool TW>
__device__ __forceinline__ void admm3a_tile(const Fused3dArgs& a, double* __restrict__ szr, double (&red)[7], int X0,
                                            int Yh, int z0, int z1, double t_old, double c_old, double t_new,
                                            double c_prev, double rho_f) {
    constexpr int P = 3, NC = 8, IW = f3a::IW, IH = f3a::IH, NI = f3a_nimg<NB, ORD>();
    static_assert(!TW || twin_block(NB, P, ORD) >= 0, "twin blocks");
    const Geom& g = a.g;
    const int wv = int(threadIdx.x) >> 6, ln = int(threadIdx.x) & 63;
    const bool hcol = wv == IH;                 // the halo-column wave
    const int row = hcol ? ln : wv;
    const int col = hcol ? 0 : ln + 1;
    const int x = hcol ? X0 - 1 : X0 + ln, y = Yh + row;
    const int m0 = int(g.m[0]), m1 = int(g.m[1]), m2 = int(g.m[2]);
    const bool active = row < IH;               // holds an image cell
    const bool cell = active && x >= 0 && y >= 0 && x < m0 && y < m1;   // computes z_new here
    const bool inner = cell && !hcol && row > 0;                       // owns outputs here
    const uint32_t pl = uint32_t(m0) * uint32_t(m1);
    const int xc = min(max(x, 0), m0 - 1), yc = min(max(y, 0), m1 - 1);
    const uint32_t xo[2] = {uint32_t(xc), uint32_t(min(xc + 1, m0 - 1))};
    const uint32_t yo[2] = {uint32_t(yc) * uint32_t(m0), uint32_t(min(yc + 1, m1 - 1)) * uint32_t(m0)};
    const uint32_t ixy = yo[0] + xo[0];
    const bool okx = x > 0, oky = y > 0;
    const bool hrow = row == 0;
    auto sidx = [&](int buf, int slot, int r, int c) { return ((buf * NI + slot) * IH + r) * IW + c; };

    auto load_theta = [&](double (&th)[4], int e) {
        const uint32_t zo = uint32_t(e) * pl;
#pragma unroll
        for (int q = 0; q < 4; ++q) th[q] = cell ? a.theta[zo + yo[q >> 1] + xo[q & 1]] : 0.0;
    };
    // halo cells load only the blocks their neighbours read: row 0 those with dim 1 in S', the halo
    // column those with dim 0, the corner both
    auto load_z = [&](double (&zo)[NB], int e) {
        const uint32_t i = uint32_t(e) * pl + ixy;
        static_for<0, NB>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            constexpr int S = sprime_mask(block_code(k, P, ORD), P);
            const bool need = cell && (!hrow || (S & 2)) && (!hcol || (S & 1));
            if constexpr (TW && twin_of(k, P, ORD) != k) zo[k] = 0.0;
            else zo[k] = need ? a.z_old[eix(g, k, i)] : 0.0;
        });
    };
    auto edge_cell = [&](int e, const double (&th0)[4], const double (&th1)[4], const double (&zo)[NB],
                         double (&zn)[NB], bool own) {
        const uint32_t i = uint32_t(e) * pl + ixy;
        double v[NC];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            v[q] = th0[q];
            v[q | 4] = th1[q];
        }
        if constexpr (DTH)
            if (own) red[3] = fmax(red[3], fabs(v[0] - a.theta_old[i]));
#pragma unroll
        for (int j = 0; j < P; ++j)
#pragma unroll
            for (int q = 0; q < NC; ++q)
                if (!((q >> j) & 1)) v[q | (1 << j)] = v[q] - v[q | (1 << j)];
        static_for<0, NB>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            constexpr int S = sprime_mask(block_code(k, P, ORD), P);
            if constexpr (TW && twin_of(k, P, ORD) != k) {
                zn[k] = 0.0;
            } else {
                const double d = g.w[k] * v[S];
                const double uo = (UM == U_EXPLICIT) ? zo[k] : -c_old * clampd(zo[k], t_old);
                const double z = cell ? d - uo : 0.0;
                zn[k] = z;
                if (own) {
                    const double al = z - clampd(z, t_new);
                    const double r = al - d;
                    __builtin_nontemporal_store(z, a.z_new + eix(g, k, i));
                    constexpr double m = TW ? double(twin_count(k, NB, P, ORD)) : 1.0;   // the twins' rows: the same terms
                    red[0] = fma(m * r, r, red[0]);
                    red[1] = fma(m * d, d, red[1]);
                    red[2] = fma(m * al, al, red[2]);
                }
            }
        });
    };
    auto to_image = [&](int buf, const double (&zn)[NB]) {
        if (!active) return;
        static_for<0, NB>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            constexpr int sl = f3a_slot<NB, ORD>(k);
            if constexpr (sl >= 0 && !(TW && twin_of(k, P, ORD) != k)) szr[sidx(buf, sl, row, col)] = zn[k];
        });
    };
    // in-plane backward sums Q_k of an owned cell: its own value from the register, the neighbours
    // (x-1, y), (x, y-1), (x-1, y-1) from the image
    auto plane_q = [&](auto kc, int buf, double own_z, double& qa, double& qu) {
        constexpr int k = decltype(kc)::value;
        constexpr int S = sprime_mask(block_code(k, P, ORD), P);
        constexpr int SI = S & 3;
        constexpr int sl = f3a_slot<NB, ORD>(k);
        qa = 0.0;
        qu = 0.0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if ((q & ~SI) != 0) continue;
            double v;
            if (q == 0) {
                v = own_z;
            } else {
                const bool ok = (!(q & 1) || okx) && (!(q & 2) || oky);
                if constexpr (sl >= 0) v = ok ? szr[sidx(buf, sl, row - ((q >> 1) & 1), col - (q & 1))] : 0.0;
                else v = 0.0;
            }
            const bool neg = __builtin_popcount(q) & 1;
            const double cl = clampd(v, t_new);
            const double al = v - cl;
            qa = neg ? qa - al : qa + al;
            qu = neg ? qu + cl : qu - cl;   // u = -clamp
        }
    };
    double qa_prev = 0.0, qu_prev = 0.0;
    double th0[4], th1[4], zo[NB], zn[NB];
    if (z0 > 0) {   // carried sums of plane z0 - 1: recompute its z_new from the old state
        load_theta(th0, z0 - 1);
        load_theta(th1, z0);
        load_z(zo, z0 - 1);
        edge_cell(z0 - 1, th0, th1, zo, zn, false);
        to_image(1, zn);
        lds_barrier();
        if (inner) {
            static_for<0, NB>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                constexpr int S = sprime_mask(block_code(k, P, ORD), P);
                if constexpr ((S & 4) != 0 && !(TW && twin_of(k, P, ORD) != k)) {
                    constexpr double mk = TW ? double(twin_count(k, NB, P, ORD)) : 1.0;   // exact for 2
                    double qa, qu;
                    plane_q(kc, 1, zn[k], qa, qu);
                    qa_prev = fma(mk * g.w[k], qa, qa_prev);
                    qu_prev = fma(mk * g.w[k], qu, qu_prev);
                }
            });
        }
        lds_barrier();
    }
    load_theta(th0, z0);
    load_theta(th1, min(z0 + 1, m2 - 1));
    load_z(zo, z0);
    double gp = inner ? __builtin_nontemporal_load(a.g_uprev + uint32_t(z0) * pl + ixy) : 0.0;
    for (int e = z0; e < z1; ++e) {
        const int buf = (e - z0) & 1;
        edge_cell(e, th0, th1, zo, zn, inner);
        to_image(buf, zn);
        double nth[4], nzo[NB], ngp = 0.0;   // prefetch step e+1 while this step's gather runs
        if (e + 1 < z1) {
            load_theta(nth, min(e + 2, m2 - 1));
            load_z(nzo, e + 1);
            ngp = inner ? __builtin_nontemporal_load(a.g_uprev + uint32_t(e + 1) * pl + ixy) : 0.0;
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) nth[q] = 0.0;
#pragma unroll
            for (int k = 0; k < NB; ++k) nzo[k] = 0.0;
        }
        lds_barrier();
        if (inner) {
            double ga = 0.0, gu = 0.0, na = 0.0, nu = 0.0;
            static_for<0, NB>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                constexpr int S = sprime_mask(block_code(k, P, ORD), P);
                if constexpr (!(TW && twin_of(k, P, ORD) != k)) {
                    constexpr double mk = TW ? double(twin_count(k, NB, P, ORD)) : 1.0;
                    const double wk = mk * g.w[k];
                    double qa, qu;
                    plane_q(kc, buf, zn[k], qa, qu);
                    ga = fma(wk, qa, ga);
                    gu = fma(wk, qu, gu);
                    if constexpr ((S & 4) != 0) {
                        na = fma(wk, qa, na);
                        nu = fma(wk, qu, nu);
                    }
                }
            });
            ga -= qa_prev;
            gu -= qu_prev;
            qa_prev = na;
            qu_prev = nu;
            const uint32_t i = uint32_t(e) * pl + ixy;
            __builtin_nontemporal_store(a.fold ? rho_f * (ga + gu) : ga, a.g_alpha + i);
            __builtin_nontemporal_store(gu, a.g_u + i);
            const double gpc = c_prev * gp;
            const double db = gu - gpc, da = ga + gpc;
            red[4] = fma(gu, gu, red[4]);
            red[5] = fma(db, db, red[5]);
            red[6] = fma(da, da, red[6]);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            th0[q] = th1[q];
            th1[q] = nth[q];
        }
#pragma unroll
        for (int k = 0; k < NB; ++k) zo[k] = nzo[k];
        gp = ngp;
    }
}

template <int ORD, int UM, bool DTH, int NB, bool TW>
__global__ __launch_bounds__(f3a::NT) void k_admm3a(const Fused3dArgs a) {
    constexpr int NT = f3a::NT, NI = f3a_nimg<NB, ORD>();
    double t_old = a.t_old, c_old = a.c_old, t_new = a.t_new, c_prev = a.c_prev, rho_f = 0.0;
    if (a.ctl) {
        if (a.ctl->done) return;
        t_old = a.ctl->t_z;
        c_old = a.ctl->c_prev;
        t_new = a.ctl->t_next;
        c_prev = a.ctl->c_prev;
        rho_f = a.ctl->rho;
    }
    __shared__ double szr[2 * NI * f3a::IH * f3a::IW];
    double red[7] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    const int bid = a.xcd ? int((blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3)) : int(blockIdx.x);
    const bool valid = bid < a.nblocks;
    if (valid) {
        const int tz = bid / a.tpz, rem = bid - tz * a.tpz;
        const int z0 = a.zlo + tz * a.zchunk, z1 = min(a.zhi, z0 + a.zchunk);
        const int tyi = rem / a.tiles_x, txi = rem - tyi * a.tiles_x;
        admm3a_tile<ORD, UM, DTH, NB, TW>(a, szr, red, txi * 64, tyi * f3a::TY - 1, z0, z1, t_old, c_old, t_new,
                                          c_prev, rho_f);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
#pragma unroll
        for (int k = 0; k < 7; ++k) {
            const double o = __shfl_down(red[k], off, 64);
            red[k] = k == 3 ? fmax(red[k], o) : red[k] + o;
        }
    }
    __shared__ double rs[NT / 64][7];
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0)
        for (int k = 0; k < 7; ++k) rs[w][k] = valid ? red[k] : 0.0;
    __syncthreads();
    if (threadIdx.x < 7) {
        const int k = threadIdx.x;
        double acc = rs[0][k];
        for (int ww = 1; ww < NT / 64; ++ww) acc = k == 3 ? fmax(acc, rs[ww][k]) : acc + rs[ww][k];
        a.partials[blockIdx.x * 7 + k] = acc;
    }
}

namespace {
// compute units of the current device (the fused kernel's concurrent workgroups: one per CU)
int device_cus() {
    static thread_local int dev = -1, cus = 256;
    int d = 0;
    if (hipGetDevice(&d) == hipSuccess && d != dev) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, d) == hipSuccess && prop.multiProcessorCount > 0) cus = prop.multiProcessorCount;
        dev = d;
    }
    return cus;
}

Fused3dArgs f3d_args(const Geom& g) {
    Fused3dArgs a{};
    a.g = g;
    a.zlo = int(g.ibeg / (g.m[0] * g.m[1]));
    a.zhi = int(g.iend / (g.m[0] * g.m[1]));
    const char* xe = probe_env("MVTV_F3D_XCD");
    a.xcd = !xe || std::atoi(xe) != 0;
    a.tiles_x = int((g.m[0] + 63) / 64);
    a.tiles_y = int((int(g.m[1]) + f3a::TY - 1) / f3a::TY);
    a.tpz = a.tiles_x * a.tiles_y;
    const int tiles = a.tpz;
    // dim-2 chunks. A workgroup (1024 threads, 94 KB of LDS: one per CU) marches zc planes and recomputes
    // one at its start, so the launch costs ~ waves x (zc + 1 + c0), waves = ceil(workgroups / CUs). Among
    // chunkings of <= 32 planes that give >= 2.5 waves (fewer leave the tail of the last wave exposed; longer
    // chunks measured slower at 512^3: 6 chunks of 86 planes 2 % behind 16 of 32, round 1) the one minimising
    // that cost with c0 = 1; tiny meshes: the cheapest of all. Measured per setting in one process
    // (tools/zchunk_probe.py, profiles/r03/v2_zchunk): 256^3 0.549 ms at the old ~4096-workgroup target
    // (5-plane chunks) -> 0.488 ms (26 planes, 760 workgroups); a 512^3 slab rank of 64 planes (8 GPUs)
    // 0.59 -> 0.513 ms (16 planes); 512^3 unchanged (32 planes, 3.53 ms, the best of six settings).
    const char* wge = probe_env("MVTV_F3D_WG");   // read per launch set-up: the probe varies it
    const int nzp = std::max(1, a.zhi - a.zlo);
    int nz = 1;
    if (wge) {
        nz = std::max(1, std::min(nzp, std::atoi(wge) / std::max(1, tiles)));
    } else {
        const int cus = device_cus();
        auto cost_of = [&](int nzr, int zc) { return ((long(tiles) * nzr + cus - 1) / cus) * (zc + 2); };
        for (int pass = 0; pass < 2 && nz == 1; ++pass) {
            auto ok = [&](int nzr, int zc) { return pass == 1 || (zc <= 32 && 2L * tiles * nzr >= 5L * cus); };
            long best = -1;
            for (int c = 1; c <= nzp; ++c) {
                const int zc = (nzp + c - 1) / c, nzr = (nzp + zc - 1) / zc;
                if (nzr == c && ok(nzr, zc) && (best < 0 || cost_of(nzr, zc) < best)) best = cost_of(nzr, zc);
            }
            // the longest chunks within 2 % of the cheapest (the model's resolution)
            for (int c = 1; c <= nzp && best >= 0; ++c) {
                const int zc = (nzp + c - 1) / c, nzr = (nzp + zc - 1) / zc;
                if (nzr == c && ok(nzr, zc) && 50 * cost_of(nzr, zc) <= 51 * best) {
                    nz = nzr;
                    break;
                }
            }
        }
    }
    while (nz > 1 && ((nz * tiles + 7) / 8 * 8) * 7 > kMaxCgBlocks * kMaxRed) --nz;
    a.zchunk = (nzp + nz - 1) / nz;
    nz = (nzp + a.zchunk - 1) / a.zchunk;
    a.nblocks = tiles * nz;
    return a;
}
}  // namespace

bool fused2d_ok(const Geom& g);
hipError_t launch_admm2d(const Geom& g, int order, int umode, hipStream_t s, const double* theta, const double* z_old,
                         double* z_new, double t_old, double c_old, double t_new, double c_prev,
                         const double* theta_old, double* g_alpha, double* g_u, const double* g_uprev,
                         double* partials, int* nparts, const AdmmCtl* ctl, bool fold);

bool fused3d_ok(const Geom& g) {
    if (g.p == 2) return fused2d_ok(g);
    if (g.p != 3 || probe_env("MVTV_F3D_OFF")) return false;
    const Fused3dArgs a = f3d_args(g);
    return ((a.nblocks + 7) / 8 * 8) * 7 <= kMaxCgBlocks * kMaxRed;
}

hipError_t launch_admm3d(const Geom& g, int order, int umode, hipStream_t s, const double* theta, const double* z_old,
                         double* z_new, double t_old, double c_old, double t_new, double c_prev,
                         const double* theta_old, double* g_alpha, double* g_u, const double* g_uprev,
                         double* partials, int* nparts, const AdmmCtl* ctl, bool fold, bool twin) {
    if (fold && ((g.p != 2 && g.p != 3) || !ctl)) return hipErrorInvalidValue;   // the folded b: asynchronous loop
    if (twin && (g.p != 3 || !twin_weights_equal(g, order)))   // twins must carry one weight (the host checks the state)
        return hipErrorInvalidValue;
    if (g.p == 2)
        return launch_admm2d(g, order, umode, s, theta, z_old, z_new, t_old, c_old, t_new, c_prev, theta_old, g_alpha,
                             g_u, g_uprev, partials, nparts, ctl, fold);
    Fused3dArgs a = f3d_args(g);
    a.theta = theta;
    a.z_old = z_old;
    a.z_new = z_new;
    a.theta_old = theta_old;
    a.g_alpha = g_alpha;
    a.g_u = g_u;
    a.g_uprev = g_uprev;
    a.partials = partials;
    a.t_old = t_old;
    a.c_old = c_old;
    a.t_new = t_new;
    a.c_prev = c_prev;
    a.ctl = ctl;
    a.fold = fold ? 1 : 0;
    const int grid = (a.nblocks + 7) / 8 * 8;
    *nparts = grid;
    const bool dth = theta_old != nullptr;
    auto go = [&](auto kern) {
        klaunch(kern, dim3(grid), dim3(f3a::NT), 0, s, a);
        return hipGetLastError();
    };
    auto pick = [&](auto ordc, auto nbc, auto twc) {
        constexpr int O = decltype(ordc)::value, NB = decltype(nbc)::value;
        constexpr bool T = decltype(twc)::value;
        if (umode == U_EXPLICIT)
            return dth ? go(k_admm3a<O, U_EXPLICIT, true, NB, T>) : go(k_admm3a<O, U_EXPLICIT, false, NB, T>);
        return dth ? go(k_admm3a<O, U_FROM_Z, true, NB, T>) : go(k_admm3a<O, U_FROM_Z, false, NB, T>);
    };
    using std::integral_constant;
    using T1 = integral_constant<bool, true>;
    using T0 = integral_constant<bool, false>;
    if (order == 0)
        return twin ? pick(integral_constant<int, 0>{}, integral_constant<int, 7>{}, T1{})
                    : pick(integral_constant<int, 0>{}, integral_constant<int, 7>{}, T0{});
    if (g.nb == 6)
        return twin ? pick(integral_constant<int, 1>{}, integral_constant<int, 6>{}, T1{})
                    : pick(integral_constant<int, 1>{}, integral_constant<int, 6>{}, T0{});
    return twin ? pick(integral_constant<int, 1>{}, integral_constant<int, 7>{}, T1{})
                : pick(integral_constant<int, 1>{}, integral_constant<int, 7>{}, T0{});
}

// Fill block kdst of an edge state from block ksrc at nodes [i0, i1) (the twin block after a run that skipped it)
__global__ __launch_bounds__(256) void k_edges_copy_block(const Geom g, double* __restrict__ edges, int kdst, int ksrc,
                                                          uint32_t i0, uint32_t i1) {
    for (uint32_t i = i0 + blockIdx.x * 256u + threadIdx.x; i < i1; i += gridDim.x * 256u)
        edges[eix(g, kdst, i)] = edges[eix(g, ksrc, i)];
}

hipError_t launch_edges_copy_block(const Geom& g, hipStream_t s, double* edges, int kdst, int ksrc, uint32_t i0,
                                   uint32_t i1) {
    i1 = std::min(i1, g.N);
    if (i0 >= i1) return hipSuccess;
    const uint32_t blocks = std::min<uint32_t>((i1 - i0 + 255u) / 256u, 4096u);
    klaunch(k_edges_copy_block, dim3(std::max(blocks, 1u)), dim3(256), 0, s, g, edges, kdst, ksrc, i0, i1);
    return hipGetLastError();
}

// fill every twin block of the state from its group's first block at nodes [i0, i1): after a run that skipped the
// twins (the whole state), or before a 4-D slab rank hands its last plane to the next rank (whose ghost-plane pass A
// reads every block)
hipError_t fill_twins(const Geom& g, int order, hipStream_t s, double* edges, uint32_t i0, uint32_t i1) {
    for (int k = 0; k < g.nb; ++k) {
        const int c = twin_of(k, g.p, order);
        if (c != k) {
            const hipError_t e = launch_edges_copy_block(g, s, edges, k, c, i0, i1);
            if (e != hipSuccess) return e;
        }
    }
    return hipSuccess;
}

// =============================================================================================
// 4-D (config 5, 128^4): the same marching scheme one dimension up. A thread owns an (x, y, z)
// cell of the 3-D "plane" of dims 0..2 and walks dim 3; its in-plane neighbours (x+1, y+1, z+1
// for D, x-1, y-1, z-1 for D^T) are other threads' own cells of the same step (L1/L2 hits), the
// dim-3 neighbours come from registers (carried theta plane / carried backward sums).
struct Edge4dArgs {
    Geom g;
    const double* theta;
    double* edges;
    const double* theta_old;
    double* g_alpha;
    double* g_u;
    const double* g_uprev;
    double* partials;
    double t_old, c_old, t_new, t, c_prev;
    const AdmmCtl* ctl;
    int tiles_x, tiles_y, tiles_z, wchunk, nblocks, wlo, whi;
};
namespace e4d {
constexpr int TX = 64, TY = 4, NT = TX * TY;
}
struct Tile4 {
    int x, y, z, w0, w1;
    bool valid;
};
__device__ __forceinline__ Tile4 tile4(const Edge4dArgs& a) {
    Tile4 t{};
    const int bid = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
    t.valid = bid < a.nblocks;
    if (!t.valid) return t;
    const int nt = a.tiles_x * a.tiles_y * a.tiles_z;
    const int tw = bid / nt;
    int rem = bid - tw * nt;
    const int tz = rem / (a.tiles_x * a.tiles_y);
    rem -= tz * a.tiles_x * a.tiles_y;
    const int ty = rem / a.tiles_x, tx = rem - ty * a.tiles_x;
    t.x = tx * e4d::TX + int(threadIdx.x & 63);
    t.y = ty * e4d::TY + int(threadIdx.x >> 6);
    t.z = tz;
    t.w0 = a.wlo + tw * a.wchunk;
    t.w1 = min(a.whi, t.w0 + a.wchunk);
    return t;
}

template <int ORD, int UM, bool DTH, int NB>
__global__ __launch_bounds__(e4d::NT) void k_edge4d(const Edge4dArgs a) {
    constexpr int P = 4, NC = 16, PC = 8;
    const Geom& g = a.g;
    double t_old = a.t_old, c_old = a.c_old, t_new = a.t_new;
    if (a.ctl) {
        if (a.ctl->done) return;
        t_old = a.ctl->t_z;
        c_old = a.ctl->c_prev;
        t_new = a.ctl->t_next;
    }
    double red[ER_N] = {0.0, 0.0, 0.0, 0.0};
    const Tile4 T = tile4(a);
    if (T.valid && T.x < int(g.m[0]) && T.y < int(g.m[1])) {
        const uint32_t m0 = g.m[0], m01 = g.m[0] * g.m[1], pl = m01 * g.m[2];
        const uint32_t xo[2] = {uint32_t(T.x), uint32_t(min(T.x + 1, int(g.m[0]) - 1))};
        const uint32_t yo[2] = {uint32_t(T.y) * m0, uint32_t(min(T.y + 1, int(g.m[1]) - 1)) * m0};
        const uint32_t zo[2] = {uint32_t(T.z) * m01, uint32_t(min(T.z + 1, int(g.m[2]) - 1)) * m01};
        double th0[PC], th1[PC];
        auto load_plane = [&](double (&th)[PC], int w) {
            const uint32_t wo = uint32_t(w) * pl;
#pragma unroll
            for (int q = 0; q < PC; ++q) th[q] = a.theta[wo + zo[(q >> 2) & 1] + yo[(q >> 1) & 1] + xo[q & 1]];
        };
        load_plane(th0, T.w0);
        for (int w = T.w0; w < T.w1; ++w) {
            load_plane(th1, min(w + 1, int(g.m[3]) - 1));
            const uint32_t i = uint32_t(w) * pl + zo[0] + yo[0] + xo[0];
            double v[NC];
#pragma unroll
            for (int q = 0; q < PC; ++q) {
                v[q] = th0[q];
                v[q | PC] = th1[q];
            }
            if constexpr (DTH) red[ER_DTH] = fmax(red[ER_DTH], fabs(v[0] - a.theta_old[i]));
#pragma unroll
            for (int j = 0; j < P; ++j)
#pragma unroll
                for (int q = 0; q < NC; ++q)
                    if (!((q >> j) & 1)) v[q | (1 << j)] = v[q] - v[q | (1 << j)];
            static_for<0, NB>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                constexpr int S = sprime_mask(block_code(k, P, ORD), P);
                const double d = g.w[k] * v[S];
                double* ep = a.edges + eix(g, k, i);
                const double stored = __builtin_nontemporal_load(ep);
                const double uo = (UM == U_EXPLICIT) ? stored : -c_old * clampd(stored, t_old);
                const double z = d - uo;
                const double al = z - clampd(z, t_new);
                const double r = al - d;
                __builtin_nontemporal_store(z, ep);
                red[ER_R2] = fma(r, r, red[ER_R2]);
                red[ER_D2] = fma(d, d, red[ER_D2]);
                red[ER_A2] = fma(al, al, red[ER_A2]);
            });
#pragma unroll
            for (int q = 0; q < PC; ++q) th0[q] = th1[q];
        }
    }
    if (!T.valid)
        for (int k = 0; k < ER_N; ++k) red[k] = 0.0;
    block_reduce_store<ER_N, 1, e4d::NT>(red, a.partials);
}

template <int ORD, int UM, bool PREV, int NB>
__global__ __launch_bounds__(e4d::NT) void k_gather4d(const Edge4dArgs a) {
    constexpr int P = 4, PC = 8;
    const Geom& g = a.g;
    double tt = a.t, c_prev = a.c_prev;
    if (a.ctl) {
        if (a.ctl->done) return;
        tt = a.ctl->t_next;
        c_prev = a.ctl->c_prev;
    }
    double red[GR_N] = {0.0, 0.0, 0.0};
    const Tile4 T = tile4(a);
    if (T.valid && T.x < int(g.m[0]) && T.y < int(g.m[1])) {
        const uint32_t m0 = g.m[0], m01 = g.m[0] * g.m[1], pl = m01 * g.m[2];
        const bool okx = T.x > 0, oky = T.y > 0, okz = T.z > 0;
        const uint32_t base = uint32_t(T.z) * m01 + uint32_t(T.y) * m0 + uint32_t(T.x);
        uint32_t qoff[PC];
        bool qok[PC];
#pragma unroll
        for (int q = 0; q < PC; ++q) {
            const bool bx = q & 1, by = (q >> 1) & 1, bz = (q >> 2) & 1;
            qok[q] = (!bx || okx) && (!by || oky) && (!bz || okz);
            qoff[q] = qok[q] ? (bx ? 1u : 0u) + (by ? m0 : 0u) + (bz ? m01 : 0u) : 0u;
        }
        double qa_prev[NB], qu_prev[NB];
#pragma unroll
        for (int k = 0; k < NB; ++k) qa_prev[k] = qu_prev[k] = 0.0;
        auto plane_q = [&](auto kc, int w, double& qa, double& qu) {
            constexpr int k = decltype(kc)::value;
            constexpr int S = sprime_mask(block_code(k, P, ORD), P);
            constexpr int SI = S & 7;
            const uint32_t ib = uint32_t(w) * pl + base;
            qa = 0.0;
            qu = 0.0;
#pragma unroll
            for (int q = 0; q < PC; ++q) {
                if ((q & ~SI) != 0) continue;
                const double vv = a.edges[eix(g, k, ib - qoff[q])];
                const double v = qok[q] ? vv : 0.0;
                const bool neg = __builtin_popcount(q) & 1;
                if constexpr (UM == U_FROM_Z) {
                    const double cl = clampd(v, tt);
                    const double al = v - cl;
                    qa = neg ? qa - al : qa + al;
                    qu = neg ? qu + cl : qu - cl;
                } else {
                    qu = neg ? qu - v : qu + v;
                }
            }
        };
        if (T.w0 > 0) {
            static_for<0, NB>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                constexpr int S = sprime_mask(block_code(k, P, ORD), P);
                if constexpr ((S & 8) != 0) plane_q(kc, T.w0 - 1, qa_prev[k], qu_prev[k]);
            });
        }
        for (int w = T.w0; w < T.w1; ++w) {
            double ga = 0.0, gu = 0.0;
            static_for<0, NB>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                constexpr int S = sprime_mask(block_code(k, P, ORD), P);
                double qa, qu;
                plane_q(kc, w, qa, qu);
                double ca = qa, cu = qu;
                if constexpr ((S & 8) != 0) {
                    ca -= qa_prev[k];
                    cu -= qu_prev[k];
                    qa_prev[k] = qa;
                    qu_prev[k] = qu;
                }
                ga = fma(g.w[k], ca, ga);
                gu = fma(g.w[k], cu, gu);
            });
            const uint32_t i = uint32_t(w) * pl + base;
            if constexpr (UM == U_FROM_Z) __builtin_nontemporal_store(ga, a.g_alpha + i);
            __builtin_nontemporal_store(gu, a.g_u + i);
            red[GR_GU2] = fma(gu, gu, red[GR_GU2]);
            if constexpr (PREV) {
                const double gp = c_prev * __builtin_nontemporal_load(a.g_uprev + i);
                const double db = gu - gp, da = ga + gp;
                red[GR_S2B] = fma(db, db, red[GR_S2B]);
                red[GR_S2A] = fma(da, da, red[GR_S2A]);
            }
        }
    }
    if (!T.valid)
        for (int k = 0; k < GR_N; ++k) red[k] = 0.0;
    block_reduce_store<GR_N, 0, e4d::NT>(red, a.partials);
}

namespace {
Edge4dArgs e4d_args(const Geom& g) {
    Edge4dArgs a{};
    a.g = g;
    const uint32_t pl = g.m[0] * g.m[1] * g.m[2];
    a.wlo = int(g.ibeg / pl);
    a.whi = int(g.iend / pl);
    a.tiles_x = int((g.m[0] + e4d::TX - 1) / e4d::TX);
    a.tiles_y = int((g.m[1] + e4d::TY - 1) / e4d::TY);
    a.tiles_z = int(g.m[2]);
    const int tiles = a.tiles_x * a.tiles_y * a.tiles_z;
    const int nwp = std::max(1, a.whi - a.wlo);
    int nw = std::max(1, std::min(nwp, 8192 / std::max(1, tiles)));
    while (nw > 1 && ((nw * tiles + 7) / 8 * 8) > kMaxCgBlocks) --nw;
    a.wchunk = (nwp + nw - 1) / nw;
    nw = (nwp + a.wchunk - 1) / a.wchunk;
    a.nblocks = tiles * nw;
    return a;
}
}  // namespace

bool edge4d_ok(const Geom& g) {
    if (g.p != 4 || probe_env("MVTV_E3D_OFF")) return false;
    const Edge4dArgs a = e4d_args(g);
    return (a.nblocks + 7) / 8 * 8 <= kMaxCgBlocks;
}

hipError_t launch_edge4d(const Geom& g, int order, int umode, hipStream_t s, const double* theta, double* edges,
                         double t_old, double c_old, double t_new, const double* theta_old, double* partials,
                         int* nparts, const AdmmCtl* ctl) {
    Edge4dArgs a = e4d_args(g);
    a.theta = theta;
    a.edges = edges;
    a.theta_old = theta_old;
    a.partials = partials;
    a.t_old = t_old;
    a.c_old = c_old;
    a.t_new = t_new;
    a.ctl = ctl;
    const int grid = (a.nblocks + 7) / 8 * 8;
    *nparts = grid;
    const bool dth = theta_old != nullptr;
    auto go = [&](auto kern) {
        klaunch(kern, dim3(grid), dim3(e4d::NT), 0, s, a);
        return hipGetLastError();
    };
    if (order == 0) {
        if (umode == U_EXPLICIT) return dth ? go(k_edge4d<0, U_EXPLICIT, true, 15>) : go(k_edge4d<0, U_EXPLICIT, false, 15>);
        return dth ? go(k_edge4d<0, U_FROM_Z, true, 15>) : go(k_edge4d<0, U_FROM_Z, false, 15>);
    }
    if (g.nb == 14) {
        if (umode == U_EXPLICIT) return dth ? go(k_edge4d<1, U_EXPLICIT, true, 14>) : go(k_edge4d<1, U_EXPLICIT, false, 14>);
        return dth ? go(k_edge4d<1, U_FROM_Z, true, 14>) : go(k_edge4d<1, U_FROM_Z, false, 14>);
    }
    if (umode == U_EXPLICIT) return dth ? go(k_edge4d<1, U_EXPLICIT, true, 15>) : go(k_edge4d<1, U_EXPLICIT, false, 15>);
    return dth ? go(k_edge4d<1, U_FROM_Z, true, 15>) : go(k_edge4d<1, U_FROM_Z, false, 15>);
}

hipError_t launch_gather4d(const Geom& g, int order, int umode, hipStream_t s, const double* edges, double t,
                           double* g_alpha, double* g_u, const double* g_uprev, double c_prev, double* partials,
                           int* nparts, const AdmmCtl* ctl) {
    Edge4dArgs a = e4d_args(g);
    a.edges = const_cast<double*>(edges);   // read only in k_gather4d
    a.g_alpha = g_alpha;
    a.g_u = g_u;
    a.g_uprev = g_uprev;
    a.partials = partials;
    a.t = t;
    a.c_prev = c_prev;
    a.ctl = ctl;
    const int grid = (a.nblocks + 7) / 8 * 8;
    *nparts = grid;
    const bool prev = g_uprev != nullptr;
    auto go = [&](auto kern) {
        klaunch(kern, dim3(grid), dim3(e4d::NT), 0, s, a);
        return hipGetLastError();
    };
    if (order == 0) {
        if (umode == U_EXPLICIT) return prev ? go(k_gather4d<0, U_EXPLICIT, true, 15>) : go(k_gather4d<0, U_EXPLICIT, false, 15>);
        return prev ? go(k_gather4d<0, U_FROM_Z, true, 15>) : go(k_gather4d<0, U_FROM_Z, false, 15>);
    }
    if (g.nb == 14) {
        if (umode == U_EXPLICIT) return prev ? go(k_gather4d<1, U_EXPLICIT, true, 14>) : go(k_gather4d<1, U_EXPLICIT, false, 14>);
        return prev ? go(k_gather4d<1, U_FROM_Z, true, 14>) : go(k_gather4d<1, U_FROM_Z, false, 14>);
    }
    if (umode == U_EXPLICIT) return prev ? go(k_gather4d<1, U_EXPLICIT, true, 15>) : go(k_gather4d<1, U_EXPLICIT, false, 15>);
    return prev ? go(k_gather4d<1, U_FROM_Z, true, 15>) : go(k_gather4d<1, U_FROM_Z, false, 15>);
}

// ---------------------------------------------------------------------------------------------
// 4-D gather in two passes (default for p = 4). D^T is separable per block: the dim-3 (w) backward
// difference factors out, D^T(alpha) = G0 + (1 - s_w) Gw, where G0 / Gw sum the (x, y, z) gathers
// of the blocks without / with dim 3 in S'. Pass A marches dim 2 at a fixed w like k_gather3d
// (x-1, y-1 from L1/L2, z-1 from carried sums) and writes G0 and Gw (alpha and u parts); pass B
// walks w with Gw(w-1) in registers and forms g_alpha, g_u and the dual-residual sums. Both passes
// stream; no neighbour along dim 3 (16 MB away at 128^4) is ever re-read from HBM.
struct Gather4Args {
    Geom g;
    const double* edges;
    double* s0a;     // G0 alpha / u and Gw alpha / u: 4 N-arrays of scratch
    double* s0u;
    double* swa;
    double* swu;
    double* g_alpha;
    double* g_u;
    const double* g_uprev;
    double* partials;
    double t, c_prev;
    const AdmmCtl* ctl;
    int fold;        // pass B stores s = rho (g_alpha + g_u) in g_alpha (the folded right-hand side)
    int tiles_x, tiles_y, zchunk, nzc, nblocks, wa, wb;   // pass A: planes w in [wa, wb)
    int wlo, whi, wchunk, nwc, n3, nblocks_b;            // pass B: owned planes [wlo, whi)
};
namespace g4 {
constexpr int TX = 64, NTB = 256;   // pass A: 64-column tiles of g4_ty() rows; pass B: 256 threads
}

template <int ORD, int UM, int NB, int TYV>
__global__ __launch_bounds__(64 * TYV) void k_gather4a(const Gather4Args a) {
    constexpr int P = 4;
    const Geom& g = a.g;
    double tt = a.t;
    if (a.ctl) {
        if (a.ctl->done) return;
        tt = a.ctl->t_next;
    }
    const int bid = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
    if (bid >= a.nblocks) return;
    const int nt = a.tiles_x * a.tiles_y;
    const int tw = bid / (nt * a.nzc);
    int rem = bid - tw * nt * a.nzc;
    const int tz = rem / nt;
    rem -= tz * nt;
    const int ty = rem / a.tiles_x, tx = rem - ty * a.tiles_x;
    const int x = tx * g4::TX + int(threadIdx.x & 63), y = ty * TYV + int(threadIdx.x >> 6);
    const int w = a.wa + tw;
    const int z0 = tz * a.zchunk, z1 = min(int(g.m[2]), z0 + a.zchunk);
    if (x >= int(g.m[0]) || y >= int(g.m[1])) return;
    const uint32_t m0 = g.m[0], m01 = g.m[0] * g.m[1], pl = m01 * g.m[2];
    const bool okx = x > 0, oky = y > 0;
    const uint32_t base = uint32_t(w) * pl + uint32_t(y) * m0 + uint32_t(x);
    const uint32_t qoff[4] = {0u, okx ? 1u : 0u, oky ? m0 : 0u, (okx ? 1u : 0u) + (oky ? m0 : 0u)};
    const bool qok[4] = {true, okx, oky, okx && oky};
    // the dim-2 difference is carried per output group, not per block: for each of G0 / Gw (alpha
    // and u) the weighted in-plane sums of the blocks with dim 2 in S' at plane e - 1
    double ca0 = 0.0, cu0 = 0.0, caw = 0.0, cuw = 0.0;
    auto plane_q = [&](auto kc, int e, double& qa, double& qu) {
        constexpr int k = decltype(kc)::value;
        constexpr int S = sprime_mask(block_code(k, P, ORD), P);
        constexpr int SI = S & 3;
        const uint32_t ib = uint32_t(e) * m01 + base;
        qa = 0.0;
        qu = 0.0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if ((q & ~SI) != 0) continue;
            const double vv = a.edges[eix(g, k, ib - qoff[q])];
            const double v = qok[q] ? vv : 0.0;
            const bool neg = __builtin_popcount(q) & 1;
            if constexpr (UM == U_FROM_Z) {
                const double cl = clampd(v, tt);
                const double al = v - cl;
                qa = neg ? qa - al : qa + al;
                qu = neg ? qu + cl : qu - cl;
            } else {
                qu = neg ? qu - v : qu + v;
            }
        }
    };
    if (z0 > 0) {
        static_for<0, NB>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            constexpr int S = sprime_mask(block_code(k, P, ORD), P);
            if constexpr ((S & 4) != 0) {
                double qa, qu;
                plane_q(kc, z0 - 1, qa, qu);
                if constexpr ((S & 8) != 0) {
                    caw = fma(g.w[k], qa, caw);
                    cuw = fma(g.w[k], qu, cuw);
                } else {
                    ca0 = fma(g.w[k], qa, ca0);
                    cu0 = fma(g.w[k], qu, cu0);
                }
            }
        });
    }
    for (int e = z0; e < z1; ++e) {
        // this plane's sums: all blocks (s*) and those with dim 2 in S' (n*, carried to plane e + 1)
        double sa0 = 0.0, su0 = 0.0, saw = 0.0, suw = 0.0, na0 = 0.0, nu0 = 0.0, naw = 0.0, nuw = 0.0;
        static_for<0, NB>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            constexpr int S = sprime_mask(block_code(k, P, ORD), P);
            double qa, qu;
            plane_q(kc, e, qa, qu);
            if constexpr ((S & 8) != 0) {
                saw = fma(g.w[k], qa, saw);
                suw = fma(g.w[k], qu, suw);
                if constexpr ((S & 4) != 0) {
                    naw = fma(g.w[k], qa, naw);
                    nuw = fma(g.w[k], qu, nuw);
                }
            } else {
                sa0 = fma(g.w[k], qa, sa0);
                su0 = fma(g.w[k], qu, su0);
                if constexpr ((S & 4) != 0) {
                    na0 = fma(g.w[k], qa, na0);
                    nu0 = fma(g.w[k], qu, nu0);
                }
            }
        });
        const double a0 = sa0 - ca0, u0 = su0 - cu0, aw = saw - caw, uw = suw - cuw;
        ca0 = na0;
        cu0 = nu0;
        caw = naw;
        cuw = nuw;
        const uint32_t i = uint32_t(e) * m01 + base;
        if constexpr (UM == U_FROM_Z) {
            __builtin_nontemporal_store(a0, a.s0a + i);
            __builtin_nontemporal_store(aw, a.swa + i);
        }
        __builtin_nontemporal_store(u0, a.s0u + i);
        __builtin_nontemporal_store(uw, a.swu + i);
    }
}

template <int UM, bool PREV>
__global__ __launch_bounds__(g4::NTB) void k_gather4b(const Gather4Args a) {
    double c_prev = a.c_prev, rho_f = 0.0;
    if (a.ctl) {
        if (a.ctl->done) return;
        c_prev = a.ctl->c_prev;
        rho_f = a.ctl->rho;
    }
    double red[GR_N] = {0.0, 0.0, 0.0};
    const int bid = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
    const int per = (a.n3 + g4::NTB - 1) / g4::NTB;   // workgroups per w-chunk
    const int wc = bid / per;
    const int i3 = (bid - wc * per) * g4::NTB + int(threadIdx.x);
    if (bid < a.nblocks_b && i3 < a.n3) {
        const uint32_t pl = uint32_t(a.n3);
        const int w0 = a.wlo + wc * a.wchunk, w1 = min(a.whi, w0 + a.wchunk);
        double pa = 0.0, pu = 0.0;   // Gw at plane w - 1 (zero below the mesh)
        if (w0 > 0) {
            const uint32_t j = uint32_t(w0 - 1) * pl + uint32_t(i3);
            if constexpr (UM == U_FROM_Z) pa = a.swa[j];
            pu = a.swu[j];
        }
        for (int w = w0; w < w1; ++w) {
            const uint32_t i = uint32_t(w) * pl + uint32_t(i3);
            double ga = 0.0, wa_ = 0.0;
            if constexpr (UM == U_FROM_Z) {
                wa_ = __builtin_nontemporal_load(a.swa + i);
                ga = __builtin_nontemporal_load(a.s0a + i) + (wa_ - pa);
                pa = wa_;
            }
            const double wu = __builtin_nontemporal_load(a.swu + i);
            const double gu = __builtin_nontemporal_load(a.s0u + i) + (wu - pu);
            pu = wu;
            if constexpr (UM == U_FROM_Z) __builtin_nontemporal_store(a.fold ? rho_f * (ga + gu) : ga, a.g_alpha + i);
            __builtin_nontemporal_store(gu, a.g_u + i);
            red[GR_GU2] = fma(gu, gu, red[GR_GU2]);
            if constexpr (PREV) {
                const double gp = c_prev * __builtin_nontemporal_load(a.g_uprev + i);
                const double db = gu - gp, da = ga + gp;
                red[GR_S2B] = fma(db, db, red[GR_S2B]);
                red[GR_S2A] = fma(da, da, red[GR_S2A]);
            }
        }
    }
    block_reduce_store<GR_N, 0, g4::NTB>(red, a.partials);
}

bool gather4_ok(const Geom& g) {
    if (g.p != 4 || probe_env("MVTV_G4D") || probe_env("MVTV_G4_OFF")) return false;
    const uint32_t pl = g.m[0] * g.m[1] * g.m[2];
    const int nwp = int(g.iend / pl) - int(g.ibeg / pl);
    const int per = int((pl + g4::NTB - 1) / g4::NTB);
    // pass B: at least one w-chunk per workgroup row, within the partials buffer
    return per <= kMaxCgBlocks && nwp >= 1;
}

// rows (waves) of a pass-A tile: the y - 1 neighbours of all but the first row are the tile's own loads.
// 128^4, same box: 4 rows 9.39-9.42 ms, 8 rows 9.05, 16 rows 11.4 (profiles/r02/v14_gather4_rows)
static int g4_ty() {
    static const int ty = [] {
        const char* e = probe_env("MVTV_G4_TY");
        const int v = e ? std::atoi(e) : 8;
        return (v == 4 || v == 16) ? v : 8;
    }();
    return ty;
}

hipError_t launch_gather4(const Geom& g, int order, int umode, hipStream_t s, const double* edges, double t,
                          double* g_alpha, double* g_u, const double* g_uprev, double c_prev, double* partials,
                          int* nparts, const AdmmCtl* ctl, double* scratch, bool fold, int passes) {
    Gather4Args a{};
    a.g = g;
    a.fold = fold ? 1 : 0;
    a.edges = edges;
    a.s0a = scratch;
    a.s0u = scratch + size_t(g.N);
    a.swa = scratch + 2 * size_t(g.N);
    a.swu = scratch + 3 * size_t(g.N);
    a.g_alpha = g_alpha;
    a.g_u = g_u;
    a.g_uprev = g_uprev;
    a.partials = partials;
    a.t = t;
    a.c_prev = c_prev;
    a.ctl = ctl;
    const uint32_t pl = g.m[0] * g.m[1] * g.m[2];
    a.wlo = int(g.ibeg / pl);
    a.whi = int(g.iend / pl);
    a.wa = std::max(0, a.wlo - 1);   // Gw of the plane below the owned range (slab ghost) too
    a.wb = a.whi;
    if (passes & 4) a.wb = a.wlo;    // pass A on that ghost plane only (the fused 4-D slab pass did the owned ones)
    if ((passes & 4) && a.wb <= a.wa) passes &= ~4;
    a.tiles_x = int((g.m[0] + g4::TX - 1) / g4::TX);
    a.tiles_y = int((g.m[1] + g4_ty() - 1) / g4_ty());
    const int per_w = a.tiles_x * a.tiles_y;
    const int nw = a.wb - a.wa;
    a.nzc = std::max(1, std::min(int(g.m[2]), 8192 / std::max(1, per_w * nw)));
    a.zchunk = int((g.m[2] + a.nzc - 1) / a.nzc);
    a.nzc = int((g.m[2] + a.zchunk - 1) / a.zchunk);
    a.nblocks = per_w * a.nzc * nw;
    // pass B: w-chunks so that the grid fills the chip a few times, within the partials rows
    a.n3 = int(pl);
    const int per = (a.n3 + g4::NTB - 1) / g4::NTB;
    const int nwo = std::max(1, a.whi - a.wlo);
    a.nwc = std::max(1, std::min(nwo, std::min(4096, kMaxCgBlocks) / std::max(1, per)));
    a.wchunk = (nwo + a.nwc - 1) / a.nwc;
    a.nwc = (nwo + a.wchunk - 1) / a.wchunk;
    a.nblocks_b = per * a.nwc;
    const bool expl = umode == U_EXPLICIT;
    auto goa = [&](auto kern) {
        klaunch(kern, dim3((a.nblocks + 7) / 8 * 8), dim3(64 * g4_ty()), 0, s, a);
        return hipGetLastError();
    };
    auto pick = [&](auto tc) {
        constexpr int T = decltype(tc)::value;
        if (order == 0) return expl ? goa(k_gather4a<0, U_EXPLICIT, 15, T>) : goa(k_gather4a<0, U_FROM_Z, 15, T>);
        if (g.nb == 14) return expl ? goa(k_gather4a<1, U_EXPLICIT, 14, T>) : goa(k_gather4a<1, U_FROM_Z, 14, T>);
        return expl ? goa(k_gather4a<1, U_EXPLICIT, 15, T>) : goa(k_gather4a<1, U_FROM_Z, 15, T>);
    };
    const int ty = g4_ty();
    const hipError_t e = !(passes & 5) ? hipSuccess
                                       : (ty == 16 ? pick(std::integral_constant<int, 16>{})
                                                   : (ty == 8 ? pick(std::integral_constant<int, 8>{})
                                                              : pick(std::integral_constant<int, 4>{})));
    if (e != hipSuccess || !(passes & 2)) return e;
    if (g_timed_b.start) {   // the caller timed both passes
        g_timed = g_timed_b;
        g_timed_b = TimedLaunch{};
    }
    const int gridb = (a.nblocks_b + 7) / 8 * 8;
    *nparts = gridb;
    const bool prev = g_uprev != nullptr;
    auto gob = [&](auto kern) {
        klaunch(kern, dim3(gridb), dim3(g4::NTB), 0, s, a);
        return hipGetLastError();
    };
    if (expl) return prev ? gob(k_gather4b<U_EXPLICIT, true>) : gob(k_gather4b<U_EXPLICIT, false>);
    return prev ? gob(k_gather4b<U_FROM_Z, true>) : gob(k_gather4b<U_FROM_Z, false>);
}

// ---------------------------------------------------------------------------------------------
// k_admm4a (4-D, config 5): the edge update and the gather's pass A in ONE pass over the edge state, the
// k_admm3a scheme one dimension up. A workgroup owns a 64 x 6 tile of the (dim 0, dim 1) plane at a fixed w
// (dim 3) and marches dim 2 over a chunk of z planes: at every step it forms z_new of its cells (theta at the 16
// corners (x + a, y + b, z + c, w + d): the w + 1 corners are a second theta row, the z + 1 ones the next step's
// plane, carried), stores it to the ping-pong partner buffer, stages the blocks whose S' has dim 0 or 1 in LDS,
// and forms pass A's outputs from the in-plane backward corners (x - 1, y - 1 from the image; the halo row and
// the halo column recompute the neighbouring tiles' z_new from the previous iterate and never store it) and the
// dim-2 corner from per-group sums carried from the previous plane: G0 (blocks without dim 3 in S') and Gw
// (with), alpha and u parts. k_gather4b then takes the dim-3 difference as before. Against k_edge4d + k_gather4a
// the edge state is read once instead of twice: 8 (2E + 5N) bytes instead of 8 (3E + 5N) (+ theta twice: the
// w + 1 corners come from another plane, 16 MB away at 128^4, read as a second stream).
// 512 threads: waves 0..6 hold image rows 0..6 (row 0 the y - 1 halo), wave 7 the x - 1 halo column (lanes
// 0..6); the image holds 13 of the 15 blocks (S' = {2} and {3} are read by their own cell only) in two plane
// buffers: 13 x 7 x 65 x 8 B x 2 = 95 KB, one workgroup per CU, up to 256 VGPRs a lane (the 1024-thread form of
// round 2 spilled at 128).
// With the twins skipped (TW) the image holds 9 of the 13 blocks, so the tile grows to 10 owned rows (11 image rows,
// 768 threads: 12 waves a CU instead of 8, 103 KB of LDS, <= 170 VGPRs a lane): 128^4 launch 12.22 -> 11.87 ms, same
// box (profiles/r04/v16_f4a_tall)).
namespace f4a {
constexpr int IW = 65;
constexpr int ih(bool tw) { return tw ? 11 : 7; }
constexpr int nt(bool tw) { return (ih(tw) + 1) * 64; }
}

// image slots: the blocks whose S' has dim 0 or 1, minus the twins when they are skipped
template <int NB, int ORD, bool TW = false>
__host__ __device__ constexpr bool f4a_in_image(int k) {
    return (sprime_mask(block_code(k, 4, ORD), 4) & 3) != 0 && !(TW && twin_of(k, 4, ORD) != k);
}
template <int NB, int ORD, bool TW = false>
__host__ __device__ constexpr int f4a_nimg() {
    int n = 0;
    for (int k = 0; k < NB; ++k)
        if (f4a_in_image<NB, ORD, TW>(k)) ++n;
    return n;
}
template <int NB, int ORD, bool TW = false>
__host__ __device__ constexpr int f4a_slot(int k) {
    int n = 0;
    for (int j = 0; j < k; ++j)
        if (f4a_in_image<NB, ORD, TW>(j)) ++n;
    return f4a_in_image<NB, ORD, TW>(k) ? n : -1;
}

struct Fused4Args {
    Geom g;
    const double* theta;
    const double* z_old;
    double* z_new;
    const double* theta_old;
    double* s0a;   // pass A's outputs (k_gather4b's inputs): G0 / Gw, alpha and u parts
    double* s0u;
    double* swa;
    double* swu;
    double* partials;
    const AdmmCtl* ctl;
    double t_old, c_old, t_new;
    int tiles_x, tiles_y, zchunk, nzc, nblocks, wa;
};

// TW: the twin blocks (mvtv_internal.h twin_of) are skipped as in k_admm3a, their group's first block counting for all
template <int ORD, int UM, bool DTH, int NB, bool TW>
__global__ __launch_bounds__(f4a::nt(TW)) void k_admm4a(const Fused4Args a) {
    constexpr int P = 4, NC = 16, IW = f4a::IW, IH = f4a::ih(TW), TY = IH - 1, NI = f4a_nimg<NB, ORD, TW>();
    static_assert(!TW || twin_block(NB, P, ORD) >= 0, "twin blocks");
    double t_old = a.t_old, c_old = a.c_old, t_new = a.t_new;
    if (a.ctl) {
        if (a.ctl->done) return;
        t_old = a.ctl->t_z;
        c_old = a.ctl->c_prev;
        t_new = a.ctl->t_next;
    }
    __shared__ double szr[2 * NI * IH * IW];
    double red[ER_N] = {0.0, 0.0, 0.0, 0.0};
    const Geom& g = a.g;
    const int bid = int((blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3));   // XCD runs of tiles
    if (bid < a.nblocks) {
        const int nt = a.tiles_x * a.tiles_y;
        const int tw = bid / (nt * a.nzc);
        int rem = bid - tw * nt * a.nzc;
        const int tz = rem / nt;
        rem -= tz * nt;
        const int tyi = rem / a.tiles_x, txi = rem - tyi * a.tiles_x;
        const int X0 = txi * 64, Yh = tyi * TY - 1;
        const int w = a.wa + tw;
        const int m0 = int(g.m[0]), m1 = int(g.m[1]), m2 = int(g.m[2]), m3 = int(g.m[3]);
        const int z0 = tz * a.zchunk, z1 = min(m2, z0 + a.zchunk);
        const int wv = int(threadIdx.x) >> 6, ln = int(threadIdx.x) & 63;
        const bool hcol = wv == IH;
        const int row = hcol ? ln : wv;
        const int col = hcol ? 0 : ln + 1;
        const int x = hcol ? X0 - 1 : X0 + ln, y = Yh + row;
        const bool active = row < IH;
        const bool cell = active && x >= 0 && y >= 0 && x < m0 && y < m1;
        const bool inner = cell && !hcol && row > 0;
        const bool hrow = row == 0;
        const uint32_t pl = uint32_t(m0) * uint32_t(m1), pl3 = pl * uint32_t(m2);
        const int xc = min(max(x, 0), m0 - 1), yc = min(max(y, 0), m1 - 1);
        const uint32_t xo[2] = {uint32_t(xc), uint32_t(min(xc + 1, m0 - 1))};
        const uint32_t yo[2] = {uint32_t(yc) * uint32_t(m0), uint32_t(min(yc + 1, m1 - 1)) * uint32_t(m0)};
        const uint32_t wo[2] = {uint32_t(w) * pl3, uint32_t(min(w + 1, m3 - 1)) * pl3};
        const uint32_t ixy = yo[0] + xo[0];
        const bool okx = x > 0, oky = y > 0;
        auto sidx = [&](int buf, int slot, int r, int c) { return ((buf * NI + slot) * IH + r) * IW + c; };

        // theta at (x + a, y + b, w + d) of plane e: index a | b << 1 | d << 2
        auto load_theta = [&](double (&th)[8], int e) {
            const uint32_t zo = uint32_t(e) * pl;
#pragma unroll
            for (int q = 0; q < 8; ++q) th[q] = cell ? a.theta[wo[q >> 2] + zo + yo[(q >> 1) & 1] + xo[q & 1]] : 0.0;
        };
        auto load_z = [&](double (&zo)[NB], int e) {
            const uint32_t i = wo[0] + uint32_t(e) * pl + ixy;
            static_for<0, NB>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                constexpr int S = sprime_mask(block_code(k, P, ORD), P);
                const bool need = cell && (!hrow || (S & 2)) && (!hcol || (S & 1));
                if constexpr (TW && twin_of(k, P, ORD) != k) zo[k] = 0.0;
                else zo[k] = need ? a.z_old[eix(g, k, i)] : 0.0;
            });
        };
        auto edge_cell = [&](int e, const double (&th0)[8], const double (&th1)[8], const double (&zo)[NB],
                             double (&zn)[NB], bool own) {
            const uint32_t i = wo[0] + uint32_t(e) * pl + ixy;
            double v[NC];   // corner a | b << 1 | c << 2 | d << 3
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int qq = (q & 3) | ((q & 4) << 1);
                v[qq] = th0[q];
                v[qq | 4] = th1[q];
            }
            if constexpr (DTH)
                if (own) red[ER_DTH] = fmax(red[ER_DTH], fabs(v[0] - a.theta_old[i]));
#pragma unroll
            for (int j = 0; j < P; ++j)
#pragma unroll
                for (int q = 0; q < NC; ++q)
                    if (!((q >> j) & 1)) v[q | (1 << j)] = v[q] - v[q | (1 << j)];
            static_for<0, NB>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                constexpr int S = sprime_mask(block_code(k, P, ORD), P);
                if constexpr (TW && twin_of(k, P, ORD) != k) {
                    zn[k] = 0.0;
                } else {
                    const double d = g.w[k] * v[S];
                    const double uo = (UM == U_EXPLICIT) ? zo[k] : -c_old * clampd(zo[k], t_old);
                    const double z = cell ? d - uo : 0.0;
                    zn[k] = z;
                    if (own) {
                        const double al = z - clampd(z, t_new);
                        const double r = al - d;
                        __builtin_nontemporal_store(z, a.z_new + eix(g, k, i));
                        constexpr double m = TW ? double(twin_count(k, NB, P, ORD)) : 1.0;   // the twins' terms
                        red[ER_R2] = fma(m * r, r, red[ER_R2]);
                        red[ER_D2] = fma(m * d, d, red[ER_D2]);
                        red[ER_A2] = fma(m * al, al, red[ER_A2]);
                    }
                }
            });
        };
        auto to_image = [&](int buf, const double (&zn)[NB]) {
            if (!active) return;
            static_for<0, NB>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                constexpr int sl = f4a_slot<NB, ORD, TW>(k);
                if constexpr (sl >= 0 && !(TW && twin_of(k, P, ORD) != k)) szr[sidx(buf, sl, row, col)] = zn[k];
            });
        };
        auto plane_q = [&](auto kc, int buf, double own_z, double& qa, double& qu) {
            constexpr int k = decltype(kc)::value;
            constexpr int S = sprime_mask(block_code(k, P, ORD), P);
            constexpr int SI = S & 3;
            constexpr int sl = f4a_slot<NB, ORD, TW>(k);
            qa = 0.0;
            qu = 0.0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if ((q & ~SI) != 0) continue;
                double v;
                if (q == 0) {
                    v = own_z;
                } else {
                    const bool ok = (!(q & 1) || okx) && (!(q & 2) || oky);
                    if constexpr (sl >= 0) v = ok ? szr[sidx(buf, sl, row - ((q >> 1) & 1), col - (q & 1))] : 0.0;
                    else v = 0.0;
                }
                const bool neg = __builtin_popcount(q) & 1;
                const double cl = clampd(v, t_new);
                const double al = v - cl;
                qa = neg ? qa - al : qa + al;
                qu = neg ? qu + cl : qu - cl;   // u = -clamp
            }
        };
        // per-group sums of the blocks with dim 2 in S' at the previous plane (G0 / Gw, alpha / u)
        double ca0 = 0.0, cu0 = 0.0, caw = 0.0, cuw = 0.0;
        auto carry = [&](int buf, const double (&zn)[NB], double& na0, double& nu0, double& naw, double& nuw) {
            static_for<0, NB>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                constexpr int S = sprime_mask(block_code(k, P, ORD), P);
                if constexpr ((S & 4) != 0 && !(TW && twin_of(k, P, ORD) != k)) {
                    constexpr double mk = TW ? double(twin_count(k, NB, P, ORD)) : 1.0;
                    const double wk = mk * g.w[k];
                    double qa, qu;
                    plane_q(kc, buf, zn[k], qa, qu);
                    if constexpr ((S & 8) != 0) {
                        naw = fma(wk, qa, naw);
                        nuw = fma(wk, qu, nuw);
                    } else {
                        na0 = fma(wk, qa, na0);
                        nu0 = fma(wk, qu, nu0);
                    }
                }
            });
        };
        double th0[8], th1[8], zo[NB], zn[NB];
        if (z0 > 0) {   // the carried sums of plane z0 - 1, from its z_new recomputed from the old state
            load_theta(th0, z0 - 1);
            load_theta(th1, z0);
            load_z(zo, z0 - 1);
            edge_cell(z0 - 1, th0, th1, zo, zn, false);
            to_image(1, zn);
            lds_barrier();
            if (inner) carry(1, zn, ca0, cu0, caw, cuw);
            lds_barrier();
        }
        load_theta(th0, z0);
        load_theta(th1, min(z0 + 1, m2 - 1));
        load_z(zo, z0);
        for (int e = z0; e < z1; ++e) {
            const int buf = (e - z0) & 1;
            edge_cell(e, th0, th1, zo, zn, inner);
            to_image(buf, zn);
            double nth[8], nzo[NB];   // the next step's loads in flight during this step's gather
            if (e + 1 < z1) {
                load_theta(nth, min(e + 2, m2 - 1));
                load_z(nzo, e + 1);
            } else {
#pragma unroll
                for (int q = 0; q < 8; ++q) nth[q] = 0.0;
#pragma unroll
                for (int k = 0; k < NB; ++k) nzo[k] = 0.0;
            }
            lds_barrier();
            if (inner) {
                double sa0 = 0.0, su0 = 0.0, saw = 0.0, suw = 0.0, na0 = 0.0, nu0 = 0.0, naw = 0.0, nuw = 0.0;
                static_for<0, NB>([&](auto kc) {
                    constexpr int k = decltype(kc)::value;
                    constexpr int S = sprime_mask(block_code(k, P, ORD), P);
                    if constexpr (!(TW && twin_of(k, P, ORD) != k)) {
                        constexpr double mk = TW ? double(twin_count(k, NB, P, ORD)) : 1.0;
                        const double wk = mk * g.w[k];
                        double qa, qu;
                        plane_q(kc, buf, zn[k], qa, qu);
                        if constexpr ((S & 8) != 0) {
                            saw = fma(wk, qa, saw);
                            suw = fma(wk, qu, suw);
                            if constexpr ((S & 4) != 0) {
                                naw = fma(wk, qa, naw);
                                nuw = fma(wk, qu, nuw);
                            }
                        } else {
                            sa0 = fma(wk, qa, sa0);
                            su0 = fma(wk, qu, su0);
                            if constexpr ((S & 4) != 0) {
                                na0 = fma(wk, qa, na0);
                                nu0 = fma(wk, qu, nu0);
                            }
                        }
                    }
                });
                const uint32_t i = wo[0] + uint32_t(e) * pl + ixy;
                __builtin_nontemporal_store(sa0 - ca0, a.s0a + i);
                __builtin_nontemporal_store(su0 - cu0, a.s0u + i);
                __builtin_nontemporal_store(saw - caw, a.swa + i);
                __builtin_nontemporal_store(suw - cuw, a.swu + i);
                ca0 = na0;
                cu0 = nu0;
                caw = naw;
                cuw = nuw;
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                th0[q] = th1[q];
                th1[q] = nth[q];
            }
#pragma unroll
            for (int k = 0; k < NB; ++k) zo[k] = nzo[k];
        }
    }
    block_reduce_store<ER_N, 1, f4a::nt(TW)>(red, a.partials);
}

// ---------------------------------------------------------------------------------------------
// k_admm2d: the fused edge update + D^T gather for p = 2 (configs 2 and 4). A wave owns 64 columns
// (lane 0 on x = X0-1 as halo, 63 interior) over a chunk of rows and marches dim 1: the x-1
// neighbour of the gather comes from the lane below (shuffle), the y-1 neighbour from two carried
// group sums. No LDS and no barrier; waves are independent. z ping-pongs like k_admm3d.
namespace f2d {
constexpr int TX = 63, NT = 256;
}
template <int ORD, int UM, bool DTH, int NB>
__global__ __launch_bounds__(f2d::NT) void k_admm2d(const Fused3dArgs a) {
    constexpr int P = 2, NC = 4;
    const Geom& g = a.g;
    double t_old = a.t_old, c_old = a.c_old, t_new = a.t_new, c_prev = a.c_prev, rho_f = 0.0;
    if (a.ctl) {
        if (a.ctl->done) return;
        t_old = a.ctl->t_z;
        c_old = a.ctl->c_prev;
        t_new = a.ctl->t_next;
        c_prev = a.ctl->c_prev;
        rho_f = a.ctl->rho;
    }
    double red[7] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    const int bid = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
    const int wv = bid * (f2d::NT / 64) + int(threadIdx.x >> 6);   // this wave's (tile, chunk)
    const int nwaves = a.nblocks;
    if (bid * (f2d::NT / 64) < nwaves && wv < nwaves) {
        const int lane = int(threadIdx.x & 63);
        const int tc = wv / a.tiles_x, txi = wv - tc * a.tiles_x;
        const int x = txi * f2d::TX - 1 + lane;
        const int m0 = int(g.m[0]), m1 = int(g.m[1]);
        const int y0 = tc * a.zchunk, y1 = min(m1, y0 + a.zchunk);
        const bool cell = x >= 0 && x < m0;
        const bool own = cell && lane > 0;
        const int xc = min(max(x, 0), m0 - 1);
        const uint32_t xo[2] = {uint32_t(xc), uint32_t(min(xc + 1, m0 - 1))};
        const bool okx = x > 0;
        auto load_row = [&](double (&th)[2], int y) {
            const uint32_t yo = uint32_t(min(y, m1 - 1)) * uint32_t(m0);
            th[0] = cell ? a.theta[yo + xo[0]] : 0.0;
            th[1] = cell ? a.theta[yo + xo[1]] : 0.0;
        };
        auto load_z = [&](double (&zo)[NB], int y) {
            const uint32_t i = uint32_t(y) * uint32_t(m0) + uint32_t(xc);
#pragma unroll
            for (int k = 0; k < NB; ++k) zo[k] = cell ? a.z_old[uint64_t(k) * g.N + i] : 0.0;
        };
        // z_new of this cell at row y from theta rows y (r0), y+1 (r1) and the old z
        auto edge_cell = [&](int y, const double (&r0)[2], const double (&r1)[2], const double (&zo)[NB],
                             double (&zn)[NB], bool mine) {
            const uint32_t i = uint32_t(y) * uint32_t(m0) + uint32_t(xc);
            double v[NC] = {r0[0], r0[1], r1[0], r1[1]};
            if constexpr (DTH)
                if (mine) red[3] = fmax(red[3], fabs(v[0] - a.theta_old[i]));
#pragma unroll
            for (int j = 0; j < P; ++j)
#pragma unroll
                for (int q = 0; q < NC; ++q)
                    if (!((q >> j) & 1)) v[q | (1 << j)] = v[q] - v[q | (1 << j)];
            static_for<0, NB>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                constexpr int S = sprime_mask(block_code(k, P, ORD), P);
                const double d = g.w[k] * v[S];
                const double uo = (UM == U_EXPLICIT) ? zo[k] : -c_old * clampd(zo[k], t_old);
                const double z = cell ? d - uo : 0.0;
                zn[k] = z;
                if (mine) {
                    const double al = z - clampd(z, t_new);
                    const double r = al - d;
                    __builtin_nontemporal_store(z, a.z_new + uint64_t(k) * g.N + i);
                    red[0] = fma(r, r, red[0]);
                    red[1] = fma(d, d, red[1]);
                    red[2] = fma(al, al, red[2]);
                }
            });
        };
        // in-row sums of block k at this cell: own z_new and (dim 0 in S') the lane below's
        auto row_q = [&](auto kc, const double (&zn)[NB], double& qa, double& qu) {
            constexpr int k = decltype(kc)::value;
            constexpr int S = sprime_mask(block_code(k, P, ORD), P);
            const double v0 = zn[k];
            const double cl0 = clampd(v0, t_new);
            qa = v0 - cl0;
            qu = -cl0;
            if constexpr ((S & 1) != 0) {
                const double vl = __shfl_up(v0, 1, 64);
                const double v1 = okx ? vl : 0.0;
                const double cl1 = clampd(v1, t_new);
                qa -= v1 - cl1;
                qu += cl1;
            }
        };
        double ca = 0.0, cu = 0.0;   // carried: weighted row sums of the blocks with dim 1 in S' at y-1
        double r0[2], r1[2], zo[NB], zn[NB];
        if (y0 > 0) {
            load_row(r0, y0 - 1);
            load_row(r1, y0);
            load_z(zo, y0 - 1);
            edge_cell(y0 - 1, r0, r1, zo, zn, false);
            static_for<0, NB>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                constexpr int S = sprime_mask(block_code(k, P, ORD), P);
                double qa, qu;
                row_q(kc, zn, qa, qu);
                if constexpr ((S & 2) != 0) {
                    ca = fma(g.w[k], qa, ca);
                    cu = fma(g.w[k], qu, cu);
                }
            });
        }
        load_row(r0, y0);
        load_row(r1, y0 + 1);
        load_z(zo, y0);
        double gp = own ? __builtin_nontemporal_load(a.g_uprev + uint32_t(y0) * uint32_t(m0) + uint32_t(xc)) : 0.0;
        for (int y = y0; y < y1; ++y) {
            edge_cell(y, r0, r1, zo, zn, own);
            double nr[2], nzo[NB], ngp = 0.0;
            if (y + 1 < y1) {
                load_row(nr, y + 2);
                load_z(nzo, y + 1);
                ngp = own ? __builtin_nontemporal_load(a.g_uprev + uint32_t(y + 1) * uint32_t(m0) + uint32_t(xc)) : 0.0;
            } else {
                nr[0] = nr[1] = 0.0;
#pragma unroll
                for (int k = 0; k < NB; ++k) nzo[k] = 0.0;
            }
            double ga = 0.0, gu = 0.0, na = 0.0, nu = 0.0;
            static_for<0, NB>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                constexpr int S = sprime_mask(block_code(k, P, ORD), P);
                double qa, qu;
                row_q(kc, zn, qa, qu);
                ga = fma(g.w[k], qa, ga);
                gu = fma(g.w[k], qu, gu);
                if constexpr ((S & 2) != 0) {
                    na = fma(g.w[k], qa, na);
                    nu = fma(g.w[k], qu, nu);
                }
            });
            ga -= ca;
            gu -= cu;
            ca = na;
            cu = nu;
            if (own) {
                const uint32_t i = uint32_t(y) * uint32_t(m0) + uint32_t(xc);
                __builtin_nontemporal_store(a.fold ? rho_f * (ga + gu) : ga, a.g_alpha + i);
                __builtin_nontemporal_store(gu, a.g_u + i);
                const double gpc = c_prev * gp;
                const double db = gu - gpc, da = ga + gpc;
                red[4] = fma(gu, gu, red[4]);
                red[5] = fma(db, db, red[5]);
                red[6] = fma(da, da, red[6]);
            }
            r0[0] = r1[0];
            r0[1] = r1[1];
            r1[0] = nr[0];
            r1[1] = nr[1];
#pragma unroll
            for (int k = 0; k < NB; ++k) zo[k] = nzo[k];
            gp = ngp;
        }
    }
    // block reduction (max in slot 3)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
#pragma unroll
        for (int k = 0; k < 7; ++k) {
            const double o = __shfl_down(red[k], off, 64);
            red[k] = k == 3 ? fmax(red[k], o) : red[k] + o;
        }
    }
    __shared__ double rs[f2d::NT / 64][7];
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0)
        for (int k = 0; k < 7; ++k) rs[w][k] = red[k];
    __syncthreads();
    if (threadIdx.x < 7) {
        const int k = threadIdx.x;
        double acc = rs[0][k];
        for (int ww = 1; ww < f2d::NT / 64; ++ww) acc = k == 3 ? fmax(acc, rs[ww][k]) : acc + rs[ww][k];
        a.partials[blockIdx.x * 7 + k] = acc;
    }
}

namespace {
Fused3dArgs f2d_args(const Geom& g) {
    Fused3dArgs a{};
    a.g = g;
    a.tiles_x = int((g.m[0] + f2d::TX - 1) / f2d::TX);
    static const int want = [] {
        const char* e = probe_env("MVTV_F2D_WAVES");
        return e ? std::atoi(e) : 2048;   // 2048^2: 2048 waves 75.8 us, 4096 81.8, 8192 81.0
    }();
    const int m1 = int(g.m[1]);
    int nc = std::max(1, std::min(m1 / 8, want / std::max(1, a.tiles_x)));   // rows per chunk >= 8
    const int wpb = f2d::NT / 64;
    while (nc > 1 && ((nc * a.tiles_x + wpb - 1) / wpb + 7) / 8 * 8 * 7 > kMaxCgBlocks * kMaxRed) --nc;
    a.zchunk = (m1 + nc - 1) / nc;
    nc = (m1 + a.zchunk - 1) / a.zchunk;
    a.nblocks = a.tiles_x * nc;   // waves
    return a;
}
}  // namespace

bool fused2d_ok(const Geom& g) {
    if (g.p != 2 || probe_env("MVTV_F2D_OFF") || g.ibeg != 0 || g.iend != g.N) return false;
    const Fused3dArgs a = f2d_args(g);
    const int wg = (a.nblocks + f2d::NT / 64 - 1) / (f2d::NT / 64);
    return ((wg + 7) / 8 * 8) * 7 <= kMaxCgBlocks * kMaxRed;
}

hipError_t launch_admm2d(const Geom& g, int order, int umode, hipStream_t s, const double* theta, const double* z_old,
                         double* z_new, double t_old, double c_old, double t_new, double c_prev,
                         const double* theta_old, double* g_alpha, double* g_u, const double* g_uprev,
                         double* partials, int* nparts, const AdmmCtl* ctl, bool fold) {
    Fused3dArgs a = f2d_args(g);
    a.fold = fold ? 1 : 0;
    a.theta = theta;
    a.z_old = z_old;
    a.z_new = z_new;
    a.theta_old = theta_old;
    a.g_alpha = g_alpha;
    a.g_u = g_u;
    a.g_uprev = g_uprev;
    a.partials = partials;
    a.t_old = t_old;
    a.c_old = c_old;
    a.t_new = t_new;
    a.c_prev = c_prev;
    a.ctl = ctl;
    const int wg = (a.nblocks + f2d::NT / 64 - 1) / (f2d::NT / 64);
    const int grid = (wg + 7) / 8 * 8;
    *nparts = grid;
    const bool dth = theta_old != nullptr;
    auto go = [&](auto kern) {
        klaunch(kern, dim3(grid), dim3(f2d::NT), 0, s, a);
        return hipGetLastError();
    };
    if (order == 0) {
        if (umode == U_EXPLICIT) return dth ? go(k_admm2d<0, U_EXPLICIT, true, 3>) : go(k_admm2d<0, U_EXPLICIT, false, 3>);
        return dth ? go(k_admm2d<0, U_FROM_Z, true, 3>) : go(k_admm2d<0, U_FROM_Z, false, 3>);
    }
    if (g.nb == 2) {
        if (umode == U_EXPLICIT) return dth ? go(k_admm2d<1, U_EXPLICIT, true, 2>) : go(k_admm2d<1, U_EXPLICIT, false, 2>);
        return dth ? go(k_admm2d<1, U_FROM_Z, true, 2>) : go(k_admm2d<1, U_FROM_Z, false, 2>);
    }
    if (umode == U_EXPLICIT) return dth ? go(k_admm2d<1, U_EXPLICIT, true, 3>) : go(k_admm2d<1, U_EXPLICIT, false, 3>);
    return dth ? go(k_admm2d<1, U_FROM_Z, true, 3>) : go(k_admm2d<1, U_FROM_Z, false, 3>);
}


// ------------------------------------------------------------------------------------------------ k_admm4a
namespace {
Fused4Args f4a_args(const Geom& g, bool tw = false) {
    Fused4Args a{};
    a.g = g;
    const uint32_t pl3 = g.m[0] * g.m[1] * g.m[2];
    a.wa = int(g.ibeg / pl3);
    const int nw = std::max(1, int(g.iend / pl3) - a.wa);
    const int ty = f4a::ih(tw) - 1;
    a.tiles_x = int((g.m[0] + 63) / 64);
    a.tiles_y = int((int(g.m[1]) + ty - 1) / ty);
    const int tiles = a.tiles_x * a.tiles_y * nw;
    // z chunks only when the (tile, w) items alone leave the chip under ~4 waves (one workgroup per CU): every chunk
    // start recomputes one plane
    a.nzc = std::max(1, std::min(int(g.m[2]), (1024 + tiles - 1) / tiles));
    a.zchunk = int((g.m[2] + uint32_t(a.nzc) - 1) / uint32_t(a.nzc));
    a.nzc = int((g.m[2] + uint32_t(a.zchunk) - 1) / uint32_t(a.zchunk));
    a.nblocks = tiles * a.nzc;
    return a;
}
}  // namespace

bool fused4_ok(const Geom& g) {
    if (g.p != 4 || probe_env("MVTV_F4D_OFF") || !gather4_ok(g) || g.iend <= g.ibeg) return false;
    const Fused4Args a = f4a_args(g);
    // partial rows: ER_N words per workgroup within the partials buffer
    return size_t((a.nblocks + 7) / 8 * 8) * ER_N <= size_t(kMaxCgBlocks) * kMaxRed;
}

hipError_t launch_admm4a(const Geom& g, int order, int umode, hipStream_t s, const double* theta, const double* z_old,
                         double* z_new, double t_old, double c_old, double t_new, const double* theta_old,
                         double* scratch4, double* partials, int* nparts, const AdmmCtl* ctl, bool twin) {
    if (!fused4_ok(g) || !scratch4 || z_old == z_new) return hipErrorInvalidValue;
    if (twin && !twin_weights_equal(g, order)) return hipErrorInvalidValue;
    Fused4Args a = f4a_args(g, twin);
    a.t_old = t_old;
    a.c_old = c_old;
    a.t_new = t_new;
    a.theta = theta;
    a.z_old = z_old;
    a.z_new = z_new;
    a.theta_old = theta_old;
    a.s0a = scratch4;
    a.s0u = scratch4 + size_t(g.N);
    a.swa = scratch4 + 2 * size_t(g.N);
    a.swu = scratch4 + 3 * size_t(g.N);
    a.partials = partials;
    a.ctl = ctl;
    const int grid = (a.nblocks + 7) / 8 * 8;
    *nparts = grid;
    const bool dth = theta_old != nullptr;
    auto go = [&](auto kern) {
        klaunch(kern, dim3(grid), dim3(f4a::nt(twin)), 0, s, a);
        return hipGetLastError();
    };
    auto pick = [&](auto ordc, auto nbc, auto twc) {
        constexpr int O = decltype(ordc)::value, NB = decltype(nbc)::value;
        constexpr bool T = decltype(twc)::value;
        if (umode == U_EXPLICIT)
            return dth ? go(k_admm4a<O, U_EXPLICIT, true, NB, T>) : go(k_admm4a<O, U_EXPLICIT, false, NB, T>);
        return dth ? go(k_admm4a<O, U_FROM_Z, true, NB, T>) : go(k_admm4a<O, U_FROM_Z, false, NB, T>);
    };
    using std::integral_constant;
    using T1 = integral_constant<bool, true>;
    using T0 = integral_constant<bool, false>;
    if (order == 0)
        return twin ? pick(integral_constant<int, 0>{}, integral_constant<int, 15>{}, T1{})
                    : pick(integral_constant<int, 0>{}, integral_constant<int, 15>{}, T0{});
    if (g.nb == 14)
        return twin ? pick(integral_constant<int, 1>{}, integral_constant<int, 14>{}, T1{})
                    : pick(integral_constant<int, 1>{}, integral_constant<int, 14>{}, T0{});
    return twin ? pick(integral_constant<int, 1>{}, integral_constant<int, 15>{}, T1{})
                : pick(integral_constant<int, 1>{}, integral_constant<int, 15>{}, T0{});
}

hipError_t launch_gather4b(const Geom& g, int umode, hipStream_t s, double* g_alpha, double* g_u, const double* g_uprev,
                           double c_prev, double* partials, int* nparts, const AdmmCtl* ctl, double* scratch4,
                           bool fold) {
    return launch_gather4(g, 0, umode, s, nullptr, 0.0, g_alpha, g_u, g_uprev, c_prev, partials, nparts, ctl, scratch4,
                          fold, 2);
}

hipError_t launch_gather4a_ghost(const Geom& g, int order, hipStream_t s, const double* edges, double* scratch4,
                                 const AdmmCtl* ctl) {
    int np = 0;
    return launch_gather4(g, order, U_FROM_Z, s, edges, 0.0, nullptr, nullptr, nullptr, 1.0, nullptr, &np, ctl, scratch4,
                          false, 4);
}
}  // namespace mvtv

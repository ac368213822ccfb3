// mvtv_cg3d.hip — fused Jacobi-PCG iteration for 3-D meshes (the BASELINE 512^3 path).
//
// Replaces spsolve(W + rho D^T D, b) of rcpp-code/MultivarTV/src/solvers.cpp:113 by the
// single-reduction (Chronopoulos-Gear) form of Jacobi-preconditioned CG, one launch per CG
// iteration, with everything that needs a neighbour RECOMPUTED on chip instead of stored:
//
//   iteration i, state (x_i, r_i, p_{i-1}), scalars alpha_i, beta_i from the previous launch:
//     p_i     = M^-1 r_i + beta_i p_{i-1}      needed on the tile + 2-cell halo
//     s_i     = A p_i                          tile + 1 halo      (27-point stencil)
//     r_{i+1} = r_i - alpha_i s_i              tile + 1 halo
//     u_{i+1} = M^-1 r_{i+1}                   tile + 1 halo
//     w_{i+1} = A u_{i+1}                      tile               (27-point stencil)
//     x_{i+1} = x_i + alpha_i p_i              tile
//   reductions: gamma = (r_{i+1}, u_{i+1}), delta = (w_{i+1}, u_{i+1}), |r_{i+1}|^2
//   next (k_finalize op 5): beta = gamma'/gamma, alpha = gamma' / (delta' - beta gamma'/alpha)
//
// x is needed only at the end, and iteration i+1 reads p_i anyway (as p_{i-1} of its direction), so
// x moves every other iteration: even iterations leave it alone, odd ones apply both steps,
// x += alpha_{i-1} p_{i-1} + alpha_i p_i (the same two fmas in the same order as one step per
// iteration, so x is bit-identical), and k_cg_xflush applies a pending step once the solve ends on
// an even iteration. HBM traffic per iteration is 4N words (read r, p; write r, p) and 6N (x too)
// alternately, 5N on average, against 11N for the three-kernel PCG. r and p ping-pong between two
// buffers: a launch reads neighbour halos of r_i and p_{i-1} that their owning workgroups overwrite.
//
// Geometry. A 512-thread workgroup owns a 60 x 20 column of the (dim 0, dim 1) plane over a
// chunk of dim-2 planes and marches through dim 2. Each plane is staged in LDS as a 64 x 24
// image (tile + 2-cell halo): ONE IMAGE ROW IS ONE WAVEFRONT ROW, and wave w owns image rows
// 3w .. 3w+2 in every stage. So the thread that loads a cell is the thread that finishes it
// (r_i never goes through LDS), rows are wave-uniform (row bounds and row addresses are scalar
// work), and a thread's three rows share the five image rows their stencils read.
//
// D^T D's 27-point stencil is reflection-symmetric per axis, so it has 8 distinct weights
// K(|dx|,|dy|,|dz|) and its dz = -1 and dz = +1 layers are equal: a plane contributes one
// in-plane 9-point sum k0 to output z and one sum k1 to outputs z-1 and z+1, accumulated in
// register queues. Boundaries: the reference's D^T D is a sum of Kronecker products of 1-D
// Neumann Laplacians (clamped neighbours). In dims 0 and 1 the image holds the mesh's
// half-sample MIRROR outside the mesh (cell -1 = cell 0, -2 = 1): the Neumann Laplacian
// commutes with that extension, so the plain stencil on the mirrored image gives the clamped
// result on the mesh AND the mirror of it on the ghost cells, which is exactly what the
// second stencil (w = A u) needs. In dim 2 the z-march duplicates the k1 term at planes 0 and
// m2-1. With W = I the identity is folded into the centre weight. The Jacobi diagonal takes
// one of 8 values by boundary pattern (interior / face along each dimension), tabulated in LDS.
#include <algorithm>
#include <cstdint>
#include <cstdlib>

#include "mvtv_device.h"

namespace mvtv {

namespace cg3d {
constexpr int IW = 64;                   // image row = one wavefront
constexpr int RPW = 3;                   // image rows per wave
constexpr int TX = IW - 4;               // 60 output columns
// NWV waves per workgroup: 8 -> 24 image rows (60 x 20 output tile), 16 -> 48 rows (60 x 44): the
// taller tile re-reads fewer halo rows of r and p (64 x 48 / (60 x 44) = 1.16 loads per owned cell
// against 64 x 24 / (60 x 20) = 1.28)
template <int NWV>
struct Shape {
    static constexpr int NT = NWV * 64, NW = NWV;
    static constexpr int IH = NW * RPW;
    static constexpr int TY = IH - 4;
    static constexpr int IMG = (IH + 2) * IW + 2;   // + a guard row above and below, + 1 word each end
};
}  // namespace cg3d

struct Cg3dArgs {
    const double* wdiag;
    double* x;
    const double* r_in;
    const double* p_in;
    double* r_out;
    double* p_out;
    const double* oty;
    const double* ga;
    const double* gb;
    const PcgState* st;
    double* partials;
    double K[8];     // sigma * D^T D weight at |dx| + 2 |dy| + 4 |dz| (+1 at [0] when W = I)
    double acc[8];   // sigma * diag(D^T D) by boundary pattern (bit j: interior along dim j)
    double ca, cb;
    int m0, m1, m2, tiles_x, tiles_y, zchunk, nblocks;
    int full_sync;   // probe builds (MVTV_CG3D_SYNC=1): __syncthreads in the plane loop instead of LDS-only barriers
};

// Half-sample mirror into [0, m): -1 -> 0, -2 -> 1, m -> m-1, m+1 -> m-2; clamped beyond.
__device__ __forceinline__ int mirror(int g, int m) {
    g = g < 0 ? -1 - g : g;
    g = g >= m ? 2 * m - 1 - g : g;
    return min(max(g, 0), m - 1);
}

// The 3 output rows of a wave from the 5 image rows around them: in-plane sums k0 (dz = 0
// layer) and k1 (dz = +-1 layer), and the centre value. img points at the wave's first row.
__device__ __forceinline__ void wave_rows(const double* img, const double* K, double (&k0)[cg3d::RPW],
                                          double (&k1)[cg3d::RPW], double (&ctr)[cg3d::RPW]) {
    using namespace cg3d;
    double c[RPW + 2], h[RPW + 2];
#pragma unroll
    for (int j = 0; j < RPW + 2; ++j) {
        const double* q = img + (j - 1) * IW;
        c[j] = q[0];
        h[j] = q[-1] + q[1];
    }
#pragma unroll
    for (int k = 0; k < RPW; ++k) {
        const double cv = c[k] + c[k + 2], hv = h[k] + h[k + 2];
        k0[k] = fma(K[0], c[k + 1], fma(K[1], h[k + 1], fma(K[2], cv, K[3] * hv)));
        k1[k] = fma(K[4], c[k + 1], fma(K[5], h[k + 1], fma(K[6], cv, K[7] * hv)));
        ctr[k] = c[k + 1];
    }
}

// MODE 0: prologue (r0 = b - A x0 with b = oty + ca ga + cb gb; reductions gamma0, delta0,
// |r0|^2, |b|^2); MODE 1: first iteration (beta = 0, p_{-1} not read); MODE 2: iteration;
// MODE 3: iteration that also moves x by both its own step and the previous one's.
template <int WM, int MODE, int NWV>
__global__ __launch_bounds__(cg3d::Shape<NWV>::NT, 32 / NWV) void k_cg3d(const Cg3dArgs a) {
    using namespace cg3d;
    using Sh = Shape<NWV>;
    constexpr int NT = Sh::NT, IH = Sh::IH, TY = Sh::TY, IMG = Sh::IMG;
    __shared__ double sP[IMG];   // plane z of p_i (x_0 in the prologue)
    __shared__ double sU[IMG];   // u_{i+1} of one plane
    __shared__ double sD[8];     // 1 / diag (W = I) or sigma diag(D^T D) (W diagonal), by pattern
    if (MODE != 0 && a.st->done) return;
    const double alpha = MODE == 0 ? 0.0 : a.st->alpha;
    const double alpha_prev = MODE == 3 ? a.st->alpha_prev : 0.0;
    const double beta = MODE >= 2 ? a.st->beta : 0.0;
    if (threadIdx.x < 8) sD[threadIdx.x] = WM == W_DIAG ? a.acc[threadIdx.x] : 1.0 / (1.0 + a.acc[threadIdx.x]);
    // the plane loop's barriers order the LDS images only: nothing this launch writes to HBM is read in it (r, p
    // ping-pong; x is written only where the same thread read it), so they need not wait for the global loads and
    // stores in flight — with __syncthreads the second barrier of a plane waited for the next plane's loads
    const bool full_sync = a.full_sync != 0;
    auto bar = [&]() {
        if (full_sync) __syncthreads();
        else lds_barrier();
    };

    const int m0 = a.m0, m1 = a.m1, m2 = a.m2;
    const size_t pl = size_t(m0) * size_t(m1);
    const int nt = a.tiles_x * a.tiles_y;
    // XCD-aware order: workgroups are dealt round-robin over the 8 XCDs (b and b+8 share one),
    // so give each XCD a contiguous run of tiles (a compact patch of tile rows): a tile's halo
    // lines are then its neighbours' own lines, fetched once into that XCD's L2. The grid is
    // padded to a multiple of 8; padding workgroups contribute zero partials. Placement
    // affects speed only, never results.
    const int bid = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
    if (bid >= a.nblocks) {
        if (threadIdx.x < 4) a.partials[blockIdx.x * 4 + threadIdx.x] = 0.0;
        return;
    }
    const int tz = bid / nt, trem = bid - tz * nt;
    const int ty = trem / a.tiles_x, tx = trem - ty * a.tiles_x;
    const int X0 = tx * TX, Y0 = ty * TY;
    const int z0 = tz * a.zchunk, z1 = min(m2, z0 + a.zchunk);

    // per-lane geometry (dim 0), fixed for the launch
    const int lane = threadIdx.x & 63;
    const int gx = X0 - 2 + lane;
    const int gxm = mirror(gx, m0);
    const uint32_t boff = uint32_t(gxm) * 8u;   // byte offset inside a mesh row
    const bool own_x = lane >= 2 && lane < IW - 2 && gx < m0;
    const int xb = int(gxm > 0 && gxm + 1 < m0);
    // per-row geometry (dim 1): wave-uniform
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int row0 = wv * RPW;
    size_t rowoff[RPW], xrowoff[RPW];
    int ypat[RPW];
    bool own_y[RPW];
#pragma unroll
    for (int k = 0; k < RPW; ++k) {
        const int rho = row0 + k, gy = Y0 - 2 + rho, gym = mirror(gy, m1);
        rowoff[k] = size_t(gym) * size_t(m0);
        // x is needed on tile rows only; halo rows load a tile row's lines instead (L2 hits)
        xrowoff[k] = size_t(mirror(Y0 - 2 + min(max(rho, 2), IH - 3), m1)) * size_t(m0);
        ypat[k] = int(gym > 0 && gym + 1 < m1) << 1;
        own_y[k] = rho >= 2 && rho < IH - 2 && gy < m1;
    }
    const int li = 1 + (row0 + 1) * IW + lane;   // LDS index of (row0, lane)

    // global element (plane z, slot k) at this lane
    auto ld = [&](const double* base, size_t zoff, int k) {
        return *reinterpret_cast<const double*>(reinterpret_cast<const char*>(base + zoff + rowoff[k]) + boff);
    };
    // stores are non-temporal: nothing written is read again in this launch, and keeping them
    // out of L2 leaves it to the halo lines that neighbouring tiles read
    auto st = [&](double* base, size_t zoff, int k, double v) {
        __builtin_nontemporal_store(v, reinterpret_cast<double*>(reinterpret_cast<char*>(base + zoff + rowoff[k]) + boff));
    };
    auto zpat = [&](int z) { return int(z > 0 && z + 1 < m2) << 2; };
    // M^-1 v at (slot k, pattern bits of the plane)
    auto minv = [&](double v, double wvv, int k, int zp) {
        const double d = sD[xb | ypat[k] | zp];
        return WM == W_DIAG ? v / (wvv + d) : v * d;
    };

    double bm1[RPW], b0[RPW], pcm1[RPW], pc0[RPW];   // s accumulators and p centres, outputs z-1, z
    double cm1[RPW], c0[RPW], ucm1[RPW];             // w accumulators (outputs e-1, e), u centre at e-1
    double rm1[RPW], rz[RPW];                        // r_i at planes z-1, z (own loads, never in LDS)
#pragma unroll
    for (int k = 0; k < RPW; ++k) bm1[k] = b0[k] = pcm1[k] = pc0[k] = cm1[k] = c0[k] = ucm1[k] = rm1[k] = rz[k] = 0.0;
    double red[4] = {0.0, 0.0, 0.0, 0.0};   // gamma, delta, |r|^2, |b|^2

    const int zs = max(0, z0 - 2), ze = min(m2 - 1, z1 + 1);
    const int ulo = max(0, z0 - 1), uhi = min(m2 - 1, z1);   // planes of s and u formed here

    // s of plane e is complete: r_{i+1}, u_{i+1} on tile + 1, then accumulate w = A u.
    auto finish_plane = [&](int e, bool last) {
        const size_t eoff = size_t(e) * pl;
        const bool own = e >= z0 && e < z1;
        const int zp = zpat(e);
        double uc[RPW];
#pragma unroll
        for (int k = 0; k < RPW; ++k) {
            const double wvv = WM == W_DIAG ? ld(a.wdiag, eoff, k) : 1.0;
            double se = last ? b0[k] : bm1[k];
            if (WM == W_DIAG) se = fma(wvv, last ? pc0[k] : pcm1[k], se);
            const bool tile = own && own_y[k] && own_x;
            double rn;
            if (MODE == 0) {
                const double b = fma(a.cb, ld(a.gb, eoff, k), fma(a.ca, ld(a.ga, eoff, k), ld(a.oty, eoff, k)));
                rn = b - se;
                if (tile) red[3] = fma(b, b, red[3]);
            } else {
                rn = fma(-alpha, se, last ? rz[k] : rm1[k]);
            }
            const double un = minv(rn, wvv, k, zp);
            sU[li + k * IW] = un;
            uc[k] = un;
            if (tile) {
                st(a.r_out, eoff, k, rn);
                red[0] = fma(rn, un, red[0]);
                red[2] = fma(rn, rn, red[2]);
            }
        }
        bar();
        double k0v[RPW], k1v[RPW], ctr[RPW];
        wave_rows(sU + li, a.K, k0v, k1v, ctr);
        const bool prev_own = e - 1 >= z0 && e - 1 < z1;   // w(e-1) is complete
        const bool end_own = e == m2 - 1 && own;             // last mesh plane: w(e) is complete too
#pragma unroll
        for (int k = 0; k < RPW; ++k) {
            cm1[k] += k1v[k];
            c0[k] += k0v[k] + (e == 0 ? k1v[k] : 0.0) + (e == m2 - 1 ? k1v[k] : 0.0);
            if (own_y[k] && own_x) {
                if (prev_own) {
                    double wq = cm1[k];
                    if (WM == W_DIAG) wq = fma(ld(a.wdiag, eoff - pl, k), ucm1[k], wq);
                    red[1] = fma(wq, ucm1[k], red[1]);
                }
                if (end_own) {
                    double wq = c0[k];
                    if (WM == W_DIAG) wq = fma(ld(a.wdiag, eoff, k), uc[k], wq);
                    red[1] = fma(wq, uc[k], red[1]);
                }
            }
            cm1[k] = c0[k];
            c0[k] = k1v[k];
            ucm1[k] = uc[k];
        }
        // no closing barrier: the next write of sU follows the next plane's post-commit barrier
    };

    // Stage A is split: issue() loads plane z's inputs into registers one plane ahead, so the HBM
    // latency of plane z+1 overlaps the stencil work of plane z; commit() forms p_i into LDS.
    double qr[RPW], qp[RPW], qx[RPW], qw[RPW];
#pragma unroll
    for (int k = 0; k < RPW; ++k) qr[k] = qp[k] = qx[k] = qw[k] = 0.0;
    auto issue = [&](int z) {
        const size_t zoff = size_t(z) * pl;
#pragma unroll
        for (int k = 0; k < RPW; ++k) {
            if (MODE == 0) {
                qx[k] = ld(a.x, zoff, k);
            } else {
                qr[k] = ld(a.r_in, zoff, k);
                if (MODE >= 2) qp[k] = ld(a.p_in, zoff, k);
                if (WM == W_DIAG) qw[k] = ld(a.wdiag, zoff, k);
                // unconditional (every address is valid): a conditional load into the queue
                // gets its stores merged with a dynamic index, which demotes qx to scratch
                if (MODE == 3)
                    qx[k] = *reinterpret_cast<const double*>(
                        reinterpret_cast<const char*>(a.x + zoff + xrowoff[k]) + boff);
            }
        }
    };
    auto commit = [&](int z) {
        const size_t zoff = size_t(z) * pl;
        const bool ownz = z >= z0 && z < z1;
        const int zp = zpat(z);
#pragma unroll
        for (int k = 0; k < RPW; ++k) {
            if (MODE == 0) {
                sP[li + k * IW] = qx[k];
            } else {
                double pi = minv(qr[k], qw[k], k, zp);
                if (MODE >= 2) pi = fma(beta, qp[k], pi);
                sP[li + k * IW] = pi;
                rz[k] = qr[k];
                if (ownz && own_y[k] && own_x) {
                    st(a.p_out, zoff, k, pi);
                    if (MODE == 3) st(a.x, zoff, k, fma(alpha, pi, fma(alpha_prev, qp[k], qx[k])));
                }
            }
        }
    };

    __syncthreads();   // sD
    issue(zs);
    for (int z = zs; z <= ze; ++z) {
        // ---------------- stage A: plane z of p_i (x_0 in the prologue) on tile + 2
        commit(z);
        bar();
        if (z + 1 <= ze) issue(z + 1);
        // ---------------- stage B: plane z feeds s at outputs z-1 (k1), z (k0), z+1 (k1); clamped
        // dim-2 neighbours: plane 0 is its own dz=-1 layer, plane m2-1 its own dz=+1 layer
        double k0v[RPW], k1v[RPW], ctr[RPW], bp1[RPW];
        wave_rows(sP + li, a.K, k0v, k1v, ctr);
#pragma unroll
        for (int k = 0; k < RPW; ++k) {
            bm1[k] += k1v[k];
            b0[k] += k0v[k] + (z == 0 ? k1v[k] : 0.0) + (z == m2 - 1 ? k1v[k] : 0.0);
            bp1[k] = k1v[k];
            pc0[k] = ctr[k];
        }
        bool synced = false;
        if (z - 1 >= ulo && z - 1 <= uhi) {
            finish_plane(z - 1, false);
            synced = true;
        }
        if (z == m2 - 1 && z >= ulo && z <= uhi) {
            if (synced) bar();   // sU is still being read by the previous plane's stage C
            finish_plane(z, true);
            synced = true;
        }
        if (!synced) bar();   // stage B's reads of sP before the next commit
#pragma unroll
        for (int k = 0; k < RPW; ++k) {
            bm1[k] = b0[k];
            b0[k] = bp1[k];
            pcm1[k] = pc0[k];
            rm1[k] = rz[k];
        }
    }
    block_reduce_store<4, 0, NT>(red, a.partials);
}

// ------------------------------------------------------------------------------------ launcher
hipError_t launch_cg3d(const Geom& g, hipStream_t s, int mode, double sigma, int wmode, const double* wdiag,
                       double* x, const double* r_in, const double* p_in, double* r_out, double* p_out,
                       const double* oty, const double* ga, double ca, const double* gb, double cb,
                       const PcgState* st, double* partials, int* nblocks_out) {
    using namespace cg3d;
    static const int nwv = [] {
        const char* e = probe_env("MVTV_CG3D_NW");
        return e && std::atoi(e) == 8 ? 8 : 16;
    }();
    const int TY = nwv == 16 ? Shape<16>::TY : Shape<8>::TY;
    Cg3dArgs a{};
    static const bool full_sync = probe_env("MVTV_CG3D_SYNC") != nullptr;
    a.full_sync = full_sync ? 1 : 0;
    a.m0 = int(g.m[0]);
    a.m1 = int(g.m[1]);
    a.m2 = int(g.m[2]);
    a.tiles_x = (a.m0 + TX - 1) / TX;
    a.tiles_y = (a.m1 + TY - 1) / TY;
    const int tiles = a.tiles_x * a.tiles_y;
    // dim-2 chunks: each costs 3 extra plane steps (halo planes); workgroups run in rounds of
    // `slots` (resident workgroups per CU x CUs), so pick the chunk count with the fewest plane steps per
    // slot. At 128 VGPRs a CU holds 16 waves: one 1024-thread workgroup (round 2's model assumed two, and
    // chose 4 chunks = 432 workgroups = 1.7 rounds at 512^3; the occupancy query picks 7 = 2.95 rounds,
    // 1.209 -> 1.193 ms per launch in a probe sweep, profiles/r04/v8_cg3d_chunks)
    static const int slots = [] {
        int dev = 0, cus = 256, per_cu = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            cus = 256;
        const hipError_t e = nwv == 16
            ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_cg3d<W_IDENTITY, 2, 16>, 1024, 0)
            : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_cg3d<W_IDENTITY, 2, 8>, 512, 0);
        if (e != hipSuccess || per_cu < 1) {
            (void)hipGetLastError();
            per_cu = 1;
        }
        return per_cu * std::max(1, cus);
    }();
    static const int nz_env = [] {
        const char* e = probe_env("MVTV_CG3D_NZ");
        return e ? atoi(e) : 0;
    }();
    int nz = 1;
    long best = -1;
    for (int c = 1; c <= a.m2 && c * tiles + 7 <= kMaxCgBlocks; ++c) {
        const int zc = (a.m2 + c - 1) / c;
        if ((a.m2 + zc - 1) / zc != c) continue;   // same chunking as a smaller count
        const long cost = long((c * tiles + slots - 1) / slots) * (zc + 3);
        if (best < 0 || cost < best) best = cost, nz = c;
    }
    if (nz_env > 0) nz = std::min(nz_env, a.m2);
    a.zchunk = (a.m2 + nz - 1) / nz;
    nz = (a.m2 + a.zchunk - 1) / a.zchunk;
    a.nblocks = tiles * nz;
    const int nblocks = (a.nblocks + 7) / 8 * 8;   // grid, padded for the XCD mapping
    if (nblocks > kMaxCgBlocks) return hipErrorInvalidValue;
    if (nblocks_out) *nblocks_out = nblocks;
    // K(o) = sum_S cS[S] prod_j f_j(o_j) with f = (j in S) ? (o == 0 ? 2 : -1) : (o == 0 ? 1 : 0):
    // even in every o_j, so it depends on |o_j| only. diag: l_j = 1 on a face, 2 inside.
    for (int t = 0; t < 8; ++t) {
        double kk = 0.0, dd = 0.0;
        for (int S = 1; S < 8; ++S) {
            double prod = g.cS[S], dprod = g.cS[S];
            for (int j = 0; j < 3; ++j) {
                const bool off = (t >> j) & 1;
                const bool inS = (S >> j) & 1;
                prod *= inS ? (off ? -1.0 : 2.0) : (off ? 0.0 : 1.0);
                if (inS) dprod *= ((t >> j) & 1) ? 2.0 : 1.0;
            }
            kk += prod;
            dd += dprod;
        }
        a.K[t] = sigma * kk;
        a.acc[t] = sigma * dd;
    }
    if (wmode != W_DIAG) a.K[0] += 1.0;   // W = I folded into the centre weight
    a.wdiag = wdiag;
    a.x = x;
    a.r_in = r_in;
    a.p_in = p_in;
    a.r_out = r_out;
    a.p_out = p_out;
    a.oty = oty;
    a.ga = ga;
    a.gb = gb;
    a.ca = ca;
    a.cb = cb;
    a.st = st;
    a.partials = partials;
    auto go = [&](auto kern) {
        klaunch(kern, dim3(nblocks), dim3(nwv * 64), 0, s, a);
        return hipGetLastError();
    };
    auto pick = [&](auto nc) {
        constexpr int NV = decltype(nc)::value;
        if (wmode == W_DIAG) {
            if (mode == 0) return go(k_cg3d<W_DIAG, 0, NV>);
            if (mode == 1) return go(k_cg3d<W_DIAG, 1, NV>);
            if (mode == 2) return go(k_cg3d<W_DIAG, 2, NV>);
            return go(k_cg3d<W_DIAG, 3, NV>);
        }
        if (mode == 0) return go(k_cg3d<W_IDENTITY, 0, NV>);
        if (mode == 1) return go(k_cg3d<W_IDENTITY, 1, NV>);
        if (mode == 2) return go(k_cg3d<W_IDENTITY, 2, NV>);
        return go(k_cg3d<W_IDENTITY, 3, NV>);
    };
    if (mode < 0 || mode > 3) return hipErrorInvalidValue;
    return nwv == 16 ? pick(std::integral_constant<int, 16>{}) : pick(std::integral_constant<int, 8>{});
}

// x += alpha_prev p when the solve stopped after an even iteration (st->iter odd): that iteration's step is the one
// k_cg3d left pending. Enqueued once after the iterations; a no-op otherwise.
__global__ __launch_bounds__(256) void k_cg_xflush(uint64_t n, double* __restrict__ x, const double* __restrict__ p,
                                                   const PcgState* __restrict__ st) {
    if ((st->iter & 1) == 0) return;
    const double al = st->alpha_prev;
    for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += uint64_t(gridDim.x) * 256)
        x[i] = fma(al, p[i], x[i]);
}

hipError_t launch_cg_xflush(hipStream_t s, uint64_t n, double* x, const double* p, const PcgState* st) {
    const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, 8192);
    klaunch(k_cg_xflush, dim3(uint32_t(std::max<uint64_t>(blocks, 1))), dim3(256), 0, s, n, x, p, st);
    return hipGetLastError();
}


// ------------------------------------------------------------------------------------ k_apply3d
// q = (W + sigma D^T D) x on a whole 3-D mesh: the ADMM start's g_alpha = D^T D theta_0
// (rcpp…/solvers.cpp:101, alpha_0 = D theta_0) and the operator checks. A thread owns one
// (dim 0, dim 1) column over a chunk of dim-2 planes and marches dim 2: each plane is read once
// per thread as its 3 x 3 in-plane neighbourhood (L1/L2 serve the 8 neighbours) and reduced to the
// two in-plane sums of the 8-weight symmetric stencil (dz = 0 layer, dz = +-1 layer); q(z) =
// s1(z-1) + s0(z) + s1(z+1) with half-sample mirrored neighbours (the Neumann structure of
// D^T D, as in k_cg3d). 2N words of HBM traffic against ~27 L2 reads per cell of the generic
// grid-stride k_apply_A. DOT (the PCG operator step): x.q per workgroup into `partials` (every
// workgroup of the grid writes its row) and a no-op once the PCG state is done.
struct Apply3dArgs {
    const double* x;
    double* q;
    const double* wdiag;
    double* partials;
    const PcgState* st;
    double K[8];
    int m0, m1, m2, tiles_x, tiles_y, zchunk, nblocks;
};

template <int WM, bool DOT>
__global__ __launch_bounds__(256) void k_apply3d(const Apply3dArgs a) {
    if (DOT && a.st->done) return;
    const int bid = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
    const int nt = a.tiles_x * a.tiles_y;
    const int tz = bid / nt, rem = bid - tz * nt;
    const int ty = rem / a.tiles_x, tx = rem - ty * a.tiles_x;
    const int x = tx * 64 + int(threadIdx.x & 63), y = ty * 4 + int(threadIdx.x >> 6);
    const int m0 = a.m0, m1 = a.m1, m2 = a.m2;
    double red[1] = {0.0};
    const bool act = bid < a.nblocks && x < m0 && y < m1;
    if (!DOT && !act) return;   // no barriers below without DOT
    const int z0 = tz * a.zchunk, z1 = act ? min(m2, z0 + a.zchunk) : z0;
    const size_t pl = size_t(m0) * size_t(m1);
    const size_t yd = size_t(mirror(y - 1, m1)) * m0, yc = size_t(y) * m0, yu = size_t(mirror(y + 1, m1)) * m0;
    const double K0 = a.K[0], K1 = a.K[1], K2 = a.K[2], K3 = a.K[3];
    const double K4 = a.K[4], K5 = a.K[5], K6 = a.K[6], K7 = a.K[7];
    // a wave is one 64-cell x-run of a row: the x +- 1 neighbours come from the adjacent lanes (wave
    // shuffles), only lanes 0 / 63 load the cell past the run; a mirrored neighbour is the cell itself.
    // Exited lanes (x >= m0) are never read: their active neighbour takes the mirror (itself).
    const int lane = int(threadIdx.x & 63);
    const bool has_l = x > 0, has_r = x + 1 < m0;
    const bool hload = (lane == 0 && has_l) || (lane == 63 && has_r);
    const int xh = lane == 0 ? x - 1 : x + 1;
    auto hsum = [&](const double* R, double c) {   // x-1 + x+1 neighbours of this lane's cell in row R
        const double e = hload ? R[xh] : 0.0;
        const double up = __shfl_up(c, 1), dn = __shfl_down(c, 1);
        const double l = has_l ? (lane == 0 ? e : up) : c;
        const double r = has_r ? (lane == 63 ? e : dn) : c;
        return l + r;
    };
    // in-plane sums of plane e: s0 (dz = 0 weights), s1 (dz = +-1 weights)
    auto sums = [&](int e, double& s0, double& s1) {
        const double* P = a.x + size_t(e) * pl;
        const double c = P[yc + x], cd = P[yd + x], cu = P[yu + x];
        const double h = hsum(P + yc, c);
        const double v = cd + cu;
        const double d = hsum(P + yd, cd) + hsum(P + yu, cu);
        s0 = fma(K0, c, fma(K1, h, fma(K2, v, K3 * d)));
        s1 = fma(K4, c, fma(K5, h, fma(K6, v, K7 * d)));
    };
    double s0c = 0.0, s1c = 0.0, s0n = 0.0, s1n = 0.0, s1m = 0.0;
    if (act) {
        sums(z0, s0c, s1c);
        if (z0 > 0) sums(z0 - 1, s0n, s1m);
        else s1m = s1c;
    }
    for (int z = z0; z < z1; ++z) {
        if (z + 1 < m2) sums(z + 1, s0n, s1n);
        else s1n = s1c, s0n = s0c;
        const size_t i = size_t(z) * pl + yc + x;
        double out = s1m + s0c + s1n;
        if (WM == W_DIAG) out = fma(a.wdiag[i], a.x[i], out);
        __builtin_nontemporal_store(out, a.q + i);
        if constexpr (DOT) red[0] = fma(a.x[i], out, red[0]);
        s1m = s1c;
        s0c = s0n;
        s1c = s1n;
    }
    if constexpr (DOT) block_reduce_store<1, 0>(red, a.partials);
}

// The same with two adjacent cells a lane (m0 even, 16-B aligned vectors): a wave covers a 128-cell x-run with 16-B
// loads and stores, so each of its march steps keeps twice the bytes in flight (the one-cell kernel waits a full
// memory latency per plane step: 0.72 ms at 512^3 for 2N words). The sums per cell are the one-cell kernel's, in the
// same order.
typedef double a3v2 __attribute__((ext_vector_type(2)));

template <int WM, bool DOT>
__global__ __launch_bounds__(256) void k_apply3d2(const Apply3dArgs a) {
    if (DOT && a.st->done) return;
    const int bid = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
    const int nt = a.tiles_x * a.tiles_y;
    const int tz = bid / nt, rem = bid - tz * nt;
    const int ty = rem / a.tiles_x, tx = rem - ty * a.tiles_x;
    const int lane = int(threadIdx.x & 63);
    const int x = tx * 128 + 2 * lane, y = ty * 4 + int(threadIdx.x >> 6);   // cells x, x + 1 (m0 even)
    const int m0 = a.m0, m1 = a.m1, m2 = a.m2;
    double red[1] = {0.0};
    const bool act = bid < a.nblocks && x < m0 && y < m1;
    if (!DOT && !act) return;   // no barriers below without DOT
    const int z0 = tz * a.zchunk, z1 = act ? min(m2, z0 + a.zchunk) : z0;
    const size_t pl = size_t(m0) * size_t(m1);
    const size_t yd = size_t(mirror(y - 1, m1)) * m0, yc = size_t(y) * m0, yu = size_t(mirror(y + 1, m1)) * m0;
    const double K0 = a.K[0], K1 = a.K[1], K2 = a.K[2], K3 = a.K[3];
    const double K4 = a.K[4], K5 = a.K[5], K6 = a.K[6], K7 = a.K[7];
    // cell x's right neighbour and cell x + 1's left one are the lane's own pair; x - 1 is the previous lane's
    // second cell, x + 2 the next lane's first (lanes 0 / 63 load them past the run); mirrored: the cell itself
    const bool has_l = x > 0, has_r = x + 2 < m0;
    const bool hload = (lane == 0 && has_l) || (lane == 63 && has_r);
    const int xh = lane == 0 ? x - 1 : x + 2;
    auto ld = [](const double* p) { return *reinterpret_cast<const a3v2*>(p); };
    auto hsum = [&](const double* R, a3v2 c) {
        const double e = hload ? R[xh] : 0.0;
        const double up = __shfl_up(c.y, 1), dn = __shfl_down(c.x, 1);
        const double l = has_l ? (lane == 0 ? e : up) : c.x;
        const double r = has_r ? (lane == 63 ? e : dn) : c.y;
        a3v2 h;
        h.x = l + c.y;
        h.y = c.x + r;
        return h;
    };
    auto comb = [](double k0, double k1, double k2, double k3, a3v2 c, a3v2 h, a3v2 v, a3v2 d) {
        a3v2 s;
        s.x = fma(k0, c.x, fma(k1, h.x, fma(k2, v.x, k3 * d.x)));
        s.y = fma(k0, c.y, fma(k1, h.y, fma(k2, v.y, k3 * d.y)));
        return s;
    };
    auto sums = [&](int e, a3v2& s0, a3v2& s1) {
        const double* P = a.x + size_t(e) * pl;
        const a3v2 c = ld(P + yc + x), cd = ld(P + yd + x), cu = ld(P + yu + x);
        const a3v2 h = hsum(P + yc, c);
        const a3v2 v = cd + cu;
        const a3v2 d = hsum(P + yd, cd) + hsum(P + yu, cu);
        s0 = comb(K0, K1, K2, K3, c, h, v, d);
        s1 = comb(K4, K5, K6, K7, c, h, v, d);
    };
    a3v2 s0c = 0.0, s1c = 0.0, s0n = 0.0, s1n = 0.0, s1m = 0.0;
    if (act) {
        sums(z0, s0c, s1c);
        if (z0 > 0) sums(z0 - 1, s0n, s1m);
        else s1m = s1c;
    }
    for (int z = z0; z < z1; ++z) {
        if (z + 1 < m2) sums(z + 1, s0n, s1n);
        else s1n = s1c, s0n = s0c;
        const size_t i = size_t(z) * pl + yc + x;
        a3v2 out = s1m + s0c + s1n;
        if (WM == W_DIAG) {
            const a3v2 w = ld(a.wdiag + i), xv = ld(a.x + i);
            out.x = fma(w.x, xv.x, out.x);
            out.y = fma(w.y, xv.y, out.y);
        }
        __builtin_nontemporal_store(out, reinterpret_cast<a3v2*>(a.q + i));
        if constexpr (DOT) {
            const a3v2 xv = ld(a.x + i);
            red[0] = fma(xv.y, out.y, fma(xv.x, out.x, red[0]));
        }
        s1m = s1c;
        s0c = s0n;
        s1c = s1n;
    }
    if constexpr (DOT) block_reduce_store<1, 0>(red, a.partials);
}

hipError_t launch_apply3d(const Geom& g, hipStream_t s, double sigma, int wmode, const double* wdiag,
                          const double* x, double* q, double* partials, const PcgState* st, int* nparts) {
    Apply3dArgs a{};
    a.m0 = int(g.m[0]);
    a.m1 = int(g.m[1]);
    a.m2 = int(g.m[2]);
    // two cells a lane where every row starts 16-B aligned (MVTV_APPLY3D_V1=1 in probe builds: one cell a lane)
    static const bool v1_env = probe_env("MVTV_APPLY3D_V1") != nullptr;
    const bool two = !v1_env && a.m0 % 2 == 0 &&
                     ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(q) |
                       reinterpret_cast<uintptr_t>(wmode == W_DIAG ? wdiag : nullptr)) & 15) == 0;
    a.tiles_x = two ? (a.m0 + 127) / 128 : (a.m0 + 63) / 64;
    a.tiles_y = (a.m1 + 3) / 4;
    const int tiles = a.tiles_x * a.tiles_y;
    int nz = std::max(1, std::min(a.m2, (two ? 4096 : 8192) / std::max(1, tiles)));
    a.zchunk = (a.m2 + nz - 1) / nz;
    nz = (a.m2 + a.zchunk - 1) / a.zchunk;
    a.nblocks = tiles * nz;
    const int grid = (a.nblocks + 7) / 8 * 8;
    for (int t = 0; t < 8; ++t) {   // the k_cg3d weights: K(o) = sigma sum_S cS[S] prod_j f_j(o_j)
        double kk = 0.0;
        for (int S = 1; S < 8; ++S) {
            double prod = g.cS[S];
            for (int j = 0; j < 3; ++j) {
                const bool off = (t >> j) & 1;
                prod *= ((S >> j) & 1) ? (off ? -1.0 : 2.0) : (off ? 0.0 : 1.0);
            }
            kk += prod;
        }
        a.K[t] = sigma * kk;
    }
    if (wmode == W_IDENTITY) a.K[0] += 1.0;
    a.x = x;
    a.q = q;
    a.wdiag = wdiag;
    a.partials = partials;
    a.st = st;
    if (partials) {
        if (!st || !nparts) return hipErrorInvalidValue;
        *nparts = grid;
        if (two && wmode == W_DIAG) klaunch(k_apply3d2<W_DIAG, true>, dim3(grid), dim3(256), 0, s, a);
        else if (two) klaunch(k_apply3d2<W_NONE, true>, dim3(grid), dim3(256), 0, s, a);
        else if (wmode == W_DIAG) klaunch(k_apply3d<W_DIAG, true>, dim3(grid), dim3(256), 0, s, a);
        else klaunch(k_apply3d<W_NONE, true>, dim3(grid), dim3(256), 0, s, a);
        return hipGetLastError();
    }
    if (two && wmode == W_DIAG) klaunch(k_apply3d2<W_DIAG, false>, dim3(grid), dim3(256), 0, s, a);
    else if (two) klaunch(k_apply3d2<W_NONE, false>, dim3(grid), dim3(256), 0, s, a);
    else if (wmode == W_DIAG) klaunch(k_apply3d<W_DIAG, false>, dim3(grid), dim3(256), 0, s, a);
    else klaunch(k_apply3d<W_NONE, false>, dim3(grid), dim3(256), 0, s, a);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------ k_apply4d
// The same for p = 4 (config 5's run start g_alpha = D^T D theta_0, rcpp…/solvers.cpp:101, and the PCG operator step
// of a 4-D W != I solve): a thread owns an (x, y, z) cell and marches dim 3. D^T D's 81-point stencil is even in every
// offset, so with K[|dx| + 2|dy| + 4|dz| + 8|dw|] a w-plane contributes one 27-point sum s0 (dw = 0 weights) to its own
// output and one s1 (dw = 1 weights) to the outputs w - 1 and w + 1: q(w) = s1(w - 1) + s0(w) + s1(w + 1), mirrored
// at the ends. The 27 neighbours of a plane come through L1 / L2 (a 64 x 4 tile's rows are whole 512-B runs);
// 2N words of HBM traffic against the generic grid-stride k_apply_A's 81 L2 reads per cell (10.2 ms at 128^4).
struct Apply4dArgs {
    const double* x;
    double* q;
    const double* wdiag;
    double* partials;
    const PcgState* st;
    double K[16];
    int m0, m1, m2, m3, tiles_x, tiles_y, wchunk, nblocks;
};

template <int WM, bool DOT>
__global__ __launch_bounds__(256) void k_apply4d(const Apply4dArgs a) {
    if (DOT && a.st->done) return;
    const int bid = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
    const int nxy = a.tiles_x * a.tiles_y, per_w = nxy * a.m2;
    const int tw = bid / per_w, rem = bid - tw * per_w;
    const int z = rem / nxy, rxy = rem - z * nxy;
    const int ty = rxy / a.tiles_x, tx = rxy - ty * a.tiles_x;
    const int x = tx * 64 + int(threadIdx.x & 63), y = ty * 4 + int(threadIdx.x >> 6);
    const int m0 = a.m0, m1 = a.m1, m2 = a.m2, m3 = a.m3;
    double red[1] = {0.0};
    const bool act = bid < a.nblocks && x < m0 && y < m1;
    if (!DOT && !act) return;   // no barriers below without DOT
    const int w0 = tw * a.wchunk, w1 = act ? min(m3, w0 + a.wchunk) : w0;
    const size_t pl = size_t(m0) * size_t(m1), pl3 = pl * size_t(m2);
    const int xs[3] = {mirror(x - 1, m0), x, mirror(x + 1, m0)};
    const size_t ys[3] = {size_t(mirror(y - 1, m1)) * m0, size_t(y) * m0, size_t(mirror(y + 1, m1)) * m0};
    const size_t zs[3] = {size_t(mirror(z - 1, m2)) * pl, size_t(z) * pl, size_t(mirror(z + 1, m2)) * pl};
    double K[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) K[t] = a.K[t];
    // in-plane (x, y, z) sums of plane w by offset class c = |dx| + 2|dy| + 4|dz|
    auto sums = [&](int w, double& s0, double& s1) {
        const double* P = a.x + size_t(w) * pl3;
        double v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int dz = 0; dz < 3; ++dz)
#pragma unroll
            for (int dy = 0; dy < 3; ++dy) {
                const double* R = P + zs[dz] + ys[dy];
                const int c = (dy != 1 ? 2 : 0) + (dz != 1 ? 4 : 0);
                v[c] += R[xs[1]];
                v[c | 1] += R[xs[0]] + R[xs[2]];
            }
        s0 = 0.0;
        s1 = 0.0;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            s0 = fma(K[c], v[c], s0);
            s1 = fma(K[8 + c], v[c], s1);
        }
    };
    double s0c = 0.0, s1c = 0.0, s0n = 0.0, s1n = 0.0, s1m = 0.0;
    if (act) {
        sums(w0, s0c, s1c);
        if (w0 > 0) sums(w0 - 1, s0n, s1m);
        else s1m = s1c;
    }
    const size_t cell = zs[1] + ys[1] + size_t(x);
    for (int w = w0; w < w1; ++w) {
        if (w + 1 < m3) sums(w + 1, s0n, s1n);
        else s1n = s1c, s0n = s0c;
        const size_t i = size_t(w) * pl3 + cell;
        double out = s1m + s0c + s1n;
        if (WM == W_DIAG) out = fma(a.wdiag[i], a.x[i], out);
        __builtin_nontemporal_store(out, a.q + i);
        if constexpr (DOT) red[0] = fma(a.x[i], out, red[0]);
        s1m = s1c;
        s0c = s0n;
        s1c = s1n;
    }
    if constexpr (DOT) block_reduce_store<1, 0>(red, a.partials);
}

hipError_t launch_apply4d(const Geom& g, hipStream_t s, double sigma, int wmode, const double* wdiag,
                          const double* x, double* q, double* partials, const PcgState* st, int* nparts) {
    Apply4dArgs a{};
    a.m0 = int(g.m[0]);
    a.m1 = int(g.m[1]);
    a.m2 = int(g.m[2]);
    a.m3 = int(g.m[3]);
    a.tiles_x = (a.m0 + 63) / 64;
    a.tiles_y = (a.m1 + 3) / 4;
    const long items = long(a.tiles_x) * a.tiles_y * a.m2;   // (tile, z) columns, each marching dim 3
    int nw = int(std::max<long>(1, std::min<long>(a.m3, 8192 / std::max<long>(1, items))));
    a.wchunk = (a.m3 + nw - 1) / nw;
    nw = (a.m3 + a.wchunk - 1) / a.wchunk;
    if (items * nw > long(kMaxCgBlocks) * kMaxRed) return hipErrorInvalidValue;
    a.nblocks = int(items * nw);
    const int grid = (a.nblocks + 7) / 8 * 8;
    for (int t = 0; t < 16; ++t) {   // K(o) = sigma sum_S cS[S] prod_j f_j(o_j), t = |dx| + 2|dy| + 4|dz| + 8|dw|
        double kk = 0.0;
        for (int S = 1; S < 16; ++S) {
            double prod = g.cS[S];
            for (int j = 0; j < 4; ++j) {
                const bool off = (t >> j) & 1;
                prod *= ((S >> j) & 1) ? (off ? -1.0 : 2.0) : (off ? 0.0 : 1.0);
            }
            kk += prod;
        }
        a.K[t] = sigma * kk;
    }
    if (wmode == W_IDENTITY) a.K[0] += 1.0;
    a.x = x;
    a.q = q;
    a.wdiag = wdiag;
    a.partials = partials;
    a.st = st;
    if (partials) {
        if (!st || !nparts) return hipErrorInvalidValue;
        *nparts = grid;
        if (wmode == W_DIAG) klaunch(k_apply4d<W_DIAG, true>, dim3(grid), dim3(256), 0, s, a);
        else klaunch(k_apply4d<W_NONE, true>, dim3(grid), dim3(256), 0, s, a);
        return hipGetLastError();
    }
    if (wmode == W_DIAG) klaunch(k_apply4d<W_DIAG, false>, dim3(grid), dim3(256), 0, s, a);
    else klaunch(k_apply4d<W_NONE, false>, dim3(grid), dim3(256), 0, s, a);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------ k_apply2d
// The same for p = 2 (configs 2 and 4: the PCG operator step of a CV fold): a thread owns one dim-0
// column over a chunk of >= 8 rows and marches dim 1; a row contributes s0 = K0 c + K1 (l + r) to its own
// output and s1 = K2 c + K3 (l + r) to the rows above and below (K indexed by |dx| + 2 |dy|), with the
// half-sample mirror at the ends. 2N words against the 9 L2 reads per cell of the generic stencil.
struct Apply2dArgs {
    const double* x;
    double* q;
    const double* wdiag;
    double* partials;
    const PcgState* st;
    double K[4];
    int m0, m1, tiles_x, ychunk, nblocks;
};

template <int WM, bool DOT>
__global__ __launch_bounds__(256) void k_apply2d(const Apply2dArgs a) {
    if (DOT && a.st->done) return;
    const int bid = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
    const int ty = bid / a.tiles_x, tx = bid - ty * a.tiles_x;
    const int x = tx * 256 + int(threadIdx.x);
    const int m0 = a.m0, m1 = a.m1;
    double red[1] = {0.0};
    const bool act = bid < a.nblocks && x < m0;
    if (!DOT && !act) return;   // no barriers below without DOT
    const int y0 = ty * a.ychunk, y1 = act ? min(m1, y0 + a.ychunk) : y0;
    const int xl = mirror(x - 1, m0), xr = mirror(x + 1, m0);
    const double K0 = a.K[0], K1 = a.K[1], K2 = a.K[2], K3 = a.K[3];
    auto sums = [&](int y, double& s0, double& s1) {
        const double* R = a.x + size_t(y) * size_t(m0);
        const double c = R[x], h = R[xl] + R[xr];
        s0 = fma(K0, c, K1 * h);
        s1 = fma(K2, c, K3 * h);
    };
    double s0c = 0.0, s1c = 0.0, s0n = 0.0, s1n = 0.0, s1m = 0.0;
    if (act) {
        sums(y0, s0c, s1c);
        if (y0 > 0) sums(y0 - 1, s0n, s1m);
        else s1m = s1c;
    }
    for (int y = y0; y < y1; ++y) {
        if (y + 1 < m1) sums(y + 1, s0n, s1n);
        else s1n = s1c, s0n = s0c;
        const size_t i = size_t(y) * size_t(m0) + size_t(x);
        double out = s1m + s0c + s1n;
        if (WM == W_DIAG) out = fma(a.wdiag[i], a.x[i], out);
        __builtin_nontemporal_store(out, a.q + i);
        if constexpr (DOT) red[0] = fma(a.x[i], out, red[0]);
        s1m = s1c;
        s0c = s0n;
        s1c = s1n;
    }
    if constexpr (DOT) block_reduce_store<1, 0>(red, a.partials);
}

hipError_t launch_apply2d(const Geom& g, hipStream_t s, double sigma, int wmode, const double* wdiag,
                          const double* x, double* q, double* partials, const PcgState* st, int* nparts) {
    Apply2dArgs a{};
    a.m0 = int(g.m[0]);
    a.m1 = int(g.m[1]);
    a.tiles_x = (a.m0 + 255) / 256;
    int ny = std::max(1, std::min(std::max(1, a.m1 / 8), 8192 / a.tiles_x));   // >= 8 rows per chunk
    a.ychunk = (a.m1 + ny - 1) / ny;
    ny = (a.m1 + a.ychunk - 1) / a.ychunk;
    a.nblocks = a.tiles_x * ny;
    const int grid = (a.nblocks + 7) / 8 * 8;
    for (int t = 0; t < 4; ++t) {   // K(|dx|, |dy|) = sigma sum_S cS[S] prod_j f_j, t = |dx| + 2 |dy|
        double kk = 0.0;
        for (int S = 1; S < 4; ++S) {
            double prod = g.cS[S];
            for (int j = 0; j < 2; ++j) {
                const bool off = (t >> j) & 1;
                prod *= ((S >> j) & 1) ? (off ? -1.0 : 2.0) : (off ? 0.0 : 1.0);
            }
            kk += prod;
        }
        a.K[t] = sigma * kk;
    }
    if (wmode == W_IDENTITY) a.K[0] += 1.0;
    a.x = x;
    a.q = q;
    a.wdiag = wdiag;
    a.partials = partials;
    a.st = st;
    if (partials) {
        if (!st || !nparts || grid > kMaxCgBlocks * kMaxRed) return hipErrorInvalidValue;
        *nparts = grid;
        if (wmode == W_DIAG) klaunch(k_apply2d<W_DIAG, true>, dim3(grid), dim3(256), 0, s, a);
        else klaunch(k_apply2d<W_NONE, true>, dim3(grid), dim3(256), 0, s, a);
        return hipGetLastError();
    }
    if (wmode == W_DIAG) klaunch(k_apply2d<W_DIAG, false>, dim3(grid), dim3(256), 0, s, a);
    else klaunch(k_apply2d<W_NONE, false>, dim3(grid), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace mvtv

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
// HBM traffic per iteration is 6N words (read x, r, p; write x, r, p) against 11N for the
// three-kernel PCG. r and p ping-pong between two buffers: a launch reads neighbour halos of
// r_i and p_{i-1} that their owning workgroups overwrite. A 512-thread workgroup owns a 64 x 16
// column of the (dim 0, dim 1) plane over a chunk of dim-2 planes and marches through dim 2:
// each plane is loaded once into LDS (with a 2-cell halo). D^T D's 27-point stencil is
// reflection-symmetric per axis, so it has 8 distinct weights K(|dx|,|dy|,|dz|) and its
// dz = -1 and dz = +1 layers are equal: a plane contributes one in-plane 9-point sum k0 to
// output z and one sum k1 to outputs z-1 and z+1, accumulated in register queues (9 LDS reads
// per cell per plane). Neighbours outside the mesh are clamped (1-D Neumann Laplacians,
// x_{-1} := x_0), which is exactly the reference's D^T D. The Jacobi diagonal takes one of 8
// values by boundary pattern (interior / face along each dimension), tabulated in LDS.
#include <algorithm>

#include "mvtv_device.h"

namespace mvtv {

namespace cg3d {
constexpr int NT = 512;                   // threads per workgroup
constexpr int TX = 64, TY = 16;
constexpr int AX = TX + 4, AY = TY + 4;   // tile + 2 halo
constexpr int BX = TX + 2, BY = TY + 2;   // tile + 1 halo
constexpr int NA = AX * AY, NB = BX * BY, NC = TX * TY;
constexpr int SA = (NA + NT - 1) / NT;
constexpr int SB = (NB + NT - 1) / NT;
constexpr int SC = NC / NT;
static_assert(NC % NT == 0, "tile must be a multiple of the block");
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
    double K[8];     // sigma * D^T D weight at |dx| + 2 |dy| + 4 |dz|
    double acc[8];   // sigma * diag(D^T D) by boundary pattern (bit j: interior along dim j)
    double ca, cb;
    int m0, m1, m2, tiles_x, tiles_y, zchunk;
};

// One cell of a RX-wide region with origin (ox, oy), reading neighbours from an LDS image of
// row length IX with origin (iox, ioy); neighbour offsets are 0 where the mesh clamps them.
struct Cell {
    int gx, gy, c, xl, xr, yl, yr;
    bool in;
};

// INT: the workgroup's tile + 2 halo lies inside the mesh in dims 0 and 1, so no neighbour is
// clamped and every cell is in the mesh (about 70 % of the workgroups at 512^3).
template <int RX, int NREG, int IX, bool INT>
__device__ __forceinline__ Cell cell_of(int cell, int ox, int oy, int iox, int ioy, int m0, int m1) {
    Cell s;
    const int ly = cell / RX, lx = cell - ly * RX;
    s.gx = ox + lx;
    s.gy = oy + ly;
    s.c = (s.gy - ioy) * IX + (s.gx - iox);
    if constexpr (INT) {
        s.in = cell < NREG;
        s.xl = -1;
        s.xr = 1;
        s.yl = -IX;
        s.yr = IX;
    } else {
        s.in = cell < NREG && s.gx >= 0 && s.gx < m0 && s.gy >= 0 && s.gy < m1;
        s.xl = s.gx > 0 ? -1 : 0;
        s.xr = s.gx + 1 < m0 ? 1 : 0;
        s.yl = s.gy > 0 ? -IX : 0;
        s.yr = s.gy + 1 < m1 ? IX : 0;
    }
    return s;
}

template <bool INT>
__device__ __forceinline__ int bpat(int gx, int gy, int gz, int m0, int m1, int m2) {
    const int zb = int(gz > 0 && gz + 1 < m2) << 2;
    if constexpr (INT) return 3 | zb;
    return int(gx > 0 && gx + 1 < m0) | (int(gy > 0 && gy + 1 < m1) << 1) | zb;
}

// In-plane sums of the dz = 0 layer (k0) and of the dz = +-1 layers (k1) around cell s.
__device__ __forceinline__ void plane_sums(const double* img, const Cell& s, const double* K, double& k0,
                                           double& k1, double& centre) {
    const int r0 = s.c + s.yl, r2 = s.c + s.yr;
    const double c1 = img[s.c], h1 = img[s.c + s.xl] + img[s.c + s.xr];
    const double cv = img[r0] + img[r2];
    const double hv = img[r0 + s.xl] + img[r0 + s.xr] + img[r2 + s.xl] + img[r2 + s.xr];
    centre = c1;
    k0 = fma(K[0], c1, fma(K[1], h1, fma(K[2], cv, K[3] * hv)));
    k1 = fma(K[4], c1, fma(K[5], h1, fma(K[6], cv, K[7] * hv)));
}

// MODE 0: prologue (r0 = b - A x0 with b = oty + ca ga + cb gb; reductions gamma0, delta0,
// |r0|^2, |b|^2); MODE 1: first iteration (beta = 0, p_{-1} not read); MODE 2: iteration.
template <int WM, int MODE, bool INT>
__device__ __forceinline__ void cg3d_body(const Cg3dArgs& a, double* sP, double (*sR)[cg3d::NB], double* sU,
                                          const double* sD, int X0, int Y0, int z0, int z1, double alpha,
                                          double beta) {
    using namespace cg3d;
    int tid = threadIdx.x;   // re-hidden from the optimiser every plane (see the z loop)
    const int m0 = a.m0, m1 = a.m1, m2 = a.m2;
    const size_t pl = size_t(m0) * size_t(m1);

    // M^-1 v at a cell (W = I: table of reciprocals; W diagonal: one division)
    auto minv = [&](double v, double wv, int pat) {
        return WM == W_DIAG ? v / (wv + sD[pat]) : v * sD[pat];
    };

    double bm1[SB], b0[SB], pcm1[SB], pc0[SB];   // s accumulators and p centres, outputs z-1, z
    double cm1[SC], c0[SC], ucm1[SC];            // w accumulators (outputs e-1, e), u centre at e-1
#pragma unroll
    for (int k = 0; k < SB; ++k) bm1[k] = b0[k] = pcm1[k] = pc0[k] = 0.0;
#pragma unroll
    for (int k = 0; k < SC; ++k) cm1[k] = c0[k] = ucm1[k] = 0.0;
    double red[4] = {0.0, 0.0, 0.0, 0.0};   // gamma, delta, |r|^2, |b|^2

    const int zs = max(0, z0 - 2), ze = min(m2 - 1, z1 + 1);
    const int ulo = max(0, z0 - 1), uhi = min(m2 - 1, z1);   // planes of s and u formed here

    // s of plane e is complete: r_{i+1}, u_{i+1} on tile + 1, then accumulate w = A u.
    auto finish_plane = [&](int e, bool last) {
        const size_t eoff = size_t(e) * pl;
        const bool own = e >= z0 && e < z1;
#pragma unroll
        for (int k = 0; k < SB; ++k) {
            const int bc = tid + k * NT;
            const Cell s = cell_of<BX, NB, AX, INT>(bc, X0 - 1, Y0 - 1, X0 - 2, Y0 - 2, m0, m1);
            if (s.in) {
                const size_t gi = eoff + size_t(s.gy) * m0 + s.gx;
                const double wv = WM == W_DIAG ? a.wdiag[gi] : 1.0;
                const double se = fma(wv, last ? pc0[k] : pcm1[k], last ? b0[k] : bm1[k]);
                const bool tile = own && s.gx >= X0 && s.gx < X0 + TX && s.gy >= Y0 && s.gy < Y0 + TY;
                double rn;
                if (MODE == 0) {
                    const double b = fma(a.cb, a.gb[gi], fma(a.ca, a.ga[gi], a.oty[gi]));
                    rn = b - se;
                    if (tile) red[3] = fma(b, b, red[3]);
                } else {
                    rn = fma(-alpha, se, sR[e & 1][bc]);
                }
                const double un = minv(rn, wv, bpat<INT>(s.gx, s.gy, e, m0, m1, m2));
                sU[bc] = un;
                if (tile) {
                    a.r_out[gi] = rn;
                    red[0] = fma(rn, un, red[0]);
                    red[2] = fma(rn, rn, red[2]);
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < SC; ++k) {
            const Cell s = cell_of<TX, NC, BX, INT>(tid + k * NT, X0, Y0, X0 - 1, Y0 - 1, m0, m1);
            double k0v = 0.0, k1v = 0.0, ctr = 0.0;
            if (s.in) plane_sums(sU, s, a.K, k0v, k1v, ctr);
            cm1[k] += k1v;
            c0[k] += k0v + (e == 0 ? k1v : 0.0) + (e == m2 - 1 ? k1v : 0.0);
            if (s.in) {
                if (e - 1 >= z0 && e - 1 < z1) {   // w(e-1) is complete
                    const double wv = WM == W_DIAG ? a.wdiag[size_t(e - 1) * pl + size_t(s.gy) * m0 + s.gx] : 1.0;
                    red[1] = fma(fma(wv, ucm1[k], cm1[k]), ucm1[k], red[1]);
                }
                if (e == m2 - 1 && own) {          // last mesh plane: w(e) is complete too
                    const double wv = WM == W_DIAG ? a.wdiag[eoff + size_t(s.gy) * m0 + s.gx] : 1.0;
                    red[1] = fma(fma(wv, ctr, c0[k]), ctr, red[1]);
                }
            }
            cm1[k] = c0[k];
            c0[k] = k1v;
            ucm1[k] = ctr;
        }
        __syncthreads();
    };

    // Stage A is split: issue() loads plane z's inputs into registers one plane ahead, so the HBM
    // latency of plane z+1 overlaps the stencil work of plane z; commit() forms p_i into LDS.
    double qr[SA], qp[SA], qx[SA], qw[SA];
#pragma unroll
    for (int k = 0; k < SA; ++k) qr[k] = qp[k] = qx[k] = qw[k] = 0.0;
    auto a_cell = [&](int k, int& lx, int& ly, int& gx, int& gy) {
        const int cell = tid + k * NT;
        ly = cell / AX;
        lx = cell - ly * AX;
        gx = X0 - 2 + lx;
        gy = Y0 - 2 + ly;
        if constexpr (INT) return cell < NA;
        return cell < NA && gx >= 0 && gx < m0 && gy >= 0 && gy < m1;
    };
    auto issue = [&](int z) {
        const size_t zoff = size_t(z) * pl;
        const bool ownz = z >= z0 && z < z1;
#pragma unroll
        for (int k = 0; k < SA; ++k) {
            int lx, ly, gx, gy;
            if (a_cell(k, lx, ly, gx, gy)) {
                const size_t gi = zoff + size_t(gy) * m0 + gx;
                if (MODE == 0) {
                    qx[k] = a.x[gi];
                } else {
                    qr[k] = a.r_in[gi];
                    if (MODE == 2) qp[k] = a.p_in[gi];
                    if (WM == W_DIAG) qw[k] = a.wdiag[gi];
                    if (ownz && lx >= 2 && lx < TX + 2 && ly >= 2 && ly < TY + 2) qx[k] = a.x[gi];
                }
            }
        }
    };
    auto commit = [&](int z) {
        const size_t zoff = size_t(z) * pl;
        const bool ownz = z >= z0 && z < z1;
#pragma unroll
        for (int k = 0; k < SA; ++k) {
            int lx, ly, gx, gy;
            if (a_cell(k, lx, ly, gx, gy)) {
                const int cell = tid + k * NT;
                if (MODE == 0) {
                    sP[cell] = qx[k];
                } else {
                    const double ri = qr[k];
                    double pi = minv(ri, qw[k], bpat<INT>(gx, gy, z, m0, m1, m2));
                    if (MODE == 2) pi = fma(beta, qp[k], pi);
                    sP[cell] = pi;
                    if (lx >= 1 && lx <= BX && ly >= 1 && ly <= BY) sR[z & 1][(ly - 1) * BX + (lx - 1)] = ri;
                    if (ownz && lx >= 2 && lx < TX + 2 && ly >= 2 && ly < TY + 2) {
                        const size_t gi = zoff + size_t(gy) * m0 + gx;
                        a.p_out[gi] = pi;
                        a.x[gi] = fma(alpha, pi, qx[k]);
                    }
                }
            }
        }
    };

    issue(zs);
    for (int z = zs; z <= ze; ++z) {
        // Make tid opaque per plane so the per-slot cell geometry is recomputed instead of hoisted
        // out of the loop (hoisting it costs ~80 VGPRs and halves the workgroups per CU).
        asm volatile("" : "+v"(tid));
        // ---------------- stage A: plane z of p_i (x_0 in the prologue) on tile + 2, r_i on tile + 1
        commit(z);
        __syncthreads();
        if (z + 1 <= ze) issue(z + 1);
        // ---------------- stage B: plane z feeds s at outputs z-1 (k1), z (k0), z+1 (k1); clamped
        // dim-2 neighbours: plane 0 is its own dz=-1 layer, plane m2-1 its own dz=+1 layer
        double bp1[SB];
#pragma unroll
        for (int k = 0; k < SB; ++k) {
            const Cell s = cell_of<BX, NB, AX, INT>(tid + k * NT, X0 - 1, Y0 - 1, X0 - 2, Y0 - 2, m0, m1);
            double k0v = 0.0, k1v = 0.0, ctr = 0.0;
            if (s.in) plane_sums(sP, s, a.K, k0v, k1v, ctr);
            bm1[k] += k1v;
            b0[k] += k0v + (z == 0 ? k1v : 0.0) + (z == m2 - 1 ? k1v : 0.0);
            bp1[k] = k1v;
            pc0[k] = ctr;
        }
        bool synced = false;
        if (z - 1 >= ulo && z - 1 <= uhi) {
            finish_plane(z - 1, false);
            synced = true;
        }
        if (z == m2 - 1 && z >= ulo && z <= uhi) {
            finish_plane(z, true);
            synced = true;
        }
        if (!synced) __syncthreads();
#pragma unroll
        for (int k = 0; k < SB; ++k) {
            bm1[k] = b0[k];
            b0[k] = bp1[k];
            pcm1[k] = pc0[k];
        }
    }
    block_reduce_store<4, 0, NT>(red, a.partials);
}

template <int WM, int MODE>
__global__ __launch_bounds__(cg3d::NT, 4) void k_cg3d(const Cg3dArgs a) {
    using namespace cg3d;
    __shared__ double sP[NA];      // plane z of p_i (x_0 in the prologue), tile + 2
    __shared__ double sR[2][NB];   // r_i of planes z-1, z (ping-pong), tile + 1
    __shared__ double sU[NB];      // u_{i+1} of one plane, tile + 1
    __shared__ double sD[8];       // 1 / diag (W = I) or sigma diag(D^T D) (W diagonal), by pattern
    if (MODE != 0 && a.st->done) return;
    const double alpha = MODE == 0 ? 0.0 : a.st->alpha;
    const double beta = MODE == 2 ? a.st->beta : 0.0;
    if (threadIdx.x < 8) sD[threadIdx.x] = WM == W_DIAG ? a.acc[threadIdx.x] : 1.0 / (1.0 + a.acc[threadIdx.x]);
    const int nt = a.tiles_x * a.tiles_y;
    // XCD-aware order: workgroups are dealt round-robin over the 8 XCDs (b and b+8 share one),
    // so give each XCD a contiguous run of tiles; neighbouring tiles then share their halo
    // lines in that XCD's L2. Placement affects speed only, never results.
    int bid = blockIdx.x;
    if ((gridDim.x & 7) == 0) bid = (bid & 7) * (gridDim.x >> 3) + (bid >> 3);
    const int tz = bid / nt, trem = bid - tz * nt;
    const int ty = trem / a.tiles_x, tx = trem - ty * a.tiles_x;
    const int X0 = tx * TX, Y0 = ty * TY;
    const int z0 = tz * a.zchunk, z1 = min(a.m2, z0 + a.zchunk);
    __syncthreads();
    if (X0 >= 2 && X0 + AX - 2 <= a.m0 && Y0 >= 2 && Y0 + AY - 2 <= a.m1)
        cg3d_body<WM, MODE, true>(a, sP, sR, sU, sD, X0, Y0, z0, z1, alpha, beta);
    else
        cg3d_body<WM, MODE, false>(a, sP, sR, sU, sD, X0, Y0, z0, z1, alpha, beta);
}

// ------------------------------------------------------------------------------------ launcher
hipError_t launch_cg3d(const Geom& g, hipStream_t s, int mode, double sigma, int wmode, const double* wdiag,
                       double* x, const double* r_in, const double* p_in, double* r_out, double* p_out,
                       const double* oty, const double* ga, double ca, const double* gb, double cb,
                       const PcgState* st, double* partials, int* nblocks_out) {
    using namespace cg3d;
    Cg3dArgs a{};
    a.m0 = int(g.m[0]);
    a.m1 = int(g.m[1]);
    a.m2 = int(g.m[2]);
    a.tiles_x = (a.m0 + TX - 1) / TX;
    a.tiles_y = (a.m1 + TY - 1) / TY;
    const int tiles = a.tiles_x * a.tiles_y;
    int nz = std::max(1, std::min(a.m2 / 16, (1024 + tiles - 1) / tiles));
    a.zchunk = (a.m2 + nz - 1) / nz;
    nz = (a.m2 + a.zchunk - 1) / a.zchunk;
    const int nblocks = tiles * nz;
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
        hipLaunchKernelGGL(kern, dim3(nblocks), dim3(NT), 0, s, a);
        return hipGetLastError();
    };
    if (wmode == W_DIAG) {
        if (mode == 0) return go(k_cg3d<W_DIAG, 0>);
        if (mode == 1) return go(k_cg3d<W_DIAG, 1>);
        return go(k_cg3d<W_DIAG, 2>);
    }
    if (mode == 0) return go(k_cg3d<W_IDENTITY, 0>);
    if (mode == 1) return go(k_cg3d<W_IDENTITY, 1>);
    return go(k_cg3d<W_IDENTITY, 2>);
}

}  // namespace mvtv

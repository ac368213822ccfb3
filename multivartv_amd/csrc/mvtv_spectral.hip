// mvtv_spectral.hip — exact theta-solve by fast cosine transforms (W = I, power-of-two meshes).
//
// The reference solves (O^T O + rho D^T D) theta = b with SuperLU every ADMM iteration
// (rcpp-code/MultivarTV/src/solvers.cpp:113; cpp-code/solvers.cpp:116). On a mesh fit
// (mesh == data, O = I) that matrix is a sum of Kronecker products of 1-D Neumann Laplacians
// (SURVEY Appendix A):
//
//     A = I + sigma * sum_S cS[S] (x)_{j in S} L_j,      L_j = D1^T D1 (m_j x m_j)
//
// and every L_j is diagonalised by the DCT-II: L_j = C^T diag(lam_j) C with
// lam_j(k) = 4 sin^2(pi k / (2 m_j)). So A^-1 b = IDCT( DCT(b) / mu ), with
// mu(k) = 1 + sigma * sum_S cS[S] prod_{j in S} lam_j(k_j): a direct solve, exact to
// rounding, in 2p - 1 streaming passes over the mesh instead of K PCG iterations.
//
// One pass transforms every line of the mesh along one dimension d. A workgroup owns TQ
// lines (TQ consecutive line indices: for d > 0 they are TQ adjacent dim-0 cells, so every
// line position is a contiguous 8*TQ-byte row and loads are coalesced; for d = 0 each line
// is contiguous itself). Lines are paired as the real and imaginary parts of one complex
// sequence, so a length-m real DCT costs half a length-m complex FFT:
//
//   forward (DCT-II, Makhoul):  v[n] = x[2n], v[m-1-n] = x[2n+1];  Z = FFT(v_a + i v_b)
//                               A = (Z[k] + conj Z[m-k]) / 2, B = (Z[k] - conj Z[m-k]) / 2i
//                               X[k] = Re(e^{-i pi k/2m} A[k])   (same for B)
//   inverse (DCT-III):          V[k] = e^{i pi k/2m} (X[k] - i X[m-k]),  X[m] = 0
//                               v_a + i v_b = IFFT(V_a + i V_b), un-permute
//
// The FFT runs in LDS: radix-2^2 in-place stages, decimation in time on input loaded in
// bit-reversed order (forward), decimation in frequency leaving bit-reversed output (inverse),
// so both permutations fold into the global load/store index. The pass along the last
// dimension does forward, the divide by mu (and the 1/N of the inverse transforms) and the
// inverse in one launch. The first pass forms b = oty + ca*ga + cb*gb on load.
//
// HBM traffic per solve: 8 * (4N + 2N*(2p - 2)) bytes = 12N words at p = 3 (against 6N words
// per fused PCG iteration x ~44 iterations).
#include <algorithm>
#include <cmath>
#include <cstdint>

#include "mvtv_device.h"

namespace mvtv {

namespace spec {
constexpr int NT = 256;               // threads per workgroup
constexpr int LDS_WORDS = 8192;       // real doubles per workgroup tile (64 KB): TQ * m <= 8192
constexpr int PAD = 1;                // complex slots of padding per line (bank spread)
}  // namespace spec

struct SpecArgs {
    const double* in;        // input lines (FORMB: oty)
    const double* ga;        // FORMB: b = in + ca * ga + cb * gb
    const double* gb;
    double ca, cb;
    double* out;
    const double2* tw;       // FFT twiddles e^{-2 pi i k / m}, k < m/2
    const double2* twq;      // quarter-wave twiddles e^{-i pi k / 2m}, k < m
    const double* lam;       // MID: per-dim eigenvalue tables, lam + lam_off[j]
    uint32_t lam_off[kMaxDims];
    uint32_t m[kMaxDims];
    FastDiv fd[kMaxDims - 1];
    double cS[16];
    double sigma, w0, inv_n;
    uint32_t stride;         // element stride along the line (1 for d = 0)
    uint32_t nlines;         // N / m
    int32_t d, p, L, tq;     // line dimension, dims, log2 m, lines per workgroup
    int32_t ls;              // log2 stride
};

enum SpecMode { SPEC_FWD = 0, SPEC_INV = 1, SPEC_MID = 2 };

__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
    return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 csub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double2 cconj(double2 a) { return make_double2(a.x, -a.y); }
// multiply by -i (forward) or +i (inverse)
template <bool INV>
__device__ __forceinline__ double2 crot(double2 a) {
    return INV ? make_double2(-a.y, a.x) : make_double2(a.y, -a.x);
}

// Position of DCT input sample k in the bit-reversed Makhoul sequence.
__device__ __forceinline__ uint32_t perm_pos(uint32_t k, uint32_t m, int L) {
    const uint32_t n = (k & 1u) ? m - 1u - (k >> 1) : (k >> 1);
    return L ? (__brev(n) >> (32 - L)) : 0u;
}

// In-place radix-2^2 FFT over ncl complex lines of length m = 2^L at line pitch LP.
// DIT: bit-reversed in, natural out. DIF: natural in, bit-reversed out. INV conjugates twiddles.
template <bool DIF, bool INV>
__device__ __forceinline__ void fft_lines(double2* __restrict__ buf, const double2* __restrict__ tw, int ncl, int L,
                                          int LP) {
    const uint32_t m = 1u << L;
    auto twid = [&](uint32_t k) { return INV ? cconj(tw[k]) : tw[k]; };
    auto radix2 = [&]() {
        const int nb = ncl << (L - 1);
        for (int t = threadIdx.x; t < nb; t += spec::NT) {
            const int line = t >> (L - 1);
            const uint32_t j = uint32_t(t & ((1 << (L - 1)) - 1)) << 1;
            double2* x = buf + line * LP;
            const double2 a = x[j], b = x[j + 1];
            x[j] = cadd(a, b);
            x[j + 1] = csub(a, b);
        }
        __syncthreads();
    };
    if (L < 2) {
        if (L == 1) radix2();
        return;
    }
    const int nbf = ncl << (L - 2);   // radix-4 butterflies per stage
    if (!DIF) {
        uint32_t s = 1;
        if (L & 1) {
            radix2();
            s = 2;
        }
        for (; s < m; s <<= 2) {
            const uint32_t sh2 = m / (2 * s), sh4 = m / (4 * s);
            for (int t = threadIdx.x; t < nbf; t += spec::NT) {
                const int line = t >> (L - 2);
                const uint32_t bf = uint32_t(t & ((1 << (L - 2)) - 1));
                const uint32_t r = bf & (s - 1);
                const uint32_t j = (bf - r) * 4 + r;
                double2* x = buf + line * LP;
                const double2 w1 = twid(r * sh2), w2 = twid(r * sh4);
                const double2 a0 = x[j], a1 = cmul(x[j + s], w1), a2 = x[j + 2 * s], a3 = cmul(x[j + 3 * s], w1);
                const double2 b0 = cadd(a0, a1), b1 = csub(a0, a1), b2 = cadd(a2, a3), b3 = csub(a2, a3);
                const double2 t2 = cmul(w2, b2), t3 = crot<INV>(cmul(w2, b3));
                x[j] = cadd(b0, t2);
                x[j + 2 * s] = csub(b0, t2);
                x[j + s] = cadd(b1, t3);
                x[j + 3 * s] = csub(b1, t3);
            }
            __syncthreads();
        }
    } else {
        for (uint32_t s = m >> 2; s >= 1; s >>= 2) {
            const uint32_t sh2 = m / (2 * s), sh4 = m / (4 * s);
            for (int t = threadIdx.x; t < nbf; t += spec::NT) {
                const int line = t >> (L - 2);
                const uint32_t bf = uint32_t(t & ((1 << (L - 2)) - 1));
                const uint32_t r = bf & (s - 1);
                const uint32_t j = (bf - r) * 4 + r;
                double2* x = buf + line * LP;
                const double2 w4 = twid(r * sh4), w2 = twid(r * sh2);
                const double2 a0 = x[j], a1 = x[j + s], a2 = x[j + 2 * s], a3 = x[j + 3 * s];
                const double2 b0 = cadd(a0, a2), b2 = cmul(csub(a0, a2), w4);
                const double2 b1 = cadd(a1, a3), b3 = crot<INV>(cmul(csub(a1, a3), w4));
                x[j] = cadd(b0, b1);
                x[j + s] = cmul(csub(b0, b1), w2);
                x[j + 2 * s] = cadd(b2, b3);
                x[j + 3 * s] = cmul(csub(b2, b3), w2);
            }
            __syncthreads();
            if (s < 4) break;
        }
        if (L & 1) radix2();
    }
}

// Global element offset of (line ql of the tile starting at line q0, position k).
template <bool D0>
__device__ __forceinline__ uint32_t line_addr(const SpecArgs& a, uint32_t q0, uint32_t ql, uint32_t k) {
    if (D0) return ((q0 + ql) << a.L) + k;
    const uint32_t q = q0 + ql;                 // q0 .. q0+tq-1 lie in one stride block (tq | stride)
    return (q & (a.stride - 1)) + ((q >> a.ls) << (a.ls + a.L)) + (k << a.ls);
}

template <int MODE, bool D0, bool FORMB>
__global__ __launch_bounds__(spec::NT) void k_dct(SpecArgs a) {
    __shared__ double2 buf[spec::LDS_WORDS / 2 + 8 * spec::PAD];
    __shared__ double lc0[16], lc1[16];     // MID: per-line eigenvalue coefficients
    const int L = a.L;
    const uint32_t m = 1u << L;
    const int tq = a.tq, ncl = tq >> 1;
    const int LP = int(m) + spec::PAD;
    const uint32_t q0 = blockIdx.x * uint32_t(tq);
    const int log2tq = __ffs(tq) - 1;

    if (MODE == SPEC_MID && threadIdx.x < uint32_t(tq)) {
        // line q indexes dims 0..p-2 column-major (d = p - 1): split mu into c0 + c1 * lam_d(k)
        const uint32_t q = q0 + threadIdx.x;
        double lamv[kMaxDims] = {0, 0, 0, 0};
        uint32_t rest = q < a.nlines ? q : 0u;
        for (int j = 0; j < a.p - 1; ++j) {
            const uint32_t qq = (j < a.p - 2) ? a.fd[j].div(rest) : 0u;
            const uint32_t c = rest - qq * a.m[j];
            lamv[j] = a.lam[a.lam_off[j] + c];
            rest = qq;
        }
        double c0 = a.w0, c1 = 0.0;
        const int dbit = 1 << a.d;
        for (int S = 1; S < (1 << a.p); ++S) {
            if (a.cS[S] == 0.0) continue;
            double prod = a.sigma * a.cS[S];
            for (int j = 0; j < a.p; ++j)
                if (j != a.d && ((S >> j) & 1)) prod *= lamv[j];
            if (S & dbit) c1 += prod;
            else c0 += prod;
        }
        lc0[threadIdx.x] = c0;
        lc1[threadIdx.x] = c1;
    }

    // ---- load (forward: bit-reversed Makhoul order; inverse: natural order) ----------------
    double* bw = reinterpret_cast<double*>(buf);
    const int total = tq << L;
    for (int e = threadIdx.x; e < total; e += spec::NT) {
        uint32_t ql, k;
        if (D0) {
            ql = uint32_t(e) >> L;
            k = uint32_t(e) & (m - 1);
        } else {
            ql = uint32_t(e) & uint32_t(tq - 1);
            k = uint32_t(e) >> log2tq;
        }
        double v = 0.0;
        if (q0 + ql < a.nlines) {
            const uint32_t gi = line_addr<D0>(a, q0, ql, k);
            v = __builtin_nontemporal_load(a.in + gi);
            if (FORMB) v += a.ca * __builtin_nontemporal_load(a.ga + gi) + a.cb * __builtin_nontemporal_load(a.gb + gi);
        }
        const uint32_t pos = (MODE == SPEC_INV) ? k : perm_pos(k, m, L);
        bw[2 * ((ql >> 1) * LP + pos) + (ql & 1)] = v;
    }
    __syncthreads();

    if (MODE != SPEC_INV) fft_lines<false, false>(buf, a.tw, ncl, L, LP);

    // ---- spectrum <-> DCT coefficients, paired (k, m-k) in registers ---------------------------
    {
        const uint32_t half = m >> 1;
        const int npairs = ncl << (L - 1);
        for (int t = threadIdx.x; t < npairs; t += spec::NT) {
            const int line = t >> (L - 1);
            const uint32_t k = uint32_t(t) & (half - 1);
            double2* x = buf + line * LP;
            // indices handled by this thread: k and m-k (k >= 1), or the self-pairs 0 and m/2
            const uint32_t ka = k, kb = k ? m - k : half;
            const bool self = (k == 0);
            double2 Xk, Xmk;   // (X_a, X_b) at ka and kb
            if (MODE != SPEC_INV) {
                const double2 Z1 = x[ka], Z2 = x[kb];
                const double2 q1 = a.twq[ka], q2 = a.twq[kb];
                if (self) {
                    // Z[0] and Z[m/2] pair with themselves: A = Re Z, B = Im Z
                    Xk = make_double2(q1.x * Z1.x, q1.x * Z1.y);
                    Xmk = make_double2(q2.x * Z2.x, q2.x * Z2.y);
                } else {
                    const double2 Ap = make_double2(0.5 * (Z1.x + Z2.x), 0.5 * (Z1.y - Z2.y));   // (Z1 + conj Z2)/2
                    const double2 Bp = make_double2(0.5 * (Z1.y + Z2.y), -0.5 * (Z1.x - Z2.x));  // (Z1 - conj Z2)/2i
                    // X[k] = Re(q1 A), X[m-k] = Re(q2 conj A)
                    Xk = make_double2(q1.x * Ap.x - q1.y * Ap.y, q1.x * Bp.x - q1.y * Bp.y);
                    Xmk = make_double2(q2.x * Ap.x + q2.y * Ap.y, q2.x * Bp.x + q2.y * Bp.y);
                }
            } else {
                Xk = x[ka];
                Xmk = x[kb];
            }
            if (MODE == SPEC_MID) {
                const double* lamd = a.lam + a.lam_off[a.d];
                const double la = lamd[ka], lb = lamd[kb];
                const int l0 = 2 * line, l1 = 2 * line + 1;
                Xk.x *= a.inv_n / (lc0[l0] + lc1[l0] * la);
                Xk.y *= a.inv_n / (lc0[l1] + lc1[l1] * la);
                Xmk.x *= a.inv_n / (lc0[l0] + lc1[l0] * lb);
                Xmk.y *= a.inv_n / (lc0[l1] + lc1[l1] * lb);
            }
            if (MODE == SPEC_FWD) {
                x[ka] = Xk;
                x[kb] = Xmk;
                continue;
            }
            // V[k] = conj(q[k]) (X[k] - i X[m-k]); Z = V_a + i V_b
            const double2 q1 = cconj(a.twq[ka]), q2 = cconj(a.twq[kb]);
            double2 Za, Zb;
            if (self) {
                // k = 0: X[m] = 0 -> V = X[0].  k = m/2: V = q (X - i X)
                Za = make_double2(Xk.x, Xk.y);   // V_a[0] = Xa[0], V_b[0] = Xb[0] -> Z = Xa + i Xb
                const double2 va = cmul(q2, make_double2(Xmk.x, -Xmk.x));
                const double2 vb = cmul(q2, make_double2(Xmk.y, -Xmk.y));
                Zb = make_double2(va.x - vb.y, va.y + vb.x);
                x[0] = Za;
                x[half] = Zb;
            } else {
                const double2 va1 = cmul(q1, make_double2(Xk.x, -Xmk.x));
                const double2 vb1 = cmul(q1, make_double2(Xk.y, -Xmk.y));
                const double2 va2 = cmul(q2, make_double2(Xmk.x, -Xk.x));
                const double2 vb2 = cmul(q2, make_double2(Xmk.y, -Xk.y));
                x[ka] = make_double2(va1.x - vb1.y, va1.y + vb1.x);
                x[kb] = make_double2(va2.x - vb2.y, va2.y + vb2.x);
            }
        }
        __syncthreads();
    }

    if (MODE != SPEC_FWD) fft_lines<true, true>(buf, a.tw, ncl, L, LP);

    // ---- store (forward: natural order; inverse: un-permute from bit-reversed order) ------------
    for (int e = threadIdx.x; e < total; e += spec::NT) {
        uint32_t ql, k;
        if (D0) {
            ql = uint32_t(e) >> L;
            k = uint32_t(e) & (m - 1);
        } else {
            ql = uint32_t(e) & uint32_t(tq - 1);
            k = uint32_t(e) >> log2tq;
        }
        if (q0 + ql >= a.nlines) continue;
        const uint32_t pos = (MODE == SPEC_FWD) ? k : perm_pos(k, m, L);
        __builtin_nontemporal_store(bw[2 * ((ql >> 1) * LP + pos) + (ql & 1)], a.out + line_addr<D0>(a, q0, ql, k));
    }
}

// ------------------------------------------------------------------------------ launcher
hipError_t launch_dct_pass(const SpecPlan& sp, const Geom& g, hipStream_t s, int mode, int d, const double* in,
                           const double* ga, double ca, const double* gb, double cb, double* out, double sigma,
                           double w0) {
    SpecArgs a{};
    a.in = in;
    a.ga = ga;
    a.gb = gb;
    a.ca = ca;
    a.cb = cb;
    a.out = out;
    a.tw = reinterpret_cast<const double2*>(sp.tw + sp.tw_off[d]);
    a.twq = reinterpret_cast<const double2*>(sp.twq + sp.twq_off[d]);
    a.lam = sp.lam;
    for (int j = 0; j < kMaxDims; ++j) {
        a.lam_off[j] = sp.lam_off[j];
        a.m[j] = g.m[j];
    }
    for (int j = 0; j < kMaxDims - 1; ++j) a.fd[j] = g.fd[j];
    for (int S = 0; S < 16; ++S) a.cS[S] = g.cS[S];
    a.sigma = sigma;
    a.w0 = w0;
    a.inv_n = 1.0 / double(g.N);
    a.stride = g.stride[d];
    a.ls = 0;
    while ((1u << a.ls) < a.stride) ++a.ls;
    const uint32_t m = g.m[d];
    a.nlines = g.N / m;
    a.d = d;
    a.p = g.p;
    a.L = 0;
    while ((1u << a.L) < m) ++a.L;
    int tq = std::max(2, std::min(16, int(spec::LDS_WORDS / m)));
    if (d > 0) tq = std::min<int>(tq, int(g.stride[d]));
    if (tq < 2 || (1u << a.L) != m || m > 4096) return hipErrorInvalidValue;
    a.tq = tq;
    const bool formb = ga != nullptr;
    const dim3 grid((a.nlines + uint32_t(tq) - 1) / uint32_t(tq)), block(spec::NT);
#define MVTV_DCT_LAUNCH(MODE, D0, FB) klaunch(k_dct<MODE, D0, FB>, grid, block, 0, s, a)
    if (mode == SPEC_FWD) {
        if (d == 0) {
            if (formb) MVTV_DCT_LAUNCH(SPEC_FWD, true, true);
            else MVTV_DCT_LAUNCH(SPEC_FWD, true, false);
        } else {
            MVTV_DCT_LAUNCH(SPEC_FWD, false, false);
        }
    } else if (mode == SPEC_INV) {
        if (d == 0) MVTV_DCT_LAUNCH(SPEC_INV, true, false);
        else MVTV_DCT_LAUNCH(SPEC_INV, false, false);
    } else {
        if (d == 0) {   // p = 1: the only pass
            if (formb) MVTV_DCT_LAUNCH(SPEC_MID, true, true);
            else MVTV_DCT_LAUNCH(SPEC_MID, true, false);
        } else {
            MVTV_DCT_LAUNCH(SPEC_MID, false, false);
        }
    }
#undef MVTV_DCT_LAUNCH
    return hipGetLastError();
}

}  // namespace mvtv

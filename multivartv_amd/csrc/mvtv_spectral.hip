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
#include <cstdio>
#include <cstdlib>

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
    uint32_t q_off;          // MID: global index of line 0
    const int32_t* skip;     // != nullptr and *skip: return at once (preconditioner of a converged PCG)
    const AdmmCtl* ctl;      // asynchronous ADMM loop: sigma, ca = rho, cb = rho c_prev from the device
    // mixed-radix lengths (k_dctg): the FFT's radices in stage order, division by the line stride
    int32_t nrad;
    int32_t rad[8];
    FastDiv fds;              // division by the line stride
    FastDiv fm;               // division by m
    FastDiv fper[8], fL[8];   // stage s: butterflies per line (m / rad[s]) and the span before it
    const uint32_t* perm;     // position of sample k in the digit-reversed Makhoul order (this dim)
    int32_t xcd;              // k_dct8: tiles dealt to the XCDs in contiguous runs (grid a multiple of 8)
    int32_t xrun;             // k_dctg / k_dctm / k_dctb / k_dctb8 / k_trig: the same for any grid (xcd_run)
    PcgFuse pf;               // k_dct8 PC = 1 / 2: the PCG vector work of the preconditioner's d = 0 passes
    int32_t fold;             // FORMB from the folded s (k_dct8, ctl): b = in + fold_ka ga [+ fold_kb gb if ctl->fix]
    int32_t pair16;           // k_dct8 d = 0 forward / inverse: coefficients through LDS as 16-B pairs (dct_pair16)
    // Bluestein lengths (k_dctb; L = log2 M then, tw = the length-M FFT twiddles): the chirp c[n] = e^{-i pi n^2/m}
    // and the transforms / M of the forward / inverse convolution kernels
    const double2* bchirp;
    const double2* bvf;
    const double2* bvi;
};

// Workgroup b of G runs on XCD b % 8. The tile it takes when the tiles are dealt to the XCDs in contiguous runs, for
// any G (XCD x takes G / 8 tiles, one more when x < G % 8): the tiles that share the 128-B lines of a strided row —
// a line pitch that is not a multiple of 128 B (500, 251, 100 points ...) — are then read through one L2 instead of
// two, where round-robin dealing put neighbouring tiles on different XCDs and each straddled line came from HBM twice
__device__ __forceinline__ uint32_t xcd_run(uint32_t b, uint32_t G) {
    const uint32_t x = b & 7u, i = b >> 3, q = G >> 3, r = G & 7u;
    return x * q + (x < r ? x : r) + i;
}

enum SpecMode { SPEC_FWD = 0, SPEC_INV = 1, SPEC_MID = 2 };

typedef double dvec2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double2 ldnt2(const double* p) {
    const dvec2 v = __builtin_nontemporal_load(reinterpret_cast<const dvec2*>(p));
    return make_double2(v.x, v.y);
}
__device__ __forceinline__ void stnt2(double* p, double2 v) {
    dvec2 w;
    w.x = v.x;
    w.y = v.y;
    __builtin_nontemporal_store(w, reinterpret_cast<dvec2*>(p));
}

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
__global__ __launch_bounds__(spec::NT) void k_dct(const SpecArgs a) {
    double sigma = a.sigma, ca = a.ca, cb = a.cb;   // locals: see k_dct8
    if (a.skip && *a.skip) return;
    if (a.ctl) {
        if (a.ctl->done) return;
        sigma = a.ctl->sigma;
        ca = a.ctl->rho;
        cb = a.ctl->rho * a.ctl->c_prev;
    }
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
        const uint32_t q = a.q_off + q0 + threadIdx.x;
        double lamv[kMaxDims] = {0, 0, 0, 0};
        uint32_t rest = (q - a.q_off) < a.nlines ? q : a.q_off;
        const int jlast = a.d == a.p - 1 ? a.p - 2 : a.p - 1;
        for (int j = 0; j < a.p; ++j) {
            if (j == a.d) continue;
            const uint32_t qq = (j < jlast) ? a.fd[j].div(rest) : 0u;
            const uint32_t c = rest - qq * a.m[j];
            lamv[j] = a.lam[a.lam_off[j] + c];
            rest = qq;
        }
        double c0 = a.w0, c1 = 0.0;
        const int dbit = 1 << a.d;
        for (int S = 1; S < (1 << a.p); ++S) {
            if (a.cS[S] == 0.0) continue;
            double prod = sigma * a.cS[S];
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
            if (FORMB) v += ca * __builtin_nontemporal_load(a.ga + gi) + cb * __builtin_nontemporal_load(a.gb + gi);
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

// =============================================================================================
// Register-radix Stockham version (m >= 8): every thread holds 8 complex values of one complex
// line (two real lines) and runs radix-8 butterflies in registers (one radix-2/4 stage first
// when log2 m is not a multiple of 3); LDS only carries the exchange between stages. The first
// forward stage reads the Makhoul-permuted input straight from HBM and the last inverse stage
// stores the un-permuted output straight to HBM.
//
// Thread -> (complex line c, butterfly column j), j < m/8. For d > 0 lanes run over c first,
// so the two real lines of a complex line are one 16-B access and the 2*NCL lines of a tile
// make one contiguous row per mesh position; for d = 0 lanes run over j (lines are contiguous).
namespace spec8 {
template <int L>
struct Shape {
    static constexpr int M = 1 << L;
    static constexpr int TPL = M / 8;                                     // threads per complex line
    static constexpr int TQ = (8192 / M) < 16 ? (8192 / M) : 16;          // real lines per workgroup
    static constexpr int NCL = TQ / 2;                                    // complex lines per workgroup
    static constexpr int NT = NCL * TPL;
    // line pitch (complex slots): a multiple of 8 plus 8 mod 16, and slot = pidx(pos) ^ (c & 7), so
    // c-fastest lanes (d > 0) hit distinct banks for the 16-B reads (16-lane groups) and writes
    // (8-lane groups); j-fastest lanes (d = 0) are spread by pidx
    static constexpr int LP = (M + M / 8 + 15) / 16 * 16 + 8;
    static constexpr int R0 = (L % 3 == 0) ? 8 : (L % 3 == 1 ? 2 : 4);    // radix of the first stage
};
// kernel-level shape with an optional smaller tile (TQW real lines per workgroup)
template <int L, int TQW>
struct ShapeK : Shape<L> {
    static constexpr int TQ = TQW > 0 ? TQW : Shape<L>::TQ;
    static constexpr int NCL = TQ / 2;
    static constexpr int NT = NCL * Shape<L>::TPL;
};
__device__ __forceinline__ int pidx(int pos) { return pos + (pos >> 3); }   // one pad slot per 8
__device__ __forceinline__ int slot(int pos, int cx) { return pidx(pos) ^ cx; }
}  // namespace spec8

template <bool INV>
__device__ __forceinline__ void fft4r(double2& z0, double2& z1, double2& z2, double2& z3) {
    const double2 t0 = cadd(z0, z2), t1 = csub(z0, z2), t2 = cadd(z1, z3), t3 = crot<INV>(csub(z1, z3));
    z0 = cadd(t0, t2);
    z2 = csub(t0, t2);
    z1 = cadd(t1, t3);
    z3 = csub(t1, t3);
}

// natural-order radix-R DFT of z[0..R-1] in registers
template <int R, bool INV>
__device__ __forceinline__ void dft_r(double2* z) {
    if constexpr (R == 2) {
        const double2 a = z[0], b = z[1];
        z[0] = cadd(a, b);
        z[1] = csub(a, b);
    } else if constexpr (R == 4) {
        fft4r<INV>(z[0], z[1], z[2], z[3]);
    } else {
        double2 e0 = z[0], e1 = z[2], e2 = z[4], e3 = z[6];
        double2 o0 = z[1], o1 = z[3], o2 = z[5], o3 = z[7];
        fft4r<INV>(e0, e1, e2, e3);
        fft4r<INV>(o0, o1, o2, o3);
        constexpr double h = 0.70710678118654752440;
        // w8^k o_k, w8 = e^{-+ i pi/4}
        const double2 p1 = INV ? make_double2(h * (o1.x - o1.y), h * (o1.x + o1.y))
                               : make_double2(h * (o1.x + o1.y), h * (o1.y - o1.x));
        const double2 p2 = crot<INV>(o2);
        const double2 p3 = INV ? make_double2(-h * (o3.x + o3.y), h * (o3.x - o3.y))
                               : make_double2(h * (o3.y - o3.x), -h * (o3.x + o3.y));
        z[0] = cadd(e0, o0);
        z[4] = csub(e0, o0);
        z[1] = cadd(e1, p1);
        z[5] = csub(e1, p1);
        z[2] = cadd(e2, p2);
        z[6] = csub(e2, p2);
        z[3] = cadd(e3, p3);
        z[7] = csub(e3, p3);
    }
}

// One Stockham stage of radix R on this thread's 8/R butterflies b_s = j + s*TPL. Register
// z[s*R + r] holds input position b_s + r*M/R. Twiddles, then the DFT; output position of
// z[s*R + r] is (b_s / NS) * NS * R + b_s % NS + r * NS.
template <int L, int R, int NS, bool INV>
__device__ __forceinline__ void stage_compute(double2* z, int j, const double2* __restrict__ tw) {
    using S = spec8::Shape<L>;
#pragma unroll
    for (int s = 0; s < 8 / R; ++s) {
        if constexpr (NS > 1) {
            const int kk = (j + s * S::TPL) % NS;
            constexpr int step = S::M / (NS * R);
#pragma unroll
            for (int r = 1; r < R; ++r) {
                double2 w = tw[kk * r * step];
                if (INV) w = cconj(w);
                z[s * R + r] = cmul(z[s * R + r], w);
            }
        }
        dft_r<R, INV>(z + s * R);
    }
}
template <int L, int R>
__device__ __forceinline__ int stage_in_pos(int j, int i) {
    using S = spec8::Shape<L>;
    const int s = i / R, r = i % R;
    return j + S::TPL * (s + r * (8 / R));
}
template <int L, int R, int NS>
__device__ __forceinline__ int stage_out_pos(int j, int i) {
    using S = spec8::Shape<L>;
    const int s = i / R, r = i % R;
    const int b = j + s * S::TPL;
    return (b / NS) * NS * R + (b % NS) + r * NS;
}

// Barrier policies of the FFT exchanges: 0 __syncthreads, 1 LDS-only workgroup barrier (lds_barrier: global loads
// issued before the stages stay in flight), 2 the wave alone — for tiles where every complex line's threads are one
// wave's lanes (d = 0 passes with m / 8 <= 64 threads per line), whose exchange slots no other wave touches: a
// wave's LDS accesses complete in issue order, so only the compiler must not move them across the point
template <int BAR>
__device__ __forceinline__ void xbar() {
    if constexpr (BAR == 0) {
        __syncthreads();
    } else if constexpr (BAR == 1) {
        lds_barrier();
    } else {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    }
}

// Stages after the first (the first is peeled: its input comes from HBM or the caller's LDS).
// STAGE counts radix-8 stages done after R0. Writes the outputs of stage NS_IN's butterflies
// to LDS, then (if more stages remain) reads the next stage's inputs. BAR: the barrier policy (xbar); true (1):
// LDS-only barriers (lds_barrier), so global loads issued before the stages stay in flight
template <int L, int R, int NS, bool INV, bool LAST_TO_REGS, int BAR = 0>
__device__ __forceinline__ void stages_from(double2* z, int j, double2* X, int cx, const double2* __restrict__ tw) {
    using S = spec8::Shape<L>;
    stage_compute<L, R, NS, INV>(z, j, tw);
    constexpr int NS_NEXT = NS * R;
    if constexpr (NS_NEXT == S::M && LAST_TO_REGS) {
        return;   // caller stores z (output positions stage_out_pos<L, R, NS>)
    } else {
        xbar<BAR>();   // everyone has read this stage's inputs
#pragma unroll
        for (int i = 0; i < 8; ++i) X[spec8::slot(stage_out_pos<L, R, NS>(j, i), cx)] = z[i];
        xbar<BAR>();
        if constexpr (NS_NEXT < S::M) {
#pragma unroll
            for (int i = 0; i < 8; ++i) z[i] = X[spec8::slot(stage_in_pos<L, 8>(j, i), cx)];
            stages_from<L, 8, NS_NEXT, INV, LAST_TO_REGS, BAR>(z, j, X, cx, tw);
        }
    }
}
// radix of the last stage and its NS (for the register-resident output positions)
template <int L>
struct LastStage {
    static constexpr int R = (L == 1 || L == 2) ? (1 << L) : 8;   // L >= 3 always ends with radix 8
    static constexpr int NS = (1 << L) / R;
};

// PC (PcgFuse, d = 0 passes of a preconditioner solve): 1 = first pass, r -= alpha q and x += alpha p on
// load with r and x written back, input sinv * r; 2 = last pass, out = sinv * transform, r.z and |r|^2 per
// workgroup
template <int L, int MODE, bool D0, bool FORMB, int TQW = 0, int PC = 0>
__global__ __launch_bounds__((spec8::ShapeK<L, TQW>::NT)) void k_dct8(const SpecArgs a) {
    using S = spec8::ShapeK<L, TQW>;
    static_assert(PC == 0 || (D0 && !FORMB && (PC == 1 ? MODE == SPEC_FWD : MODE == SPEC_INV)),
                  "PCG fusion: d = 0 forward (PC 1) / inverse (PC 2) passes only");
    // scalars into locals: writing into the by-value argument struct would demote it to scratch
    double sigma = a.sigma, ca = a.ca, cb = a.cb;
    if (a.skip && *a.skip) return;
    const double alpha = PC == 1 ? a.pf.st->alpha : 0.0;
    double rz = 0.0, rr = 0.0;   // PC 2 reductions
    bool rd_gb = true;   // FORMB reads gb (the folded form only after a rho change)
    if (a.ctl) {
        if (a.ctl->done) return;
        sigma = a.ctl->sigma;
        ca = a.ctl->rho;
        cb = a.ctl->rho * a.ctl->c_prev;
        if (a.fold) {
            ca = a.ctl->fold_ka;
            cb = a.ctl->fold_kb;
            rd_gb = a.ctl->fix != 0;
        }
    }
    constexpr int M = S::M, TPL = S::TPL, NCL = S::NCL;
    // d = 0 with <= 64 threads per complex line: each line's exchanges stay inside one wave (no workgroup barrier;
    // MID keeps them: its line constants are shared)
    constexpr int BAR = (D0 && TPL <= 64 && 64 % TPL == 0 && MODE != SPEC_MID) ? 2 : 0;
    __shared__ double2 buf[NCL * S::LP];
    __shared__ double lc0[2 * NCL], lc1[2 * NCL];
    const int t = threadIdx.x;
    const int j = D0 ? (t % TPL) : (t / NCL);
    const int c = D0 ? (t / TPL) : (t % NCL);
    // xcd: workgroup b runs on XCD b % 8; dealing tiles in contiguous runs per XCD keeps the tiles that
    // share a 128-B row of a strided pass (d > 0, < 16 lines per tile) in one L2
    const uint32_t bx = a.xcd ? (blockIdx.x & 7u) * (gridDim.x >> 3) + (blockIdx.x >> 3) : blockIdx.x;
    const uint32_t q0 = bx * uint32_t(a.tq);
    const int la = 2 * c, lb = 2 * c + 1;
    const bool va = la < a.tq && q0 + la < a.nlines;
    const bool vb = lb < a.tq && q0 + lb < a.nlines;
    double2* X = buf + c * S::LP;
    const int cx = c & 7;
    const double2* __restrict__ tw = a.tw;

    for (int l = t; MODE == SPEC_MID && l < a.tq; l += S::NT) {
        const uint32_t q = a.q_off + q0 + l;
        double lamv[kMaxDims] = {0, 0, 0, 0};
        uint32_t rest = (q - a.q_off) < a.nlines ? q : a.q_off;
        // line q enumerates the dims other than d, dim 0 fastest
        const int jlast = a.d == a.p - 1 ? a.p - 2 : a.p - 1;
        for (int jj = 0; jj < a.p; ++jj) {
            if (jj == a.d) continue;
            const uint32_t qq = (jj < jlast) ? a.fd[jj].div(rest) : 0u;
            lamv[jj] = a.lam[a.lam_off[jj] + (rest - qq * a.m[jj])];
            rest = qq;
        }
        double c0 = a.w0, c1 = 0.0;
        for (int Sm = 1; Sm < (1 << a.p); ++Sm) {
            if (a.cS[Sm] == 0.0) continue;
            double prod = sigma * a.cS[Sm];
            for (int jj = 0; jj < a.p; ++jj)
                if (jj != a.d && ((Sm >> jj) & 1)) prod *= lamv[jj];
            if ((Sm >> a.d) & 1) c1 += prod;
            else c0 += prod;
        }
        lc0[l] = c0;
        lc1[l] = c1;
    }

    // element k of real line ql (local) -> global offset
    auto gaddr = [&](int ql, uint32_t k) -> uint32_t {
        const uint32_t q = q0 + uint32_t(ql);
        if (D0) return (q << L) + k;
        return (q & (a.stride - 1)) + ((q >> a.ls) << (a.ls + L)) + (k << a.ls);
    };
    auto ld2 = [&](uint32_t k) -> double2 {   // (line la, line lb) at position k, b formed if FORMB
        double2 v = make_double2(0.0, 0.0);
        if (D0) {
            if (va) {
                const uint32_t g = gaddr(la, k);
                v.x = __builtin_nontemporal_load(a.in + g);
                if (FORMB && !rd_gb) v.x += ca * __builtin_nontemporal_load(a.ga + g);
                else if (FORMB) v.x += ca * __builtin_nontemporal_load(a.ga + g) + cb * __builtin_nontemporal_load(a.gb + g);
            }
            if (vb) {
                const uint32_t g = gaddr(lb, k);
                v.y = __builtin_nontemporal_load(a.in + g);
                if (FORMB && !rd_gb) v.y += ca * __builtin_nontemporal_load(a.ga + g);
                else if (FORMB) v.y += ca * __builtin_nontemporal_load(a.ga + g) + cb * __builtin_nontemporal_load(a.gb + g);
            }
        } else if (va) {   // d > 0: lines la, lb are adjacent words (vb == va)
            const uint32_t g = gaddr(la, k);
            v = ldnt2(a.in + g);
            if (FORMB && !rd_gb) {
                const double2 x1 = ldnt2(a.ga + g);
                v.x += ca * x1.x;
                v.y += ca * x1.y;
            } else if (FORMB) {
                const double2 x1 = ldnt2(a.ga + g);
                const double2 x2 = ldnt2(a.gb + g);
                v.x += ca * x1.x + cb * x2.x;
                v.y += ca * x1.y + cb * x2.y;
            }
        }
        return v;
    };
    auto st2 = [&](uint32_t k, double2 v) {
        if (D0) {
            if (va) __builtin_nontemporal_store(v.x, a.out + gaddr(la, k));
            if (vb) __builtin_nontemporal_store(v.y, a.out + gaddr(lb, k));
        } else if (va) {
            stnt2(a.out + gaddr(la, k), v);
        }
    };

    double2 z[8];
    if (MODE != SPEC_INV) {
        // ---- forward FFT of the Makhoul sequence z[n] = x[2n] | x[2(M-1-n)+1] -----------------
        constexpr int R0 = S::R0;
        if (D0) {
            // contiguous lines: 16-B loads of (x[2n], x[2n+1]) land at Makhoul positions n, M-1-n
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) {
                const int n = j + s4 * TPL;
                double2 xa = make_double2(0.0, 0.0), xb = make_double2(0.0, 0.0);
                auto ld_in = [&](uint32_t g) -> double2 {
                    if constexpr (PC == 1) {   // the operations of k_pcgs_vec op 1
                        double2 rv = ldnt2(a.pf.r + g);
                        const double2 qv = ldnt2(a.pf.q + g);
                        double2 xv = ldnt2(a.pf.x + g);
                        const double2 pv = ldnt2(a.pf.p + g);
                        rv.x = fma(-alpha, qv.x, rv.x);
                        rv.y = fma(-alpha, qv.y, rv.y);
                        xv.x = fma(alpha, pv.x, xv.x);
                        xv.y = fma(alpha, pv.y, xv.y);
                        stnt2(a.pf.r + g, rv);
                        stnt2(a.pf.x + g, xv);
                        if (a.pf.sinv) {
                            const double2 sv = ldnt2(a.pf.sinv + g);
                            rv.x *= sv.x;
                            rv.y *= sv.y;
                        }
                        return rv;
                    } else {
                        double2 v = ldnt2(a.in + g);
                        if (FORMB && !rd_gb) {
                            const double2 g1 = ldnt2(a.ga + g);
                            v.x += ca * g1.x;
                            v.y += ca * g1.y;
                        } else if (FORMB) {
                            const double2 g1 = ldnt2(a.ga + g), g2 = ldnt2(a.gb + g);
                            v.x += ca * g1.x + cb * g2.x;
                            v.y += ca * g1.y + cb * g2.y;
                        }
                        return v;
                    }
                };
                if (va) xa = ld_in(gaddr(la, uint32_t(2 * n)));
                if (vb) xb = ld_in(gaddr(lb, uint32_t(2 * n)));
                X[spec8::slot(n, cx)] = make_double2(xa.x, xb.x);
                X[spec8::slot(M - 1 - n, cx)] = make_double2(xa.y, xb.y);
            }
            xbar<BAR>();
#pragma unroll
            for (int i = 0; i < 8; ++i) z[i] = X[spec8::slot(stage_in_pos<L, R0>(j, i), cx)];
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int n = stage_in_pos<L, R0>(j, i);
                const uint32_t k = n < M / 2 ? uint32_t(2 * n) : uint32_t(2 * (M - 1 - n) + 1);
                z[i] = ld2(k);
            }
        }
        stages_from<L, R0, 1, false, false, BAR>(z, j, X, cx, tw);   // natural-order spectrum in LDS
    }

    // ---- spectrum <-> DCT coefficients for the pairs (k, M-k); k = 0 also takes M/2 -------------
    // the inverse pass issues all 8 coefficient loads before the first LDS write (issued inside the loop,
    // each group waited for its loads before writing LDS: four HBM round trips per workgroup instead of one)
    // d = 0 with a.pair16: the coefficients of the two real lines cross LDS (the line's exchange slots as M + M doubles)
    // so that they arrive / leave as 16-B pairs (k, k + 1) of one line, as the other side of these passes does; read or
    // written directly they are 8-B accesses at positions k and M - k (round 6: the d = 0 forward pass 540 us for 2N
    // words against 383 for a strided one at 512^3)
    double* const Xd = reinterpret_cast<double*>(X);
    double2 pre[8];
    if constexpr (MODE == SPEC_INV) {
        if (D0 && a.pair16) {
            double2 qa[4], qb[4];
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) {
                const uint32_t i2 = uint32_t(2 * (j + s4 * TPL));
                qa[s4] = va ? ldnt2(a.in + gaddr(la, i2)) : make_double2(0.0, 0.0);
                qb[s4] = vb ? ldnt2(a.in + gaddr(lb, i2)) : make_double2(0.0, 0.0);
            }
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) {
                const int i2 = 2 * (j + s4 * TPL);
                *reinterpret_cast<double2*>(Xd + i2) = qa[s4];
                *reinterpret_cast<double2*>(Xd + M + i2) = qb[s4];
            }
            xbar<BAR>();
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int k = j + s * TPL, kb = k ? M - k : M / 2;
                pre[2 * s] = make_double2(Xd[k], Xd[M + k]);
                pre[2 * s + 1] = make_double2(Xd[kb], Xd[M + kb]);
            }
            xbar<BAR>();   // every coefficient read before the IFFT input is written over them
        } else {
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int k = j + s * TPL;
                pre[2 * s] = ld2(uint32_t(k));
                pre[2 * s + 1] = ld2(uint32_t(k ? M - k : M / 2));
            }
        }
    }
    double2 fco[8];   // d = 0 forward with a.pair16: the coefficient pairs, written after the loop
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const int k = j + s * TPL;
        const int ka = k, kb = k ? M - k : M / 2;
        const bool self = k == 0;
        double2 Xk, Xmk;
        if (MODE != SPEC_INV) {
            const double2 Z1 = X[spec8::slot(ka, cx)], Z2 = X[spec8::slot(kb, cx)];
            const double2 q1 = a.twq[ka], q2 = a.twq[kb];
            if (self) {
                Xk = make_double2(q1.x * Z1.x, q1.x * Z1.y);
                Xmk = make_double2(q2.x * Z2.x, q2.x * Z2.y);
            } else {
                const double2 Ap = make_double2(0.5 * (Z1.x + Z2.x), 0.5 * (Z1.y - Z2.y));
                const double2 Bp = make_double2(0.5 * (Z1.y + Z2.y), -0.5 * (Z1.x - Z2.x));
                Xk = make_double2(q1.x * Ap.x - q1.y * Ap.y, q1.x * Bp.x - q1.y * Bp.y);
                Xmk = make_double2(q2.x * Ap.x + q2.y * Ap.y, q2.x * Bp.x + q2.y * Bp.y);
            }
        } else {
            Xk = pre[2 * s];
            Xmk = pre[2 * s + 1];
        }
        if (MODE == SPEC_FWD) {
            if (D0 && a.pair16) {
                fco[2 * s] = Xk;
                fco[2 * s + 1] = Xmk;
            } else {
                st2(uint32_t(ka), Xk);
                st2(uint32_t(kb), Xmk);
            }
            continue;
        }
        if (MODE == SPEC_MID) {
            const double* lamd = a.lam + a.lam_off[a.d];
            const double l1 = lamd[ka], l2 = lamd[kb];
            Xk.x *= a.inv_n / (lc0[la] + lc1[la] * l1);
            Xk.y *= a.inv_n / (lc0[lb] + lc1[lb] * l1);
            Xmk.x *= a.inv_n / (lc0[la] + lc1[la] * l2);
            Xmk.y *= a.inv_n / (lc0[lb] + lc1[lb] * l2);
        }
        const double2 q1 = cconj(a.twq[ka]), q2 = cconj(a.twq[kb]);
        if (self) {
            const double2 va2 = cmul(q2, make_double2(Xmk.x, -Xmk.x));
            const double2 vb2 = cmul(q2, make_double2(Xmk.y, -Xmk.y));
            X[spec8::slot(0, cx)] = Xk;
            X[spec8::slot(M / 2, cx)] = make_double2(va2.x - vb2.y, va2.y + vb2.x);
        } else {
            const double2 va1 = cmul(q1, make_double2(Xk.x, -Xmk.x));
            const double2 vb1 = cmul(q1, make_double2(Xk.y, -Xmk.y));
            const double2 va2 = cmul(q2, make_double2(Xmk.x, -Xk.x));
            const double2 vb2 = cmul(q2, make_double2(Xmk.y, -Xk.y));
            X[spec8::slot(ka, cx)] = make_double2(va1.x - vb1.y, va1.y + vb1.x);
            X[spec8::slot(kb, cx)] = make_double2(va2.x - vb2.y, va2.y + vb2.x);
        }
    }
    if (MODE == SPEC_FWD) {
        if (D0 && a.pair16) {
            xbar<BAR>();   // every spectrum read before the coefficients are written over it
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int k = j + s * TPL, kb = k ? M - k : M / 2;
                Xd[k] = fco[2 * s].x;
                Xd[M + k] = fco[2 * s].y;
                Xd[kb] = fco[2 * s + 1].x;
                Xd[M + kb] = fco[2 * s + 1].y;
            }
            xbar<BAR>();
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) {
                const int i2 = 2 * (j + s4 * TPL);
                if (va) stnt2(a.out + gaddr(la, uint32_t(i2)), *reinterpret_cast<const double2*>(Xd + i2));
                if (vb) stnt2(a.out + gaddr(lb, uint32_t(i2)), *reinterpret_cast<const double2*>(Xd + M + i2));
            }
        }
        return;
    }
    xbar<BAR>();

    // ---- inverse FFT, natural in; the last stage's outputs go straight to HBM, un-permuted ------
    {
        constexpr int R0 = S::R0;
#pragma unroll
        for (int i = 0; i < 8; ++i) z[i] = X[spec8::slot(stage_in_pos<L, R0>(j, i), cx)];
        if (D0) {
            // contiguous lines: the output goes through LDS so (x[2n], x[2n+1]) leave as one 16-B store
            stages_from<L, R0, 1, true, false, BAR>(z, j, X, cx, tw);
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) {
                const int n = j + s4 * TPL;
                const double2 v0 = X[spec8::slot(n, cx)], v1 = X[spec8::slot(M - 1 - n, cx)];
                auto st_out = [&](uint32_t g, double2 v) {
                    if constexpr (PC == 2) {   // the operations of k_pcgs_vec op 2
                        if (a.pf.sinv) {
                            const double2 sv = ldnt2(a.pf.sinv + g);
                            v.x *= sv.x;
                            v.y *= sv.y;
                        }
                        const double2 rv = ldnt2(a.pf.r + g);
                        rz = fma(rv.x, v.x, rz);
                        rr = fma(rv.x, rv.x, rr);
                        rz = fma(rv.y, v.y, rz);
                        rr = fma(rv.y, rv.y, rr);
                        stnt2(a.out + g, v);
                    } else {
                        stnt2(a.out + g, v);
                    }
                };
                if (va) st_out(gaddr(la, uint32_t(2 * n)), make_double2(v0.x, v1.x));
                if (vb) st_out(gaddr(lb, uint32_t(2 * n)), make_double2(v0.y, v1.y));
            }
            if constexpr (PC == 2) {
                double red[2] = {rz, rr};
                block_reduce_store<2, 0, S::NT>(red, a.pf.partials);
            }
        } else {
            stages_from<L, R0, 1, true, true>(z, j, X, cx, tw);
            using LS = LastStage<L>;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int n = stage_out_pos<L, LS::R, LS::NS>(j, i);
                const uint32_t k = n < M / 2 ? uint32_t(2 * n) : uint32_t(2 * (M - 1 - n) + 1);
                st2(k, z[i]);
            }
        }
    }
}

// =============================================================================================
// Two in-plane passes in one launch (m0 = m1 = 2^L, L <= 7): a workgroup owns one (dim 0, dim 1) plane,
// 128 KB at L = 7, and keeps it on chip between the two 1-D transforms, so the spectral solve of a 4-D
// 128^4 mesh makes 5 passes over HBM instead of 7 (3 instead of 5 at 128^3). NCL = M / 2 complex lines x
// TPL = M / 8 threads: the whole plane is one k_dct8 tile of M lines. Between the passes the coefficients go
// through a plane image in LDS (aliasing the FFT exchange buffer, barriers on both sides). Every barrier orders
// LDS only (lds_barrier): __syncthreads would also wait for the next plane's loads.
//   forward: dim-0 DCT of the rows (b formed on load as k_dct8's first pass), dim-1 DCT of the columns;
//   inverse: dim-1 inverse of the columns, dim-0 inverse of the rows.
template <int L, int MODE, bool FORMB>
__global__ __launch_bounds__((1 << L) / 2 * (1 << L) / 8) void k_plane8(const SpecArgs a, uint32_t nplanes) {
    using S = spec8::Shape<L>;
    constexpr int M = S::M, TPL = S::TPL, NCL = M / 2, R0 = S::R0;
    static_assert(L >= 4 && L <= 7, "the plane must fit the exchange buffer of one workgroup");
    static_assert(TPL <= 64 && 64 % TPL == 0, "a row pair's threads are lanes of one wave (xbar<2> on the rows)");
    // plane image pitch PP = M + M / 16 doubles (18 at M = 16): a wave's row accesses (8-B words, TPL = M / 8
    // lanes per row, 8 rows a wave at M = 64, 4 at 128) then start 16 PP bytes apart = M bytes mod 256, so the rows
    // of one wave instruction fall on different LDS banks; with pitch M every row started on bank 0 (rows 2 KB
    // apart at M = 128: 4-way conflicts on the transposes). Column accesses stay 16-B aligned (PP even).
    constexpr int PP = M + (M / 16 > 2 ? M / 16 : 2);
    static_assert(size_t(NCL) * S::LP * 16 >= size_t(M) * PP * 8, "plane image aliases the exchange buffer");
    static_assert(MODE == SPEC_FWD || !FORMB, "b is formed by the forward pass");
    double ca = a.ca, cb = a.cb;
    bool rd_gb = true;
    if (a.skip && *a.skip) return;
    if (a.ctl) {
        if (a.ctl->done) return;
        ca = a.ctl->rho;
        cb = a.ctl->rho * a.ctl->c_prev;
        if (a.fold) {
            ca = a.ctl->fold_ka;
            cb = a.ctl->fold_kb;
            rd_gb = a.ctl->fix != 0;
        }
    }
    __shared__ double2 buf[NCL * S::LP];
    double* const PI = reinterpret_cast<double*>(buf);   // plane image [row x1][column x0], pitch PP
    // rows mapping (dim-0 lines: lanes over j) and columns mapping (dim-1 lines: lanes over the line pair); the
    // loop below re-derives them from an opaque copy of the thread index each plane, so the many per-thread LDS
    // offsets are not hoisted out of it (kept live across the loop they spill)
    int t = threadIdx.x;
    int jr = t % TPL, cr = t / TPL, jc = t / NCL, cc = t % NCL;
    double2 z[8];
    // the workgroup walks planes blockIdx.x, + gridDim.x, ...; the next plane's loads are issued as soon as this
    // plane's have been moved to LDS, so they are in flight during both transforms
    double2 lv[8], lg1[8];   // forward: in, ga at (row 2cr + r, 2n) (gb, read only after a rho change or without the
                             // fold, is loaded when used); inverse: the coefficient pairs
    auto issue = [&](uint32_t e) {
        const uint32_t pb = e << (2 * L);
        if constexpr (MODE == SPEC_FWD) {
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    const uint32_t g = pb + uint32_t(2 * cr + r) * M + uint32_t(2 * (jr + s4 * TPL));
                    lv[2 * s4 + r] = ldnt2(a.in + g);
                    if (FORMB) lg1[2 * s4 + r] = ldnt2(a.ga + g);
                }
        } else {
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int k = jc + s * TPL;
                lv[2 * s] = ldnt2(a.in + pb + uint32_t(k) * M + uint32_t(2 * cc));
                lv[2 * s + 1] = ldnt2(a.in + pb + uint32_t(k ? M - k : M / 2) * M + uint32_t(2 * cc));
            }
        }
    };
    uint32_t e = blockIdx.x;
    if (e < nplanes) issue(e);
    for (; e < nplanes; e += gridDim.x) {
        const uint32_t pb = e << (2 * L);
        const uint32_t en = e + gridDim.x;
        // the twiddle tables through opaque pointers: their loads stay in the loop (hoisted out of it, the
        // per-plane values would all stay live and spill)
        const double2* tw = a.tw;
        const double2* twq = a.twq;
        asm volatile("" : "+s"(tw), "+s"(twq));
        asm volatile("" : "+v"(t));
        jr = t % TPL;
        cr = t / TPL;
        jc = t / NCL;
        cc = t % NCL;
        double2* const Xr = buf + cr * S::LP;
        double2* const Xc = buf + cc * S::LP;
        const int cxr = cr & 7, cxc = cc & 7;
        // coefficients (k, M - k) -> the IFFT input of the Makhoul sequence, in X
        auto inv_spectrum = [&](double2* X, int cx, int k, double2 Xk, double2 Xmk) {
            const int ka = k, kb = k ? M - k : M / 2;
            const double2 q1 = cconj(twq[ka]), q2 = cconj(twq[kb]);
            if (k == 0) {
                const double2 va2 = cmul(q2, make_double2(Xmk.x, -Xmk.x));
                const double2 vb2 = cmul(q2, make_double2(Xmk.y, -Xmk.y));
                X[spec8::slot(0, cx)] = Xk;
                X[spec8::slot(M / 2, cx)] = make_double2(va2.x - vb2.y, va2.y + vb2.x);
            } else {
                const double2 va1 = cmul(q1, make_double2(Xk.x, -Xmk.x));
                const double2 vb1 = cmul(q1, make_double2(Xk.y, -Xmk.y));
                const double2 va2 = cmul(q2, make_double2(Xmk.x, -Xk.x));
                const double2 vb2 = cmul(q2, make_double2(Xmk.y, -Xk.y));
                X[spec8::slot(ka, cx)] = make_double2(va1.x - vb1.y, va1.y + vb1.x);
                X[spec8::slot(kb, cx)] = make_double2(va2.x - vb2.y, va2.y + vb2.x);
            }
        };
        // the natural-order spectrum in X -> DCT-II coefficients (k, M - k) for k = j + s TPL
        auto fwd_coeff = [&](const double2* X, int cx, int k, double2& Xk, double2& Xmk) {
            const int ka = k, kb = k ? M - k : M / 2;
            const double2 Z1 = X[spec8::slot(ka, cx)], Z2 = X[spec8::slot(kb, cx)];
            const double2 q1 = twq[ka], q2 = twq[kb];
            if (k == 0) {
                Xk = make_double2(q1.x * Z1.x, q1.x * Z1.y);
                Xmk = make_double2(q2.x * Z2.x, q2.x * Z2.y);
            } else {
                const double2 Ap = make_double2(0.5 * (Z1.x + Z2.x), 0.5 * (Z1.y - Z2.y));
                const double2 Bp = make_double2(0.5 * (Z1.y + Z2.y), -0.5 * (Z1.x - Z2.x));
                Xk = make_double2(q1.x * Ap.x - q1.y * Ap.y, q1.x * Bp.x - q1.y * Bp.y);
                Xmk = make_double2(q2.x * Ap.x + q2.y * Ap.y, q2.x * Bp.x + q2.y * Bp.y);
            }
        };
        if constexpr (MODE == SPEC_FWD) {
            // ---- dim 0: rows 2cr, 2cr + 1 as one complex line ----------------------------------------------
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) {
                const int n = jr + s4 * TPL;
                double2 xv[2];
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    double2 v = lv[2 * s4 + r];
                    if (FORMB && !rd_gb) {
                        v.x += ca * lg1[2 * s4 + r].x;
                        v.y += ca * lg1[2 * s4 + r].y;
                    } else if (FORMB) {
                        const double2 g2 = ldnt2(a.gb + pb + uint32_t(2 * cr + r) * M + uint32_t(2 * n));
                        v.x += ca * lg1[2 * s4 + r].x + cb * g2.x;
                        v.y += ca * lg1[2 * s4 + r].y + cb * g2.y;
                    }
                    xv[r] = v;
                }
                Xr[spec8::slot(n, cxr)] = make_double2(xv[0].x, xv[1].x);
                Xr[spec8::slot(M - 1 - n, cxr)] = make_double2(xv[0].y, xv[1].y);
            }
            if (en < nplanes) issue(en);
            // a row pair's 16 threads are lanes of one wave and its exchange slots are that wave's alone: the row
            // transforms sync the wave only (xbar<2>); the plane image and the columns need the workgroup
            xbar<2>();
#pragma unroll
            for (int i = 0; i < 8; ++i) z[i] = Xr[spec8::slot(stage_in_pos<L, R0>(jr, i), cxr)];
            stages_from<L, R0, 1, false, false, 2>(z, jr, Xr, cxr, tw);   // natural-order spectrum in X
#pragma unroll
            for (int s = 0; s < 4; ++s) fwd_coeff(Xr, cxr, jr + s * TPL, z[2 * s], z[2 * s + 1]);
            lds_barrier();   // every spectrum read before the plane image (same LDS) is written
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int k = jr + s * TPL, ka = k, kb = k ? M - k : M / 2;
                PI[(2 * cr) * PP + ka] = z[2 * s].x;
                PI[(2 * cr + 1) * PP + ka] = z[2 * s].y;
                PI[(2 * cr) * PP + kb] = z[2 * s + 1].x;
                PI[(2 * cr + 1) * PP + kb] = z[2 * s + 1].y;
            }
            lds_barrier();
            // ---- dim 1: columns 2cc, 2cc + 1 as one complex line -------------------------------------------
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int n = stage_in_pos<L, R0>(jc, i);
                const int k = n < M / 2 ? 2 * n : 2 * (M - 1 - n) + 1;
                z[i] = *reinterpret_cast<const double2*>(&PI[k * PP + 2 * cc]);
            }
            stages_from<L, R0, 1, false, false, true>(z, jc, Xc, cxc, tw);   // its first barrier ends the image reads
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int k = jc + s * TPL, ka = k, kb = k ? M - k : M / 2;
                double2 Xk, Xmk;
                fwd_coeff(Xc, cxc, k, Xk, Xmk);
                stnt2(a.out + pb + uint32_t(ka) * M + uint32_t(2 * cc), Xk);
                stnt2(a.out + pb + uint32_t(kb) * M + uint32_t(2 * cc), Xmk);
            }
            lds_barrier();   // every spectrum read before the next plane's rows are written
        } else {
            // ---- dim 1 inverse: columns 2cc, 2cc + 1 --------------------------------------------------------
#pragma unroll
            for (int s = 0; s < 4; ++s) inv_spectrum(Xc, cxc, jc + s * TPL, lv[2 * s], lv[2 * s + 1]);
            if (en < nplanes) issue(en);
            lds_barrier();
#pragma unroll
            for (int i = 0; i < 8; ++i) z[i] = Xc[spec8::slot(stage_in_pos<L, R0>(jc, i), cxc)];
            stages_from<L, R0, 1, true, true, true>(z, jc, Xc, cxc, tw);   // outputs in registers
            lds_barrier();   // every exchange read before the plane image is written
            using LS = LastStage<L>;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int n = stage_out_pos<L, LS::R, LS::NS>(jc, i);
                const int k = n < M / 2 ? 2 * n : 2 * (M - 1 - n) + 1;
                *reinterpret_cast<double2*>(&PI[k * PP + 2 * cc]) = z[i];
            }
            lds_barrier();
            // ---- dim 0 inverse: rows 2cr, 2cr + 1 -----------------------------------------------------------
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int k = jr + s * TPL, kb = k ? M - k : M / 2;
                z[2 * s] = make_double2(PI[(2 * cr) * PP + k], PI[(2 * cr + 1) * PP + k]);
                z[2 * s + 1] = make_double2(PI[(2 * cr) * PP + kb], PI[(2 * cr + 1) * PP + kb]);
            }
            lds_barrier();   // every image read before the exchange buffer (same LDS) is written
#pragma unroll
            for (int s = 0; s < 4; ++s) inv_spectrum(Xr, cxr, jr + s * TPL, z[2 * s], z[2 * s + 1]);
            xbar<2>();   // the row transforms: one wave's slots (as forward)
#pragma unroll
            for (int i = 0; i < 8; ++i) z[i] = Xr[spec8::slot(stage_in_pos<L, R0>(jr, i), cxr)];
            stages_from<L, R0, 1, true, false, 2>(z, jr, Xr, cxr, tw);   // output through X
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) {
                const int n = jr + s4 * TPL;
                const double2 v0 = Xr[spec8::slot(n, cxr)], v1 = Xr[spec8::slot(M - 1 - n, cxr)];
                stnt2(a.out + pb + uint32_t(2 * cr) * M + uint32_t(2 * n), make_double2(v0.x, v1.x));
                stnt2(a.out + pb + uint32_t(2 * cr + 1) * M + uint32_t(2 * n), make_double2(v0.y, v1.y));
            }
            lds_barrier();   // every exchange read before the next plane's spectrum is written
        }
    }
}

// =============================================================================================
// 3-D meshes: the dim-0 transforms and the tridiagonal solve along dim 1 in two marching passes.
//
// Transforms along different dimensions commute, so a 3-D solve can run the dim-2 forward transform first (b formed
// on load) and leave dims 0 and 1 for last: after the dim-0 and dim-2 transforms, line (k0, k2) along dim 1 carries
// c0 I + c1 T (k_tri's operator). A workgroup owns one dim-2 frequency plane (m0 x m1, contiguous) and marches
// its rows (dim-1 positions), NR at a time:
//   forward  (k_march<L, false>): DCT-II of the NR rows along dim 0 (k_dct8's register radix-8 stages), then one
//            Thomas forward-elimination step per row for every k0 line, x'_i = (g_i - A x'_{i-1}) / den_i, the
//            previous row's x' carried in registers; x' written in place;
//   backward (k_march<L, true>): rows in reverse, x_i = x'_i - (A / den_i) x_{i+1}, then the inverse DCT along
//            dim 0 of the NR rows; theta written in place (scaled by inv_n m1).
// The dim-1 forward / inverse transform passes and the separate tridiagonal pass become these two: a 3-D solve
// moves 9N words instead of 11N (the first pass 3N, then 2N each).
//
// The backward sweep needs den_i in reverse order, which the forward recurrence den_i = B - A^2 / den_{i-1}
// cannot give without storing it. Its closed form does: den_i = p_{i+1} / p_i with p_{i+1} = B p_i - A^2 p_{i-1},
// p_0 = 1, p_1 = B0 = c0 + c1 (the Neumann first row), so with the roots l1 > l2 of l^2 - B l + A^2 and
// q = l2 / l1, r = beta / alpha:
//     den_i = l1 (1 + r q^{i+1}) / (1 + r q^i),  l1 = (B + s) / 2,  s = sqrt(c0 (c0 + 4 c1)),
//     r = 4 c0 c1 / (c0 + s)^2,  q = 4 c1^2 / (B + s)^2,  1 - q = (c0 + s)(B + s + 2 c1) / (B + s)^2
//     (B = c0 + 2 c1, A = -c1)
// every term free of cancellation (a numpy study against long-double Thomas: as accurate as fp64 Thomas for
// c1 / c0 from 1e-2 to 1e7). The last row subtracts c1 (Neumann end). Both sweeps evaluate the same closed form,
// so they apply one factorisation; q^i comes from one exp per line per step, then q-multiplications over the
// step's rows.
namespace march {
template <int L>
struct Shape {
    static constexpr int M = 1 << L;
    static constexpr int TPL = M / 8;          // FFT threads per complex line (k_dct8's D0 mapping)
    static constexpr int NCL = 2048 / M;       // complex lines = row pairs per step
    static constexpr int NR = 2 * NCL;         // rows per step
    static constexpr int NT = NCL * TPL;       // 256 threads
    static constexpr int LPT = M / NT;         // k0 lines per thread in the elimination
};
}  // namespace march

template <int L, bool BWD>
__global__ __launch_bounds__(256) void k_march(const SpecArgs a, uint32_t m1) {
    using S = spec8::Shape<L>;
    using T = march::Shape<L>;
    constexpr int M = T::M, TPL = T::TPL, NCL = T::NCL, NR = T::NR, NT = T::NT, LPT = T::LPT, R0 = S::R0;
    static_assert(NT == 256 && LPT >= 1, "k_march: 256 threads, m0 in [256, 2048]");
    double sigma = a.sigma;
    if (a.skip && *a.skip) return;
    if (a.ctl) {
        if (a.ctl->done) return;
        sigma = a.ctl->sigma;
    }
    __shared__ double2 buf[NCL * S::LP];   // FFT exchange (k_dct8's slot layout)
    __shared__ double C[NR * M];          // the step's coefficients [row][k0]
    const uint32_t e = blockIdx.x;        // dim-2 frequency
    const uint32_t pb = e * (uint32_t(M) * m1);
    const int t = threadIdx.x;
    const int j = t % TPL, c = t / TPL;
    double2* const X = buf + c * S::LP;
    const int cx = c & 7;
    const double2* __restrict__ tw = a.tw;
    const double2* __restrict__ twq = a.twq;

    // line constants of k0 = t + l NT: c0 + c1 T along dim 1 (dims 0 and 2 transformed), then the closed form
    double A[LPT], il1[LPT], rr[LPT], qq[LPT], lq[LPT], c1v[LPT];
    {
        const double lam2 = a.lam[a.lam_off[2] + e];
#pragma unroll
        for (int l = 0; l < LPT; ++l) {
            const double lam0 = a.lam[a.lam_off[0] + uint32_t(t + l * NT)];
            double c0 = a.w0, c1 = 0.0;
            for (int Sm = 1; Sm < 8; ++Sm) {
                if (a.cS[Sm] == 0.0) continue;
                double prod = sigma * a.cS[Sm];
                if (Sm & 1) prod *= lam0;
                if (Sm & 4) prod *= lam2;
                if (Sm & 2) c1 += prod;
                else c0 += prod;
            }
            const double B = c0 + 2.0 * c1, sq = sqrt(c0 * (c0 + 4.0 * c1));
            const double l1 = 0.5 * (B + sq);
            const double cs = c0 + sq, bs = B + sq;
            A[l] = -c1;
            c1v[l] = c1;
            il1[l] = 1.0 / l1;
            rr[l] = 4.0 * c0 * c1 / (cs * cs);
            // log q: from q = 4 c1^2 / (B + s)^2 while q is small (-inf when c1 = 0), from 1 - q near 1 (where the
            // rounding of 1 - q ~ 1 could also push log1p's argument below -1)
            const double qd = 4.0 * c1 * c1 / (bs * bs);
            lq[l] = qd < 0.5 ? log(qd) : log1p(-(cs * (bs + 2.0 * c1)) / (bs * bs));
            qq[l] = qd < 0.5 ? qd : exp(lq[l]);
        }
    }
    // q^i at the first row of a step (exact start: no drift over the march)
    auto qpow = [&](int l, uint32_t i) -> double { return i == 0 ? 1.0 : exp(double(i) * lq[l]); };

    // the natural-order spectrum in X -> DCT-II coefficients (k, M - k) for k = j + s TPL (k_plane8's fwd_coeff)
    auto fwd_coeff = [&](int k, double2& Xk, double2& Xmk) {
        const int ka = k, kb = k ? M - k : M / 2;
        const double2 Z1 = X[spec8::slot(ka, cx)], Z2 = X[spec8::slot(kb, cx)];
        const double2 q1 = twq[ka], q2 = twq[kb];
        if (k == 0) {
            Xk = make_double2(q1.x * Z1.x, q1.x * Z1.y);
            Xmk = make_double2(q2.x * Z2.x, q2.x * Z2.y);
        } else {
            const double2 Ap = make_double2(0.5 * (Z1.x + Z2.x), 0.5 * (Z1.y - Z2.y));
            const double2 Bp = make_double2(0.5 * (Z1.y + Z2.y), -0.5 * (Z1.x - Z2.x));
            Xk = make_double2(q1.x * Ap.x - q1.y * Ap.y, q1.x * Bp.x - q1.y * Bp.y);
            Xmk = make_double2(q2.x * Ap.x + q2.y * Ap.y, q2.x * Bp.x + q2.y * Bp.y);
        }
    };
    // coefficients (k, M - k) -> the IFFT input of the Makhoul sequence, in X (k_plane8's inv_spectrum)
    auto inv_spectrum = [&](int k, double2 Xk, double2 Xmk) {
        const int ka = k, kb = k ? M - k : M / 2;
        const double2 q1 = cconj(twq[ka]), q2 = cconj(twq[kb]);
        if (k == 0) {
            const double2 va2 = cmul(q2, make_double2(Xmk.x, -Xmk.x));
            const double2 vb2 = cmul(q2, make_double2(Xmk.y, -Xmk.y));
            X[spec8::slot(0, cx)] = Xk;
            X[spec8::slot(M / 2, cx)] = make_double2(va2.x - vb2.y, va2.y + vb2.x);
        } else {
            const double2 va1 = cmul(q1, make_double2(Xk.x, -Xmk.x));
            const double2 vb1 = cmul(q1, make_double2(Xk.y, -Xmk.y));
            const double2 va2 = cmul(q2, make_double2(Xmk.x, -Xk.x));
            const double2 vb2 = cmul(q2, make_double2(Xmk.y, -Xk.y));
            X[spec8::slot(ka, cx)] = make_double2(va1.x - vb1.y, va1.y + vb1.x);
            X[spec8::slot(kb, cx)] = make_double2(va2.x - vb2.y, va2.y + vb2.x);
        }
    };

    double2 z[8];
    if constexpr (!BWD) {
        double xs[LPT];   // x'_{i-1} per line
#pragma unroll
        for (int l = 0; l < LPT; ++l) xs[l] = 0.0;
        double2 lv[8];    // the step's rows (2c, 2c + 1) at (2n, 2n + 1), n = j + s4 TPL
        auto issue = [&](uint32_t i0) {
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
                for (int r = 0; r < 2; ++r)
                    lv[2 * s4 + r] = ldnt2(a.in + pb + (i0 + uint32_t(2 * c + r)) * uint32_t(M) +
                                           uint32_t(2 * (j + s4 * TPL)));
        };
        issue(0);
        for (uint32_t i0 = 0; i0 < m1; i0 += NR) {
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) {
                const int n = j + s4 * TPL;
                X[spec8::slot(n, cx)] = make_double2(lv[2 * s4].x, lv[2 * s4 + 1].x);
                X[spec8::slot(M - 1 - n, cx)] = make_double2(lv[2 * s4].y, lv[2 * s4 + 1].y);
            }
            if (i0 + NR < m1) issue(i0 + NR);   // in flight during this step (LDS-only barriers below)
            lds_barrier();
#pragma unroll
            for (int i = 0; i < 8; ++i) z[i] = X[spec8::slot(stage_in_pos<L, R0>(j, i), cx)];
            stages_from<L, R0, 1, false, false, true>(z, j, X, cx, tw);   // natural-order spectrum in X
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int k = j + s * TPL, kb = k ? M - k : M / 2;
                double2 Xk, Xmk;
                fwd_coeff(k, Xk, Xmk);
                C[(2 * c) * M + k] = Xk.x;
                C[(2 * c + 1) * M + k] = Xk.y;
                C[(2 * c) * M + kb] = Xmk.x;
                C[(2 * c + 1) * M + kb] = Xmk.y;
            }
            lds_barrier();
            // forward elimination along dim 1, rows i0 .. i0 + NR - 1
#pragma unroll
            for (int l = 0; l < LPT; ++l) {
                const uint32_t k0 = uint32_t(t + l * NT);
                double qi = qpow(l, i0);
                double u = 1.0 + rr[l] * qi;
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    const uint32_t i = i0 + uint32_t(r);
                    qi *= qq[l];
                    const double u1 = 1.0 + rr[l] * qi;
                    // 1 / den_i = u_i / (l1 u_{i+1}); the last row: den - c1
                    const double w = (i + 1 == m1) ? 1.0 / (u1 / (u * il1[l]) - c1v[l]) : u * il1[l] / u1;
                    xs[l] = (C[r * M + int(k0)] - A[l] * xs[l]) * w;
                    __builtin_nontemporal_store(xs[l], a.out + pb + i * uint32_t(M) + k0);
                    u = u1;
                }
            }
            // (the next step's first LDS writes touch X, whose reads ended before the barrier above; its C
            // writes come after its first barrier)
        }
    } else {
        const double sc = a.inv_n * double(m1);   // the dim-0 and dim-2 transforms are unnormalised
        double xn[LPT];   // x_{i+1} per line
#pragma unroll
        for (int l = 0; l < LPT; ++l) xn[l] = 0.0;
        double lx[LPT][NR];   // the step's x' rows at this thread's lines
        auto issue = [&](uint32_t i0) {
#pragma unroll
            for (int l = 0; l < LPT; ++l)
#pragma unroll
                for (int r = 0; r < NR; ++r)
                    lx[l][r] = __builtin_nontemporal_load(a.in + pb + (i0 + uint32_t(r)) * uint32_t(M) + uint32_t(t + l * NT));
        };
        issue(m1 - NR);
        for (int i0 = int(m1) - NR; i0 >= 0; i0 -= NR) {
            double cur[LPT][NR];
#pragma unroll
            for (int l = 0; l < LPT; ++l)
#pragma unroll
                for (int r = 0; r < NR; ++r) cur[l][r] = lx[l][r];
            if (i0 >= NR) issue(uint32_t(i0 - NR));
            // back substitution, rows i0 + NR - 1 down to i0
#pragma unroll
            for (int l = 0; l < LPT; ++l) {
                const uint32_t k0 = uint32_t(t + l * NT);
                double u[NR + 1];
                double qi = qpow(l, uint32_t(i0));
                u[0] = 1.0 + rr[l] * qi;
#pragma unroll
                for (int r = 1; r <= NR; ++r) {
                    qi *= qq[l];
                    u[r] = 1.0 + rr[l] * qi;
                }
#pragma unroll
                for (int r = NR - 1; r >= 0; --r) {
                    const uint32_t i = uint32_t(i0 + r);
                    double x = cur[l][r];
                    if (i + 1 < m1) x -= A[l] * u[r] * il1[l] / u[r + 1] * xn[l];   // e_i = A / den_i
                    xn[l] = x;
                    C[r * M + int(k0)] = x * sc;
                }
            }
            lds_barrier();
            // inverse DCT along dim 0 of rows (2c, 2c + 1)
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int k = j + s * TPL, kb = k ? M - k : M / 2;
                inv_spectrum(k, make_double2(C[(2 * c) * M + k], C[(2 * c + 1) * M + k]),
                             make_double2(C[(2 * c) * M + kb], C[(2 * c + 1) * M + kb]));
            }
            lds_barrier();
#pragma unroll
            for (int i = 0; i < 8; ++i) z[i] = X[spec8::slot(stage_in_pos<L, R0>(j, i), cx)];
            stages_from<L, R0, 1, true, false, true>(z, j, X, cx, tw);   // output through X
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) {
                const int n = j + s4 * TPL;
                const double2 v0 = X[spec8::slot(n, cx)], v1 = X[spec8::slot(M - 1 - n, cx)];
                stnt2(a.out + pb + uint32_t(i0 + 2 * c) * uint32_t(M) + uint32_t(2 * n), make_double2(v0.x, v1.x));
                stnt2(a.out + pb + uint32_t(i0 + 2 * c + 1) * uint32_t(M) + uint32_t(2 * n), make_double2(v0.y, v1.y));
            }
            // (the next step writes C before its first barrier: every C read of this step came before this step's
            // second barrier; its X writes come after its first barrier, which every thread reaches only after its
            // stores above)
        }
    }
}

// =============================================================================================
// Mixed-radix lengths: m = 2^a 3^b 5^c 7^d <= 4096 that is not a power of two (meshes such as
// 24 x 40, 100^3 or 1000^2). Same Makhoul pairing and pass structure as k_dct8, with the complex
// FFT of length m run in LDS as in-place Cooley-Tukey stages of radix 8, 4, 2, 3, 5, 7: decimation
// in time on input stored at digit-reversed positions (forward), decimation in frequency leaving
// digit-reversed output (inverse), so both permutations fold into the load / store index as the
// bit reversal does for k_dct. Line addresses take a general stride (FastDiv).
namespace dctg {
constexpr int NT = 512;   // threads per workgroup: 16 lines of <= 512 points (two workgroups per CU)
// cos / sin (2 pi k / R), k < R
__device__ __constant__ const double c3[3] = {1.0, -0.5, -0.5};
__device__ __constant__ const double s3[3] = {0.0, 0.86602540378443864676, -0.86602540378443864676};
__device__ __constant__ const double c5[5] = {1.0, 0.30901699437494742410, -0.80901699437494742410,
                                             -0.80901699437494742410, 0.30901699437494742410};
__device__ __constant__ const double s5[5] = {0.0, 0.95105651629515357212, 0.58778525229247312917,
                                             -0.58778525229247312917, -0.95105651629515357212};
__device__ __constant__ const double c7[7] = {1.0, 0.62348980185873353053, -0.22252093395631440429,
                                             -0.90096886790241912624, -0.90096886790241912624,
                                             -0.22252093395631440429, 0.62348980185873353053};
__device__ __constant__ const double s7[7] = {0.0, 0.78183148246802980871, 0.97492791218182360702,
                                             0.43388373911755812048, -0.43388373911755812048,
                                             -0.97492791218182360702, -0.78183148246802980871};
}  // namespace dctg

// natural-order DFT of z[0..R-1] for R in {3, 5, 7}
template <int R, bool INV>
__device__ __forceinline__ void dft_odd(double2* z) {
    const double* C = R == 3 ? dctg::c3 : (R == 5 ? dctg::c5 : dctg::c7);
    const double* Sn = R == 3 ? dctg::s3 : (R == 5 ? dctg::s5 : dctg::s7);
    double2 y[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        double2 acc = z[0];
#pragma unroll
        for (int q = 1; q < R; ++q) {
            const int k = (q * r) % R;
            const double c = C[k], s = INV ? Sn[k] : -Sn[k];   // e^{-+ i 2 pi k / R}
            acc.x += z[q].x * c - z[q].y * s;
            acc.y += z[q].x * s + z[q].y * c;
        }
        y[r] = acc;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) z[r] = y[r];
}

template <int R, bool INV>
__device__ __forceinline__ void dft_any(double2* z) {
    if constexpr (R == 2 || R == 4 || R == 8) dft_r<R, INV>(z);
    else dft_odd<R, INV>(z);
}

// One in-place stage over ncl lines of pitch LP: butterflies (block b of L1 = L R, column j < L) on
// elements b L1 + j + r L. DIT: twiddle w^{r j m / L1} then DFT; DIF: DFT then twiddle.
template <int R, bool DIF, bool INV>
__device__ __forceinline__ void mr_stage(double2* __restrict__ buf, const double2* __restrict__ tw, int ncl, int m,
                                         int LP, int L, const FastDiv& fper, const FastDiv& fL) {
    const int L1 = L * R, per = m / R, nb = ncl * per, tstep = m / L1;
    for (int t = threadIdx.x; t < nb; t += dctg::NT) {
        const int line = int(fper.div(uint32_t(t))), bi = t - line * per;
        const int b = int(fL.div(uint32_t(bi))), j = bi - b * L;
        double2* x = buf + line * LP + b * L1 + j;
        double2 z[R];
#pragma unroll
        for (int r = 0; r < R; ++r) z[r] = x[r * L];
        if (!DIF) {
#pragma unroll
            for (int r = 1; r < R; ++r) {
                const double2 w = tw[r * j * tstep];   // r j m / L1 < m
                z[r] = cmul(z[r], INV ? cconj(w) : w);
            }
        }
        dft_any<R, INV>(z);
        if (DIF) {
#pragma unroll
            for (int r = 1; r < R; ++r) {
                const double2 w = tw[r * j * tstep];
                z[r] = cmul(z[r], INV ? cconj(w) : w);
            }
        }
#pragma unroll
        for (int r = 0; r < R; ++r) x[r * L] = z[r];
    }
    __syncthreads();
}

template <bool DIF, bool INV>
__device__ __forceinline__ void mr_fft(double2* buf, const double2* tw, int ncl, int m, int LP, const SpecArgs& a) {
    auto stage = [&](int s, int L) {
        switch (a.rad[s]) {
            case 2: mr_stage<2, DIF, INV>(buf, tw, ncl, m, LP, L, a.fper[s], a.fL[s]); break;
            case 3: mr_stage<3, DIF, INV>(buf, tw, ncl, m, LP, L, a.fper[s], a.fL[s]); break;
            case 4: mr_stage<4, DIF, INV>(buf, tw, ncl, m, LP, L, a.fper[s], a.fL[s]); break;
            case 5: mr_stage<5, DIF, INV>(buf, tw, ncl, m, LP, L, a.fper[s], a.fL[s]); break;
            case 7: mr_stage<7, DIF, INV>(buf, tw, ncl, m, LP, L, a.fper[s], a.fL[s]); break;
            default: mr_stage<8, DIF, INV>(buf, tw, ncl, m, LP, L, a.fper[s], a.fL[s]); break;
        }
    };
    if (!DIF) {
        for (int s = 0, L = 1; s < a.nrad; ++s) {
            stage(s, L);
            L *= a.rad[s];
        }
    } else {
        for (int s = a.nrad - 1, L1 = m; s >= 0; --s) {
            const int L = L1 / a.rad[s];
            stage(s, L);
            L1 = L;
        }
    }
}

template <int MODE, bool D0, bool FORMB>
__global__ __launch_bounds__(dctg::NT) __attribute__((amdgpu_waves_per_eu(4))) void k_dctg(const SpecArgs a) {
    double sigma = a.sigma, ca = a.ca, cb = a.cb;
    if (a.skip && *a.skip) return;
    if (a.ctl) {
        if (a.ctl->done) return;
        sigma = a.ctl->sigma;
        ca = a.ctl->rho;
        cb = a.ctl->rho * a.ctl->c_prev;
    }
    extern __shared__ double2 buf[];   // tq / 2 lines of m + PAD complex slots (launch-time size)
    __shared__ double lc0[16], lc1[16];
    const int m = int(a.m[a.d]);
    const int tq = a.tq, ncl = tq >> 1;
    const int LP = m + spec::PAD;
    const uint32_t q0 = (a.xrun ? xcd_run(blockIdx.x, gridDim.x) : blockIdx.x) * uint32_t(tq);

    if (MODE == SPEC_MID && threadIdx.x < uint32_t(tq)) {
        const uint32_t q = a.q_off + q0 + threadIdx.x;
        double lamv[kMaxDims] = {0, 0, 0, 0};
        uint32_t rest = (q - a.q_off) < a.nlines ? q : a.q_off;
        const int jlast = a.d == a.p - 1 ? a.p - 2 : a.p - 1;
        for (int j = 0; j < a.p; ++j) {
            if (j == a.d) continue;
            const uint32_t qq = (j < jlast) ? a.fd[j].div(rest) : 0u;
            lamv[j] = a.lam[a.lam_off[j] + (rest - qq * a.m[j])];
            rest = qq;
        }
        double c0 = a.w0, c1 = 0.0;
        for (int S = 1; S < (1 << a.p); ++S) {
            if (a.cS[S] == 0.0) continue;
            double prod = sigma * a.cS[S];
            for (int j = 0; j < a.p; ++j)
                if (j != a.d && ((S >> j) & 1)) prod *= lamv[j];
            if ((S >> a.d) & 1) c1 += prod;
            else c0 += prod;
        }
        lc0[threadIdx.x] = c0;
        lc1[threadIdx.x] = c1;
    }

    // global offset of (local line ql, position k): line q = (block q / stride, offset q % stride)
    auto gaddr = [&](uint32_t ql, uint32_t k) -> uint32_t {
        const uint32_t q = q0 + ql;
        if (D0) return q * uint32_t(m) + k;
        const uint32_t hi = a.fds.div(q);
        return (q - hi * a.stride) + hi * a.stride * uint32_t(m) + k * a.stride;
    };
    const int ltq = __ffs(tq) - 1;   // tq is a power of two

    double* bw = reinterpret_cast<double*>(buf);
    const int total = tq * m;
    for (int e = threadIdx.x; e < total; e += dctg::NT) {
        const int ql = D0 ? int(a.fm.div(uint32_t(e))) : (e & (tq - 1));
        const int k = D0 ? e - ql * m : (e >> ltq);
        double v = 0.0;
        if (q0 + uint32_t(ql) < a.nlines) {
            const uint32_t gi = gaddr(uint32_t(ql), uint32_t(k));
            v = __builtin_nontemporal_load(a.in + gi);
            if (FORMB) v += ca * __builtin_nontemporal_load(a.ga + gi) + cb * __builtin_nontemporal_load(a.gb + gi);
        }
        const int pos = MODE == SPEC_INV ? k : int(a.perm[k]);
        bw[2 * ((ql >> 1) * LP + pos) + (ql & 1)] = v;
    }
    __syncthreads();

    const double2* tw = a.tw;
    if (MODE != SPEC_INV) mr_fft<false, false>(buf, tw, ncl, m, LP, a);

    // spectrum <-> DCT coefficients over the pairs (k, m-k); k = 0 pairs with itself, and so does
    // k = m/2 for even m (handled with k = 0)
    {
        const int half = m >> 1, npl = (m & 1) ? half + 1 : half;
        const int npairs = ncl * npl;
        for (int t = threadIdx.x; t < npairs; t += dctg::NT) {
            const int line = t / npl, k = t - line * npl;
            double2* x = buf + line * LP;
            const bool self = k == 0;
            const bool mid = self && !(m & 1);   // also the self pair m/2
            const int ka = k, kb = self ? half : m - k;
            double2 Xk, Xmk = make_double2(0.0, 0.0);
            if (MODE != SPEC_INV) {
                const double2 Z1 = x[ka], q1 = a.twq[ka];
                if (self) {
                    Xk = make_double2(q1.x * Z1.x, q1.x * Z1.y);
                    if (mid) {
                        const double2 Z2 = x[kb], q2 = a.twq[kb];
                        Xmk = make_double2(q2.x * Z2.x, q2.x * Z2.y);
                    }
                } else {
                    const double2 Z2 = x[kb], q2 = a.twq[kb];
                    const double2 Ap = make_double2(0.5 * (Z1.x + Z2.x), 0.5 * (Z1.y - Z2.y));
                    const double2 Bp = make_double2(0.5 * (Z1.y + Z2.y), -0.5 * (Z1.x - Z2.x));
                    Xk = make_double2(q1.x * Ap.x - q1.y * Ap.y, q1.x * Bp.x - q1.y * Bp.y);
                    Xmk = make_double2(q2.x * Ap.x + q2.y * Ap.y, q2.x * Bp.x + q2.y * Bp.y);
                }
            } else {
                Xk = x[ka];
                if (!self || mid) Xmk = x[kb];
            }
            if (MODE == SPEC_MID) {
                const double* lamd = a.lam + a.lam_off[a.d];
                const int l0 = 2 * line, l1 = 2 * line + 1;
                const double la = lamd[ka];
                Xk.x *= a.inv_n / (lc0[l0] + lc1[l0] * la);
                Xk.y *= a.inv_n / (lc0[l1] + lc1[l1] * la);
                if (!self || mid) {
                    const double lb = lamd[kb];
                    Xmk.x *= a.inv_n / (lc0[l0] + lc1[l0] * lb);
                    Xmk.y *= a.inv_n / (lc0[l1] + lc1[l1] * lb);
                }
            }
            if (MODE == SPEC_FWD) {
                x[ka] = Xk;
                if (!self || mid) x[kb] = Xmk;
                continue;
            }
            const double2 q2 = cconj(a.twq[kb]);
            if (self) {
                x[0] = Xk;   // X[m] = 0: V[0] = X[0]
                if (mid) {
                    const double2 va2 = cmul(q2, make_double2(Xmk.x, -Xmk.x));
                    const double2 vb2 = cmul(q2, make_double2(Xmk.y, -Xmk.y));
                    x[half] = make_double2(va2.x - vb2.y, va2.y + vb2.x);
                }
            } else {
                const double2 q1 = cconj(a.twq[ka]);
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

    if (MODE != SPEC_FWD) mr_fft<true, true>(buf, tw, ncl, m, LP, a);

    for (int e = threadIdx.x; e < total; e += dctg::NT) {
        const int ql = D0 ? int(a.fm.div(uint32_t(e))) : (e & (tq - 1));
        const int k = D0 ? e - ql * m : (e >> ltq);
        if (q0 + uint32_t(ql) >= a.nlines) continue;
        const int pos = MODE == SPEC_FWD ? k : int(a.perm[k]);
        __builtin_nontemporal_store(bw[2 * ((ql >> 1) * LP + pos) + (ql & 1)], a.out + gaddr(uint32_t(ql), uint32_t(k)));
    }
}

// ---------------------------------------------------------------------------------------------
// k_dctm: register-resident mixed-radix passes for the lengths of the BASELINE-adjacent meshes (500 = 4 5^3,
// 1000 = 2 4 5^3): k_dct8's Stockham scheme with a compile-time radix plan. A thread holds V complex values
// of one complex line (two real lines, Makhoul pairing) and runs its V / R radix-R butterflies of each stage in
// registers; LDS carries the exchanges between stages (k_dctg: one in-place LDS stage per radix with FastDiv
// index math and a permutation-table load per element). FWD and INV passes (the last dimension takes k_trig or
// k_dctg's MID pass); TQ = 16 real lines per workgroup, lanes over the lines for a strided pass (16-B accesses
// of a line pair, 128-B rows when the tile does not straddle a stride boundary), over j for d = 0.
namespace dctm {
constexpr int NCL = 8;   // complex lines per workgroup (default tile)
// radix plan and values per thread (every radix divides V): 500 = 2 2 5^3 with V = 10 (400 threads, two
// workgroups per CU), 1000 = 2 4 5^3 with V = 20 (400 threads)
template <int M> struct Plan;
template <> struct Plan<500> {
    static constexpr int n = 5, V = 10;
    static constexpr int r[5] = {2, 2, 5, 5, 5};
};
template <> struct Plan<1000> {
    static constexpr int n = 5, V = 20;
    static constexpr int r[5] = {2, 4, 5, 5, 5};
};
template <int M> struct Shape {
    static constexpr int V = Plan<M>::V;      // complex values per thread
    static constexpr int T = M / V;           // threads per complex line
    static constexpr int NT = NCL * T;
    static constexpr int LP = M + 4;          // line pitch (complex slots)
};
}  // namespace dctm

// stage S (span NS) of the thread's butterflies b_s = j + s T; z[s R + r] holds position b_s + r M / R
template <int M, int S, int NS, bool INV>
__device__ __forceinline__ void dctm_stages(double2* z, int j, double2* X, const double2* __restrict__ tw) {
    using P = dctm::Plan<M>;
    constexpr int V = P::V, R = P::r[S], T = M / V, NB = V / R;
#pragma unroll
    for (int s = 0; s < NB; ++s) {
        if constexpr (NS > 1) {
            const int kk = (j + s * T) % NS;
            constexpr int step = M / (NS * R);
#pragma unroll
            for (int r = 1; r < R; ++r) {
                double2 w = tw[kk * r * step];
                if (INV) w = cconj(w);
                z[s * R + r] = cmul(z[s * R + r], w);
            }
        }
        dft_any<R, INV>(z + s * R);
    }
    if constexpr (S + 1 < P::n) {
        constexpr int R2 = P::r[S + 1];
        __syncthreads();   // every thread has read this stage's inputs
#pragma unroll
        for (int s = 0; s < NB; ++s) {
            const int b = j + s * T;
#pragma unroll
            for (int r = 0; r < R; ++r) X[(b / NS) * NS * R + b % NS + r * NS] = z[s * R + r];
        }
        __syncthreads();
#pragma unroll
        for (int s = 0; s < V / R2; ++s)
#pragma unroll
            for (int r = 0; r < R2; ++r) z[s * R2 + r] = X[j + s * T + r * (M / R2)];
        dctm_stages<M, S + 1, NS * R, INV>(z, j, X, tw);
    }
}
// output position of z[i] after the last stage
template <int M>
__device__ __forceinline__ int dctm_out_pos(int j, int i) {
    using P = dctm::Plan<M>;
    constexpr int R = P::r[P::n - 1], NS = M / R, T = M / P::V;
    const int s = i / R, r = i % R, b = j + s * T;
    return (b / NS) * NS * R + b % NS + r * NS;
}
// input position of z[i] of the first stage
template <int M>
__device__ __forceinline__ int dctm_in_pos(int j, int i) {
    using P = dctm::Plan<M>;
    constexpr int R = P::r[0], T = M / P::V;
    return j + (i / R) * T + (i % R) * (M / R);
}

// NCLW complex lines (2 NCLW real lines) per workgroup: 8 (128-B rows) or 4 (64-B rows, half the LDS: more workgroups
// a CU)
template <int M, int MODE, bool D0, bool FORMB, int NCLW = dctm::NCL>
__global__ __launch_bounds__(NCLW * dctm::Shape<M>::T) void k_dctm(const SpecArgs a) {
    using S = dctm::Shape<M>;
    constexpr int T = S::T, NCL = NCLW, V = S::V, TQ = 2 * NCLW;
    static_assert(MODE == SPEC_FWD || MODE == SPEC_INV, "FWD / INV passes");
    double ca = a.ca, cb = a.cb;
    bool rd_gb = true;
    if (a.skip && *a.skip) return;
    if (a.ctl) {
        if (a.ctl->done) return;
        ca = a.ctl->rho;
        cb = a.ctl->rho * a.ctl->c_prev;
        if (a.fold) {
            ca = a.ctl->fold_ka;
            cb = a.ctl->fold_kb;
            rd_gb = a.ctl->fix != 0;
        }
    }
    __shared__ double2 buf[NCL * S::LP];
    const int t = threadIdx.x;
    const int j = D0 ? (t % T) : (t / NCL);
    const int c = D0 ? (t / T) : (t % NCL);
    const uint32_t q0 = (a.xrun ? xcd_run(blockIdx.x, gridDim.x) : blockIdx.x) * uint32_t(TQ);
    const int la = 2 * c;
    const bool va = q0 + uint32_t(la) < a.nlines;   // lines come in pairs: nlines is even (launcher)
    double2* X = buf + c * S::LP;
    const double2* __restrict__ tw = a.tw;
    // global offset of (real line la of this thread's pair, position k); line la + 1 is the next word
    const uint32_t q = q0 + uint32_t(la);
    uint32_t lbase;
    if (D0) {
        lbase = q * uint32_t(M);
    } else {
        const uint32_t hi = a.fds.div(q);
        lbase = (q - hi * a.stride) + hi * a.stride * uint32_t(M);
    }
    auto gidx = [&](uint32_t k) -> uint32_t { return D0 ? lbase + k : lbase + k * a.stride; };
    auto ld_pair2 = [&](uint32_t g) -> double2 {   // b (or the input) at global offsets g, g + 1
        double2 v = ldnt2(a.in + g);
        if (FORMB && !rd_gb) {
            const double2 g1 = ldnt2(a.ga + g);
            v.x += ca * g1.x;
            v.y += ca * g1.y;
        } else if (FORMB) {
            const double2 g1 = ldnt2(a.ga + g), g2 = ldnt2(a.gb + g);
            v.x += ca * g1.x + cb * g2.x;
            v.y += ca * g1.y + cb * g2.y;
        }
        return v;
    };
    auto ld_pair = [&](uint32_t k) -> double2 {   // (line la, line la + 1) at position k, strided pass
        const uint32_t g = gidx(k);
        double2 v = ldnt2(a.in + g);
        if (FORMB && !rd_gb) {
            const double2 g1 = ldnt2(a.ga + g);
            v.x += ca * g1.x;
            v.y += ca * g1.y;
        } else if (FORMB) {
            const double2 g1 = ldnt2(a.ga + g), g2 = ldnt2(a.gb + g);
            v.x += ca * g1.x + cb * g2.x;
            v.y += ca * g1.y + cb * g2.y;
        }
        return v;
    };
    double2 z[V];
    if constexpr (MODE == SPEC_FWD) {
        // ---- Makhoul input v[n] = x[2n], v[M-1-n] = x[2n+1] into the first stage --------------------------
        if (D0) {
            // contiguous lines: 16-B loads of (x[2n], x[2n+1]) of each real line land at positions n, M-1-n
#pragma unroll
            for (int s = 0; s < M / 2 / T; ++s) {
                const int n = j + s * T;
                double2 xa = make_double2(0.0, 0.0), xb = make_double2(0.0, 0.0);
                if (va) {   // (x[2n], x[2n+1]) of lines la and la + 1: 16-B loads (M even: aligned)
                    xa = ld_pair2(lbase + uint32_t(2 * n));
                    xb = ld_pair2(lbase + uint32_t(M) + uint32_t(2 * n));
                }
                X[n] = make_double2(xa.x, xb.x);
                X[M - 1 - n] = make_double2(xa.y, xb.y);
            }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < V; ++i) z[i] = X[dctm_in_pos<M>(j, i)];
        } else {
#pragma unroll
            for (int i = 0; i < V; ++i) {
                const int n = dctm_in_pos<M>(j, i);
                const uint32_t k = n < M / 2 ? uint32_t(2 * n) : uint32_t(2 * (M - 1 - n) + 1);
                z[i] = va ? ld_pair(k) : make_double2(0.0, 0.0);
            }
        }
        dctm_stages<M, 0, 1, false>(z, j, X, tw);
        __syncthreads();   // every thread has read the last exchange
#pragma unroll
        for (int i = 0; i < V; ++i) X[dctm_out_pos<M>(j, i)] = z[i];   // natural-order spectrum
        __syncthreads();
        // ---- spectrum -> DCT-II coefficients (k, M - k); k = 0 and M / 2 pair with themselves --------------
#pragma unroll
        for (int s = 0; s < (M / 2 + T) / T; ++s) {
            const int k = j + s * T;
            if (k > M / 2) continue;
            const int ka = k, kb = k ? M - k : M / 2;
            const double2 Z1 = X[ka], Z2 = X[kb];
            const double2 q1 = a.twq[ka], q2 = a.twq[kb];
            double2 Xk, Xmk;
            if (k == 0) {
                Xk = make_double2(q1.x * Z1.x, q1.x * Z1.y);
                Xmk = make_double2(q2.x * Z2.x, q2.x * Z2.y);
            } else {
                const double2 Ap = make_double2(0.5 * (Z1.x + Z2.x), 0.5 * (Z1.y - Z2.y));
                const double2 Bp = make_double2(0.5 * (Z1.y + Z2.y), -0.5 * (Z1.x - Z2.x));
                Xk = make_double2(q1.x * Ap.x - q1.y * Ap.y, q1.x * Bp.x - q1.y * Bp.y);
                Xmk = make_double2(q2.x * Ap.x + q2.y * Ap.y, q2.x * Bp.x + q2.y * Bp.y);
            }
            if (!va || k == M / 2) continue;   // k = M/2 is written by k = 0 (its pair)
            if (D0) {
                __builtin_nontemporal_store(Xk.x, a.out + gidx(uint32_t(ka)));
                __builtin_nontemporal_store(Xk.y, a.out + gidx(uint32_t(ka)) + uint32_t(M));
                __builtin_nontemporal_store(Xmk.x, a.out + gidx(uint32_t(kb)));
                __builtin_nontemporal_store(Xmk.y, a.out + gidx(uint32_t(kb)) + uint32_t(M));
            } else {
                stnt2(a.out + gidx(uint32_t(ka)), Xk);
                stnt2(a.out + gidx(uint32_t(kb)), Xmk);
            }
        }
    } else {
        // ---- DCT-III: coefficient pairs (k, M - k) -> the Makhoul spectrum in X -----------------------------
#pragma unroll
        for (int s = 0; s < (M / 2 + T) / T; ++s) {
            const int k = j + s * T;
            if (k >= M / 2) continue;   // k = 0 also writes slot M / 2
            const int ka = k, kb = k ? M - k : M / 2;
            double2 Xk = make_double2(0.0, 0.0), Xmk = make_double2(0.0, 0.0);
            if (va) {
                if (D0) {
                    Xk = make_double2(__builtin_nontemporal_load(a.in + gidx(uint32_t(ka))),
                                      __builtin_nontemporal_load(a.in + gidx(uint32_t(ka)) + uint32_t(M)));
                    Xmk = make_double2(__builtin_nontemporal_load(a.in + gidx(uint32_t(kb))),
                                       __builtin_nontemporal_load(a.in + gidx(uint32_t(kb)) + uint32_t(M)));
                } else {
                    Xk = ldnt2(a.in + gidx(uint32_t(ka)));
                    Xmk = ldnt2(a.in + gidx(uint32_t(kb)));
                }
            }
            const double2 q1 = cconj(a.twq[ka]), q2 = cconj(a.twq[kb]);
            if (k == 0) {
                const double2 va2 = cmul(q2, make_double2(Xmk.x, -Xmk.x));
                const double2 vb2 = cmul(q2, make_double2(Xmk.y, -Xmk.y));
                X[0] = Xk;
                X[M / 2] = make_double2(va2.x - vb2.y, va2.y + vb2.x);
            } else {
                const double2 va1 = cmul(q1, make_double2(Xk.x, -Xmk.x));
                const double2 vb1 = cmul(q1, make_double2(Xk.y, -Xmk.y));
                const double2 va2 = cmul(q2, make_double2(Xmk.x, -Xk.x));
                const double2 vb2 = cmul(q2, make_double2(Xmk.y, -Xk.y));
                X[ka] = make_double2(va1.x - vb1.y, va1.y + vb1.x);
                X[kb] = make_double2(va2.x - vb2.y, va2.y + vb2.x);
            }
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < V; ++i) z[i] = X[dctm_in_pos<M>(j, i)];
        dctm_stages<M, 0, 1, true>(z, j, X, tw);
        // ---- un-permute v[n] -> x[2n] (n < M/2), x[2(M-1-n)+1] -------------------------------------------
        if (D0) {
            __syncthreads();
#pragma unroll
            for (int i = 0; i < V; ++i) X[dctm_out_pos<M>(j, i)] = z[i];
            __syncthreads();
#pragma unroll
            for (int s = 0; s < M / 2 / T; ++s) {
                const int n = j + s * T;
                const double2 v0 = X[n], v1 = X[M - 1 - n];
                if (va) {
                    stnt2(a.out + lbase + uint32_t(2 * n), make_double2(v0.x, v1.x));
                    stnt2(a.out + lbase + uint32_t(M) + uint32_t(2 * n), make_double2(v0.y, v1.y));
                }
            }
        } else if (va) {
#pragma unroll
            for (int i = 0; i < V; ++i) {
                const int n = dctm_out_pos<M>(j, i);
                const uint32_t k = n < M / 2 ? uint32_t(2 * n) : uint32_t(2 * (M - 1 - n) + 1);
                stnt2(a.out + gidx(k), z[i]);
            }
        }
    }
}

// few lines (2-D meshes): halve a tile of tq lines, down to lo, while the grid has < 512 workgroups
static int few_lines_tq(uint32_t nlines, int tq, int lo) {
    while (tq > lo && (nlines + uint32_t(tq) - 1) / uint32_t(tq) < 512u) tq /= 2;
    return tq;
}

// k_dctm serves FWD / INV passes of m = 500 / 1000 lines; false: the caller takes k_dctg
static bool launch_dctm(SpecArgs& a, hipStream_t s, int mode, bool d0, bool formb) {
    const uint32_t m = a.m[a.d];
    // the first pass (b formed on load): k_dctm at 500 (V = 10: 0.89 against k_dctg's 1.09 ms at 500^3), k_dctg at
    // 1000 (V = 20: 31 against 29 us at 1000^2; profiles/r03/v19_dctm)
    if ((m != 500 && m != 1000) || mode == SPEC_MID || (formb && m != 500) || (a.nlines & 1u) ||
        probe_env("MVTV_DCTM_OFF"))
        return false;
    if (!d0 && (a.stride & 1u)) return false;   // line pairs must be adjacent words
    // 8-line tiles (500: 32 KB of LDS, up to five workgroups a CU against two with 16 lines; 1000: two against one):
    // 500^3 137.5 / 138.3 -> 141.6 / 142.4 ADMM it/s on one box, the first pass 0.93 -> 0.86 ms
    // (profiles/r05/v11_dctm_ncl4); few lines (1000 x 1000: 125 such tiles) one line pair per workgroup. Probe builds:
    // MVTV_DCTM_NCL=8 / 4 / 1 forces the tile
    static const int ncl_env = [] {
        const char* e = probe_env("MVTV_DCTM_NCL");
        return e ? std::atoi(e) : 0;
    }();
    static const bool few_off = probe_flag("MVTV_FEW_LINES_OFF");
    const int ncl = (ncl_env == 8 || ncl_env == 4 || ncl_env == 1)
                        ? ncl_env
                        : (few_off ? 4 : few_lines_tq(a.nlines, 8, 2) / 2);
#define MVTV_DCTM(MM, NC)                                                                                       \
    do {                                                                                                        \
        const dim3 grid((a.nlines + uint32_t(2 * NC) - 1) / uint32_t(2 * NC));                                 \
        const dim3 block(NC * dctm::Shape<MM>::T);                                                              \
        if (mode == SPEC_INV) {                                                                                 \
            if (d0) klaunch(k_dctm<MM, SPEC_INV, true, false, NC>, grid, block, 0, s, a);                       \
            else klaunch(k_dctm<MM, SPEC_INV, false, false, NC>, grid, block, 0, s, a);                         \
        } else if (d0) {                                                                                        \
            if (formb) klaunch(k_dctm<MM, SPEC_FWD, true, true, NC>, grid, block, 0, s, a);                     \
            else klaunch(k_dctm<MM, SPEC_FWD, true, false, NC>, grid, block, 0, s, a);                          \
        } else {                                                                                                \
            if (formb) klaunch(k_dctm<MM, SPEC_FWD, false, true, NC>, grid, block, 0, s, a);                    \
            else klaunch(k_dctm<MM, SPEC_FWD, false, false, NC>, grid, block, 0, s, a);                         \
        }                                                                                                       \
    } while (0)
    if (m == 500) {
        if (ncl == 8) MVTV_DCTM(500, 8);
        else if (ncl == 4) MVTV_DCTM(500, 4);
        else MVTV_DCTM(500, 1);
    } else {
        if (ncl == 8) MVTV_DCTM(1000, 8);
        else if (ncl == 4) MVTV_DCTM(1000, 4);
        else MVTV_DCTM(1000, 1);
    }
#undef MVTV_DCTM
    return true;
}

static void launch_dctg(SpecArgs& a, hipStream_t s, int mode, bool d0, bool formb) {
    const dim3 grid((a.nlines + uint32_t(a.tq) - 1) / uint32_t(a.tq)), block(dctg::NT);
    const size_t smem = size_t(a.tq / 2) * (a.m[a.d] + spec::PAD) * sizeof(double2);
    // (m = 4096 over a general stride: one complex line of 4097 slots is just above 64 KB)
#define MVTV_DCTG(MODE, D0, FB)                                                                               \
    do {                                                                                                       \
        if (smem > 65536)                                                                                      \
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_dctg<MODE, D0, FB>),                    \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, int(smem));                  \
        klaunch(k_dctg<MODE, D0, FB>, grid, block, uint32_t(smem), s, a);                                      \
    } while (0)
    if (mode == SPEC_FWD) {
        if (d0) {
            if (formb) MVTV_DCTG(SPEC_FWD, true, true);
            else MVTV_DCTG(SPEC_FWD, true, false);
        } else if (formb) {
            MVTV_DCTG(SPEC_FWD, false, true);
        } else {
            MVTV_DCTG(SPEC_FWD, false, false);
        }
    } else if (mode == SPEC_INV) {
        if (d0) MVTV_DCTG(SPEC_INV, true, false);
        else MVTV_DCTG(SPEC_INV, false, false);
    } else {
        if (d0) {
            if (formb) MVTV_DCTG(SPEC_MID, true, true);
            else MVTV_DCTG(SPEC_MID, true, false);
        } else {
            MVTV_DCTG(SPEC_MID, false, false);
        }
    }
#undef MVTV_DCTG
}

// radices of m = 2^a 3^b 5^c 7^d in stage order (8s first); false if m has another prime factor
bool dct_radix_plan(uint32_t m, int* rad, int* nrad) {
    int n = 0;
    for (const uint32_t r : {8u, 4u, 2u, 3u, 5u, 7u})
        while (m % r == 0 && m > 1) {
            if (n == 8) return false;
            rad[n++] = int(r);
            m /= r;
        }
    *nrad = n;
    return m == 1;
}

// =============================================================================================
// Any other length m <= 4096 (a prime factor >= 11: 31, 37, 79, 1009 ... the released R API's default mesh
// m = floor(sqrt(n)) per dimension, rcpp-code/MultivarTV/R/MultivarTV.R:44-48, lands on such lengths). The
// length-m complex DFT of the Makhoul pairing by Bluestein's chirp-z identity nk = (n^2 + k^2 - (k - n)^2) / 2:
//
//   Y[k] = c[k] sum_n (y[n] c[n]) b[k - n],   c[n] = e^{s i pi n^2 / m},  b[j] = conj c[j]   (s = -1 / +1)
//
// a linear convolution, evaluated as a circular one of length M = 2^ceil(log2(2m - 1)) with k_dct's radix-2^2
// LDS FFT (fft_lines): the chirped input goes in at bit-reversed slots, the forward FFT leaves natural order,
// the product with the transform of b (a per-dimension table, 1/M folded in) goes through the inverse FFT,
// which leaves the convolution at bit-reversed slots again. So every length-m quantity lives at slot
// brev_M(n): the Makhoul pairing (k, m - k), the MID divide and b formed on load are k_dctg's, read and
// written there. Per line pair: two length-M FFTs per transform (four in a MID pass); fp64 round-off grows
// as log M, like the planned FFTs'.
namespace dctb {
constexpr int NT = 256;   // spec::NT: fft_lines strides over the workgroup's threads
}

template <int MODE, bool D0, bool FORMB>
__global__ __launch_bounds__(dctb::NT) void k_dctb(const SpecArgs a) {
    double sigma = a.sigma, ca = a.ca, cb = a.cb;
    if (a.skip && *a.skip) return;
    if (a.ctl) {
        if (a.ctl->done) return;
        sigma = a.ctl->sigma;
        ca = a.ctl->rho;
        cb = a.ctl->rho * a.ctl->c_prev;
    }
    extern __shared__ double2 buf[];   // tq / 2 complex lines of M + PAD slots (launch-time size)
    __shared__ double lc0[16], lc1[16];
    const int m = int(a.m[a.d]);
    const int L = a.L, M = 1 << L;     // a.L = log2 M here
    const int tq = a.tq, ncl = tq >> 1, lncl = __ffs(ncl) - 1;
    const int LP = M + spec::PAD;
    const uint32_t q0 = (a.xrun ? xcd_run(blockIdx.x, gridDim.x) : blockIdx.x) * uint32_t(tq);
    const double2* __restrict__ chirp = a.bchirp;   // c[n] = e^{-i pi n^2 / m} (s = -1), n < m

    if (MODE == SPEC_MID && threadIdx.x < uint32_t(tq)) {   // c0 + c1 lam_d(k) per line, as k_dctg
        const uint32_t q = a.q_off + q0 + threadIdx.x;
        double lamv[kMaxDims] = {0, 0, 0, 0};
        uint32_t rest = (q - a.q_off) < a.nlines ? q : a.q_off;
        const int jlast = a.d == a.p - 1 ? a.p - 2 : a.p - 1;
        for (int j = 0; j < a.p; ++j) {
            if (j == a.d) continue;
            const uint32_t qq = (j < jlast) ? a.fd[j].div(rest) : 0u;
            lamv[j] = a.lam[a.lam_off[j] + (rest - qq * a.m[j])];
            rest = qq;
        }
        double c0 = a.w0, c1 = 0.0;
        for (int S = 1; S < (1 << a.p); ++S) {
            if (a.cS[S] == 0.0) continue;
            double prod = sigma * a.cS[S];
            for (int j = 0; j < a.p; ++j)
                if (j != a.d && ((S >> j) & 1)) prod *= lamv[j];
            if ((S >> a.d) & 1) c1 += prod;
            else c0 += prod;
        }
        lc0[threadIdx.x] = c0;
        lc1[threadIdx.x] = c1;
    }

    auto gaddr = [&](uint32_t ql, uint32_t k) -> uint32_t {
        const uint32_t q = q0 + ql;
        if (D0) return q * uint32_t(m) + k;
        const uint32_t hi = a.fds.div(q);
        return (q - hi * a.stride) + hi * a.stride * uint32_t(m) + k * a.stride;
    };
    auto slot = [&](int n) { return int(__brev(uint32_t(n)) >> (32 - L)); };
    // (complex line, sample k) of work item e: lanes over k for d = 0 (contiguous lines), over the line pairs for
    // a strided pass (the pair's two words are adjacent, the tile's pairs one row)
    auto item = [&](int e, int& cl, int& k) {
        if (D0) {
            cl = int(a.fm.div(uint32_t(e)));
            k = e - cl * m;
        } else {
            cl = e & (ncl - 1);
            k = e >> lncl;
        }
    };
    auto load_pair = [&](int cl, int k) -> double2 {
        double v[2] = {0.0, 0.0};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t ql = uint32_t(2 * cl + h);
            if (q0 + ql < a.nlines) {
                const uint32_t gi = gaddr(ql, uint32_t(k));
                v[h] = __builtin_nontemporal_load(a.in + gi);
                if (FORMB)
                    v[h] += ca * __builtin_nontemporal_load(a.ga + gi) + cb * __builtin_nontemporal_load(a.gb + gi);
            }
        }
        return make_double2(v[0], v[1]);
    };
    // zero the convolution's padding slots n in [m, M)
    auto zero_pad = [&]() {
        const int np = ncl * (M - m);
        for (int e = threadIdx.x; e < np; e += dctb::NT) {
            const int cl = e / (M - m), n = m + (e - cl * (M - m));
            buf[cl * LP + slot(n)] = make_double2(0.0, 0.0);
        }
    };
    // circular convolution of every line with b (bhat = its transform / M): bit-reversed in and out
    auto convolve = [&](const double2* __restrict__ bhat) {
        fft_lines<false, false>(buf, a.tw, ncl, L, LP);
        for (int e = threadIdx.x; e < ncl * M; e += dctb::NT) {
            const int cl = e >> L, k = e & (M - 1);
            buf[cl * LP + k] = cmul(buf[cl * LP + k], bhat[k]);
        }
        __syncthreads();
        fft_lines<true, true>(buf, a.tw, ncl, L, LP);
    };

    // ---- load: forward / MID: y[n] c[n] at slot(n), n = the Makhoul position of sample k; inverse: X[k] at slot(k)
    const int total = ncl * m;
    for (int e = threadIdx.x; e < total; e += dctb::NT) {
        int cl, k;
        item(e, cl, k);
        const double2 v = load_pair(cl, k);
        if (MODE == SPEC_INV) {
            buf[cl * LP + slot(k)] = v;
        } else {
            const int n = (k & 1) ? m - 1 - (k >> 1) : (k >> 1);
            buf[cl * LP + slot(n)] = cmul(v, chirp[n]);
        }
    }
    if (MODE != SPEC_INV) zero_pad();
    __syncthreads();
    if (MODE != SPEC_INV) convolve(a.bvf);

    // ---- spectrum <-> DCT coefficients over the pairs (k, m - k) (k_dctg), at their slots ------------------
    {
        const int half = m >> 1, npl = (m & 1) ? half + 1 : half;
        const int npairs = ncl * npl;
        for (int t = threadIdx.x; t < npairs; t += dctb::NT) {
            const int line = t / npl, k = t - line * npl;
            double2* x = buf + line * LP;
            const bool self = k == 0;
            const bool mid = self && !(m & 1);
            const int ka = k, kb = self ? half : m - k;
            const int sa = slot(ka), sb = slot(kb);
            double2 Xk, Xmk = make_double2(0.0, 0.0);
            if (MODE != SPEC_INV) {   // Z[k] = c[k] conv[k]
                const double2 Z1 = cmul(x[sa], chirp[ka]), q1 = a.twq[ka];
                if (self) {
                    Xk = make_double2(q1.x * Z1.x, q1.x * Z1.y);
                    if (mid) {
                        const double2 Z2 = cmul(x[sb], chirp[kb]), q2 = a.twq[kb];
                        Xmk = make_double2(q2.x * Z2.x, q2.x * Z2.y);
                    }
                } else {
                    const double2 Z2 = cmul(x[sb], chirp[kb]), q2 = a.twq[kb];
                    const double2 Ap = make_double2(0.5 * (Z1.x + Z2.x), 0.5 * (Z1.y - Z2.y));
                    const double2 Bp = make_double2(0.5 * (Z1.y + Z2.y), -0.5 * (Z1.x - Z2.x));
                    Xk = make_double2(q1.x * Ap.x - q1.y * Ap.y, q1.x * Bp.x - q1.y * Bp.y);
                    Xmk = make_double2(q2.x * Ap.x + q2.y * Ap.y, q2.x * Bp.x + q2.y * Bp.y);
                }
            } else {
                Xk = x[sa];
                if (!self || mid) Xmk = x[sb];
            }
            if (MODE == SPEC_MID) {
                const double* lamd = a.lam + a.lam_off[a.d];
                const int l0 = 2 * line, l1 = 2 * line + 1;
                const double la = lamd[ka];
                Xk.x *= a.inv_n / (lc0[l0] + lc1[l0] * la);
                Xk.y *= a.inv_n / (lc0[l1] + lc1[l1] * la);
                if (!self || mid) {
                    const double lb = lamd[kb];
                    Xmk.x *= a.inv_n / (lc0[l0] + lc1[l0] * lb);
                    Xmk.y *= a.inv_n / (lc0[l1] + lc1[l1] * lb);
                }
            }
            if (MODE == SPEC_FWD) {
                x[sa] = Xk;
                if (!self || mid) x[sb] = Xmk;
                continue;
            }
            // V[k] = conj(q[k]) (X[k] - i X[m-k]), then the inverse transform's input chirp conj c[k]
            const double2 q2 = cconj(a.twq[kb]);
            if (self) {
                x[sa] = cmul(Xk, cconj(chirp[0]));
                if (mid) {
                    const double2 va2 = cmul(q2, make_double2(Xmk.x, -Xmk.x));
                    const double2 vb2 = cmul(q2, make_double2(Xmk.y, -Xmk.y));
                    x[sb] = cmul(make_double2(va2.x - vb2.y, va2.y + vb2.x), cconj(chirp[kb]));
                }
            } else {
                const double2 q1 = cconj(a.twq[ka]);
                const double2 va1 = cmul(q1, make_double2(Xk.x, -Xmk.x));
                const double2 vb1 = cmul(q1, make_double2(Xk.y, -Xmk.y));
                const double2 va2 = cmul(q2, make_double2(Xmk.x, -Xk.x));
                const double2 vb2 = cmul(q2, make_double2(Xmk.y, -Xk.y));
                x[sa] = cmul(make_double2(va1.x - vb1.y, va1.y + vb1.x), cconj(chirp[ka]));
                x[sb] = cmul(make_double2(va2.x - vb2.y, va2.y + vb2.x), cconj(chirp[kb]));
            }
        }
        if (MODE != SPEC_FWD) zero_pad();   // (disjoint from the pairs' slots)
        __syncthreads();
    }

    if (MODE != SPEC_FWD) convolve(a.bvi);

    // ---- store: forward: X[k] from slot(k); inverse / MID: sample k = conj c[n] conv[n], n its Makhoul position
    for (int e = threadIdx.x; e < total; e += dctb::NT) {
        int cl, k;
        item(e, cl, k);
        double2 v;
        if (MODE == SPEC_FWD) {
            v = buf[cl * LP + slot(k)];
        } else {
            const int n = (k & 1) ? m - 1 - (k >> 1) : (k >> 1);
            v = cmul(buf[cl * LP + slot(n)], cconj(chirp[n]));
        }
        const uint32_t ql = uint32_t(2 * cl);
        if (q0 + ql < a.nlines) __builtin_nontemporal_store(v.x, a.out + gaddr(ql, uint32_t(k)));
        if (q0 + ql + 1 < a.nlines) __builtin_nontemporal_store(v.y, a.out + gaddr(ql + 1, uint32_t(k)));
    }
}

// k_dctb8: the same Bluestein passes with k_dct8's register-resident radix-8 Stockham stages (stages_from) for the
// length-M FFTs: a thread holds 8 complex values of one complex line (two real lines), LDS carries only the exchanges
// between stages, both FFTs of a convolution leave natural order. The LDS-staged k_dctb spends ~20x the HBM bytes in
// LDS traffic (every radix-2^2 stage a round trip through LDS for two length-M FFTs per transform) and runs at ~0.9 TB/s
// (251^3); this keeps the working set of a stage in registers.
template <int L, int MODE, bool D0, bool FORMB, int TQW>
__global__ __launch_bounds__((spec8::ShapeK<L, TQW>::NT)) void k_dctb8(const SpecArgs a) {
    using S = spec8::ShapeK<L, TQW>;
    constexpr int M = S::M, TPL = S::TPL, NCL = S::NCL, R0 = S::R0;
    double sigma = a.sigma, ca = a.ca, cb = a.cb;
    if (a.skip && *a.skip) return;
    if (a.ctl) {
        if (a.ctl->done) return;
        sigma = a.ctl->sigma;
        ca = a.ctl->rho;
        cb = a.ctl->rho * a.ctl->c_prev;
    }
    __shared__ double2 buf[NCL * S::LP];
    __shared__ double lc0[2 * NCL], lc1[2 * NCL];
    const int m = int(a.m[a.d]);
    const int t = threadIdx.x;
    const int j = D0 ? (t % TPL) : (t / NCL);
    const int c = D0 ? (t / TPL) : (t % NCL);
    const uint32_t q0 = (a.xrun ? xcd_run(blockIdx.x, gridDim.x) : blockIdx.x) * uint32_t(TQW);
    const int la = 2 * c, lb = 2 * c + 1;
    const bool va = q0 + uint32_t(la) < a.nlines, vb = q0 + uint32_t(lb) < a.nlines;
    double2* const X = buf + c * S::LP;
    const int cx = c & 7;
    const double2* __restrict__ tw = a.tw;       // length-M twiddles
    const double2* __restrict__ chirp = a.bchirp;

    for (int l = t; MODE == SPEC_MID && l < TQW; l += S::NT) {   // c0 + c1 lam_d(k) per line (k_dct8)
        const uint32_t q = a.q_off + q0 + l;
        double lamv[kMaxDims] = {0, 0, 0, 0};
        uint32_t rest = (q - a.q_off) < a.nlines ? q : a.q_off;
        const int jlast = a.d == a.p - 1 ? a.p - 2 : a.p - 1;
        for (int jj = 0; jj < a.p; ++jj) {
            if (jj == a.d) continue;
            const uint32_t qq = (jj < jlast) ? a.fd[jj].div(rest) : 0u;
            lamv[jj] = a.lam[a.lam_off[jj] + (rest - qq * a.m[jj])];
            rest = qq;
        }
        double c0 = a.w0, c1 = 0.0;
        for (int Sm = 1; Sm < (1 << a.p); ++Sm) {
            if (a.cS[Sm] == 0.0) continue;
            double prod = sigma * a.cS[Sm];
            for (int jj = 0; jj < a.p; ++jj)
                if (jj != a.d && ((Sm >> jj) & 1)) prod *= lamv[jj];
            if ((Sm >> a.d) & 1) c1 += prod;
            else c0 += prod;
        }
        lc0[l] = c0;
        lc1[l] = c1;
    }

    auto gaddr = [&](int ql, uint32_t k) -> uint32_t {
        const uint32_t q = q0 + uint32_t(ql);
        if (D0) return q * uint32_t(m) + k;
        const uint32_t hi = a.fds.div(q);
        return (q - hi * a.stride) + hi * a.stride * uint32_t(m) + k * a.stride;
    };
    auto ld1 = [&](int ql, uint32_t k) -> double {
        const uint32_t gi = gaddr(ql, k);
        double v = __builtin_nontemporal_load(a.in + gi);
        if (FORMB) v += ca * __builtin_nontemporal_load(a.ga + gi) + cb * __builtin_nontemporal_load(a.gb + gi);
        return v;
    };
    auto ld2 = [&](uint32_t k) {
        return make_double2(va ? ld1(la, k) : 0.0, vb ? ld1(lb, k) : 0.0);
    };
    auto st2 = [&](uint32_t k, double2 v) {
        if (va) __builtin_nontemporal_store(v.x, a.out + gaddr(la, k));
        if (vb) __builtin_nontemporal_store(v.y, a.out + gaddr(lb, k));
    };
    // circular convolution with b (bhat = its transform / M) of u (u_at(n), n < M): natural order in X
    auto convolve = [&](auto&& u_at, const double2* __restrict__ bhat) {
        double2 z[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) z[i] = u_at(stage_in_pos<L, R0>(j, i));
        stages_from<L, R0, 1, false, false>(z, j, X, cx, tw);   // DFT, natural order in X
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int n = stage_in_pos<L, R0>(j, i);
            z[i] = cmul(X[spec8::slot(n, cx)], bhat[n]);
        }
        stages_from<L, R0, 1, true, false>(z, j, X, cx, tw);    // inverse DFT, natural order in X
    };
    const int half = m >> 1, npl = (m & 1) ? half + 1 : half;
    // the inverse transform's input: V[k] conj c[k] at k < m (pairs (k, m - k)), zeros at [m, M)
    auto put_v = [&](int k, double2 Xk, double2 Xmk) {
        const bool self = k == 0, mid = self && !(m & 1);
        const int ka = k, kb = self ? half : m - k;
        const double2 q2 = cconj(a.twq[kb]);
        if (self) {
            X[spec8::slot(0, cx)] = cmul(Xk, cconj(chirp[0]));
            if (mid) {
                const double2 va2 = cmul(q2, make_double2(Xmk.x, -Xmk.x));
                const double2 vb2 = cmul(q2, make_double2(Xmk.y, -Xmk.y));
                X[spec8::slot(kb, cx)] = cmul(make_double2(va2.x - vb2.y, va2.y + vb2.x), cconj(chirp[kb]));
            }
        } else {
            const double2 q1 = cconj(a.twq[ka]);
            const double2 va1 = cmul(q1, make_double2(Xk.x, -Xmk.x));
            const double2 vb1 = cmul(q1, make_double2(Xk.y, -Xmk.y));
            const double2 va2 = cmul(q2, make_double2(Xmk.x, -Xk.x));
            const double2 vb2 = cmul(q2, make_double2(Xmk.y, -Xk.y));
            X[spec8::slot(ka, cx)] = cmul(make_double2(va1.x - vb1.y, va1.y + vb1.x), cconj(chirp[ka]));
            X[spec8::slot(kb, cx)] = cmul(make_double2(va2.x - vb2.y, va2.y + vb2.x), cconj(chirp[kb]));
        }
    };
    auto zero_pad = [&]() {
        for (int n = m + j; n < M; n += TPL) X[spec8::slot(n, cx)] = make_double2(0.0, 0.0);
    };

    if (MODE != SPEC_INV) {
        // forward: u[n] = y[n] c[n], y the Makhoul sequence of the two lines (sample k(n))
        convolve(
            [&](int n) {
                if (n >= m) return make_double2(0.0, 0.0);
                const int k = 2 * n < m ? 2 * n : 2 * (m - 1 - n) + 1;
                return cmul(ld2(uint32_t(k)), chirp[n]);
            },
            a.bvf);
        for (int k = j; k < npl; k += TPL) {   // Z[k] = c[k] conv[k] -> DCT-II coefficients of the pair (k, m - k)
            const bool self = k == 0, mid = self && !(m & 1);
            const int ka = k, kb = self ? half : m - k;
            const double2 Z1 = cmul(X[spec8::slot(ka, cx)], chirp[ka]), q1 = a.twq[ka];
            double2 Xk, Xmk = make_double2(0.0, 0.0);
            if (self) {
                Xk = make_double2(q1.x * Z1.x, q1.x * Z1.y);
                if (mid) {
                    const double2 Z2 = cmul(X[spec8::slot(kb, cx)], chirp[kb]), q2 = a.twq[kb];
                    Xmk = make_double2(q2.x * Z2.x, q2.x * Z2.y);
                }
            } else {
                const double2 Z2 = cmul(X[spec8::slot(kb, cx)], chirp[kb]), q2 = a.twq[kb];
                const double2 Ap = make_double2(0.5 * (Z1.x + Z2.x), 0.5 * (Z1.y - Z2.y));
                const double2 Bp = make_double2(0.5 * (Z1.y + Z2.y), -0.5 * (Z1.x - Z2.x));
                Xk = make_double2(q1.x * Ap.x - q1.y * Ap.y, q1.x * Bp.x - q1.y * Bp.y);
                Xmk = make_double2(q2.x * Ap.x + q2.y * Ap.y, q2.x * Bp.x + q2.y * Bp.y);
            }
            if (MODE == SPEC_FWD) {
                st2(uint32_t(ka), Xk);
                if (!self || mid) st2(uint32_t(kb), Xmk);
                continue;
            }
            const double* lamd = a.lam + a.lam_off[a.d];
            const double l1 = lamd[ka];
            Xk.x *= a.inv_n / (lc0[la] + lc1[la] * l1);
            Xk.y *= a.inv_n / (lc0[lb] + lc1[lb] * l1);
            if (!self || mid) {
                const double l2 = lamd[kb];
                Xmk.x *= a.inv_n / (lc0[la] + lc1[la] * l2);
                Xmk.y *= a.inv_n / (lc0[lb] + lc1[lb] * l2);
            }
            put_v(k, Xk, Xmk);
        }
        if (MODE == SPEC_FWD) return;
    } else {
        for (int k = j; k < npl; k += TPL) {   // coefficients (k, m - k) from HBM
            const bool self = k == 0, mid = self && !(m & 1);
            const double2 Xk = ld2(uint32_t(k));
            const double2 Xmk = (!self || mid) ? ld2(uint32_t(self ? half : m - k)) : make_double2(0.0, 0.0);
            put_v(k, Xk, Xmk);
        }
    }
    zero_pad();
    __syncthreads();
    convolve([&](int n) { return X[spec8::slot(n, cx)]; }, a.bvi);
    for (int k = j; k < m; k += TPL) {   // sample k = conj c[n] conv[n], n its Makhoul position
        const int n = (k & 1) ? m - 1 - (k >> 1) : (k >> 1);
        st2(uint32_t(k), cmul(X[spec8::slot(n, cx)], cconj(chirp[n])));
    }
}

// k_dctb8's tile: k_dct8's default real lines per workgroup (16, fewer for M > 512), at least one wave of threads
template <int L>
constexpr int dctb8_tq() {
    constexpr int TQ = spec8::Shape<L>::TQ, TPL = spec8::Shape<L>::TPL;
    return TQ < 2 ? 2 : ((TQ / 2) * TPL >= 64 ? TQ : 2 * (64 / TPL));
}

template <int L, int TQW>
static void launch_dctb8_t(SpecArgs& a, hipStream_t s, int mode, bool d0, bool formb) {
    const dim3 grid((a.nlines + uint32_t(TQW) - 1) / uint32_t(TQW)), block(spec8::ShapeK<L, TQW>::NT);
#define MVTV_DCTB8(MODE, D0, FB) klaunch(k_dctb8<L, MODE, D0, FB, TQW>, grid, block, 0, s, a)
    if (mode == SPEC_FWD) {
        if (d0) {
            if (formb) MVTV_DCTB8(SPEC_FWD, true, true);
            else MVTV_DCTB8(SPEC_FWD, true, false);
        } else if (formb) {
            MVTV_DCTB8(SPEC_FWD, false, true);
        } else {
            MVTV_DCTB8(SPEC_FWD, false, false);
        }
    } else if (mode == SPEC_INV) {
        if (d0) MVTV_DCTB8(SPEC_INV, true, false);
        else MVTV_DCTB8(SPEC_INV, false, false);
    } else {
        if (d0) {
            if (formb) MVTV_DCTB8(SPEC_MID, true, true);
            else MVTV_DCTB8(SPEC_MID, true, false);
        } else if (formb) {
            MVTV_DCTB8(SPEC_MID, false, true);
        } else {
            MVTV_DCTB8(SPEC_MID, false, false);
        }
    }
#undef MVTV_DCTB8
}

// few lines (a 2-D mesh: 251 lines of 251): one line pair per workgroup where that is >= one wave of threads
// (M >= 512), the default tile is >= 8 lines (M <= 1024) and leaves < 512 workgroups: 251^2 12851 / 12874 -> 16902 /
// 16751 ADMM it/s; at M = 2048 (1009^2: 253 workgroups of 4 lines) one pair was slower, 8356 -> 8061
// (profiles/r05/v14_few_lines_bluestein; probe builds: MVTV_FEW_LINES_OFF=1)
template <int L>
static void launch_dctb8_l(SpecArgs& a, hipStream_t s, int mode, bool d0, bool formb) {
    constexpr int TQW = dctb8_tq<L>();
    static const bool few_off = probe_flag("MVTV_FEW_LINES_OFF");
    if constexpr (L >= 9 && L <= 10 && TQW > 2) {
        if (!few_off && (a.nlines + uint32_t(TQW) - 1) / uint32_t(TQW) < 512u)
            return launch_dctb8_t<L, 2>(a, s, mode, d0, formb);
    }
    launch_dctb8_t<L, TQW>(a, s, mode, d0, formb);
}

static hipError_t launch_dctb(SpecArgs& a, hipStream_t s, int mode, bool d0, bool formb) {
    const int M = 1 << a.L;
    if (!probe_env("MVTV_DCTB_LDS")) {   // the register-stage form (probe builds: MVTV_DCTB_LDS=1 keeps k_dctb)
        switch (a.L) {
            case 5: launch_dctb8_l<5>(a, s, mode, d0, formb); return hipGetLastError();
            case 6: launch_dctb8_l<6>(a, s, mode, d0, formb); return hipGetLastError();
            case 7: launch_dctb8_l<7>(a, s, mode, d0, formb); return hipGetLastError();
            case 8: launch_dctb8_l<8>(a, s, mode, d0, formb); return hipGetLastError();
            case 9: launch_dctb8_l<9>(a, s, mode, d0, formb); return hipGetLastError();
            case 10: launch_dctb8_l<10>(a, s, mode, d0, formb); return hipGetLastError();
            case 11: launch_dctb8_l<11>(a, s, mode, d0, formb); return hipGetLastError();
            case 12: launch_dctb8_l<12>(a, s, mode, d0, formb); return hipGetLastError();
            case 13: launch_dctb8_l<13>(a, s, mode, d0, formb); return hipGetLastError();
            default: break;
        }
    }
    // <= 16 lines in <= 64 KB of LDS (two complex lines' worth at least); M = 8192 takes one line pair in 128 KB
    int tq = 16;
    while (tq > 2 && size_t(tq / 2) * size_t(M + spec::PAD) * sizeof(double2) > 65536) tq /= 2;
    a.tq = tq;
    const size_t smem = size_t(tq / 2) * size_t(M + spec::PAD) * sizeof(double2);
    if (smem > 160 * 1024) return hipErrorInvalidValue;
    const dim3 grid((a.nlines + uint32_t(tq) - 1) / uint32_t(tq)), block(dctb::NT);
#define MVTV_DCTB(MODE, D0, FB)                                                                               \
    do {                                                                                                       \
        if (smem > 65536)                                                                                      \
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_dctb<MODE, D0, FB>),                    \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, int(smem));                  \
        klaunch(k_dctb<MODE, D0, FB>, grid, block, uint32_t(smem), s, a);                                      \
    } while (0)
    if (mode == SPEC_FWD) {
        if (d0) {
            if (formb) MVTV_DCTB(SPEC_FWD, true, true);
            else MVTV_DCTB(SPEC_FWD, true, false);
        } else if (formb) {
            MVTV_DCTB(SPEC_FWD, false, true);
        } else {
            MVTV_DCTB(SPEC_FWD, false, false);
        }
    } else if (mode == SPEC_INV) {
        if (d0) MVTV_DCTB(SPEC_INV, true, false);
        else MVTV_DCTB(SPEC_INV, false, false);
    } else {
        if (d0) {
            if (formb) MVTV_DCTB(SPEC_MID, true, true);
            else MVTV_DCTB(SPEC_MID, true, false);
        } else if (formb) {
            MVTV_DCTB(SPEC_MID, false, true);
        } else {
            MVTV_DCTB(SPEC_MID, false, false);
        }
    }
#undef MVTV_DCTB
    return hipGetLastError();
}

// =============================================================================================
// Last dimension by a tridiagonal solve instead of DCT / divide / inverse DCT.
//
// After the forward transforms along dims 0..p-2, line q of the last dimension d carries the 1-D
// operator c0(q) I + c1(q) T, T = D1^T D1 = tridiag(-1, [1, 2, ..., 2, 1], -1) (the Neumann
// Laplacian the DCT along d would diagonalise: mu = c0 + c1 lam_d(k)). Solving it directly costs
// ~6 flops per element against two length-m FFTs, a divide and the DCT pre/post twiddles, with the
// same 2N words of HBM traffic; the pass stops being VALU/latency bound.
//
// Partitioned Thomas: a thread owns SEG consecutive rows of one line and eliminates them with the
// left / right neighbours x[lo-1] = L, x[hi+1] = R kept symbolic: x_i = G_i + H_i L + K_i R. The
// line's Toeplitz interior makes 1/den_i, e_i, H_i, K_i the same for every segment (line constants,
// built once per workgroup in LDS); the Neumann ends are the mirror conditions x[-1] = x[0],
// x[m] = x[m-1]. One thread per line then solves the 2 x NSEG interface system (u_j = x at a
// segment's first row, v_j at its last) by block elimination, and every thread finishes its rows.
// The result is the exact solve (the system is strictly diagonally dominant: c0 > 0, c1 >= 0),
// scaled by inv_n * m_d (the normalisation of the transforms along the other dims).
namespace tri {
constexpr int TQ = 16;    // lines per workgroup: one 128-B row per position (d > 0)
template <int L, int SEG, int TQL = TQ>
struct Shape {
    static constexpr int M = 1 << L;
    static constexpr int NSEG = M / SEG;   // segments (threads) per line
    static constexpr int NT = TQL * NSEG;
};
}  // namespace tri

// TQL lines per workgroup: 16 (128-B rows) by default; 2-D meshes with few lines take 4 or 8 with the
// tiles dealt to the XCDs in contiguous runs (a.xcd), as k_dct8's strided passes
template <int L, int SEG, int TQL = tri::TQ>
__global__ __launch_bounds__((tri::Shape<L, SEG, TQL>::NT)) void k_tri(const SpecArgs a) {
    using S = tri::Shape<L, SEG, TQL>;
    constexpr int TQ = TQL, NSEG = S::NSEG;
    double sigma = a.sigma;
    if (a.skip && *a.skip) return;
    if (a.ctl) {
        if (a.ctl->done) return;
        sigma = a.ctl->sigma;
    }
    __shared__ double t_id[SEG][TQ], t_e[SEG][TQ], t_h[SEG][TQ], t_k[SEG][TQ];   // line constants
    __shared__ double s_a[TQ];                                                    // -c1 per line
    __shared__ double s_u[NSEG][TQ], s_v[NSEG][TQ], s_bu[NSEG][TQ], s_bv[NSEG][TQ];
    const int t = threadIdx.x, c = t % TQ, sj = t / TQ;
    const uint32_t bx = a.xcd ? (blockIdx.x & 7u) * (gridDim.x >> 3) + (blockIdx.x >> 3) : blockIdx.x;
    const uint32_t q0 = bx * uint32_t(TQ);
    const uint32_t q = q0 + uint32_t(c);
    const bool valid = q < a.nlines;
    const uint32_t base = (q & (a.stride - 1)) + ((q >> a.ls) << (a.ls + L)) + (uint32_t(sj * SEG) << a.ls);

    // the line's eigenvalue loads are issued before the rows, so the line constants below wait for them
    // alone (loads complete in order: issued after the rows, they would wait for all SEG row loads)
    double lamv[kMaxDims] = {0, 0, 0, 0};
    if (t < TQ) {
        // c0 + c1 T along d for this line (q indexes dims 0..p-2 column-major, as k_dct8's MID)
        const uint32_t ql = a.q_off + (valid ? q : q0);
        uint32_t rest = ql;
        const int jlast = a.d == a.p - 1 ? a.p - 2 : a.p - 1;
        for (int jj = 0; jj < a.p; ++jj) {
            if (jj == a.d) continue;
            const uint32_t qq = (jj < jlast) ? a.fd[jj].div(rest) : 0u;
            lamv[jj] = a.lam[a.lam_off[jj] + (rest - qq * a.m[jj])];
            rest = qq;
        }
    }
    double g[SEG];
#pragma unroll
    for (int i = 0; i < SEG; ++i) g[i] = valid ? __builtin_nontemporal_load(a.in + base + (uint32_t(i) << a.ls)) : 0.0;

    if (t < TQ) {
        double c0 = a.w0, c1 = 0.0;
        for (int Sm = 1; Sm < (1 << a.p); ++Sm) {
            if (a.cS[Sm] == 0.0) continue;
            double prod = sigma * a.cS[Sm];
            for (int jj = 0; jj < a.p; ++jj)
                if (jj != a.d && ((Sm >> jj) & 1)) prod *= lamv[jj];
            if ((Sm >> a.d) & 1) c1 += prod;
            else c0 += prod;
        }
        // Thomas on one interior segment: den_i = B - A e_{i-1}, e_i = A / den_i, h_i = -A h_{i-1} / den_i
        const double A = -c1, B = c0 + 2.0 * c1;
        double e = 0.0, h = 1.0;
#pragma unroll 1
        for (int i = 0; i < SEG; ++i) {
            const double id = 1.0 / (B - A * e);
            e = A * id;
            h = -A * h * id;
            t_id[i][c] = id;
            t_e[i][c] = e;
            t_h[i][c] = h;
        }
        // back substitution of the L / R responses: H_i = h_i - e_i H_{i+1}, K_i = -e_i K_{i+1}
        double H = t_h[SEG - 1][c], K = -t_e[SEG - 1][c];
        t_k[SEG - 1][c] = K;
#pragma unroll 1
        for (int i = SEG - 2; i >= 0; --i) {
            const double ei = t_e[i][c];
            H = t_h[i][c] - ei * H;
            K = -ei * K;
            t_h[i][c] = H;
            t_k[i][c] = K;
        }
        s_a[c] = A;
    }
    __syncthreads();

    // this segment with L = R = 0: forward elimination, then back substitution
    {
        const double A = s_a[c];
        g[0] *= t_id[0][c];
#pragma unroll
        for (int i = 1; i < SEG; ++i) g[i] = (g[i] - A * g[i - 1]) * t_id[i][c];
#pragma unroll
        for (int i = SEG - 2; i >= 0; --i) g[i] -= t_e[i][c] * g[i + 1];
        s_u[sj][c] = g[0];
        s_v[sj][c] = g[SEG - 1];
    }
    __syncthreads();

    if (t < TQ) {
        // interface system: u_j = G0_j + H0 L_j + K0 R_j, v_j = G1_j + H1 L_j + K1 R_j with
        // L_j = v_{j-1} (L_0 = u_0), R_j = u_{j+1} (R_last = v_last). Eliminate forward to
        // z_j = (au, av) + (bu, bv) u_{j+1}, solve the last 2 x 2 block, substitute back.
        const double H0 = t_h[0][c], K0 = t_k[0][c], H1 = t_h[SEG - 1][c], K1 = t_k[SEG - 1][c];
        double av = 0.0, bv = 0.0;   // v_{j-1} = av + bv u_j
#pragma unroll 1
        for (int j = 0; j < NSEG - 1; ++j) {
            const double g0 = s_u[j][c], g1 = s_v[j][c];
            double au, bu;
            if (j == 0) {
                const double id = 1.0 / (1.0 - H0);
                au = g0 * id;
                bu = K0 * id;
                av = g1 + H1 * au;
                bv = K1 + H1 * bu;
            } else {
                const double id = 1.0 / (1.0 - H0 * bv);
                au = (g0 + H0 * av) * id;
                bu = K0 * id;
                const double nav = g1 + H1 * av + H1 * bv * au;
                bv = K1 + H1 * bv * bu;
                av = nav;
            }
            s_u[j][c] = au;
            s_bu[j][c] = bu;
            s_v[j][c] = av;
            s_bv[j][c] = bv;
        }
        constexpr int J = NSEG - 1;
        const double a11 = 1.0 - H0 * bv, a12 = -K0, a21 = -H1 * bv, a22 = 1.0 - K1;
        const double b1 = s_u[J][c] + H0 * av, b2 = s_v[J][c] + H1 * av;
        const double idet = 1.0 / (a11 * a22 - a12 * a21);
        double u = (b1 * a22 - a12 * b2) * idet;
        s_u[J][c] = u;
        s_v[J][c] = (a11 * b2 - a21 * b1) * idet;
#pragma unroll 1
        for (int j = J - 1; j >= 0; --j) {
            const double un = u;
            u = s_u[j][c] + s_bu[j][c] * un;
            s_v[j][c] = s_v[j][c] + s_bv[j][c] * un;
            s_u[j][c] = u;
        }
    }
    __syncthreads();

    const double Lj = sj == 0 ? s_u[0][c] : s_v[sj - 1][c];
    const double Rj = sj == NSEG - 1 ? s_v[NSEG - 1][c] : s_u[sj + 1][c];
    const double sc = a.inv_n * double(S::M);
    if (!valid) return;
#pragma unroll
    for (int i = 0; i < SEG; ++i)
        __builtin_nontemporal_store(sc * (g[i] + t_h[i][c] * Lj + t_k[i][c] * Rj), a.out + base + (uint32_t(i) << a.ls));
}

// ---------------------------------------------------------------------------------------------
// k_trir: the same line solves by the factorised operator (round 6). c0 I + c1 T is, away from the ends,
// -c1 x[i-1] + (c0 + 2 c1) x[i] - c1 x[i+1] = kappa (1 - r S+)(1 - r S-) with r the root in (0, 1) of
// c1 r^2 - (c0 + 2 c1) r + c1 = 0; its Green's function is r^|k| / D with D = sqrt(c0 (c0 + 4 c1)). The
// Neumann ends are the mirror conditions, so the line's solve is the bi-infinite one on the even extension of
// the data: x_i = (F_i + B_i - f_i) / D with the two first-order recursions
//     F_i = f_i + r F_{i-1} (forward),      B_i = f_i + r B_{i+1} (backward),
// closed by the mirror: F_{-1} = B_0 and B_m = F_{m-1} (a 2 x 2 system with determinant 1 - r^2m).
// Segment-parallel: a thread runs both recursions over its SEG rows from zero (two independent chains),
// one thread per line combines the segments' sums into every segment's carries (F into its first row, B into
// its last) and closes the mirror, and every thread reruns the recursions with its carries. No divide per row,
// no per-row line constants (k_tri keeps four [SEG][TQ] tables in ~97 KB of LDS, so one workgroup fits a CU,
// and eliminates the interface on one wave with a divide per step); LDS here is 2 sums per segment and five
// constants per line. r = 2 c1 / (c0 + 2 c1 + D) and 1 - r = (c0 + D) / (c0 + 2 c1 + D) are cancellation-free;
// 1 - r^k by t_2k = t_k (2 - t_k). Against a long-double Thomas solve (numpy transcription): 1e-15 at
// c1 / c0 = 1e2, 3e-14 at 1e7 relative (an LU solve of the same system: 2e-11 at 1e7).
namespace trir {
template <int L, int SEG, int TQL>
struct Shape {
    static constexpr int M = 1 << L;
    static constexpr int NSEG = M / SEG;
    static constexpr int NT = TQL * NSEG;
};
}  // namespace trir

template <int L, int SEG, int TQL>
__global__ __launch_bounds__((trir::Shape<L, SEG, TQL>::NT), (SEG <= 16 ? 8 : 4)) void k_trir(const SpecArgs a) {
    using S = trir::Shape<L, SEG, TQL>;
    constexpr int TQ = TQL, NSEG = S::NSEG;
    double sigma = a.sigma;
    if (a.skip && *a.skip) return;
    if (a.ctl) {
        if (a.ctl->done) return;
        sigma = a.ctl->sigma;
    }
    __shared__ double s_f[NSEG][TQ], s_b[NSEG][TQ];   // segment sums from zero, then the segments' carries
    __shared__ double s_r[TQ], s_sd[TQ];               // r, scale / D per line
    const int t = threadIdx.x, c = t % TQ, sj = t / TQ;
    const uint32_t bx = a.xcd ? (blockIdx.x & 7u) * (gridDim.x >> 3) + (blockIdx.x >> 3) : blockIdx.x;
    const uint32_t q0 = bx * uint32_t(TQ);
    const uint32_t q = q0 + uint32_t(c);
    const bool valid = q < a.nlines;
    const uint32_t base = (q & (a.stride - 1)) + ((q >> a.ls) << (a.ls + L)) + (uint32_t(sj * SEG) << a.ls);

    double lamv[kMaxDims] = {0, 0, 0, 0};
    if (t < TQ) {
        const uint32_t ql = a.q_off + (valid ? q : q0);
        uint32_t rest = ql;
        const int jlast = a.d == a.p - 1 ? a.p - 2 : a.p - 1;
        for (int jj = 0; jj < a.p; ++jj) {
            if (jj == a.d) continue;
            const uint32_t qq = (jj < jlast) ? a.fd[jj].div(rest) : 0u;
            lamv[jj] = a.lam[a.lam_off[jj] + (rest - qq * a.m[jj])];
            rest = qq;
        }
    }
    double g[SEG];
#pragma unroll
    for (int i = 0; i < SEG; ++i) g[i] = valid ? __builtin_nontemporal_load(a.in + base + (uint32_t(i) << a.ls)) : 0.0;

    double rm = 0.0, idet = 1.0, rseg = 0.0;   // t < TQ: r^m, 1 / (1 - r^2m), r^SEG
    if (t < TQ) {
        double c0 = a.w0, c1 = 0.0;
        for (int Sm = 1; Sm < (1 << a.p); ++Sm) {
            if (a.cS[Sm] == 0.0) continue;
            double prod = sigma * a.cS[Sm];
            for (int jj = 0; jj < a.p; ++jj)
                if (jj != a.d && ((Sm >> jj) & 1)) prod *= lamv[jj];
            if ((Sm >> a.d) & 1) c1 += prod;
            else c0 += prod;
        }
        const double D = sqrt(c0 * (c0 + 4.0 * c1));
        const double den = 1.0 / (c0 + 2.0 * c1 + D);
        const double r = 2.0 * c1 * den;
        double pk = r, tk = (c0 + D) * den;   // r^k, 1 - r^k at k = 1
#pragma unroll
        for (int k = 1; k < SEG; k <<= 1) {
            pk *= pk;
            tk *= 2.0 - tk;
        }
        rseg = pk;
#pragma unroll
        for (int k = SEG; k < S::M; k <<= 1) {
            pk *= pk;
            tk *= 2.0 - tk;
        }
        rm = pk;
        idet = 1.0 / (tk * (2.0 - tk));   // 1 / (1 - r^2m)
        s_r[c] = r;
        s_sd[c] = a.inv_n * double(S::M) / D;
    }
    __syncthreads();

    const double r = s_r[c];
    {
        // both recursions over this segment from zero: two independent chains
        double fl = 0.0, bl = 0.0;
#pragma unroll
        for (int i = 0; i < SEG; ++i) {
            fl = fma(r, fl, g[i]);
            bl = fma(r, bl, g[SEG - 1 - i]);
        }
        s_f[sj][c] = fl;
        s_b[sj][c] = bl;
    }
    __syncthreads();

    if (t < TQ) {
        // carries: F into segment j's first row = sum_{k<j} r^{SEG(j-1-k)} fl_k + r^{SEG j} F_{-1}, B likewise from
        // the right; F_{-1} = B_0 and B_m = F_{m-1} close the mirror
        double acc = 0.0, bcc = 0.0;
#pragma unroll 8
        for (int k = 0; k < NSEG; ++k) {
            const double fk = s_f[k][c], bk = s_b[NSEG - 1 - k][c];
            s_f[k][c] = acc;
            s_b[NSEG - 1 - k][c] = bcc;
            acc = fma(acc, rseg, fk);
            bcc = fma(bcc, rseg, bk);
        }
        const double fm1 = (bcc + rm * acc) * idet, bm = (acc + rm * bcc) * idet;
        double pw = 1.0;
#pragma unroll 8
        for (int k = 0; k < NSEG; ++k) {
            s_f[k][c] = fma(pw, fm1, s_f[k][c]);
            s_b[NSEG - 1 - k][c] = fma(pw, bm, s_b[NSEG - 1 - k][c]);
            pw *= rseg;
        }
    }
    __syncthreads();

    if (!valid) return;
    const double sd = s_sd[c], bin = s_b[sj][c];
    double fv = s_f[sj][c];
    // g <- B (backward with the carry), then x_i = (B_i + r F_{i-1}) / D, F_i = B_i + r (F_{i-1} - B_{i+1})
    {
        double bv = bin;
#pragma unroll
        for (int i = SEG - 1; i >= 0; --i) {
            bv = fma(r, bv, g[i]);
            g[i] = bv;
        }
    }
#pragma unroll
    for (int i = 0; i < SEG; ++i) {
        const double gn = i + 1 < SEG ? g[i + 1] : bin;
        __builtin_nontemporal_store(sd * fma(r, fv, g[i]), a.out + base + (uint32_t(i) << a.ls));
        fv = fma(r, fv - gn, g[i]);
    }
}

// k_trig: the same solve for any line length m = (NSEG - 1) * s + sr (segment length s <= SMAX chosen at launch,
// NSEG <= NS, the last segment sr <= s rows) and any line stride (FastDiv addressing): the last-dimension pass of
// the mixed-radix and prime-length meshes. Rows past a segment's length in the fixed-size register arrays are
// predicated off. A shorter last segment (RG: m has no divisor in the segment range, e.g. a prime length) shares
// the forward-elimination constants id_i, h_i (they depend on the row's distance from the segment's top only) and
// has its own backward responses H, K (from its own last row). TQ lines per workgroup: 16 (128-B rows,
// any block of <= 64 segments) or, where the block fits 1024 threads, 32 / 64 (256- / 512-B rows) with the segment
// arrays sized to the block (k_tris's tiles; e_i = A id_i recomputed, not stored: the same double)
namespace trig {
constexpr int SMAX = 32, NSMAX = 64, TQ = 16;
}

template <int SMAX, int TQ, int NS, bool RG = false>
__global__ __launch_bounds__(1024) void k_trig(const SpecArgs a, int sl, int nseg, int sr) {
    double sigma = a.sigma;
    if (a.skip && *a.skip) return;
    if (a.ctl) {
        if (a.ctl->done) return;
        sigma = a.ctl->sigma;
    }
    __shared__ double t_id[SMAX][TQ], t_h[SMAX][TQ], t_k[SMAX][TQ];
    __shared__ double s_a[TQ];
    __shared__ double s_u[NS][TQ], s_v[NS][TQ], s_bu[NS][TQ], s_bv[NS][TQ];
    __shared__ double t_h2[RG ? SMAX : 1][TQ], t_k2[RG ? SMAX : 1][TQ];   // the last segment's H, K
    const int t = threadIdx.x, c = t % TQ, sj = t / TQ;
    const int ln = (RG && sj == nseg - 1) ? sr : sl;   // this thread's segment length
    const uint32_t m = a.m[a.d];
    const uint32_t q0 = (a.xrun ? xcd_run(blockIdx.x, gridDim.x) : blockIdx.x) * uint32_t(TQ);
    const uint32_t q = q0 + uint32_t(c);
    const bool valid = q < a.nlines;
    const uint32_t qq = valid ? q : q0;
    const uint32_t hi = a.fds.div(qq);
    const uint32_t base = (qq - hi * a.stride) + hi * a.stride * m + uint32_t(sj * sl) * a.stride;

    double g[SMAX];
#pragma unroll
    for (int i = 0; i < SMAX; ++i)
        g[i] = (valid && i < ln) ? __builtin_nontemporal_load(a.in + base + uint32_t(i) * a.stride) : 0.0;

    if (t < TQ) {
        const uint32_t ql = a.q_off + qq;
        double lamv[kMaxDims] = {0, 0, 0, 0};
        uint32_t rest = ql;
        const int jlast = a.d == a.p - 1 ? a.p - 2 : a.p - 1;
        for (int jj = 0; jj < a.p; ++jj) {
            if (jj == a.d) continue;
            const uint32_t qd = (jj < jlast) ? a.fd[jj].div(rest) : 0u;
            lamv[jj] = a.lam[a.lam_off[jj] + (rest - qd * a.m[jj])];
            rest = qd;
        }
        double c0 = a.w0, c1 = 0.0;
        for (int Sm = 1; Sm < (1 << a.p); ++Sm) {
            if (a.cS[Sm] == 0.0) continue;
            double prod = sigma * a.cS[Sm];
            for (int jj = 0; jj < a.p; ++jj)
                if (jj != a.d && ((Sm >> jj) & 1)) prod *= lamv[jj];
            if ((Sm >> a.d) & 1) c1 += prod;
            else c0 += prod;
        }
        const double A = -c1, B = c0 + 2.0 * c1;
        double e = 0.0, h = 1.0;
#pragma unroll 1
        for (int i = 0; i < sl; ++i) {
            const double id = 1.0 / (B - A * e);
            e = A * id;
            h = -A * h * id;
            t_id[i][c] = id;
            t_h[i][c] = h;
        }
        if constexpr (RG) {   // the last segment's sweep first: it reads the forward h_i that the next one replaces
            double H2 = t_h[sr - 1][c], K2 = -(A * t_id[sr - 1][c]);
            t_h2[sr - 1][c] = H2;
            t_k2[sr - 1][c] = K2;
#pragma unroll 1
            for (int i = sr - 2; i >= 0; --i) {
                const double ei = A * t_id[i][c];
                H2 = t_h[i][c] - ei * H2;
                K2 = -ei * K2;
                t_h2[i][c] = H2;
                t_k2[i][c] = K2;
            }
        }
        double H = t_h[sl - 1][c], K = -(A * t_id[sl - 1][c]);
        t_k[sl - 1][c] = K;
#pragma unroll 1
        for (int i = sl - 2; i >= 0; --i) {
            const double ei = A * t_id[i][c];
            H = t_h[i][c] - ei * H;
            K = -ei * K;
            t_h[i][c] = H;
            t_k[i][c] = K;
        }
        s_a[c] = A;
    }
    __syncthreads();

    {
        const double A = s_a[c];
        g[0] *= t_id[0][c];
#pragma unroll
        for (int i = 1; i < SMAX; ++i)
            if (i < ln) g[i] = (g[i] - A * g[i - 1]) * t_id[i][c];
        double last = 0.0;
#pragma unroll
        for (int i = SMAX - 1; i >= 0; --i) {
            if (i == ln - 1) last = g[i];
            if (i < ln - 1) g[i] -= (A * t_id[i][c]) * g[i + 1];
        }
        s_u[sj][c] = g[0];
        s_v[sj][c] = last;
    }
    __syncthreads();

    if (t < TQ) {
        const double H0 = t_h[0][c], K0 = t_k[0][c], H1 = t_h[sl - 1][c], K1 = t_k[sl - 1][c];
        double av = 0.0, bv = 0.0;
#pragma unroll 1
        for (int j = 0; j < nseg - 1; ++j) {
            const double g0 = s_u[j][c], g1 = s_v[j][c];
            double au, bu;
            if (j == 0) {
                const double id = 1.0 / (1.0 - H0);
                au = g0 * id;
                bu = K0 * id;
                av = g1 + H1 * au;
                bv = K1 + H1 * bu;
            } else {
                const double id = 1.0 / (1.0 - H0 * bv);
                au = (g0 + H0 * av) * id;
                bu = K0 * id;
                const double nav = g1 + H1 * av + H1 * bv * au;
                bv = K1 + H1 * bv * bu;
                av = nav;
            }
            s_u[j][c] = au;
            s_bu[j][c] = bu;
            s_v[j][c] = av;
            s_bv[j][c] = bv;
        }
        const int J = nseg - 1;
        const double H0J = RG ? t_h2[0][c] : H0, K0J = RG ? t_k2[0][c] : K0;
        const double H1J = RG ? t_h2[sr - 1][c] : H1, K1J = RG ? t_k2[sr - 1][c] : K1;
        const double a11 = 1.0 - H0J * bv, a12 = -K0J, a21 = -H1J * bv, a22 = 1.0 - K1J;
        const double b1 = s_u[J][c] + H0J * av, b2 = s_v[J][c] + H1J * av;
        const double idet = 1.0 / (a11 * a22 - a12 * a21);
        double u = (b1 * a22 - a12 * b2) * idet;
        s_u[J][c] = u;
        s_v[J][c] = (a11 * b2 - a21 * b1) * idet;
#pragma unroll 1
        for (int j = J - 1; j >= 0; --j) {
            const double un = u;
            u = s_u[j][c] + s_bu[j][c] * un;
            s_v[j][c] = s_v[j][c] + s_bv[j][c] * un;
            s_u[j][c] = u;
        }
    }
    __syncthreads();

    const double Lj = sj == 0 ? s_u[0][c] : s_v[sj - 1][c];
    const double Rj = sj == nseg - 1 ? s_v[nseg - 1][c] : s_u[sj + 1][c];
    const double sc = a.inv_n * double(m);
    if (!valid) return;
    const bool lastseg = RG && sj == nseg - 1;
#pragma unroll
    for (int i = 0; i < SMAX; ++i)
        if (i < ln) {
            const double h = lastseg ? t_h2[i][c] : t_h[i][c], kk = lastseg ? t_k2[i][c] : t_k[i][c];
            __builtin_nontemporal_store(sc * (g[i] + h * Lj + kk * Rj), a.out + base + uint32_t(i) * a.stride);
        }
}

// (r^k, 1 - r^k) pairs: products and powers keep 1 - r^k free of cancellation (1 - r^(a+b) = t_a + r^a t_b)
struct PowT {
    double p, t;
};
__device__ __forceinline__ PowT powt_mul(PowT a, PowT b) { return {a.p * b.p, fma(a.p, b.t, a.t)}; }
__device__ __forceinline__ PowT powt_pow(PowT x, uint32_t n) {
    PowT y{1.0, 0.0};
    while (n) {
        if (n & 1u) y = powt_mul(y, x);
        x = powt_mul(x, x);
        n >>= 1;
    }
    return y;
}

// k_trigr: k_trir's factorised solve for k_trig's lines (any length m = (nseg - 1) sl + sr, any stride; a shorter
// last segment sr <= sl). Segment j's carries go through r^len_j; the mirror closure through r^m.
template <int SMAX, int TQ, int NS>
__global__ __launch_bounds__(1024) void k_trigr(const SpecArgs a, int sl, int nseg, int sr) {
    double sigma = a.sigma;
    if (a.skip && *a.skip) return;
    if (a.ctl) {
        if (a.ctl->done) return;
        sigma = a.ctl->sigma;
    }
    __shared__ double s_f[NS][TQ], s_b[NS][TQ];
    __shared__ double s_r[TQ], s_sd[TQ];
    const int t = threadIdx.x, c = t % TQ, sj = t / TQ;
    const int ln = sj == nseg - 1 ? sr : sl;   // this thread's segment length
    const uint32_t m = a.m[a.d];
    const uint32_t q0 = (a.xrun ? xcd_run(blockIdx.x, gridDim.x) : blockIdx.x) * uint32_t(TQ);
    const uint32_t q = q0 + uint32_t(c);
    const bool valid = q < a.nlines;
    const uint32_t qq = valid ? q : q0;
    const uint32_t hi = a.fds.div(qq);
    const uint32_t base = (qq - hi * a.stride) + hi * a.stride * m + uint32_t(sj * sl) * a.stride;

    double lamv[kMaxDims] = {0, 0, 0, 0};
    if (t < TQ) {
        uint32_t rest = a.q_off + qq;
        const int jlast = a.d == a.p - 1 ? a.p - 2 : a.p - 1;
        for (int jj = 0; jj < a.p; ++jj) {
            if (jj == a.d) continue;
            const uint32_t qd = (jj < jlast) ? a.fd[jj].div(rest) : 0u;
            lamv[jj] = a.lam[a.lam_off[jj] + (rest - qd * a.m[jj])];
            rest = qd;
        }
    }
    double g[SMAX];
    {
        const double* pin = a.in + base;
#pragma unroll
        for (int i = 0; i < SMAX; ++i) {
            g[i] = (valid && i < ln) ? __builtin_nontemporal_load(pin) : 0.0;
            pin += a.stride;
        }
    }

    double rsl = 0.0, rsr = 0.0, rm = 0.0, idet = 1.0;   // t < TQ: r^sl, r^sr, r^m, 1 / (1 - r^2m)
    if (t < TQ) {
        double c0 = a.w0, c1 = 0.0;
        for (int Sm = 1; Sm < (1 << a.p); ++Sm) {
            if (a.cS[Sm] == 0.0) continue;
            double prod = sigma * a.cS[Sm];
            for (int jj = 0; jj < a.p; ++jj)
                if (jj != a.d && ((Sm >> jj) & 1)) prod *= lamv[jj];
            if ((Sm >> a.d) & 1) c1 += prod;
            else c0 += prod;
        }
        const double D = sqrt(c0 * (c0 + 4.0 * c1));
        const double den = 1.0 / (c0 + 2.0 * c1 + D);
        const PowT r1{2.0 * c1 * den, (c0 + D) * den};
        const PowT ps = powt_pow(r1, uint32_t(sl)), pr = powt_pow(r1, uint32_t(sr));
        const PowT pm = powt_mul(powt_pow(ps, uint32_t(nseg - 1)), pr);
        rsl = ps.p;
        rsr = pr.p;
        rm = pm.p;
        idet = 1.0 / powt_mul(pm, pm).t;
        s_r[c] = r1.p;
        s_sd[c] = a.inv_n * double(m) / D;
    }
    __syncthreads();

    const double r = s_r[c];
    {
        double fl = 0.0, bl = 0.0;
#pragma unroll
        for (int i = 0; i < SMAX; ++i) {
            if (i < ln) fl = fma(r, fl, g[i]);
            bl = fma(r, bl, g[SMAX - 1 - i]);   // rows past ln are 0: bl stays 0 until row ln - 1
        }
        s_f[sj][c] = fl;
        s_b[sj][c] = bl;
    }
    __syncthreads();

    if (t < TQ) {
        double acc = 0.0, bcc = 0.0;
        for (int k = 0; k < nseg; ++k) {
            const int kb = nseg - 1 - k;
            const double fk = s_f[k][c], bk = s_b[kb][c];
            s_f[k][c] = acc;
            s_b[kb][c] = bcc;
            acc = fma(acc, k == nseg - 1 ? rsr : rsl, fk);
            bcc = fma(bcc, k == 0 ? rsr : rsl, bk);
        }
        const double fm1 = (bcc + rm * acc) * idet, bm = (acc + rm * bcc) * idet;
        double pf = 1.0, pb = 1.0;
        for (int k = 0; k < nseg; ++k) {
            const int kb = nseg - 1 - k;
            s_f[k][c] = fma(pf, fm1, s_f[k][c]);
            s_b[kb][c] = fma(pb, bm, s_b[kb][c]);
            pf *= rsl;
            pb *= k == 0 ? rsr : rsl;
        }
    }
    __syncthreads();

    if (!valid) return;
    const double sd = s_sd[c], bin = s_b[sj][c];
    double fv = s_f[sj][c];
    {
        double bv = bin;
#pragma unroll
        for (int i = SMAX - 1; i >= 0; --i)
            if (i < ln) {
                bv = fma(r, bv, g[i]);
                g[i] = bv;
            }
    }
    double* pout = a.out + base;
#pragma unroll
    for (int i = 0; i < SMAX; ++i)
        if (i < ln) {
            const double gn = i + 1 < ln ? g[i + 1] : bin;
            __builtin_nontemporal_store(sd * fma(r, fv, g[i]), pout);
            pout += a.stride;
            fv = fma(r, fv - gn, g[i]);
        }
}

// =============================================================================================
// The last dimension of a slab-decomposed mesh (mvtv_slab.cpp): the same tridiagonal line solves, with
// every line cut at the rank boundaries, solved by substructuring instead of transposing the mesh.
//
// Rank r holds rows [zb_r, ze_r) of every line (its owned planes). Its local block of the line's
// operator, with the neighbours x[zb_r - 1] = L and x[ze_r] = R as unknowns (a mirror at the mesh's own
// ends), has the solution x = G + L H + R K (G: the data with L = R = 0; H, K: the responses to L = 1 and
// R = 1). Phase 1 (k_tris<1>) computes, per line, the first and last rows of G, H and K (6 numbers) without
// writing the mesh; the interface system that couples the ranks' (first, last) rows of a line is solved
// where the line's chunk lives (k_tris_iface: one thread per line, O(G)); phase 3 (k_tris<3>) solves the
// local block again with the now known L and R and writes x. The ranks exchange 6 + 2 numbers per line
// instead of the 2 x (owned planes) numbers per line of two transposes: at 512^3 over 8 ranks 15 MB
// instead of 235 MB per rank per iteration. Within a rank the block is cut into nseg segments of sl rows,
// one thread each, as k_trig (Toeplitz interior: the segment constants are line constants in LDS).
namespace tris {
constexpr int NSMAX = 64, TQ = 16;
}

// TQ lines per workgroup (16: 128-B rows; 64: 512-B rows, one full run per wave load), NS >= nseg segments (the LDS
// of the interface arrays is sized by it: with NS = 64 for every block, a 4-segment block of a G = 8 rank at 512^3
// took 48 KB for one wave, 3 waves per CU, and moved 0.9-1.5 TB/s)
template <int PHASE, int SMAX, int TQ = tris::TQ, int NS = tris::NSMAX>
__global__ __launch_bounds__(1024) void k_tris(const SpecArgs a, int sl, int nseg, double* __restrict__ x,
                                               double* __restrict__ coef, const double* __restrict__ lr,
                                               uint32_t chunk, int lo_ext, int hi_ext, double scale) {
    double sigma = a.sigma;
    if (a.skip && *a.skip) return;
    if (a.ctl) {
        if (a.ctl->done) return;
        sigma = a.ctl->sigma;
    }
    __shared__ double t_id[SMAX][TQ], t_h[SMAX][TQ], t_k[SMAX][TQ];   // e_i = A id_i: recomputed, not stored
    __shared__ double s_a[TQ];
    __shared__ double s_u[NS][TQ], s_v[NS][TQ], s_bu[NS][TQ];
    // phase 1: the forward-eliminated u of the L- and R-response tracks; phase 3: the slopes of v_j on u_{j+1}
    __shared__ double s_u1[PHASE == 1 ? NS : 1][TQ], s_u2[PHASE == 1 ? NS : 1][TQ], s_bv[PHASE == 3 ? NS : 1][TQ];
    const int t = threadIdx.x, c = t % TQ, sj = t / TQ;
    const uint32_t q0 = blockIdx.x * uint32_t(TQ);
    const uint32_t q = q0 + uint32_t(c);
    const bool valid = q < a.nlines;
    const uint32_t qq = valid ? q : q0;
    const size_t base = size_t(qq) + size_t(sj * sl) * a.stride;   // lines are contiguous: stride = plane

    double g[SMAX];
#pragma unroll
    for (int i = 0; i < SMAX; ++i)
        g[i] = (valid && i < sl) ? __builtin_nontemporal_load(x + base + size_t(i) * a.stride) : 0.0;
    double lx = 0.0, rx = 0.0;   // phase 3: the neighbours' values (the interface solve's result)
    if (PHASE == 3 && t < TQ) {
        const uint32_t s = qq / chunk, l = qq - s * chunk;
        if (lo_ext) lx = lr[(size_t(s) * 2) * chunk + l];
        if (hi_ext) rx = lr[(size_t(s) * 2 + 1) * chunk + l];
    }

    if (t < TQ) {   // c0 + c1 T along the last dim for line qq (dims 0..p-2 column-major)
        double lamv[kMaxDims] = {0, 0, 0, 0};
        uint32_t rest = qq;
        for (int jj = 0; jj < a.p - 1; ++jj) {
            const uint32_t qd = (jj < a.p - 2) ? a.fd[jj].div(rest) : 0u;
            lamv[jj] = a.lam[a.lam_off[jj] + (rest - qd * a.m[jj])];
            rest = qd;
        }
        double c0 = a.w0, c1 = 0.0;
        for (int Sm = 1; Sm < (1 << a.p); ++Sm) {
            if (a.cS[Sm] == 0.0) continue;
            double prod = sigma * a.cS[Sm];
            for (int jj = 0; jj < a.p - 1; ++jj)
                if ((Sm >> jj) & 1) prod *= lamv[jj];
            if ((Sm >> (a.p - 1)) & 1) c1 += prod;
            else c0 += prod;
        }
        const double A = -c1, B = c0 + 2.0 * c1;
        double e = 0.0, h = 1.0;
#pragma unroll 1
        for (int i = 0; i < sl; ++i) {
            const double id = 1.0 / (B - A * e);
            e = A * id;
            h = -A * h * id;
            t_id[i][c] = id;
            t_h[i][c] = h;
        }
        double H = t_h[sl - 1][c], K = -(A * t_id[sl - 1][c]);
        t_k[sl - 1][c] = K;
#pragma unroll 1
        for (int i = sl - 2; i >= 0; --i) {
            const double ei = A * t_id[i][c];
            H = t_h[i][c] - ei * H;
            K = -ei * K;
            t_h[i][c] = H;
            t_k[i][c] = K;
        }
        s_a[c] = A;
    }
    __syncthreads();

    {   // this segment with zero neighbours
        const double A = s_a[c];
        g[0] *= t_id[0][c];
#pragma unroll
        for (int i = 1; i < SMAX; ++i)
            if (i < sl) g[i] = (g[i] - A * g[i - 1]) * t_id[i][c];
        double last = 0.0;
#pragma unroll
        for (int i = SMAX - 1; i >= 0; --i) {
            if (i == sl - 1) last = g[i];
            if (i < sl - 1) g[i] -= (A * t_id[i][c]) * g[i + 1];
        }
        s_u[sj][c] = g[0];
        s_v[sj][c] = last;
    }
    __syncthreads();

    if (t < TQ) {
        // segments' interface system as k_trig, with the block's ends either the mesh's mirror (v_{-1} = u_0,
        // R_last = v_last) or a neighbour rank's value. Eliminated forward to v_{j-1} = av + bv u_j (bv is the
        // same for every right-hand side: phase 1 carries three, the data and the responses to L = 1, R = 1).
        const double H0 = t_h[0][c], K0 = t_k[0][c], H1 = t_h[sl - 1][c], K1 = t_k[sl - 1][c];
        constexpr int NR = PHASE == 1 ? 3 : 1;
        double av[NR], bv = lo_ext ? 0.0 : 1.0;
        av[0] = lo_ext ? lx : 0.0;
        if constexpr (NR == 3) {
            av[1] = lo_ext ? 1.0 : 0.0;
            av[2] = 0.0;
        }
#pragma unroll 1
        for (int j = 0; j < nseg - 1; ++j) {
            const double id = 1.0 / (1.0 - H0 * bv);
            const double bu = K0 * id;
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const double g0 = r == 0 ? s_u[j][c] : 0.0, g1 = r == 0 ? s_v[j][c] : 0.0;
                const double au = (g0 + H0 * av[r]) * id;
                av[r] = g1 + H1 * av[r] + H1 * bv * au;
                if (r == 0) s_u[j][c] = au;
                if constexpr (NR == 3) {
                    if (r == 1) s_u1[j][c] = au;
                    if (r == 2) s_u2[j][c] = au;
                }
                if (r == 0) s_v[j][c] = av[0];
            }
            bv = K1 + H1 * bv * bu;
            s_bu[j][c] = bu;
            if constexpr (PHASE == 3) s_bv[j][c] = bv;
        }
        // last segment: R_J = cr v_J + Rx (mirror: cr = 1, Rx = 0; neighbour: cr = 0, Rx = its value)
        const int J = nseg - 1;
        const double cr = hi_ext ? 0.0 : 1.0;
        const double a11 = 1.0 - H0 * bv, a12 = -K0 * cr, a21 = -H1 * bv, a22 = 1.0 - K1 * cr;
        const double idet = 1.0 / (a11 * a22 - a12 * a21);
        double uJ[NR], vJ[NR];
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const double gJ0 = r == 0 ? s_u[J][c] : 0.0, gJ1 = r == 0 ? s_v[J][c] : 0.0;
            const double rxr = r == 0 ? (hi_ext ? rx : 0.0) : (r == 2 && hi_ext ? 1.0 : 0.0);
            const double b1 = gJ0 + H0 * av[r] + K0 * rxr, b2 = gJ1 + H1 * av[r] + K1 * rxr;
            uJ[r] = (b1 * a22 - a12 * b2) * idet;
            vJ[r] = (a11 * b2 - a21 * b1) * idet;
        }
        if constexpr (PHASE == 1) {
            // first row of the block: back-substitute u_j = au_j + bu_j u_{j+1} down to u_0 for each track
            double u[3] = {uJ[0], uJ[1], uJ[2]};
#pragma unroll 1
            for (int j = J - 1; j >= 0; --j) {
                const double bu = s_bu[j][c];
                u[0] = s_u[j][c] + bu * u[0];
                u[1] = s_u1[j][c] + bu * u[1];
                u[2] = s_u2[j][c] + bu * u[2];
            }
            if (valid) {   // [chunk s][6][line in chunk]: Gf Gl Hf Hl Kf Kl
                const uint32_t s = q / chunk, l = q - s * chunk;
                double* o = coef + size_t(s) * 6 * chunk + l;
                o[0] = u[0];
                o[size_t(chunk)] = vJ[0];
                o[2 * size_t(chunk)] = u[1];
                o[3 * size_t(chunk)] = vJ[1];
                o[4 * size_t(chunk)] = u[2];
                o[5 * size_t(chunk)] = vJ[2];
            }
        } else {
            // every segment's (u_j, v_j) by back substitution
            s_u[J][c] = uJ[0];
            s_v[J][c] = vJ[0];
            double un = uJ[0];
#pragma unroll 1
            for (int j = J - 1; j >= 0; --j) {
                const double u = s_u[j][c] + s_bu[j][c] * un;
                s_v[j][c] = s_v[j][c] + s_bv[j][c] * un;
                s_u[j][c] = u;
                un = u;
            }
        }
    }
    if constexpr (PHASE == 3) {
        __shared__ double s_lx[TQ], s_rx[TQ];
        if (t < TQ) {
            s_lx[c] = lx;
            s_rx[c] = rx;
        }
        __syncthreads();
        const double Lj = sj == 0 ? (lo_ext ? s_lx[c] : s_u[0][c]) : s_v[sj - 1][c];
        const double Rj = sj == nseg - 1 ? (hi_ext ? s_rx[c] : s_v[nseg - 1][c]) : s_u[sj + 1][c];
        if (!valid) return;
#pragma unroll
        for (int i = 0; i < SMAX; ++i)
            if (i < sl)
                __builtin_nontemporal_store(scale * (g[i] + t_h[i][c] * Lj + t_k[i][c] * Rj), x + base + size_t(i) * a.stride);
    }
}

// the interface systems of the lines of one chunk (on the rank that owns the chunk): from every rank r's
// (Gf, Gl, Hf, Hl, Kf, Kl) [r][6][chunk] the first row u_r and last row v_r of each rank's block,
//   u_r = Gf_r + Hf_r v_{r-1} + Kf_r u_{r+1},  v_r = Gl_r + Hl_r v_{r-1} + Kl_r u_{r+1}
// (Hf_0 = Hl_0 = 0, Kf_{G-1} = Kl_{G-1} = 0: the mesh's ends), eliminated forward to
// u_r = ga_r + de_r u_{r+1}, v_r = al_r + be_r u_{r+1} (kept in the input's first four rows), then
// substituted back. Out [r][2][chunk]: (L, R) of rank r = (v_{r-1}, u_{r+1}).
__global__ __launch_bounds__(256) void k_tris_iface(double* __restrict__ co, double* __restrict__ lr, uint32_t chunk,
                                                    int G, const AdmmCtl* ctl, const int32_t* skip) {
    if (ctl && ctl->done) return;
    if (skip && *skip) return;
    const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= chunk) return;
    const size_t C = chunk;
    double al = 0.0, be = 0.0;
    for (int r = 0; r < G; ++r) {
        double* c = co + size_t(r) * 6 * C + l;
        const double Gf = c[0], Gl = c[C], Hf = c[2 * C], Hl = c[3 * C], Kf = c[4 * C], Kl = c[5 * C];
        const double id = 1.0 / (1.0 - Hf * be);
        const double ga = (Gf + Hf * al) * id, de = Kf * id;
        const double nal = Gl + Hl * al + Hl * be * ga, nbe = Kl + Hl * be * de;
        c[0] = ga;
        c[C] = de;
        c[2 * C] = nal;
        c[3 * C] = nbe;
        al = nal;
        be = nbe;
    }
    double un = 0.0;   // u_{r+1}
    for (int r = G - 1; r >= 0; --r) {
        const double* c = co + size_t(r) * 6 * C + l;
        const double u = c[0] + c[C] * un, v = c[2 * C] + c[3 * C] * un;
        lr[(size_t(r) * 2 + 1) * C + l] = r < G - 1 ? un : 0.0;          // R of rank r
        if (r + 1 < G) lr[(size_t(r + 1) * 2) * C + l] = v;               // L of rank r + 1
        un = u;
    }
    lr[l] = 0.0;   // L of rank 0 (the mesh's end)
}

// ---------------------------------------------------------------------------------------------
// The slab line solves by the factorised operator (round 6; k_trir's recursions F_i = f_i + r F_{i-1},
// B_i = f_i + r B_{i+1}, x = (F + B - f) / D). A rank's block of a line enters the global recursions only through
// two numbers: F at its last row and B at its first row, each from zero carries (phase 1). The chunk owner combines
// the ranks' pairs with the multipliers r^n_r of the block lengths and closes the mirror (k_trisr_iface): every
// block's carries, F into its first row and B into its last. Phase 3 reruns the block's recursions from them. Two
// numbers per line cross the ranks each way (6 + 2 with the Thomas responses of k_tris), and no step divides per row.
template <int PHASE, int SMAX, int TQ = tris::TQ, int NS = tris::NSMAX>
__global__ __launch_bounds__(1024) void k_trisr(const SpecArgs a, int sl, int nseg, double* __restrict__ x,
                                                double* __restrict__ coef, const double* __restrict__ lr,
                                                uint32_t chunk, int, int, double scale) {
    double sigma = a.sigma;
    if (a.skip && *a.skip) return;
    if (a.ctl) {
        if (a.ctl->done) return;
        sigma = a.ctl->sigma;
    }
    __shared__ double s_f[NS][TQ], s_b[NS][TQ];
    __shared__ double s_r[TQ], s_sd[TQ];
    const int t = threadIdx.x, c = t % TQ, sj = t / TQ;
    const uint32_t q0 = blockIdx.x * uint32_t(TQ);
    const uint32_t q = q0 + uint32_t(c);
    const bool valid = q < a.nlines;
    const uint32_t qq = valid ? q : q0;
    const size_t base = size_t(qq) + size_t(sj * sl) * a.stride;   // lines are contiguous: stride = plane

    double lamv[kMaxDims] = {0, 0, 0, 0};
    if (t < TQ) {
        uint32_t rest = qq;
        for (int jj = 0; jj < a.p - 1; ++jj) {
            const uint32_t qd = (jj < a.p - 2) ? a.fd[jj].div(rest) : 0u;
            lamv[jj] = a.lam[a.lam_off[jj] + (rest - qd * a.m[jj])];
            rest = qd;
        }
    }
    double g[SMAX];
#pragma unroll
    for (int i = 0; i < SMAX; ++i)
        g[i] = (valid && i < sl) ? __builtin_nontemporal_load(x + base + size_t(i) * a.stride) : 0.0;
    double fin = 0.0, bout = 0.0, rsl = 0.0;   // t < TQ, phase 3: the block's carries; r^sl
    if (t < TQ) {
        if (PHASE == 3) {
            const uint32_t s = qq / chunk, l = qq - s * chunk;
            fin = lr[(size_t(s) * 2) * chunk + l];
            bout = lr[(size_t(s) * 2 + 1) * chunk + l];
        }
        double c0 = a.w0, c1 = 0.0;
        for (int Sm = 1; Sm < (1 << a.p); ++Sm) {
            if (a.cS[Sm] == 0.0) continue;
            double prod = sigma * a.cS[Sm];
            for (int jj = 0; jj < a.p - 1; ++jj)
                if ((Sm >> jj) & 1) prod *= lamv[jj];
            if ((Sm >> (a.p - 1)) & 1) c1 += prod;
            else c0 += prod;
        }
        const double D = sqrt(c0 * (c0 + 4.0 * c1));
        const double den = 1.0 / (c0 + 2.0 * c1 + D);
        const PowT r1{2.0 * c1 * den, (c0 + D) * den};
        rsl = powt_pow(r1, uint32_t(sl)).p;
        s_r[c] = r1.p;
        s_sd[c] = scale / D;
    }
    __syncthreads();

    const double r = s_r[c];
    {
        double fl = 0.0, bl = 0.0;
#pragma unroll
        for (int i = 0; i < SMAX; ++i) {
            if (i < sl) fl = fma(r, fl, g[i]);
            bl = fma(r, bl, g[SMAX - 1 - i]);   // rows past sl are 0
        }
        s_f[sj][c] = fl;
        s_b[sj][c] = bl;
    }
    __syncthreads();

    if (t < TQ) {
        // phase 1: the block's F at its last row and B at its first row from zero carries; phase 3: every
        // segment's carries from the block's
        double acc = PHASE == 3 ? fin : 0.0, bcc = PHASE == 3 ? bout : 0.0;
        for (int k = 0; k < nseg; ++k) {
            const int kb = nseg - 1 - k;
            const double fk = s_f[k][c], bk = s_b[kb][c];
            if (PHASE == 3) {
                s_f[k][c] = acc;
                s_b[kb][c] = bcc;
            }
            acc = fma(acc, rsl, fk);
            bcc = fma(bcc, rsl, bk);
        }
        if (PHASE == 1 && valid) {   // [chunk s][2][line in chunk]: F_last, B_first
            const uint32_t s = q / chunk, l = q - s * chunk;
            coef[(size_t(s) * 2) * chunk + l] = acc;
            coef[(size_t(s) * 2 + 1) * chunk + l] = bcc;
        }
    }
    if constexpr (PHASE == 3) {
        __syncthreads();
        if (!valid) return;
        const double sd = s_sd[c], bin = s_b[sj][c];
        double fv = s_f[sj][c];
        {
            double bv = bin;
#pragma unroll
            for (int i = SMAX - 1; i >= 0; --i)
                if (i < sl) {
                    bv = fma(r, bv, g[i]);
                    g[i] = bv;
                }
        }
#pragma unroll
        for (int i = 0; i < SMAX; ++i)
            if (i < sl) {
                const double gn = i + 1 < sl ? g[i + 1] : bin;
                __builtin_nontemporal_store(sd * fma(r, fv, g[i]), x + base + size_t(i) * a.stride);
                fv = fma(r, fv - gn, g[i]);
            }
    }
}

// the chunk owner's lines (global line q = rank * chunk + l): from every rank's (F_last, B_first) [r][2][chunk] the
// carries of every rank's block, (F into its first row, B into its last) [r][2][chunk], with the mirror closure at the
// mesh's ends. Rank k's block: planes [floor(mg k / G), floor(mg (k + 1) / G)).
__global__ __launch_bounds__(256) void k_trisr_iface(const SpecArgs a, const double* __restrict__ co,
                                                     double* __restrict__ lr, uint32_t chunk, int G, int rank,
                                                     uint32_t mg) {
    double sigma = a.sigma;
    if (a.skip && *a.skip) return;
    if (a.ctl) {
        if (a.ctl->done) return;
        sigma = a.ctl->sigma;
    }
    const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= chunk) return;
    const size_t C = chunk;
    double lamv[kMaxDims] = {0, 0, 0, 0};
    uint32_t rest = uint32_t(rank) * chunk + l;
    for (int jj = 0; jj < a.p - 1; ++jj) {
        const uint32_t qd = (jj < a.p - 2) ? a.fd[jj].div(rest) : 0u;
        lamv[jj] = a.lam[a.lam_off[jj] + (rest - qd * a.m[jj])];
        rest = qd;
    }
    double c0 = a.w0, c1 = 0.0;
    for (int Sm = 1; Sm < (1 << a.p); ++Sm) {
        if (a.cS[Sm] == 0.0) continue;
        double prod = sigma * a.cS[Sm];
        for (int jj = 0; jj < a.p - 1; ++jj)
            if ((Sm >> jj) & 1) prod *= lamv[jj];
        if ((Sm >> (a.p - 1)) & 1) c1 += prod;
        else c0 += prod;
    }
    const double D = sqrt(c0 * (c0 + 4.0 * c1));
    const double den = 1.0 / (c0 + 2.0 * c1 + D);
    const PowT r1{2.0 * c1 * den, (c0 + D) * den};
    // the multipliers r^n_k of the blocks: n_k = floor(mg (k + 1) / G) - floor(mg k / G) takes two values at most
    const uint32_t nlo = mg / uint32_t(G);
    const PowT plo = powt_pow(r1, nlo);
    const double rlo = plo.p, rhi = plo.p * r1.p;
    auto rblk = [&](int k) {
        const uint32_t n = uint32_t(uint64_t(mg) * uint64_t(k + 1) / uint64_t(G) - uint64_t(mg) * uint64_t(k) / uint64_t(G));
        return n == nlo ? rlo : rhi;
    };
    // forward: F into block k's first row from the blocks before it (zero at the mesh's start)
    double acc = 0.0;
    for (int k = 0; k < G; ++k) {
        lr[(size_t(k) * 2) * C + l] = acc;
        acc = fma(acc, rblk(k), co[(size_t(k) * 2) * C + l]);
    }
    double bcc = 0.0;
    for (int k = G - 1; k >= 0; --k) {
        lr[(size_t(k) * 2 + 1) * C + l] = bcc;
        bcc = fma(bcc, rblk(k), co[(size_t(k) * 2 + 1) * C + l]);
    }
    const PowT pm = powt_pow(r1, mg);
    const double idet = 1.0 / powt_mul(pm, pm).t;
    const double fm1 = (bcc + pm.p * acc) * idet, bm = (acc + pm.p * bcc) * idet;
    double pf = 1.0, pb = 1.0;
    for (int k = 0; k < G; ++k) {
        const int kb = G - 1 - k;
        lr[(size_t(k) * 2) * C + l] = fma(pf, fm1, lr[(size_t(k) * 2) * C + l]);
        lr[(size_t(kb) * 2 + 1) * C + l] = fma(pb, bm, lr[(size_t(kb) * 2 + 1) * C + l]);
        pf *= rblk(k);
        pb *= rblk(kb);
    }
}

static void tris_seg(uint32_t n, int* sl, int* nseg) {
    // >= 4 segments when the block allows it, segments of <= 16 rows (32 past 1024 rows), <= 64 segments
    uint32_t s = std::max<uint32_t>(1u, std::min<uint32_t>(n > 1024u ? 32u : 16u, n / 4u));
    while (s > 1 && n % s) --s;
    *sl = int(s);
    *nseg = int(n / s);
}

bool tri_slab_ok(uint32_t n) {
    int sl = 0, nseg = 0;
    tris_seg(n, &sl, &nseg);
    return n >= 1 && sl <= 32 && nseg <= tris::NSMAX;
}

static bool tris_thomas() {   // probe builds: MVTV_TRI_IIR=0 keeps the Thomas form (k_tris, 6 + 2 numbers per line)
    static const bool th = [] {
        const char* e = probe_env("MVTV_TRI_IIR");
        return e && std::atoi(e) == 0;
    }();
    return th;
}
int tri_slab_ncoef() { return tris_thomas() ? 6 : 2; }

hipError_t launch_tri_slab(const SpecPlan& sp, const Geom& og, hipStream_t s, int phase, double* x, double* coef,
                           const double* lr, uint32_t chunk, int lo_ext, int hi_ext, double scale,
                           const AdmmCtl* ctl, double sigma, double w0, const int32_t* skip) {
    const int p = og.p, d = p - 1;
    SpecArgs a{};
    a.ctl = ctl;
    a.skip = skip;
    a.sigma = sigma;
    a.w0 = w0;
    a.lam = sp.lam;
    for (int j = 0; j < kMaxDims; ++j) {
        a.lam_off[j] = sp.lam_off[j];
        a.m[j] = og.m[j];
    }
    for (int j = 0; j < kMaxDims - 1; ++j) a.fd[j] = og.fd[j];
    for (int S = 0; S < 16; ++S) a.cS[S] = og.cS[S];
    a.d = d;
    a.p = p;
    a.stride = og.stride[d];
    a.nlines = og.stride[d];
    const uint32_t n = og.m[d];
    int sl = 0, nseg = 0;
    tris_seg(n, &sl, &nseg);
    if (!tri_slab_ok(n) || chunk == 0 || a.nlines % chunk != 0)
        return hipErrorInvalidValue;
    if (phase != 1 && phase != 3) return hipErrorInvalidValue;
    // 64-line tiles with the segment arrays sized to the block (<= 16 segments: <= 1024 threads) where the lines
    // fill >= 128 such workgroups; otherwise 16-line tiles sized for any block (<= 64 segments)
    static const bool wide_off = probe_env("MVTV_TRIS_NARROW") != nullptr;
    const bool thomas = tris_thomas();
    auto go = [&](auto kern, uint32_t tq) {
        klaunch(kern, dim3((a.nlines + tq - 1) / tq), dim3(tq * uint32_t(nseg)), 0, s, a, sl, nseg, x, coef, lr, chunk,
                lo_ext, hi_ext, scale);
        return hipGetLastError();
    };
    if (!wide_off && nseg <= 16 && a.nlines >= 64u * 128u) {
        // segments of <= 16 rows keep the row registers at 16 (blocks up to 256 planes here); <= 4 rows (blocks of
        // <= 16 planes: a 4-D rank at G = 8) size the line constants for 4
        const int ns = nseg <= 4 ? 4 : (nseg <= 8 ? 8 : 16);
        if (sl <= 4 && ns == 4) {
            if (phase == 1) return thomas ? go(k_tris<1, 4, 64, 4>, 64u) : go(k_trisr<1, 4, 64, 4>, 64u);
            return thomas ? go(k_tris<3, 4, 64, 4>, 64u) : go(k_trisr<3, 4, 64, 4>, 64u);
        }
        if (sl <= 16) {
            if (phase == 1) {
                if (ns == 4) return thomas ? go(k_tris<1, 16, 64, 4>, 64u) : go(k_trisr<1, 16, 64, 4>, 64u);
                if (ns == 8) return thomas ? go(k_tris<1, 16, 64, 8>, 64u) : go(k_trisr<1, 16, 64, 8>, 64u);
                return thomas ? go(k_tris<1, 16, 64, 16>, 64u) : go(k_trisr<1, 16, 64, 16>, 64u);
            }
            if (ns == 4) return thomas ? go(k_tris<3, 16, 64, 4>, 64u) : go(k_trisr<3, 16, 64, 4>, 64u);
            if (ns == 8) return thomas ? go(k_tris<3, 16, 64, 8>, 64u) : go(k_trisr<3, 16, 64, 8>, 64u);
            return thomas ? go(k_tris<3, 16, 64, 16>, 64u) : go(k_trisr<3, 16, 64, 16>, 64u);
        }
    }
    const uint32_t tq = uint32_t(tris::TQ);
    if (phase == 1 && sl <= 16) return thomas ? go(k_tris<1, 16>, tq) : go(k_trisr<1, 16>, tq);
    if (phase == 1) return thomas ? go(k_tris<1, 32>, tq) : go(k_trisr<1, 32>, tq);
    if (sl <= 16) return thomas ? go(k_tris<3, 16>, tq) : go(k_trisr<3, 16>, tq);
    return thomas ? go(k_tris<3, 32>, tq) : go(k_trisr<3, 32>, tq);
}


hipError_t launch_tri_iface(const SpecPlan& sp, const Geom& og, hipStream_t s, double* coef_in, double* lr_out,
                            uint32_t chunk, int G, int rank, uint32_t mg, const AdmmCtl* ctl, double sigma, double w0,
                            const int32_t* skip) {
    if (G < 1 || chunk == 0) return hipErrorInvalidValue;
    if (tris_thomas()) {
        klaunch(k_tris_iface, dim3((chunk + 255) / 256), dim3(256), 0, s, coef_in, lr_out, chunk, G, ctl, skip);
        return hipGetLastError();
    }
    SpecArgs a{};
    a.ctl = ctl;
    a.skip = skip;
    a.sigma = sigma;
    a.w0 = w0;
    a.lam = sp.lam;
    for (int j = 0; j < kMaxDims; ++j) {
        a.lam_off[j] = sp.lam_off[j];
        a.m[j] = og.m[j];
    }
    for (int j = 0; j < kMaxDims - 1; ++j) a.fd[j] = og.fd[j];
    for (int S = 0; S < 16; ++S) a.cS[S] = og.cS[S];
    a.p = og.p;
    a.d = og.p - 1;
    klaunch(k_trisr_iface, dim3((chunk + 255) / 256), dim3(256), 0, s, a, coef_in, lr_out, chunk, G, rank, mg);
    return hipGetLastError();
}

// segment length for k_trig: the smallest divisor of m in [16, 32], else the largest in [4, 16),
// with at most 64 segments; else (no such divisor: a prime length, 2 x a prime ...; probe builds keep the
// Bluestein MID pass with MVTV_TRIG_EXACT=1) 16 rows (32 past 1024 points; m / 4 rounded up below 64 points) with a
// shorter last segment; 0 when there is none (m < 8, m > 2048)
static int trig_seg(uint32_t m) {
    static const int force = [] {   // probe builds: MVTV_TRIG_SL=s forces the segment length (a shorter last one
        const char* e = probe_env("MVTV_TRIG_SL");   // when s does not divide m)
        return e ? std::atoi(e) : 0;
    }();
    if (force >= 4 && force <= trig::SMAX && m / uint32_t(force) >= 2 &&
        (m + uint32_t(force) - 1) / uint32_t(force) <= uint32_t(trig::NSMAX))
        return force;
    for (uint32_t sl = 16; sl <= uint32_t(trig::SMAX); ++sl)
        if (m % sl == 0 && m / sl <= uint32_t(trig::NSMAX) && m / sl >= 2) return int(sl);
    for (uint32_t sl = 15; sl >= 4; --sl)
        if (m % sl == 0 && m / sl <= uint32_t(trig::NSMAX) && m / sl >= 2) return int(sl);
    static const bool exact = probe_flag("MVTV_TRIG_EXACT");
    if (exact || m < 8 || m > 2048) return 0;
    if (m < 64) return int((m + 3) / 4);
    return m > 1024 ? 32 : 16;
}

// k_trig's tile: 64 / 32 lines (512- / 256-B rows) with the segment arrays sized to the block where it fits 1024
// threads and the lines fill >= 256 such workgroups, else 16 lines for any block (round 4's form; probe builds:
// MVTV_TRIG_NARROW=1). sr < sl: a shorter last segment (RG)
static void launch_trig(const SpecArgs& a, hipStream_t s, int sl, int nseg, int sr) {
    static const bool narrow = probe_flag("MVTV_TRIG_NARROW");
    auto go = [&](auto kern, uint32_t tq) {
        klaunch(kern, dim3((a.nlines + tq - 1) / tq), dim3(tq * uint32_t(nseg)), 0, s, a, sl, nseg, sr);
    };
    // the factorised solve (k_trigr, round 6) unless a probe build asks for k_trig (MVTV_TRI_IIR=0)
    static const bool thomas = [] {
        const char* e = probe_env("MVTV_TRI_IIR");
        return e && std::atoi(e) == 0;
    }();
#define MVTV_TRIG(SM, TQ, NS)                                                                                   \
    do {                                                                                                        \
        if (!thomas) go(k_trigr<SM, TQ, NS>, uint32_t(TQ));                                                     \
        else if (sr != sl) go(k_trig<SM, TQ, NS, true>, uint32_t(TQ));                                          \
        else go(k_trig<SM, TQ, NS, false>, uint32_t(TQ));                                                       \
        return;                                                                                                 \
    } while (0)
    if (!narrow) {
        if (nseg <= 16 && a.nlines / 64u >= 256u) {
            if (sl <= 16) {
                if (nseg <= 8) MVTV_TRIG(16, 64, 8);
                MVTV_TRIG(16, 64, 16);
            }
            if (nseg <= 8) MVTV_TRIG(32, 64, 8);
            MVTV_TRIG(32, 64, 16);
        }
        if (nseg <= 32 && a.nlines / 32u >= 256u) {
            if (sl <= 16) MVTV_TRIG(16, 32, 32);
            MVTV_TRIG(32, 32, 32);
        }
        // few lines (the last dimension of a 2-D mesh: 1009 lines): 8- / 4-line tiles, >= 128 / 256 workgroups
        if (a.nlines / uint32_t(trig::TQ) < 256u) {
            const int tq = few_lines_tq(a.nlines, trig::TQ, 4);
            if (tq == 4) MVTV_TRIG(trig::SMAX, 4, trig::NSMAX);
            if (tq == 8) MVTV_TRIG(trig::SMAX, 8, trig::NSMAX);
        }
    }
    MVTV_TRIG(trig::SMAX, trig::TQ, trig::NSMAX);
#undef MVTV_TRIG
}

// k_tri serves the last-dimension pass when the lines are long enough for >= 4 segments and short enough
// for <= 64 (16 rows per segment up to 1024 points, 32 at 2048), the stride holds the tile's lines, and
// either 16-line tiles fill the chip (>= 256 workgroups: 3-D and 4-D meshes) or, for the few 2048-point
// lines of a 2-D mesh, 8-line tiles in XCD runs (2048^2: 4844 -> 5145 ADMM it/s on one box; at 1024^2 the
// FFT pass stays faster: 9866 against 9381 with 8-line and 9050 with 4-line tiles, profiles/r02/v19_tri2d). Round 6, with
// the factorised line solve (k_trir): 1024- and 512-point lines take it too, on 4-line tiles (one box, two reps each,
// profiles/r06/v8_tri2d: 1024^2 12928 / 12925 -> 14312 / 14249 ADMM it/s, 512^2 18185 / 18166 -> 20543 / 20357; 8-line
// tiles 14173 / 20397; 2048^2 keeps 8-line tiles: 6279 / 6226, 4-line 5319).
// Probe builds: MVTV_DCT_TRI2D=0 / 4 / 8 forces the 2-D choice.
static int tri_tiles(const SpecArgs& a, int mode, bool formb) {
    if (mode != SPEC_MID || a.d == 0 || formb) return 0;
    const char* e = probe_env("MVTV_DCT_TRI");
    if (e && std::atoi(e) == 0) return 0;
    if (a.L < 6 || a.L > 11 || a.stride < 4u) return 0;
    if (a.L <= 10 && a.stride >= uint32_t(tri::TQ) && a.nlines / uint32_t(tri::TQ) >= 256u) return tri::TQ;
    static const int t2d_env = [] {
        const char* v = probe_env("MVTV_DCT_TRI2D");
        return v ? std::atoi(v) : -1;
    }();
    const int t2d = t2d_env >= 0 ? t2d_env : (a.L == 11 ? 8 : (a.L >= 9 ? 4 : 0));
    if (t2d != 4 && t2d != 8) return 0;
    if (uint32_t(t2d) > a.stride || (a.nlines / uint32_t(t2d)) % 8u != 0u) return 0;
    return t2d;
}

template <int SEG, int TQL>
static void launch_tri_seg(SpecArgs& a, hipStream_t s) {
    const dim3 grid((a.nlines + uint32_t(TQL) - 1) / uint32_t(TQL));
    switch (a.L) {
        case 6: klaunch(k_tri<6, SEG, TQL>, grid, dim3(tri::Shape<6, SEG, TQL>::NT), 0, s, a); break;
        case 7: klaunch(k_tri<7, SEG, TQL>, grid, dim3(tri::Shape<7, SEG, TQL>::NT), 0, s, a); break;
        case 8: klaunch(k_tri<8, SEG, TQL>, grid, dim3(tri::Shape<8, SEG, TQL>::NT), 0, s, a); break;
        case 9: klaunch(k_tri<9, SEG, TQL>, grid, dim3(tri::Shape<9, SEG, TQL>::NT), 0, s, a); break;
        case 10: klaunch(k_tri<10, SEG, TQL>, grid, dim3(tri::Shape<10, SEG, TQL>::NT), 0, s, a); break;
    }
}

template <int L, int SEG, int TQL>
static bool launch_trir_l(SpecArgs& a, hipStream_t s) {
    if constexpr (trir::Shape<L, SEG, TQL>::NT <= 1024 && trir::Shape<L, SEG, TQL>::NSEG >= 2) {
        klaunch(k_trir<L, SEG, TQL>, dim3((a.nlines + uint32_t(TQL) - 1) / uint32_t(TQL)),
                dim3(trir::Shape<L, SEG, TQL>::NT), 0, s, a);
        return true;
    }
    return false;
}

template <int SEG, int TQL>
static bool launch_trir_seg(SpecArgs& a, hipStream_t s) {
    if (a.stride < uint32_t(TQL)) return false;
    a.tq = TQL;
    a.xcd = 0;
    switch (a.L) {
        case 6: return launch_trir_l<6, SEG, TQL>(a, s);
        case 7: return launch_trir_l<7, SEG, TQL>(a, s);
        case 8: return launch_trir_l<8, SEG, TQL>(a, s);
        case 9: return launch_trir_l<9, SEG, TQL>(a, s);
        case 10: return launch_trir_l<10, SEG, TQL>(a, s);
    }
    return false;
}

// The last-dimension pass of 3-D / 4-D meshes (16-line tiles in tri_tiles) by the factorised line solve. Tiles, where
// the lines fill >= 256 workgroups of 64: 64 lines (512-B rows per wave load) of 32-row segments up to 256-point lines
// (256 / 512 threads), 32 lines of 16-row segments (1024 threads, 64 VGPRs: two workgroups a CU) at 512, 32 lines of
// 32-row segments at 1024; 16 lines of 16-row segments otherwise. Against k_tri (round 6, one box, kernel trace,
// profiles/r06/v1_trir): 512^3 441 -> 392 us, 256^3 73 -> 49 us, 128^4 948 -> 797 us. Probe builds: MVTV_TRI_IIR=0
// takes k_tri, "SEG,TQ" forces a tile.
static bool launch_trir(SpecArgs& a, hipStream_t s) {
    static const int cfg = [] {
        const char* e = probe_env("MVTV_TRI_IIR");
        if (!e) return -1;
        int sg = 0, tq = 0;
        if (std::sscanf(e, "%d,%d", &sg, &tq) != 2) return 0;
        return sg * 1000 + tq;
    }();
    switch (cfg) {
        case -1: break;
        case 32064: return launch_trir_seg<32, 64>(a, s);
        case 16064: return launch_trir_seg<16, 64>(a, s);
        case 16032: return launch_trir_seg<16, 32>(a, s);
        case 32032: return launch_trir_seg<32, 32>(a, s);
        case 32016: return launch_trir_seg<32, 16>(a, s);
        case 16016: return launch_trir_seg<16, 16>(a, s);
        default: return false;
    }
    if (a.nlines / 64u >= 256u && a.stride >= 64u) {
        if (a.L <= 8) return launch_trir_seg<32, 64>(a, s);
        if (a.L == 9) return launch_trir_seg<16, 32>(a, s);
        return launch_trir_seg<32, 32>(a, s);
    }
    return launch_trir_seg<16, 16>(a, s);
}

static void launch_tri(SpecArgs& a, hipStream_t s, int tq) {
    a.tq = tq;
    if (tq == tri::TQ && launch_trir(a, s)) return;
    a.tq = tq;
    a.xcd = 0;
    if (tq == tri::TQ) {
        a.xcd = 0;
        static const int seg = [] {
            const char* e = probe_env("MVTV_TRI_SEG");
            return e && std::atoi(e) == 32 ? 32 : 16;
        }();
        // 64 lines of 32-row segments per workgroup (512-B rows: one full run per load instruction of a wave) where
        // the lines fill >= 256 such workgroups: 512^3 k_tri ~0.49 -> ~0.44 ms, 170.1 / 170.5 -> 171.8 / 172.0 ADMM it/s
        // on one box (profiles/r04/v18_tri64). Probe builds: MVTV_TRI_TQ=16 / 32 force the 16- / 32-line tiles.
        static const int tqw = [] {
            const char* e = probe_env("MVTV_TRI_TQ");
            return e ? std::atoi(e) : 64;
        }();
        if (tqw == 32 && seg == 16 && a.stride >= 32u) {
            a.tq = 32;
            launch_tri_seg<16, 32>(a, s);
        } else if (tqw == 64 && seg == 16 && a.stride >= 64u && a.L >= 7 && a.L <= 9 && a.nlines / 64u >= 256u) {
            a.tq = 64;
            const dim3 grid((a.nlines + 63u) / 64u);
            if (a.L == 7) klaunch(k_tri<7, 32, 64>, grid, dim3(tri::Shape<7, 32, 64>::NT), 0, s, a);
            else if (a.L == 8) klaunch(k_tri<8, 32, 64>, grid, dim3(tri::Shape<8, 32, 64>::NT), 0, s, a);
            else klaunch(k_tri<9, 32, 64>, grid, dim3(tri::Shape<9, 32, 64>::NT), 0, s, a);
        } else if (seg == 32) {
            launch_tri_seg<32, tri::TQ>(a, s);
        } else {
            launch_tri_seg<16, tri::TQ>(a, s);
        }
        return;
    }
    a.xcd = 1;   // 2-D: narrow tiles in XCD runs (grid a multiple of 8, tri_tiles)
    const dim3 grid(a.nlines / uint32_t(tq));
    static const bool thomas = [] {
        const char* e = probe_env("MVTV_TRI_IIR");
        return e && std::atoi(e) == 0;
    }();
    if (!thomas) {   // the factorised solve (k_trir): 2048-point lines in 64 segments of 32 rows, else 16-row segments
        if (a.L == 11) {
            if (tq == 4) klaunch(k_trir<11, 32, 4>, grid, dim3(trir::Shape<11, 32, 4>::NT), 0, s, a);
            else klaunch(k_trir<11, 32, 8>, grid, dim3(trir::Shape<11, 32, 8>::NT), 0, s, a);
            return;
        }
        switch (a.L * 16 + tq) {
            case 6 * 16 + 4: klaunch(k_trir<6, 16, 4>, grid, dim3(trir::Shape<6, 16, 4>::NT), 0, s, a); return;
            case 6 * 16 + 8: klaunch(k_trir<6, 16, 8>, grid, dim3(trir::Shape<6, 16, 8>::NT), 0, s, a); return;
            case 7 * 16 + 4: klaunch(k_trir<7, 16, 4>, grid, dim3(trir::Shape<7, 16, 4>::NT), 0, s, a); return;
            case 7 * 16 + 8: klaunch(k_trir<7, 16, 8>, grid, dim3(trir::Shape<7, 16, 8>::NT), 0, s, a); return;
            case 8 * 16 + 4: klaunch(k_trir<8, 16, 4>, grid, dim3(trir::Shape<8, 16, 4>::NT), 0, s, a); return;
            case 8 * 16 + 8: klaunch(k_trir<8, 16, 8>, grid, dim3(trir::Shape<8, 16, 8>::NT), 0, s, a); return;
            case 9 * 16 + 4: klaunch(k_trir<9, 16, 4>, grid, dim3(trir::Shape<9, 16, 4>::NT), 0, s, a); return;
            case 9 * 16 + 8: klaunch(k_trir<9, 16, 8>, grid, dim3(trir::Shape<9, 16, 8>::NT), 0, s, a); return;
            case 10 * 16 + 4: klaunch(k_trir<10, 16, 4>, grid, dim3(trir::Shape<10, 16, 4>::NT), 0, s, a); return;
            case 10 * 16 + 8: klaunch(k_trir<10, 16, 8>, grid, dim3(trir::Shape<10, 16, 8>::NT), 0, s, a); return;
            default: break;
        }
    }
    if (a.L == 11) {   // 2048-point lines: 64 segments of 32 rows
        if (tq == 4) klaunch(k_tri<11, 32, 4>, grid, dim3(tri::Shape<11, 32, 4>::NT), 0, s, a);
        else klaunch(k_tri<11, 32, 8>, grid, dim3(tri::Shape<11, 32, 8>::NT), 0, s, a);
    } else if (tq == 4) {
        launch_tri_seg<16, 4>(a, s);
    } else {
        launch_tri_seg<16, 8>(a, s);
    }
}

// ------------------------------------------------------------------------------ launcher
// One k_dct8 pass with TQW real lines per workgroup (NT = TQW / 2 * m / 8 threads).
// (tq < TQW: narrow meshes whose stride is below the tile; the extra lanes idle)
template <int L, int TQW>
static void launch_dct8_tile(SpecArgs& a, hipStream_t s, int mode, bool d0, bool formb, int tq = TQW) {
    a.tq = tq;
    const uint32_t grid = (a.nlines + uint32_t(tq) - 1) / uint32_t(tq);
    a.xcd = a.xcd && (grid & 7u) == 0u;
    const dim3 block(spec8::ShapeK<L, TQW>::NT);
    if constexpr (L >= 6 && spec8::ShapeK<L, TQW>::NT >= 64) {
        if (a.pf.mode) {   // PCG-fused d = 0 passes (dct_pcg_fusable)
            if (a.pf.mode == 2 && 2 * size_t(grid) > a.pf.cap) {   // the rows would overrun the partials
                *a.pf.nparts = -1;
                return;
            }
            if (a.pf.nparts) *a.pf.nparts = int(grid);
            if (a.pf.mode == 1) klaunch(k_dct8<L, SPEC_FWD, true, false, TQW, 1>, dim3(grid), block, 0, s, a);
            else klaunch(k_dct8<L, SPEC_INV, true, false, TQW, 2>, dim3(grid), block, 0, s, a);
            return;
        }
    }
#define MVTV_DCT8(MODE, D0, FB) klaunch(k_dct8<L, MODE, D0, FB, TQW>, dim3(grid), block, 0, s, a)
    if (mode == SPEC_FWD) {
        if (d0) {
            if (formb) MVTV_DCT8(SPEC_FWD, true, true);
            else MVTV_DCT8(SPEC_FWD, true, false);
        } else if (formb) {   // the first pass of a k_march solve (dim 2 first)
            MVTV_DCT8(SPEC_FWD, false, true);
        } else {
            MVTV_DCT8(SPEC_FWD, false, false);
        }
    } else if (mode == SPEC_INV) {
        if (d0) MVTV_DCT8(SPEC_INV, true, false);
        else MVTV_DCT8(SPEC_INV, false, false);
    } else {
        if (d0) {
            if (formb) MVTV_DCT8(SPEC_MID, true, true);
            else MVTV_DCT8(SPEC_MID, true, false);
        } else {
            MVTV_DCT8(SPEC_MID, false, false);
        }
    }
#undef MVTV_DCT8
}

// tile sizes a pass may take: a power of two in [max(2, 1024 / m), 16 * 2^(L <= 9 ? 1 : 0)], with
// NT = TQW / 2 * m / 8 in [64, 1024] and <= ~150 KB of LDS
template <int L>
constexpr bool tile_ok(int tq) {
    constexpr int M = 1 << L;
    return tq >= 2 && (tq / 2) * (M / 8) >= 64 && (tq / 2) * (M / 8) <= 1024 &&
           (tq / 2) * spec8::Shape<L>::LP * 16 <= 152 * 1024;
}
template <int L, int TQW>
static bool try_tile(SpecArgs& a, hipStream_t s, int mode, bool d0, bool formb, int want) {
    if constexpr (tile_ok<L>(TQW)) {
        if (want == TQW) {
            launch_dct8_tile<L, TQW>(a, s, mode, d0, formb);
            return true;
        }
    }
    return false;
}

// Tile choice. Default: 16 lines (128-B rows for d > 0) up to 512 points per line, then 8 / 4 / 2 for
// 1024 / 2048 / 4096 (LDS); strided passes of 1024 - 4096-point lines twice that (one ~148-KB workgroup
// per CU: 2048^2 strided passes 49 -> 28 us, 3670 -> 4320 ADMM it/s). Meshes with few lines (2-D) would
// leave CUs idle with those tiles: a d = 0 pass under 1024 workgroups takes the smallest tile (>= one wave),
// a strided pass under 128 wide workgroups takes 4 lines (32-B rows) with the tiles dealt to the XCDs in
// contiguous runs, so the 4 tiles of a 128-B row share one L2. 1024^2: 8355 -> 9650 ADMM it/s (d = 0
// passes 17.5 -> 14.8 us, strided 18.7 -> 11.8 us); 2048^2: 4797 -> 4862 (profiles/r02/v17_dct_tiles).
// Probe builds: MVTV_DCT_T0 / _T1 set the d = 0 / d > 0 tile, MVTV_DCT_XCD=0/1 the XCD runs.
template <int L>
static void launch_dct8(SpecArgs& a, hipStream_t s, int mode, bool d0, bool formb) {
    using S = spec8::Shape<L>;
    constexpr int TMIN = tile_ok<L>(2) ? 2 : (tile_ok<L>(4) ? 4 : (tile_ok<L>(8) ? 8 : 16));
    int want = S::TQ;
    bool xcd_def = false;
    if (d0) {
        if (a.nlines / uint32_t(S::TQ) < 1024u) want = std::min(TMIN, S::TQ);
    } else {
        // strided passes: tiles in XCD runs (512^3: the dim-1 passes' bucket 0.436 -> 0.405 ms, 174.7 / 174.6 ->
        // 178.3 / 178.3 ADMM it/s on one box, profiles/r05/v16_dct8_xcd; the d = 0 passes stay round-robin there)
        xcd_def = true;
        if (L >= 10 && L <= 12 && 2 * S::TQ <= int(a.stride)) {
            want = 2 * S::TQ;
            if (a.nlines / uint32_t(want) < 128u && tile_ok<L>(4) && int(a.stride) >= 4) want = 4;
        }
    }
    // (probe builds read these per launch, so a probe can vary them within one process)
    const char* e0 = probe_env("MVTV_DCT_T0");
    const char* e1 = probe_env("MVTV_DCT_T1");
    const char* ex = probe_env("MVTV_DCT_XCD");
    const int t0 = e0 ? std::atoi(e0) : 0, t1 = e1 ? std::atoi(e1) : 0, xcd_env = ex ? std::atoi(ex) : -1;
    if (d0 && t0 > 0) want = t0;
    if (!d0 && t1 > 0) want = t1;
    if (!d0) want = std::min<int>(want, int(a.stride));
    a.xcd = xcd_env >= 0 ? xcd_env : (xcd_def ? 1 : 0);
    if (try_tile<L, 2>(a, s, mode, d0, formb, want) || try_tile<L, 4>(a, s, mode, d0, formb, want) ||
        try_tile<L, 8>(a, s, mode, d0, formb, want) || try_tile<L, 16>(a, s, mode, d0, formb, want) ||
        try_tile<L, 32>(a, s, mode, d0, formb, want))
        return;
    a.xcd = 0;
    launch_dct8_tile<L, S::TQ>(a, s, mode, d0, formb, std::min(want, S::TQ));   // the default tile
}

// the fused in-plane passes (k_plane8): m0 = m1 = 2^L, 16 <= m <= 128, dims 0 and 1 transformed first
bool plane_pass_ok(const Geom& g) {
    if (g.p < 3 || g.m[0] != g.m[1] || probe_env("MVTV_PLANE_OFF") || probe_env("MVTV_DCT_LDS") ||
        probe_env("MVTV_DCT_MID"))
        return false;
    // and enough planes to fill the chip: 128^3's 128 planes (one workgroup each) ran 1 % slower than the two
    // passes, 128^4's 16384 3.5 % faster per ADMM iteration (profiles/r03/v15_plane)
    const uint32_t m = g.m[0];
    return m >= 16 && m <= 128 && (m & (m - 1)) == 0 && g.N / (uint64_t(m) * m) >= 1024;
}

// mode SPEC_FWD (dims 0 then 1; b formed on load when ga != nullptr, from the folded s when fold) or SPEC_INV
// (dims 1 then 0), in place over every (dim 0, dim 1) plane of g
hipError_t launch_plane_pass(const SpecPlan& sp, const Geom& g, hipStream_t s, int mode, const double* in,
                             const double* ga, double ca, const double* gb, double cb, double* out,
                             const AdmmCtl* ctl, const int32_t* skip, bool fold) {
    if (!plane_pass_ok(g) || (mode != SPEC_FWD && mode != SPEC_INV) || (mode == SPEC_INV && ga) ||
        (fold && (!ga || !gb || !ctl)))
        return hipErrorInvalidValue;
    SpecArgs a{};
    a.ctl = ctl;
    a.skip = skip;
    a.in = in;
    a.ga = ga;
    a.gb = gb ? gb : ga;
    a.ca = ca;
    a.cb = gb ? cb : 0.0;
    a.out = out;
    a.tw = reinterpret_cast<const double2*>(sp.tw + sp.tw_off[0]);    // m0 = m1: one table serves both dims
    a.twq = reinterpret_cast<const double2*>(sp.twq + sp.twq_off[0]);
    a.fold = fold ? 1 : 0;
    const uint32_t m = g.m[0];
    const uint32_t nplanes = g.N / (m * m);
    // persistent over the planes: one workgroup per CU (the plane's 152 KB of LDS) at m = 128, so the next
    // plane's loads overlap the transforms; smaller planes keep one workgroup per plane
    static thread_local int dev = -1, cus = 256;
    int dv = 0;
    if (hipGetDevice(&dv) == hipSuccess && dv != dev) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, dv) == hipSuccess && prop.multiProcessorCount > 0) cus = prop.multiProcessorCount;
        dev = dv;
    }
    const dim3 grid(m == 128 ? std::min<uint32_t>(nplanes, uint32_t(cus)) : nplanes);
    const bool formb = ga != nullptr;
#define MVTV_PLANE(LL)                                                                                          \
    do {                                                                                                        \
        const dim3 block((1u << LL) / 2 * (1u << LL) / 8);                                                      \
        if (mode == SPEC_INV) klaunch(k_plane8<LL, SPEC_INV, false>, grid, block, 0, s, a, nplanes);            \
        else if (formb) klaunch(k_plane8<LL, SPEC_FWD, true>, grid, block, 0, s, a, nplanes);                   \
        else klaunch(k_plane8<LL, SPEC_FWD, false>, grid, block, 0, s, a, nplanes);                             \
    } while (0)
    switch (m) {
        case 16: MVTV_PLANE(4); break;
        case 32: MVTV_PLANE(5); break;
        case 64: MVTV_PLANE(6); break;
        case 128: MVTV_PLANE(7); break;
        default: return hipErrorInvalidValue;
    }
#undef MVTV_PLANE
    return hipGetLastError();
}

// 3-D meshes whose dim-0 lines are 256 - 2048 points (a power of two) and enough dim-2 planes to fill the chip:
// dim 2 first, then the marching dim-0 transform + dim-1 tridiagonal passes (k_march). Probe builds only
// (MVTV_MARCH=1): it moves 9N words per solve instead of 11N, but its two dim-2 passes stride 2 MB (the first one
// reading three inputs) and run slower than the dim-0 / dim-1 passes they replace, and the march itself, one
// workgroup per dim-2 plane (8 waves per CU at 512^3), reaches 3.7 TB/s: 512^3 162.5-163.4 ADMM it/s against
// 165.1-165.8 for the five-pass solve, 165.2-166.4 with 32-line strided tiles, 256^3 1150 against 1170, same
// process, interleaved (profiles/r04/v2_march).
bool march_ok(const Geom& g) {
    const char* on = probe_env("MVTV_MARCH");
    if (!on || std::atoi(on) == 0) return false;
    if (g.p != 3 || probe_env("MVTV_DCT_LDS") || probe_env("MVTV_DCT_MID")) return false;
    const uint32_t m0 = g.m[0];
    if (m0 < 256 || m0 > 2048 || (m0 & (m0 - 1)) != 0) return false;
    const uint32_t nr = 2u * (2048u / m0);
    return g.m[1] % nr == 0 && g.m[2] >= 128 && g.m[2] <= 4096;
}

hipError_t launch_march(const SpecPlan& sp, const Geom& g, hipStream_t s, bool bwd, double* x, double sigma, double w0,
                        const AdmmCtl* ctl, const int32_t* skip) {
    if (!march_ok(g)) return hipErrorInvalidValue;
    SpecArgs a{};
    a.ctl = ctl;
    a.skip = skip;
    a.in = x;
    a.out = x;
    a.tw = reinterpret_cast<const double2*>(sp.tw + sp.tw_off[0]);
    a.twq = reinterpret_cast<const double2*>(sp.twq + sp.twq_off[0]);
    a.lam = sp.lam;
    for (int j = 0; j < kMaxDims; ++j) {
        a.lam_off[j] = sp.lam_off[j];
        a.m[j] = g.m[j];
    }
    for (int S = 0; S < 16; ++S) a.cS[S] = g.cS[S];
    a.sigma = sigma;
    a.w0 = w0;
    a.inv_n = 1.0 / double(g.N);
    const dim3 grid(g.m[2]), block(256);
#define MVTV_MARCH(LL)                                                                                         \
    do {                                                                                                       \
        if (bwd) klaunch(k_march<LL, true>, grid, block, 0, s, a, g.m[1]);                                     \
        else klaunch(k_march<LL, false>, grid, block, 0, s, a, g.m[1]);                                        \
    } while (0)
    switch (g.m[0]) {
        case 256: MVTV_MARCH(8); break;
        case 512: MVTV_MARCH(9); break;
        case 1024: MVTV_MARCH(10); break;
        case 2048: MVTV_MARCH(11); break;
        default: return hipErrorInvalidValue;
    }
#undef MVTV_MARCH
    return hipGetLastError();
}

bool dct_pcg_fusable(const Geom& g, size_t partial_words) {
    const uint32_t m = g.m[0];
    if (g.p < 2 || m < 64 || m > 4096 || (m & (m - 1)) != 0 || probe_env("MVTV_DCT_LDS") || probe_env("MVTV_PCGS_NINE"))
        return false;
    // partial rows of the last pass: one per tile of launch_dct8's d = 0 choice (16 lines up to m = 512,
    // 8192 / m beyond; the smallest one-wave tile, >= 1024 / m lines, when that leaves < 1024 tiles)
    const size_t nlines = g.N / m, tq = std::min<size_t>(16, 8192 / m);
    const size_t tmin = std::max<size_t>(2, 1024 / m);
    const size_t rows = nlines / tq >= 1024 ? (nlines + tq - 1) / tq : (nlines + tmin - 1) / tmin;
    return 2 * rows <= partial_words;
}

hipError_t launch_dct_pass(const SpecPlan& sp, const Geom& g, hipStream_t s, int mode, int d, const double* in,
                           const double* ga, double ca, const double* gb, double cb, double* out, double sigma,
                           double w0, const AdmmCtl* ctl, uint32_t q_off, double inv_n, const int32_t* skip,
                           const PcgFuse* pf, bool fold) {
    SpecArgs a{};
    a.ctl = ctl;
    a.skip = skip;
    a.q_off = q_off;
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
    a.inv_n = inv_n > 0.0 ? inv_n : 1.0 / double(g.N);   // 1 / (all mesh points): the inverse transforms' scale
    a.stride = g.stride[d];
    a.ls = 0;
    while ((1u << a.ls) < a.stride) ++a.ls;
    const uint32_t m = g.m[d];
    a.nlines = g.N / m;
    a.d = d;
    a.p = g.p;
    a.L = 0;
    while ((1u << a.L) < m) ++a.L;
    const bool formb = ga != nullptr;
    a.fold = fold ? 1 : 0;   // b from the folded s: k_dct8 (power-of-two m >= 8), asynchronous loop only
    static const bool pair16 = [] {   // probe builds: MVTV_DCT_P16=0 keeps the d = 0 passes' 8-B coefficient accesses
        const char* e = probe_env("MVTV_DCT_P16");
        return !(e && std::atoi(e) == 0);
    }();
    a.pair16 = pair16 ? 1 : 0;
    if (m > 4096) return hipErrorInvalidValue;
    if (a.fold && (!formb || !gb || !ctl || (1u << a.L) != m || (1u << a.ls) != a.stride || a.L < 3 ||
                   probe_env("MVTV_DCT_LDS") || mode == SPEC_MID))
        return hipErrorInvalidValue;
    if (pf && pf->mode) {   // PCG-fused d = 0 pass (dct_pcg_fusable meshes): k_dct8 only
        if (d != 0 || formb || (1u << a.L) != m || a.L < 6 || mode != (pf->mode == 1 ? SPEC_FWD : SPEC_INV) ||
            (pf->mode == 2 && !pf->nparts))
            return hipErrorInvalidValue;
        a.pf = *pf;
    }
    if ((1u << a.L) != m || (1u << a.ls) != a.stride) {   // mixed radix, or a power of two over a general stride
        const bool planned = dct_radix_plan(m, a.rad, &a.nrad);
        if (!planned && sp.blu_M[d] == 0) return hipErrorInvalidValue;
        a.fds = FastDiv(a.stride);
        a.fm = FastDiv(m);
        if (planned) {
            for (int st = 0, L = 1; st < a.nrad; ++st) {
                a.fper[st] = FastDiv(m / uint32_t(a.rad[st]));
                a.fL[st] = FastDiv(uint32_t(L));
                L *= a.rad[st];
            }
            a.perm = sp.perm + sp.lam_off[d];
        }
        static const bool few_off = probe_flag("MVTV_FEW_LINES_OFF");
        // strided passes: tiles in XCD runs (probe builds: MVTV_XRUN_OFF=1 deals them round-robin)
        static const bool xrun_off = probe_flag("MVTV_XRUN_OFF");
        a.xrun = (d > 0 && !xrun_off) ? 1 : 0;
        // the line solve along the last dimension also for the few lines of a 2-D mesh, on 4-line tiles where that
        // makes >= 250 workgroups (a Bluestein MID pass is four FFTs of twice the length per line pair): 2039^2 2070 ->
        // 3310 ADMM it/s, 1009^2 8431 -> 9086, 1000^2 10682 -> 11017; 500^2 (125 such tiles) 16059 -> 15855 keeps the
        // MID pass (profiles/r05/v15_trig_2d; probe builds: MVTV_TRIG_FEW_OFF=1)
        static const bool trig_few_off = probe_flag("MVTV_TRIG_FEW_OFF");
        const bool trig_lines = a.nlines / uint32_t(trig::TQ) >= 256u || (!trig_few_off && a.nlines >= 1000u);
        if (mode == SPEC_MID && d > 0 && !formb && trig_lines && !probe_env("MVTV_DCT_TRI0")) {
            int sl = trig_seg(m);
            // more than 16 segments keep k_trig on 32-line tiles; where 64-line tiles fill the chip, <= 32-row
            // segments with a shorter last one bring it to 16 (500: 25 x 20 -> 15 x 32 + 20 rows, 0.69 -> 0.48 ms
            // at 500^3, profiles/r05/v13_trig_sl32; probe builds: MVTV_TRIG_SL forces, MVTV_TRIG_NARROW keeps)
            static const bool sl_forced = probe_env("MVTV_TRIG_SL") != nullptr;
            if (sl > 0 && !sl_forced && (m + uint32_t(sl) - 1) / uint32_t(sl) > 16u && a.nlines / 64u >= 256u &&
                (m + 15u) / 16u <= uint32_t(trig::SMAX))
                sl = int((m + 15u) / 16u);
            if (sl > 0) {
                const int nseg = int((m + uint32_t(sl) - 1) / uint32_t(sl));
                launch_trig(a, s, sl, nseg, int(m) - (nseg - 1) * sl);
                return hipGetLastError();
            }
        }
        if (!planned) {   // Bluestein (k_dctb): L = log2 M, the length-M twiddles
            const double2* t = reinterpret_cast<const double2*>(sp.blu + sp.blu_off[d]);
            a.L = 0;
            while ((1u << a.L) < sp.blu_M[d]) ++a.L;
            a.bchirp = t;
            a.bvf = t + m;
            a.bvi = t + m + sp.blu_M[d];
            a.tw = t + m + 2 * sp.blu_M[d];
            return launch_dctb(a, s, mode, d == 0, formb);
        }
        if (launch_dctm(a, s, mode, d == 0, formb)) return hipGetLastError();
        // <= 16 lines (128-B rows for d > 0) in <= 64 KB of LDS; few lines (a 2-D mesh: 1000 lines of 1000) take
        // smaller tiles until the grid has >= 512 workgroups (two a CU) or the tile two lines (probe builds:
        // MVTV_FEW_LINES_OFF=1 keeps the LDS-sized tile)
        int tq = 16;
        while (tq > 2 && (tq / 2) * int(m + spec::PAD) > spec::LDS_WORDS / 2 + 8 * spec::PAD) tq /= 2;
        if (!few_off) tq = few_lines_tq(a.nlines, tq, 2);
        a.tq = tq;
        launch_dctg(a, s, mode, d == 0, formb);
        return hipGetLastError();
    }
    if (const int tq = tri_tiles(a, mode, formb)) {
        launch_tri(a, s, tq);
        return hipGetLastError();
    }
    if (a.L >= 3 && !probe_env("MVTV_DCT_LDS")) {
        switch (a.L) {
            case 3: launch_dct8<3>(a, s, mode, d == 0, formb); break;
            case 4: launch_dct8<4>(a, s, mode, d == 0, formb); break;
            case 5: launch_dct8<5>(a, s, mode, d == 0, formb); break;
            case 6: launch_dct8<6>(a, s, mode, d == 0, formb); break;
            case 7: launch_dct8<7>(a, s, mode, d == 0, formb); break;
            case 8: launch_dct8<8>(a, s, mode, d == 0, formb); break;
            case 9: launch_dct8<9>(a, s, mode, d == 0, formb); break;
            case 10: launch_dct8<10>(a, s, mode, d == 0, formb); break;
            case 11: launch_dct8<11>(a, s, mode, d == 0, formb); break;
            case 12: launch_dct8<12>(a, s, mode, d == 0, formb); break;
        }
        if (pf && pf->mode == 2 && *pf->nparts < 0) return hipErrorInvalidValue;
        return hipGetLastError();
    }
    int tq = std::max(2, std::min(16, int(spec::LDS_WORDS / m)));
    if (d > 0) tq = std::min<int>(tq, int(g.stride[d]));
    if (tq < 2) return hipErrorInvalidValue;
    a.tq = tq;
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

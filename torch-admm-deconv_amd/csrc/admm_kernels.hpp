// admm_kernels.hpp -- HIP kernels of the MI355X ADMM-TV solver (gfx950).
//
// Data layout in HBM (P = B*C planes, N = W/2):
//   images  float [P][H][W]      (xin, b, u_x, u_y, out)
//   spectra cf    [P][H][N]      packed real row spectra: element 0 holds
//                                (X[0], X[N]) (DC and Nyquist are real), 1..N-1 hold X[k].
//                                Exactly H*W floats per plane, rows 8N-byte aligned.
//   fcT     float [N+1][H]       Wiener factor / (2HW), transposed (column-major in ky)
//   mT      cf    [N+1][H]       centred-PSF spectrum / (2HW), transposed
//
// One ADMM iteration (deconv.py:103-115) is
//   pass B  (column pass, in place): spec = colIFFT( fc * colFFT(spec) )   -> x row spectra
//   pass A  (row pass): x = rowIFFT(spec) (+1 halo row each side), Dx, Dy, shrink,
//           dual update of u (ping-pong), v = Dx^T w_x + Dy^T w_y with w = z - u,
//           r = b + rho v, spec' = rowFFT(r)
// The row transform scaling is folded into fcT / mT.
#pragma once
#include "fft_core.hpp"

namespace admm {

// ---------------------------------------------------------------------------
// packed real-row transforms for one sub-group of L lanes (natural layout)
// ---------------------------------------------------------------------------
// Cfg: values per lane E and the radix schedule S (RowCfg<N> by default; the training backward's row
// pass runs the 256-point rows with fewer values per lane, admm_backward.hpp BwdCfg)
template <int N, class Cfg = RowCfg<N>> struct RowXf {
    static constexpr int E = Cfg::E;
    static constexpr int L = N / E;
    static constexpr int W = 2 * N;
    static_assert(L <= 64, "row transforms keep one row inside one wave");

    // p[j] = v at index N - (t + L j)  (j = 0 at t = 0 is the DC slot; unused)
    __device__ __forceinline__ static void partner(const cf (&v)[E], cf (&p)[E], int t) {
        const int src = (L - t) & (L - 1);
#pragma unroll
        for (int j = 0; j < E; ++j) {
            float a = __shfl(v[E - 1 - j].x, src, L);
            float b = __shfl(v[E - 1 - j].y, src, L);
            p[j] = (t == 0) ? v[(E - j) & (E - 1)] : mkc(a, b);
        }
    }

    // packed spectrum (== 2*rfft of a real row y) -> pixel pairs (2W * y).
    // tw: exp(-2 pi i k / W), k in [0, W)  (LDS)
    __device__ __forceinline__ static void c2r(cf (&v)[E], const RowBuf& buf, const cf* __restrict__ tw, int t) {
        cf p[E];
        partner(v, p, t);
#pragma unroll
        for (int j = 0; j < E; ++j) {
            const int k = t + L * j;
            cf z;
            if (j == 0 && t == 0) {
                z = mkc(v[0].x + v[0].y, v[0].x - v[0].y);
            } else {
                cf pc = cconj(p[j]);
                cf e = cadd(v[j], pc);
                cf o = cmulc(csub(v[j], pc), tw[k]);  // * exp(+2 pi i k/W)
                z = mkc(e.x - o.y, e.y + o.x);         // e + i o
            }
            v[j] = z;
        }
        fft_e<N, L, E, +1, 0, 2>(v, buf, tw, t, typename Cfg::S{});
    }

    // pixel pairs of a real row r -> packed spectrum 2*rfft(r)
    __device__ __forceinline__ static void r2c(cf (&v)[E], const RowBuf& buf, const cf* __restrict__ tw, int t) {
        fft_e<N, L, E, -1, 0, 2>(v, buf, tw, t, typename Cfg::S{});
        cf p[E];
        partner(v, p, t);
#pragma unroll
        for (int j = 0; j < E; ++j) {
            const int k = t + L * j;
            cf z;
            if (j == 0 && t == 0) {
                z = mkc(2.f * (v[0].x + v[0].y), 2.f * (v[0].x - v[0].y));
            } else {
                cf pc = cconj(p[j]);
                cf s = cadd(v[j], pc);
                cf d = cmul(csub(v[j], pc), tw[k]);  // w^k (Z - conj Z~)
                z = mkc(s.x + d.y, s.y - d.x);        // s - i d
            }
            v[j] = z;
        }
    }
};

// soft shrink  sign(a) max(|a| - tau, 0)   (deconv.py:15-16); NaN propagates
__device__ __forceinline__ float soft(float a, float tau) {
    float m = fabsf(a) - tau;
    m = (m < 0.f) ? 0.f : m;
    return copysignf(m, a);
}
// block-shrink factor max(1 - tau/(sqrt(s + 1e-15) + 1e-15), 0)   (deconv.py:19-24)
__device__ __forceinline__ float block_factor(float sumsq, float tau) {
    float n = sqrtf(sumsq + 1e-15f);
    float f = 1.f - tau / (n + 1e-15f);
    return f < 0.f ? 0.f : f;
}
// the reference's 1e-15 (deconv.py:20,24) in the solve's precision
template <class T> __device__ __forceinline__ constexpr T eps15() {
    if constexpr (std::is_same<T, float>::value) return 1e-15f;
    else return 1e-15;
}
// fp64 (the generic kernels' double instantiation)
__device__ __forceinline__ double soft(double a, double tau) {
    double m = fabs(a) - tau;
    m = (m < 0.0) ? 0.0 : m;
    return copysign(m, a);
}
__device__ __forceinline__ double block_factor(double sumsq, double tau) {
    double n = sqrt(sumsq + 1e-15);
    double f = 1.0 - tau / (n + 1e-15);
    return f < 0.0 ? 0.0 : f;
}

// ---------------------------------------------------------------------------
// setup kernels
// ---------------------------------------------------------------------------
// twiddle tables: twW[k] = exp(-2 pi i k/W) (k < W), twH[k] = exp(-2 pi i k/H) (k < H),
// twHd in fp64 for the PSF spectrum.
// (C = cd: the fp64 solve keeps the tables in fp64)
template <class C = cf>
__global__ void k_tables(C* __restrict__ twW, C* __restrict__ twH, double2* __restrict__ twHd, int H, int W) {
    using T = re_t<C>;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < W) {
        double s, c;
        sincospi(2.0 * i / W, &s, &c);
        twW[i] = mkx<T>((T)c, (T)-s);
    }
    if (i < H) {
        double s, c;
        sincospi(2.0 * i / H, &s, &c);
        twH[i] = mkx<T>((T)c, (T)-s);
        twHd[i] = make_double2(c, -s);
    }
}

// G[a][kx] = sum_b kern[a][b] exp(-2 pi i b kx / W), kx in [0, N], in fp64
template <class T = float>
__global__ void k_psf_rows(const T* __restrict__ kern, double2* __restrict__ G, int k, int N, int W) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= k * (N + 1)) return;
    const int a = i / (N + 1), kx = i % (N + 1);
    double re = 0.0, im = 0.0;
    for (int b = 0; b < k; ++b) {
        const long long m = ((long long)b * kx) % W;
        double s, c;
        sincospi(2.0 * (double)m / W, &s, &c);
        const double w = (double)kern[a * k + b];
        re += w * c;
        im -= w * s;
    }
    G[i] = make_double2(re, im);
}

// fcT[kx][ky] = scale / (|sigma|^2 + rho (|Dx^|^2 + |Dy^|^2));
// mT[kx][ky] = scale * sigma * exp(+2 pi i c (ky/H + kx/W))  (centred PSF, c = k/2)
// scale = 1/(2HW) for the packed power-of-two path, 1/(HW) for the generic path
template <class T = float>
__global__ void k_spectra(const double2* __restrict__ G, const double2* __restrict__ twHd,
                          const T* __restrict__ rho_p, T* __restrict__ fcT, cx_t<T>* __restrict__ mT, int k,
                          int H, int N, int W, double2* __restrict__ sigma_out, double scale) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (N + 1) * H) return;
    const int kx = i / H, ky = i % H;
    double sr = 1.0, si = 0.0;
    if (k > 0) {
        sr = 0.0;
        for (int a = 0; a < k; ++a) {
            const double2 w = twHd[((long long)a * ky) % H];
            const double2 g = G[a * (N + 1) + kx];
            sr += w.x * g.x - w.y * g.y;
            si += w.x * g.y + w.y * g.x;
        }
    }
    if (sigma_out) sigma_out[i] = make_double2(sr, si);  // kept for the PSF gradient
    const double rho = (double)rho_p[0];
    const double sx = sinpi((double)kx / W), sy = sinpi((double)ky / H);
    const double lap = 4.0 * sx * sx + 4.0 * sy * sy;
    fcT[i] = (T)(scale / (sr * sr + si * si + rho * lap));
    if (k > 0) {
        const int c = k / 2;  // ceil((k-1)/2): anchor of the reference's H_t
        const long long ph = (long long)c * ky * W + (long long)c * kx * H;  // units of 1/(H W)
        const long long HW = (long long)H * W;
        double s, co;
        sincospi(2.0 * (double)(ph % HW) / (double)HW, &s, &co);
        mT[i] = mkx<T>((T)((sr * co - si * s) * scale), (T)((sr * s + si * co) * scale));
    }
}

// ---------------------------------------------------------------------------
// row transforms of whole images (one sub-group of L lanes per row)
// ---------------------------------------------------------------------------
template <int N> struct RowKernelGeom {
    static constexpr int E = RowCfg<N>::E, L = N / E, W = 2 * N;
    static constexpr int NT = 256, SG = NT / L;
    static constexpr size_t lds_bytes() { return sizeof(cf) * (W + SG * RowBuf::slots(N)); }
};

__device__ __forceinline__ void load_tw(cf* dst, const cf* __restrict__ src, int n) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
}

// ---------------------------------------------------------------------------
// Row layouts of the internal images (u_x, u_y, b, iso norm maps).  A sub-group lane t holds the
// pixel pairs t + L j (j < E) of a row ("natural layout").  PL = false stores them in pixel
// order (8-byte accesses, one per pair).  PL = true ("lane-paired") stores the two pairs a lane
// handles in consecutive registers 2j', 2j'+1 next to each other: float4 slot t + L j' of the row
// holds pairs t + 2j' L and t + (2j'+1) L, so every such stream moves 16 bytes per lane and
// instruction (half the instructions; pass A's access pattern: 1.014 -> 0.955 ms in
// tools/membench/stream_mimic U4_SWEEP).  A pure permutation inside each row: used for the
// workspace images of the inference path, never for the caller's tensors or the training history.
// ---------------------------------------------------------------------------
typedef float f4v __attribute__((ext_vector_type(4)));
template <int E, int L, bool PL, bool NT> __device__ __forceinline__ void ld_row(const cf* row, int t, cf (&v)[E]) {
    if constexpr (PL) {
        static_assert(E % 2 == 0, "lane-paired rows need an even number of values per lane");
        const f4v* r4 = reinterpret_cast<const f4v*>(row);
#pragma unroll
        for (int j = 0; j < E / 2; ++j) {
            const f4v q = NT ? __builtin_nontemporal_load(&r4[t + L * j]) : r4[t + L * j];
            v[2 * j] = mkc(q.x, q.y);
            v[2 * j + 1] = mkc(q.z, q.w);
        }
    } else {
#pragma unroll
        for (int j = 0; j < E; ++j) v[j] = ld_pol<NT>(&row[t + L * j]);
    }
}
template <int E, int L, bool PL, bool NT> __device__ __forceinline__ void st_row(cf* row, int t, const cf (&v)[E]) {
    if constexpr (PL) {
        f4v* r4 = reinterpret_cast<f4v*>(row);
#pragma unroll
        for (int j = 0; j < E / 2; ++j) {
            const f4v q = {v[2 * j].x, v[2 * j].y, v[2 * j + 1].x, v[2 * j + 1].y};
            if constexpr (NT) __builtin_nontemporal_store(q, &r4[t + L * j]);
            else r4[t + L * j] = q;
        }
    } else {
#pragma unroll
        for (int j = 0; j < E; ++j) st_pol<NT>(&row[t + L * j], v[j]);
    }
}

// real rows -> packed row spectra
template <int N, bool PL>
__global__ void __launch_bounds__(256) k_row_r2c(const float* __restrict__ img, cf* __restrict__ spec,
                                                 const cf* __restrict__ twW_g, long long rows) {
    using G = RowKernelGeom<N>;
    constexpr int E = G::E, L = G::L;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    cf* tw = reinterpret_cast<cf*>(smem);
    load_tw(tw, twW_g, G::W);
    __syncthreads();
    const int sgl = threadIdx.x / L, t = threadIdx.x % L;
    const long long row = (long long)blockIdx.x * G::SG + sgl;
    if (row >= rows) return;
    RowBuf buf{tw + G::W + sgl * RowBuf::slots(N)};
    const cf* src = reinterpret_cast<const cf*>(img + row * G::W);
    cf v[E];
    ld_row<E, L, PL, false>(src, t, v);
    RowXf<N>::r2c(v, buf, tw, t);
    cf* dst = spec + row * N;
#pragma unroll
    for (int j = 0; j < E; ++j) dst[t + L * j] = v[j];
}

// packed row spectra -> real rows
template <int N, bool PL>
__global__ void __launch_bounds__(256) k_row_c2r(const cf* __restrict__ spec, float* __restrict__ img,
                                                 const cf* __restrict__ twW_g, long long rows) {
    using G = RowKernelGeom<N>;
    constexpr int E = G::E, L = G::L;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    cf* tw = reinterpret_cast<cf*>(smem);
    load_tw(tw, twW_g, G::W);
    __syncthreads();
    const int sgl = threadIdx.x / L, t = threadIdx.x % L;
    const long long row = (long long)blockIdx.x * G::SG + sgl;
    if (row >= rows) return;
    RowBuf buf{tw + G::W + sgl * RowBuf::slots(N)};
    const cf* src = spec + row * N;
    cf v[E];
#pragma unroll
    for (int j = 0; j < E; ++j) v[j] = src[t + L * j];
    RowXf<N>::c2r(v, buf, tw, t);
    cf* dst = reinterpret_cast<cf*>(img + row * G::W);
    st_row<E, L, PL, false>(dst, t, v);
}

// real rows in pixel order -> the lane-paired layout (b = xin on the inference path without a PSF)
template <int N>
__global__ void __launch_bounds__(256) k_row_pair(const float* __restrict__ img, float* __restrict__ out, long long rows) {
    using G = RowKernelGeom<N>;
    constexpr int E = G::E, L = G::L;
    const int sgl = threadIdx.x / L, t = threadIdx.x % L;
    const long long row = (long long)blockIdx.x * G::SG + sgl;
    if (row >= rows) return;
    cf v[E];
    ld_row<E, L, false, true>(reinterpret_cast<const cf*>(img + row * G::W), t, v);
    st_row<E, L, true, false>(reinterpret_cast<cf*>(out + row * G::W), t, v);
}

// ---------------------------------------------------------------------------
// pass B: column FFT -> multiply -> column IFFT, in place, C columns per block
// MODE 0: real Wiener factor fcT;  MODE 1: complex multiplier mT (PSF transpose H_t);
// MODE 2: conj(mT) (the adjoint of H_t, for the input gradient)
// ---------------------------------------------------------------------------
// min waves per SIMD for pass B: as many blocks per CU as the LDS admits (<= 2)
constexpr int pb_minw(int nt, size_t lds) {
    return (nt / 64 * ((160 * 1024) / lds >= 2 ? 2 : 1) + 3) / 4 > 4 ? 4
                                                                      : (nt / 64 * ((160 * 1024) / lds >= 2 ? 2 : 1) + 3) / 4;
}

template <int H, int C> struct ColGeom {
    static constexpr int E = RowCfg<H>::E, L = H / E, NT = C * L;
    static constexpr int SYNC = 1;
    static constexpr size_t lds_bytes() { return sizeof(cf) * (H + (size_t)H * C); }
};

// Packed copy of one module's Wiener factors for the column pass: fcP[(kx L + t) E + j] =
// fcT[kx H + t + L j] (the E factors a column-pass thread multiplies, contiguous)
static __global__ void k_fc_pack(const float* __restrict__ fcT, float* __restrict__ fcP, int H, int N, int E) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (N + 1) * H) return;
    const int L = H / E, kx = i / H, r = i % H, t = r / E, j = r % E;
    fcP[i] = fcT[(size_t)kx * H + t + L * j];
}

// XCD-aware remap (T1): blocks are dealt round-robin over the 8 XCDs; give each XCD a
// contiguous range of logical ids so neighbouring column blocks (which share 128-B
// lines of every row) run on the same L2 at about the same time.  Bijective for any nb.
__device__ __forceinline__ unsigned xcd_remap(unsigned b, unsigned nb) {
    const unsigned x = b & 7u, i = b >> 3, q = nb >> 3, r = nb & 7u;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

// Pair-interleaved XCD remap: hardware block b runs on XCD b % 8 at slot b / 8; logical ids are
// handed out so that the two blocks of a line-sharing pair (logical 2i, 2i + 1) run on the same
// XCD in consecutive slots, and the pair index rises with the slot across all XCDs (pair 8k + x
// on XCD x at slots 2k, 2k + 1): the launch walks its tiles in one global order instead of eight
// ranges side by side.  Identity on the last partial group of 16.  Bijective for any nb.
__device__ __forceinline__ unsigned xcd_pairs(unsigned b, unsigned nb) {
    if ((b | 15u) >= nb) return b;
    const unsigned x = b & 7u, s = b >> 3;
    return 2u * (8u * (s >> 1) + x) + (s & 1u);
}

// block -> (plane p, column block cb) in groups of G planes (G = order; 1 = plane-major): inside a
// group, consecutive ids are the two column blocks that share every 128-B line (PAIRS; one block
// column for k_pass_b2, which covers whole lines), then the same columns of the group's next plane.
// With G > 1 the blocks resident on an XCD at a time read G times fewer Wiener-factor columns (with
// G = 1 they read all 2 MB of the table at once and its lines are evicted by the streamed spectrum,
// re-read from the Infinity Cache: +51 % read requests at C3), at the cost of DRAM locality.
__device__ __forceinline__ void pb_tile(unsigned lb, int colblocks, int order, bool pairs, int& p, int& cb) {
    const unsigned P = gridDim.x / (unsigned)colblocks, G = order > 1 ? (unsigned)order : 1u;
    const unsigned per = G * (unsigned)colblocks, grp = lb / per;
    if (G == 1 || (pairs && (colblocks & 1)) || (grp + 1) * G > P) {
        p = (int)(lb / (unsigned)colblocks);
        cb = (int)(lb % (unsigned)colblocks);
        return;
    }
    const unsigned rem = lb % per;
    if (pairs) {
        const unsigned r = rem >> 1;
        p = (int)(grp * G + r % G);
        cb = (int)(2 * (r / G) + (rem & 1u));
    } else {
        p = (int)(grp * G + rem % G);
        cb = (int)(rem / G);
    }
}

#ifndef ADMM_PASSB_MHOIST
#define ADMM_PASSB_MHOIST 1
#endif
// A block runs its column block through gp planes in turn (plane group pg: planes pg*gp ...; the
// group never straddles two modules): its multipliers stay in registers and its twiddles in LDS
// for all of them, so the Wiener-factor table is read once per gp planes instead of once per
// plane (at C3 the per-plane reads were 0.40 GB of extra requests per launch, served by the
// Infinity Cache, +51 % of pass B's reads).
template <int H, int C, int MODE>
__global__ void __launch_bounds__(C * (H / RowCfg<H>::E), pb_minw(C * (H / RowCfg<H>::E), sizeof(cf) * (H + (size_t)H * C)))
    k_pass_b(const cf* spec_in, cf* spec_out, const float* __restrict__ fcT, const cf* __restrict__ mT,
             const cf* __restrict__ twH_g, int N, int colblocks, int ppm, int order, int fpack, int gp, int P,
             int pmode) {
    using G = ColGeom<H, C>;
    constexpr int E = G::E, L = G::L;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    cf* tw = reinterpret_cast<cf*>(smem);
    cf* data = tw + H;
    load_tw(tw, twH_g, H);
    const int tid = threadIdx.x;
    const int c = tid % C, t = tid / C;
    // pmode: bits 1-2 the block remap (0 none, 1 contiguous XCD ranges, 2 pair-interleaved), bit 0
    // walks the plane groups in reverse (the planes the previous pass wrote last come first)
    const unsigned rb = (pmode >> 1) == 1 ? xcd_remap(blockIdx.x, gridDim.x)
                        : (pmode >> 1) == 2 ? xcd_pairs(blockIdx.x, gridDim.x) : blockIdx.x;
    int pg, cb;
    pb_tile(rb, colblocks, order, true, pg, cb);
    if (pmode & 1) pg = (int)(gridDim.x / (unsigned)colblocks) - 1 - pg;
    const int col = cb * C + c;
    const int p0 = pg * gp;
    if (MODE == 0) fcT += (size_t)(p0 / ppm) * (N + 1) * H;  // this module's Wiener factor
    const int voff = (t * N + col) * (int)sizeof(cf);
    const int sstep = L * N * (int)sizeof(cf);
    using MT = typename std::conditional<MODE == 0, float, cf>::type;
    MT m[E];
    // multipliers of this thread's column (L2-resident tables)
    auto load_m = [&]() {
        if (MODE == 0 && fpack) {
            // the packed copy of the Wiener factors (k_fc_pack, after the G tables of this region): a
            // thread's E factors are contiguous, E/4 16-byte loads instead of E 4-byte ones
            const float* fcP = fcT + (size_t)(P / ppm) * (N + 1) * H;  // fcT: this module's
            const float4* qq = reinterpret_cast<const float4*>(fcP + ((size_t)col * L + t) * E);
    #pragma unroll
            for (int j = 0; j < E / 4; ++j) {
                const float4 f = qq[j];
                if constexpr (MODE == 0) {
                    m[4 * j] = f.x;
                    m[4 * j + 1] = f.y;
                    m[4 * j + 2] = f.z;
                    m[4 * j + 3] = f.w;
                }
            }
        } else {
            const rsrc_t rm = MODE == 0 ? make_rsrc(fcT, (unsigned)((size_t)(N + 1) * H * sizeof(float)))
                                        : make_rsrc(mT, (unsigned)((size_t)(N + 1) * H * sizeof(cf)));
            const int mo = (col * H + t) * (int)sizeof(MT);
    #pragma unroll
            for (int j = 0; j < E; ++j) {
                if constexpr (MODE == 0) m[j] = bload_f(rm, mo, j * L * (int)sizeof(float));
                else if constexpr (MODE == 1) m[j] = bload_cf(rm, mo, j * L * (int)sizeof(cf));
                else m[j] = cconj(bload_cf(rm, mo, j * L * (int)sizeof(cf)));
            }
        }
    };
    // ADMM_PASSB_MHOIST: load them once and keep them in registers for the gp planes (+16 VGPRs held
    // across the forward transform), else reload them per plane
    if (ADMM_PASSB_MHOIST) load_m();
#pragma clang loop unroll(disable)
    for (int q = 0; q < gp; ++q) {
        const int p = p0 + q;
        if (p >= P) break;  // block-uniform
        ColBuf<C> buf{data + c};
        // one plane of the spectrum = H*N*8 bytes (< 4 GiB); element (row, col) at (row*N + col)*8
        const rsrc_t rs = make_rsrc(spec_in + (size_t)p * H * N, (unsigned)((size_t)H * N * sizeof(cf)));
        const rsrc_t ro = make_rsrc(spec_out + (size_t)p * H * N, (unsigned)((size_t)H * N * sizeof(cf)));
        cf v[E];
#pragma unroll
        for (int j = 0; j < E; ++j) v[j] = bload_cf<(ADMM_NT & 8) ? 2 : 0>(rs, voff, j * sstep);
        if (!ADMM_PASSB_MHOIST) load_m();  // per plane (L2 hits after the group's first plane)
        __syncthreads();  // q = 0: the twiddles are in LDS; q > 0: the previous plane's LDS reads are done
        fft<H, L, -1, 1, 1>(v, buf, tw, t);
        if (cb == 0) {  // block-uniform: column 0 carries (DC, Nyquist) packed -> needs F[H-ky]
            __syncthreads();
#pragma unroll
            for (int j = 0; j < E; ++j) buf.at(t + L * j) = v[j];
            __syncthreads();
            if (col == 0) {
#pragma unroll
                for (int j = 0; j < E; ++j) {
                    const int ky = t + L * j;
                    const cf qv = cconj(buf.at((H - ky) & (H - 1)));
                    if constexpr (MODE == 0) {
                        const float f0 = m[j], fn = fcT[(size_t)N * H + ky];
                        const float a = 0.5f * (f0 + fn), b = 0.5f * (f0 - fn);
                        v[j] = mkc(fmaf(a, v[j].x, b * qv.x), fmaf(a, v[j].y, b * qv.y));
                    } else {
                        const cf m0 = m[j], mn = MODE == 1 ? mT[(size_t)N * H + ky] : cconj(mT[(size_t)N * H + ky]);
                        const cf a = mkc(0.5f * (m0.x + mn.x), 0.5f * (m0.y + mn.y));
                        const cf b = mkc(0.5f * (m0.x - mn.x), 0.5f * (m0.y - mn.y));
                        v[j] = cadd(cmul(v[j], a), cmul(qv, b));
                    }
                }
            }
        }
        if (col != 0) {
#pragma unroll
            for (int j = 0; j < E; ++j) {
                if constexpr (MODE == 0) v[j] = cscale(v[j], m[j]);
                else v[j] = cmul(v[j], m[j]);
            }
        }
        fft<H, L, +1, 1, 1>(v, buf, tw, t);
#pragma unroll
        for (int j = 0; j < E; ++j) bstore_cf<(ADMM_NT & 4) ? 2 : 0>(ro, voff, j * sstep, v[j]);
    }
}

// Pass B (MODE 0) with two adjacent columns per thread: 16-byte loads and stores, so the 8
// lanes of a row segment move a whole 128-byte line (the 8-column kernel above moves 64-byte
// halves).  The two column transforms of a thread run one after the other through the same
// LDS exchange buffer (CP column pairs per block, LDS as for C = CP).
#ifndef PASSB2_MINW
#define PASSB2_MINW 4
#endif
__device__ __forceinline__ float4 bload_f4(rsrc_t r, int voff, int soff) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}
__device__ __forceinline__ void bstore_f4(rsrc_t r, int voff, int soff, float4 v) {
    typedef decltype(__builtin_amdgcn_raw_buffer_load_b128(r, 0, 0, 0)) V4;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(V4, v), r, voff, soff, 0);
}

template <int H, int CP>
__global__ void __launch_bounds__(CP * (H / RowCfg<H>::E), PASSB2_MINW)
    k_pass_b2(const cf* spec_in, cf* spec_out, const float* __restrict__ fcT, const cf* __restrict__ twH_g, int N,
              int colblocks, int ppm, int order, int fpack) {
    using G = ColGeom<H, CP>;
    constexpr int E = G::E, L = G::L;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    cf* tw = reinterpret_cast<cf*>(smem);
    cf* data = tw + H;
    load_tw(tw, twH_g, H);
    const int tid = threadIdx.x;
    const int cp = tid % CP, t = tid / CP;
    int p, cb;
    pb_tile(xcd_remap(blockIdx.x, gridDim.x), colblocks, order, false, p, cb);
    const int col = cb * 2 * CP + 2 * cp;  // this thread's columns: col, col + 1
    fcT += (size_t)(p / ppm) * (N + 1) * H;  // this module's Wiener factor
    const rsrc_t rs = make_rsrc(spec_in + (size_t)p * H * N, (unsigned)((size_t)H * N * sizeof(cf)));
    const rsrc_t ro = make_rsrc(spec_out + (size_t)p * H * N, (unsigned)((size_t)H * N * sizeof(cf)));
    const int voff = (t * N + col) * (int)sizeof(cf);
    const int sstep = L * N * (int)sizeof(cf);
    cf v0[E], v1[E];
#pragma unroll
    for (int j = 0; j < E; ++j) {
        const float4 q = bload_f4(rs, voff, j * sstep);
        v0[j] = mkc(q.x, q.y);
        v1[j] = mkc(q.z, q.w);
    }
    // Wiener factors of the two columns (L2-resident table); the second set is loaded only
    // after the first column is done, to keep the register footprint at one set
    const rsrc_t rm = make_rsrc(fcT, (unsigned)((size_t)(N + 1) * H * sizeof(float)));
    const int mo = (col * H + t) * (int)sizeof(float);
    // packed Wiener factors (k_fc_pack): a thread's E factors of a column are contiguous
    const float* fcP = fcT + (size_t)(gridDim.x / colblocks / ppm) * (N + 1) * H;  // fcT: this module's
    auto packed = [&](int c, float (&m)[E]) {
        const float4* q = reinterpret_cast<const float4*>(fcP + ((size_t)c * L + t) * E);
#pragma unroll
        for (int j = 0; j < E / 4; ++j) {
            const float4 f = q[j];
            m[4 * j] = f.x;
            m[4 * j + 1] = f.y;
            m[4 * j + 2] = f.z;
            m[4 * j + 3] = f.w;
        }
    };
    float m0[E], m1[E];
    if (fpack) {
        packed(col, m0);
    } else {
#pragma unroll
        for (int j = 0; j < E; ++j) m0[j] = bload_f(rm, mo, j * L * (int)sizeof(float));
    }
    __syncthreads();
    ColBuf<CP> buf{data + cp};
    fft<H, L, -1, 1, 1>(v0, buf, tw, t);
    if (cb == 0) {  // block-uniform: column 0 carries (DC, Nyquist) packed -> needs F[H-ky]
        __syncthreads();
#pragma unroll
        for (int j = 0; j < E; ++j) buf.at(t + L * j) = v0[j];
        __syncthreads();
        if (col == 0) {
#pragma unroll
            for (int j = 0; j < E; ++j) {
                const int ky = t + L * j;
                const cf q = cconj(buf.at((H - ky) & (H - 1)));
                const float f0 = m0[j], fn = fcT[(size_t)N * H + ky];
                const float a = 0.5f * (f0 + fn), b = 0.5f * (f0 - fn);
                v0[j] = mkc(fmaf(a, v0[j].x, b * q.x), fmaf(a, v0[j].y, b * q.y));
            }
        }
    }
    if (col != 0) {
#pragma unroll
        for (int j = 0; j < E; ++j) v0[j] = cscale(v0[j], m0[j]);
    }
    fft<H, L, +1, 1, 1>(v0, buf, tw, t);
    if (fpack) {
        packed(col + 1, m1);
    } else {
#pragma unroll
        for (int j = 0; j < E; ++j) m1[j] = bload_f(rm, mo + H * (int)sizeof(float), j * L * (int)sizeof(float));
    }
    fft<H, L, -1, 1, 1>(v1, buf, tw, t);
#pragma unroll
    for (int j = 0; j < E; ++j) v1[j] = cscale(v1[j], m1[j]);
    fft<H, L, +1, 1, 1>(v1, buf, tw, t);
#pragma unroll
    for (int j = 0; j < E; ++j) bstore_f4(ro, voff, j * sstep, make_float4(v0[j].x, v0[j].y, v1[j].x, v1[j].y));
}

// ---------------------------------------------------------------------------
// pass A: the fused row pass of one ADMM iteration, one sub-group per strip of R rows
//
// State between iterations (per plane, two images):
//   inference  (HIST = false): u_{k-1} in, u_k out (ping-pong buffers)
//   training   (HIST = true) : a_{k-1} in, a_k out, a_k = D x_k + u_{k-1} kept for every k
//              (the backward needs it); u = a - S(a) and w = z - u are rebuilt in registers,
//              so both modes move the same bytes.
// ---------------------------------------------------------------------------
struct PassAArgs {
    const cf* sin;        // x row spectra (output of pass B)     [P][H][N]
    cf* sout;             // r row spectra for the next pass B     [P][H][N]
    const float* b;       // H_t(xin)                              [P][H][W]
    const float* uxi;     // u_{k-1} (or a_{k-1} when HIST), x / y [P][H][W]
    const float* uyi;
    float* uxo;           // u_k (or a_k when HIST)
    float* uyo;
    const float* nsq;     // iso: N_k     = per-pixel sum over (B,C) of a_k^2      [2][H][W]
    const float* nsq_prev;// iso + HIST: N_{k-1}
    const float* lam;
    const float* rho;
    const cf* twW;        // [W]
    int H;
    int R;                // rows per strip (divides H)
    long long nstrips;
    long long ppm;        // planes per module: with several modules solved together (desc.groups),
                          // module m = plane / ppm has lam[m], rho[m], norms at nsq + m 2HW, and
                          // all modules share b (b has ppm planes)
    int rev = 0;          // 1: walk the strips from the last one (ADMM_PASSA_REV, A/B)
};

// occupancy target of the row pass (waves per SIMD): 3 for rows up to W = 1024 (fits
// ~168 VGPRs, measured faster than 2), 1 for W = 2048 (E = 16 per lane)
#ifndef PASSA_MINW_SMALL
#define PASSA_MINW_SMALL 3
#endif
#define PASSA_MINW(n) ((n) >= 1024 ? 1 : PASSA_MINW_SMALL)

template <bool ISO, class T> __device__ __forceinline__ T shrink_z(T a, T tau, T nsum) {
    if constexpr (ISO) return block_factor(nsum, tau) * a;
    else return soft(a, tau);
}

// u_{k-1} at a pixel pair: zero (first iteration), loaded, or rebuilt from a_{k-1}
template <bool ISO, bool FIRST, bool HIST>
__device__ __forceinline__ cf prev_u(const cf* __restrict__ src, const cf* __restrict__ nsp, size_t idx, float tau) {
    if constexpr (FIRST) {
        return mkc(0.f, 0.f);
    } else {
        const cf v = lda<16>(&src[idx]);
        if constexpr (HIST) {
            const cf n = ISO ? nsp[idx] : mkc(0.f, 0.f);
            return mkc(v.x - shrink_z<ISO>(v.x, tau, n.x), v.y - shrink_z<ISO>(v.y, tau, n.y));
        } else {
            return v;
        }
    }
}

template <int N, bool ISO, bool FIRST, bool HIST, bool PL>
__global__ void __launch_bounds__(256, PASSA_MINW(N)) k_pass_a(PassAArgs a) {
    static_assert(!(PL && HIST), "the training history keeps the pixel-order layout");
    using G = RowKernelGeom<N>;
    constexpr int E = G::E, L = G::L, W = G::W;
    constexpr bool kSpecNT = (ADMM_NT & 2) != 0 || ((ADMM_NT & 32) != 0 && N >= 512);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    cf* tw = reinterpret_cast<cf*>(smem);
    load_tw(tw, a.twW, W);
    __syncthreads();
    const int sgl = threadIdx.x / L, t = threadIdx.x % L;
    // XCD remap of the strips (-DADMM_PASSA_REMAP=0/1 for A/B runs; default: W <= 512): C2
    // pass A +2 %, C3 -7 % (interleaved A/B, tools/ab_variants.sh)
#ifndef ADMM_PASSA_REMAP
#define ADMM_PASSA_REMAP -1
#endif
    constexpr bool kRemap = ADMM_PASSA_REMAP < 0 ? N <= 256 : ADMM_PASSA_REMAP != 0;
    const unsigned blk = kRemap ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
    long long strip = (long long)blk * G::SG + sgl;
    if (strip >= a.nstrips) return;
    if (a.rev) strip = a.nstrips - 1 - strip;
    const int H = a.H, R = a.R;
    const int spp = H / R;
    const long long p = strip / spp;
    const int i0 = (int)(strip % spp) * R;
    RowBuf buf{tw + W + sgl * RowBuf::slots(N)};
    const int mod = (int)(p / a.ppm);
    const float rho = a.rho[mod];
    const float tau = a.lam[mod] / rho;

    const cf* sp = a.sin + (size_t)p * H * N;
    cf* so = a.sout + (size_t)p * H * N;
    const size_t poff = (size_t)p * H * W;
    const cf* bimg = reinterpret_cast<const cf*>(a.b + (size_t)(p - (long long)mod * a.ppm) * H * W);
    const cf* uxi = reinterpret_cast<const cf*>(a.uxi + poff);
    const cf* uyi = reinterpret_cast<const cf*>(a.uyi + poff);
    cf* uxo = reinterpret_cast<cf*>(a.uxo + poff);
    cf* uyo = reinterpret_cast<cf*>(a.uyo + poff);
    const size_t moff = (size_t)mod * 2 * H * W;  // this module's norm maps
    const cf* nsx = reinterpret_cast<const cf*>(a.nsq + moff);
    const cf* nsy = reinterpret_cast<const cf*>(a.nsq + moff + (size_t)H * W);
    const cf* npx = reinterpret_cast<const cf*>(a.nsq_prev + moff);
    const cf* npy = reinterpret_cast<const cf*>(a.nsq_prev + moff + (size_t)H * W);

    cf xprev[E], xcur[E], wxp[E], wyp[E];
    {
        const int g = (i0 - 1 + H) & (H - 1);
#pragma unroll
        for (int j = 0; j < E; ++j) xprev[j] = ld_pol<kSpecNT>(&sp[(size_t)g * N + t + L * j]);
        RowXf<N>::c2r(xprev, buf, tw, t);
    }
    for (int rr = 0; rr <= R; ++rr) {
        const int g = (i0 + rr) & (H - 1);
        const size_t ro = (size_t)g * N;  // row offset in cf units (spectrum and pixel pairs alike)
#pragma unroll
        for (int j = 0; j < E; ++j) xcur[j] = ld_pol<kSpecNT>(&sp[ro + t + L * j]);
        RowXf<N>::c2r(xcur, buf, tw, t);

        // ---- y direction: a_y = x[g] - x[g-1] + u_y; z_y, u_y, w_y of row g
        cf wyc[E];
        {
            cf uy[E], fy[E];
            if constexpr (PL) {
                if constexpr (FIRST) {
#pragma unroll
                    for (int j = 0; j < E; ++j) uy[j] = mkc(0.f, 0.f);
                } else {
                    ld_row<E, L, true, (ADMM_NT & 16) != 0>(uyi + ro, t, uy);
                }
                if constexpr (ISO) ld_row<E, L, true, false>(nsy + ro, t, fy);
            } else {
#pragma unroll
                for (int j = 0; j < E; ++j) {
                    uy[j] = prev_u<ISO, FIRST, HIST>(uyi, npy, ro + t + L * j, tau);
                    if constexpr (ISO) fy[j] = nsy[ro + t + L * j];
                }
            }
#pragma unroll
            for (int j = 0; j < E; ++j) {
                const float a0 = (xcur[j].x - xprev[j].x) + uy[j].x;
                const float a1 = (xcur[j].y - xprev[j].y) + uy[j].y;
                const float z0 = shrink_z<ISO>(a0, tau, ISO ? fy[j].x : 0.f);
                const float z1 = shrink_z<ISO>(a1, tau, ISO ? fy[j].y : 0.f);
                const float n0 = a0 - z0, n1 = a1 - z1;  // u_y(new)
                uy[j] = HIST ? mkc(a0, a1) : mkc(n0, n1);
                wyc[j] = mkc(z0 - n0, z1 - n1);
            }
            if (rr < R) {
                if constexpr (PL) {
                    st_row<E, L, true, (ADMM_NT & 1) != 0>(uyo + ro, t, uy);
                } else {
#pragma unroll
                    for (int j = 0; j < E; ++j) sta(&uyo[ro + t + L * j], uy[j]);
                }
            }
        }

        // ---- finalize row g-1: v = Dx^T w_x + Dy^T w_y, r = b + rho v, row FFT
        if (rr >= 1) {
            const int gm = (g - 1 + H) & (H - 1);
            const size_t rm = (size_t)gm * N;
            cf r[E], sh[E], bv[E];
            if constexpr (PL) ld_row<E, L, true, (ADMM_NT & 16) != 0>(bimg + rm, t, bv);
#pragma unroll
            for (int j = 0; j < E; ++j) sh[j].x = __shfl(wxp[j].x, (t + 1) & (L - 1), L);
#pragma unroll
            for (int j = 0; j < E; ++j) {
                const float wr = (t == L - 1) ? sh[(j + 1) & (E - 1)].x : sh[j].x;  // w_x at pixel q1+1
                const cf bb = PL ? bv[j] : lda<16>(&bimg[rm + t + L * j]);
                const float v0 = (wxp[j].x - wxp[j].y) + (wyp[j].x - wyc[j].x);
                const float v1 = (wxp[j].y - wr) + (wyp[j].y - wyc[j].y);
                r[j] = mkc(fmaf(rho, v0, bb.x), fmaf(rho, v1, bb.y));
            }
            RowXf<N>::r2c(r, buf, tw, t);
#pragma unroll
            for (int j = 0; j < E; ++j) sta(&so[rm + t + L * j], r[j]);
        }

        // ---- x direction: a_x = x[g][j] - x[g][j-1] + u_x; z_x, u_x, w_x of row g
        if (rr < R) {
            cf ux[E], fx[E], sh[E];
            if constexpr (PL) {
                if constexpr (FIRST) {
#pragma unroll
                    for (int j = 0; j < E; ++j) ux[j] = mkc(0.f, 0.f);
                } else {
                    ld_row<E, L, true, (ADMM_NT & 16) != 0>(uxi + ro, t, ux);
                }
                if constexpr (ISO) ld_row<E, L, true, false>(nsx + ro, t, fx);
            }
#pragma unroll
            for (int j = 0; j < E; ++j) {
                if constexpr (!PL) {
                    ux[j] = prev_u<ISO, FIRST, HIST>(uxi, npx, ro + t + L * j, tau);
                    if constexpr (ISO) fx[j] = nsx[ro + t + L * j];
                }
                sh[j].x = __shfl(xcur[j].y, (t - 1) & (L - 1), L);
            }
#pragma unroll
            for (int j = 0; j < E; ++j) {
                const float xl = (t == 0) ? sh[(j - 1) & (E - 1)].x : sh[j].x;  // x at pixel q0-1
                const float a0 = (xcur[j].x - xl) + ux[j].x;
                const float a1 = (xcur[j].y - xcur[j].x) + ux[j].y;
                const float z0 = shrink_z<ISO>(a0, tau, ISO ? fx[j].x : 0.f);
                const float z1 = shrink_z<ISO>(a1, tau, ISO ? fx[j].y : 0.f);
                const float n0 = a0 - z0, n1 = a1 - z1;
                ux[j] = HIST ? mkc(a0, a1) : mkc(n0, n1);
                wxp[j] = mkc(z0 - n0, z1 - n1);
            }
            if constexpr (PL) {
                st_row<E, L, true, (ADMM_NT & 1) != 0>(uxo + ro, t, ux);
            } else {
#pragma unroll
                for (int j = 0; j < E; ++j) sta(&uxo[ro + t + L * j], ux[j]);
            }
        }
#pragma unroll
        for (int j = 0; j < E; ++j) {
            wyp[j] = wyc[j];
            xprev[j] = xcur[j];
        }
    }
}

// ---------------------------------------------------------------------------
// iso pass A1: per-pixel partial sums over a group of planes of a_x^2, a_y^2
// (a = D x + u_{k-1}), one sub-group per (plane group, row)
// ---------------------------------------------------------------------------
struct IsoArgs {
    const cf* sin;
    const float* uxi;       // u_{k-1} (or a_{k-1} when HIST)
    const float* uyi;
    const float* nsq_prev;  // HIST: N_{k-1}
    const float* lam;
    const float* rho;
    float* partial;  // [ngroups][2][H][W]
    const cf* twW;
    int P, H, ppg;   // planes per group (a plane group never straddles two modules)
    long long nitems;  // ngroups * H
    long long ppm;     // planes per module (see PassAArgs)
};

template <int N, bool FIRST, bool HIST, bool PL>
__global__ void __launch_bounds__(256) k_iso_norm(IsoArgs a) {
    static_assert(!(PL && HIST), "the training history keeps the pixel-order layout");
    using G = RowKernelGeom<N>;
    constexpr int E = G::E, L = G::L, W = G::W;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    cf* tw = reinterpret_cast<cf*>(smem);
    load_tw(tw, a.twW, W);
    __syncthreads();
    const int sgl = threadIdx.x / L, t = threadIdx.x % L;
    const long long item = (long long)blockIdx.x * G::SG + sgl;
    if (item >= a.nitems) return;
    const int H = a.H;
    const int g = (int)(item % H);
    const int grp = (int)(item / H);
    const int gm = (g - 1 + H) & (H - 1);
    RowBuf buf{tw + W + sgl * RowBuf::slots(N)};
    const int mod = (int)((long long)grp * a.ppg / a.ppm);
    const float tau = HIST ? a.lam[mod] / a.rho[mod] : 0.f;
    const size_t moff = (size_t)mod * 2 * H * W;
    const cf* npx = reinterpret_cast<const cf*>(a.nsq_prev + moff);
    const cf* npy = reinterpret_cast<const cf*>(a.nsq_prev + moff + (size_t)H * W);
    cf sx[E], sy[E];
#pragma unroll
    for (int j = 0; j < E; ++j) sx[j] = sy[j] = mkc(0.f, 0.f);
    const int p1 = min(a.P, (grp + 1) * a.ppg);
    for (int p = grp * a.ppg; p < p1; ++p) {
        const cf* sp = a.sin + (size_t)p * H * N;
        cf xp[E], xc[E];
#pragma unroll
        for (int j = 0; j < E; ++j) {
            xp[j] = sp[(size_t)gm * N + t + L * j];
            xc[j] = sp[(size_t)g * N + t + L * j];
        }
        RowXf<N>::c2r(xp, buf, tw, t);
        RowXf<N>::c2r(xc, buf, tw, t);
        const size_t ro = (size_t)p * H * N + (size_t)g * N;  // cf units == pixel pairs
        const size_t rn = (size_t)g * N;                      // norm maps are per pixel, shared by planes
        const cf* uxi = reinterpret_cast<const cf*>(a.uxi);
        const cf* uyi = reinterpret_cast<const cf*>(a.uyi);
        cf sh[E], uxv[E], uyv[E];
        if constexpr (PL && !FIRST) {
            ld_row<E, L, true, false>(uxi + ro, t, uxv);
            ld_row<E, L, true, false>(uyi + ro, t, uyv);
        }
#pragma unroll
        for (int j = 0; j < E; ++j) sh[j].x = __shfl(xc[j].y, (t - 1) & (L - 1), L);
#pragma unroll
        for (int j = 0; j < E; ++j) {
            cf ux, uy;
            if constexpr (FIRST) {
                ux = uy = mkc(0.f, 0.f);
            } else if constexpr (PL) {
                ux = uxv[j];
                uy = uyv[j];
            } else if constexpr (HIST) {
                const cf ax = uxi[ro + t + L * j], ay = uyi[ro + t + L * j];
                const cf nx = npx[rn + t + L * j], ny = npy[rn + t + L * j];
                ux = mkc(ax.x - block_factor(nx.x, tau) * ax.x, ax.y - block_factor(nx.y, tau) * ax.y);
                uy = mkc(ay.x - block_factor(ny.x, tau) * ay.x, ay.y - block_factor(ny.y, tau) * ay.y);
            } else {
                ux = uxi[ro + t + L * j];
                uy = uyi[ro + t + L * j];
            }
            const float xl = (t == 0) ? sh[(j - 1) & (E - 1)].x : sh[j].x;
            const float ax0 = (xc[j].x - xl) + ux.x, ax1 = (xc[j].y - xc[j].x) + ux.y;
            const float ay0 = (xc[j].x - xp[j].x) + uy.x, ay1 = (xc[j].y - xp[j].y) + uy.y;
            sx[j].x = fmaf(ax0, ax0, sx[j].x);
            sx[j].y = fmaf(ax1, ax1, sx[j].y);
            sy[j].x = fmaf(ay0, ay0, sy[j].x);
            sy[j].y = fmaf(ay1, ay1, sy[j].y);
        }
    }
    cf* px = reinterpret_cast<cf*>(a.partial + ((size_t)grp * 2 + 0) * H * W) + (size_t)g * N;
    cf* py = reinterpret_cast<cf*>(a.partial + ((size_t)grp * 2 + 1) * H * W) + (size_t)g * N;
    st_row<E, L, PL, false>(px, t, sx);  // the norm maps take the layout of u (pass A reads both alike)
    st_row<E, L, PL, false>(py, t, sy);
}

// nsq[k] = sum_g partial[g][k], k over 2*H*W, fixed order (deterministic)
static __global__ void k_iso_reduce(const float4* __restrict__ partial, float4* __restrict__ nsq, int ngroups,
                             long long n4) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n4) return;
    float4 s = partial[i];
    for (int g = 1; g < ngroups; ++g) {
        const float4 q = partial[(size_t)g * n4 + i];
        s.x += q.x;
        s.y += q.y;
        s.z += q.z;
        s.w += q.w;
    }
    nsq[i] = s;
}

}  // namespace admm

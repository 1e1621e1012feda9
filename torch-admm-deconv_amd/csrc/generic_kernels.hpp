// generic_kernels.hpp -- any-size path of the ADMM-TV solver.
//
// The fused two-pass kernels (admm_kernels.hpp) need power-of-two H, W (register-resident
// radix-2^k transforms).  For every other size (the reference accepts any H x W, e.g. 15 x 17)
// the iteration runs as four simpler HIP kernels:
//
//   k_grow_fwd   real rows -> half spectra X[kx], kx < Wh = W/2 + 1       (rfft along W)
//   k_gcol       per column kx: FFT along H, multiply, inverse FFT           (in place)
//   k_grow_inv   half spectra -> real rows (Hermitian completion)          (irfft along W)
//   k_gstep      per pixel: Dx, Dy, shrink, dual update, w, D^T w, r = b + rho v
//
// Transforms: LDS-resident Stockham autosort, mixed radix (4, 2, 3, 5, 7 butterflies and an
// O(R) per-output stage for any other prime R), twiddles from the same fp64-computed
// tables as the fast path (tw[i] = exp(-2 pi i i_/n), stored fp32).  Transforms are
// unnormalised; 1/(H W) is folded into the multiplier tables.
//
// Layouts: images float [P][H][W]; spectra cf [P][H][Wh]; multipliers transposed [Wh][H]
// (k_spectra's layout with N = W/2, so the setup kernels are shared with the fast path).
//
// Precision: every kernel is templated on its real type T (float, or double for fp64 inputs, which
// the reference computes in fp64: deconv.py:49,61-67,104-106); C = cx_t<T> is the complex type.
// The double instantiation runs plans without Bluestein stages and with the generic (table
// twiddle) butterflies for radices 8 and 16; the float code is unchanged by the templating.
#pragma once
#include "admm_backward.hpp"

namespace admm {

constexpr int GMAXST = 24;
// threads per block of the generic transform kernels (-DADMM_GNT=512 for A/B runs)
#ifndef ADMM_GNT
#define ADMM_GNT 256
#endif
constexpr int GNT = ADMM_GNT;  // max number of radix stages (n <= 8192 -> at most 13 factors)

// A stage whose radix is a prime R > 7 runs either as the O(R)-per-output stage (gstage_any) or,
// for R >= the Bluestein threshold (admm_capi.hip make_plan), as a chirp-z transform: the R-point
// DFT as a length-M circular convolution (M = 2^k >= 2R - 1) done with the register-resident
// power-of-two FFT of fft_core.hpp (gstage_blue).  Its tables follow the n twiddles of `tw`:
// chirp c_q = exp(-i pi q^2 / R) (R values), B = FFT_M(conj c, even-extended) / M (M values),
// and the M-point twiddles exp(-2 pi i j / M) (M values).
struct GPlan {
    int n, nst;
    int rad[GMAXST];
    int bst[GMAXST];   // Bluestein size M of stage s (0: direct stage)
    int boff[GMAXST];  // offset (complex values) of stage s's tables from the start of tw
    int ntab;          // table entries after the n twiddles
    int xslots;        // exchange slots (complex values) the Bluestein stages need
    int bm;            // the plan's Bluestein size M (all its Bluestein stages), 0: none
    int twg;           // 1: twiddles and tables are read from global memory (L1/L2), not LDS --
                       // long lines (> ~6,800 points) whose LDS image would not fit otherwise
    int glb;           // 1: even the two line buffers do not fit the LDS (lines beyond 10,240 points,
                       // 5,120 in fp64): they live in a global scratch slot per block (L2-resident),
                       // blocks walk their lines grid-stride; implies twg, no Bluestein stages
};

// values per lane of the power-of-two transform of length M (fft_core.hpp RowCfg)
__host__ __device__ constexpr int blue_e(int M) { return M <= 32 ? 4 : M <= 512 ? 8 : 16; }

// ---------------------------------------------------------------------------
// one Stockham stage over `lines` transforms of length n held in LDS as [i][lines]
// (element i of line c at src[i * lines + c]); threads stride over (line, vt) pairs.
// ---------------------------------------------------------------------------
template <int DIR, class C>
__device__ __forceinline__ C twid(const C* __restrict__ tw, int idx) {
    const C w = tw[idx];
    return DIR < 0 ? w : cconj(w);
}

// x / d for 0 <= x < 2^20, 0 < d, with rd ~ 1/d (v_rcp_f32): the float quotient is within 1 of
// the true one and one remainder test corrects it -- the transforms' index arithmetic divides by
// runtime radix products, and the compiler's exact integer division is ~20 instructions
__device__ __forceinline__ int fdiv(int x, int d, float rd) {
    int q = (int)((float)x * rd);
    const int r = x - q * d;
    q += (r < 0) ? -1 : (r >= d ? 1 : 0);
    return q;
}
__device__ __forceinline__ float frcp(int d) { return __builtin_amdgcn_rcpf((float)d); }

// cos / sin(2 pi m / R), m in [0, R), for the odd radices 3 ... 13 (fp64 literals rounded to fp32)
template <int R> struct OddTw;
template <> struct OddTw<3> {
    static constexpr double C[2] = {1.0, -0.5};
    static constexpr double S[2] = {0.0, 0.86602540378443864676};
};
template <> struct OddTw<5> {
    static constexpr double C[3] = {1.0, 0.30901699437494742410, -0.80901699437494742410};
    static constexpr double S[3] = {0.0, 0.95105651629515357212, 0.58778525229247312917};
};
template <> struct OddTw<7> {
    static constexpr double C[4] = {1.0, 0.62348980185873353053, -0.22252093395631440429, -0.90096886790241912624};
    static constexpr double S[4] = {0.0, 0.78183148246802980871, 0.97492791218182360702, 0.43388373911755812048};
};

template <> struct OddTw<11> {
    static constexpr double C[6] = {1.0, 0.8412535328311812, 0.41541501300188644, -0.142314838273285,
                                    -0.654860733945285, -0.9594929736144974};
    static constexpr double S[6] = {0.0, 0.5406408174555976, 0.9096319953545183, 0.9898214418809328,
                                    0.7557495743542583, 0.28173255684142967};
};
template <> struct OddTw<13> {
    static constexpr double C[7] = {1.0, 0.8854560256532099, 0.5680647467311559, 0.120536680255323,
                                    -0.35460488704253545, -0.7485107481711012, -0.970941817426052};
    static constexpr double S[7] = {0.0, 0.4647231720437685, 0.8229838658936564, 0.992708874098054,
                                    0.9350162426854148, 0.6631226582407952, 0.23931566428755768};
};

// cos / sin(2 pi m / R) in the real type T ((float)C[...] for T = float, as cosv / sinv)
template <int R, class T> __device__ __forceinline__ constexpr T odd_cos(int m) {
    return (T)OddTw<R>::C[m <= (R - 1) / 2 ? m : R - m];
}
template <int R, class T> __device__ __forceinline__ constexpr T odd_sin(int m) {
    return (T)(m <= (R - 1) / 2 ? OddTw<R>::S[m] : -OddTw<R>::S[R - m]);
}

template <int DIR, int R, class C>
__device__ __forceinline__ void small_dft(C (&v)[R], const C* __restrict__ tw, int n) {
    using T = re_t<C>;
    if constexpr (R == 2) {
        const C a = v[0], b = v[1];
        v[0] = cadd(a, b);
        v[1] = csub(a, b);
    } else if constexpr (R == 4) {
        const C t0 = cadd(v[0], v[2]), t1 = csub(v[0], v[2]), t2 = cadd(v[1], v[3]);
        const C t3 = mul_i<DIR>(csub(v[1], v[3]));
        v[0] = cadd(t0, t2);
        v[2] = csub(t0, t2);
        v[1] = cadd(t1, t3);
        v[3] = csub(t1, t3);
    } else if constexpr ((R == 8 || R == 16) && std::is_same<T, float>::value) {
        DFT<R, DIR>::template run<1, 0>(v);  // register DFT with exact constant twiddles (fft_core.hpp)
    } else if constexpr (R == 3 || R == 5 || R == 7 || R == 11 || R == 13) {
        // odd R with compile-time cosines / sines on the input sums / differences (the pairing of
        // gstage_any): y_k, y_{R-k} = x0 + sum_q s_q cos(qk) -+ DIR i sum_q d_q sin(qk)
        constexpr int h = (R - 1) / 2;
        C s[h + 1], d[h + 1];
        C y0 = v[0];
        static_for<1, h + 1>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            s[q] = cadd(v[q], v[R - q]);
            d[q] = csub(v[q], v[R - q]);
            y0 = cadd(y0, s[q]);
        });
        C out[R];
        out[0] = y0;
        static_for<1, h + 1>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            C a = v[0], b = mkx<T>(0, 0);
            static_for<1, h + 1>([&](auto qc) {
                constexpr int q = decltype(qc)::value;
                constexpr T c = odd_cos<R, T>((q * k) % R), sn = odd_sin<R, T>((q * k) % R);
                a.x = fmat(s[q].x, c, a.x);
                a.y = fmat(s[q].y, c, a.y);
                b.x = fmat(d[q].x, sn, b.x);
                b.y = fmat(d[q].y, sn, b.y);
            });
            // i b = (-b.y, b.x); forward (DIR < 0): y_k = a - i b
            const C ib = mkx<T>(-b.y, b.x);
            out[k] = DIR < 0 ? csub(a, ib) : cadd(a, ib);
            out[R - k] = DIR < 0 ? cadd(a, ib) : csub(a, ib);
        });
#pragma unroll
        for (int k = 0; k < R; ++k) v[k] = out[k];
        (void)tw;
        (void)n;
    } else {
        // y_k = sum_q v_q W_R^{qk}, W_R^j = tw[j n / R]
        C y[R];
        const int step = n / R;
#pragma unroll
        for (int k = 0; k < R; ++k) {
            C acc = v[0];
#pragma unroll
            for (int q = 1; q < R; ++q) {
                const C w = twid<DIR>(tw, ((q * k) % R) * step);
                const C p = cmul(v[q], w);
                acc = cadd(acc, p);
            }
            y[k] = acc;
        }
#pragma unroll
        for (int k = 0; k < R; ++k) v[k] = y[k];
    }
}

template <int DIR, int R, class C>
__device__ __forceinline__ void gstage_r(const C* __restrict__ src, C* __restrict__ dst, int n, int NS, int lines,
                                         const C* __restrict__ tw) {
    const int nb = n / R;                 // butterflies per line
    const int tstride = n / (NS * R);     // twiddle index stride of W_{NS R}
    const int lg = __ffs(lines) - 1;      // lines is a power of two
    const float rns = frcp(NS);
    for (int item = threadIdx.x; item < nb * lines; item += blockDim.x) {
        const int c = item & (lines - 1), vt = item >> lg;
        const int vq = fdiv(vt, NS, rns), m = vt - vq * NS;
        C v[R];
#pragma unroll
        for (int q = 0; q < R; ++q) {
            C x = src[(vt + q * nb) * lines + c];
            if (q > 0 && m > 0) x = cmul(x, twid<DIR>(tw, m * q * tstride));
            v[q] = x;
        }
        small_dft<DIR, R>(v, tw, n);
        const int base = vq * NS * R + m;
#pragma unroll
        for (int k = 0; k < R; ++k) dst[(base + k * NS) * lines + c] = v[k];
    }
}

// any (odd prime) radix R, in two steps:
//  1. the stage twiddles W_{NS R}^{m q} are applied to the inputs in place (src is this stage's
//     scratch), so what remains per butterfly is a plain R-point DFT;
//  2. outputs k and R - k take conjugate twiddles W_R^{+-qk}, and so do inputs q and R - q: an
//     item computes GP such output pairs of one butterfly (group 0 also output 0) from the input
//     sums and differences x_q +- x_{R-q} (real cosine / sine sums), reading each input once and
//     each table twiddle once per input pair -- four FMAs per input pair and output pair.
#ifndef ADMM_GP
#define ADMM_GP 2
#endif
#ifndef ADMM_GUNROLL
#define ADMM_GUNROLL 8
#endif
constexpr int GP = ADMM_GP;

template <int DIR, class C>
__device__ __forceinline__ void gstage_any(C* __restrict__ src, C* __restrict__ dst, int n, int NS, int R,
                                           int lines, const C* __restrict__ tw) {
    using T = re_t<C>;
    const int nb = n / R;
    const int span = NS * R;
    const int tstride = n / span;
    const int lg = __ffs(lines) - 1;
    const float rns = frcp(NS), rnb = frcp(nb);
    if (NS > 1) {
        for (int item = threadIdx.x; item < n * lines; item += blockDim.x) {
            const int c = item & (lines - 1), o = item >> lg;  // o = vt + q nb
            const int q = fdiv(o, nb, rnb), vt = o - q * nb;
            const int m = vt - fdiv(vt, NS, rns) * NS;
            if (q > 0 && m > 0) {
                C* x = src + (size_t)o * lines + c;
                *x = cmul(*x, twid<DIR>(tw, m * q * tstride));  // m q < NS R: no reduction
            }
        }
        __syncthreads();
    }
    const int npair = (R - 1) / 2;
    const int ngrp = (npair + GP - 1) / GP;
    const int rstep = n / R;  // W_R^j = tw[j n / R]
    for (int item = threadIdx.x; item < nb * ngrp * lines; item += blockDim.x) {
        const int c = item & (lines - 1), o = item >> lg;
        const int g = fdiv(o, nb, rnb), vt = o - g * nb;
        const int vq = fdiv(vt, NS, rns), m = vt - vq * NS;
        const int k0 = 1 + g * GP;
        const C* col = src + (size_t)vt * lines + c;
        const size_t qstep = (size_t)nb * lines;
        C x0 = col[0];
        C acc0 = x0;  // output 0 (group 0 only)
        // inputs q and R - q share the twiddle pair w, conj(w) (w = W_R^{qk}):
        //   x_q w + x_{R-q} conj(w) = s w.x + i d w.y,   x_q conj(w) + x_{R-q} w = s w.x - i d w.y
        // with s = x_q + x_{R-q}, d = x_q - x_{R-q}: four FMAs per input pair for both outputs
        // k and R - k (the real cosine / sine sums), half the loop trips of the per-input form
        C sa[GP], sb[GP];  // sum s w.x, sum d w.y
        int idx[GP];  // table index (q (k0 + j) mod R) * rstep, stepped without multiply or modulo
        const int wrap = R * rstep;
#pragma unroll
        for (int j = 0; j < GP; ++j) {
            sa[j] = mkx<T>(0, 0);
            sb[j] = mkx<T>(0, 0);
            idx[j] = 0;
        }
#pragma unroll ADMM_GUNROLL
        for (int q = 1; q <= npair; ++q) {
            const C xa = col[q * qstep], xb = col[(R - q) * qstep];
            const C s = cadd(xa, xb), d = csub(xa, xb);
            acc0 = cadd(acc0, s);
#pragma unroll
            for (int j = 0; j < GP; ++j) {
                idx[j] += (k0 + j) * rstep;
                if (idx[j] >= wrap) idx[j] -= wrap;
                const C w = twid<DIR>(tw, idx[j]);
                sa[j].x = fmat(s.x, w.x, sa[j].x);
                sa[j].y = fmat(s.y, w.x, sa[j].y);
                sb[j].x = fmat(d.x, w.y, sb[j].x);
                sb[j].y = fmat(d.y, w.y, sb[j].y);
            }
        }
        C* out = dst + ((size_t)vq * span + m) * lines + c;
        const size_t kstep = (size_t)NS * lines;
        if (g == 0) out[0] = acc0;
#pragma unroll
        for (int j = 0; j < GP; ++j) {
            const int k = k0 + j;
            if (k <= npair) {
                const C a = cadd(x0, sa[j]);
                out[k * kstep] = mkx<T>(a.x - sb[j].y, a.y + sb[j].x);        // a + i sb
                out[(R - k) * kstep] = mkx<T>(a.x + sb[j].y, a.y - sb[j].x);  // a - i sb
            }
        }
    }
}

// Bluestein stage (radix R prime, M = 2^k >= 2R - 1): every butterfly (vt, line) is one item,
// run by a sub-group of L = M / E lanes holding its length-M sequence in registers:
//   a_q = x_q W_{NS R}^{m q} c_q (q < R, else 0);  A = FFT_M(a);  A *= B;  a = IFFT_M(A);
//   X_k = c_k a_k  (k < R)  -- with conj(c), conj(B) for the inverse direction.
// The exchange area holds one RowBuf per sub-group; all sub-groups run the same number of
// rounds, so the wave-level exchange of fft() never diverges (idle items are masked).
template <int DIR, int M>
__device__ __forceinline__ void gstage_blue(const cf* __restrict__ src, cf* __restrict__ dst, int n, int NS, int R,
                                            int lines, const cf* __restrict__ tw, const cf* __restrict__ bt,
                                            cf* __restrict__ xbuf) {
    constexpr int E = RowCfg<M>::E, L = M / E;
    static_assert(L <= 64, "one Bluestein sequence per sub-group inside one wave");
    const int nsg = blockDim.x / L;
    const int sg = threadIdx.x / L, t = threadIdx.x % L;
    const RowBuf buf{xbuf + sg * RowBuf::slots(M)};
    const cf* chirp = bt;
    const cf* Bf = bt + R;
    const cf* twM = bt + R + M;
    const int nb = n / R, span = NS * R, tstride = n / span;
    const int items = nb * lines;
    const int rounds = (items + nsg - 1) / nsg;
    const int lg = __ffs(lines) - 1;
    const float rns = frcp(NS);
    for (int rr = 0; rr < rounds; ++rr) {
        const int item = rr * nsg + sg;
        const bool live = item < items;
        const int c = live ? item & (lines - 1) : 0, vt = live ? item >> lg : 0;
        const int vq = fdiv(vt, NS, rns), m = vt - vq * NS;
        cf v[E];
#pragma unroll
        for (int j = 0; j < E; ++j) {
            const int q = t + L * j;
            cf x = mkc(0.f, 0.f);
            if (live && q < R) {
                x = src[(vt + q * nb) * lines + c];
                if (q > 0 && m > 0) x = cmul(x, twid<DIR>(tw, m * q * tstride));
                x = DIR < 0 ? cmul(x, chirp[q]) : cmulc(x, chirp[q]);
            }
            v[j] = x;
        }
        fft<M, L, -1, 0, 1>(v, buf, twM, t);
#pragma unroll
        for (int j = 0; j < E; ++j) v[j] = DIR < 0 ? cmul(v[j], Bf[t + L * j]) : cmulc(v[j], Bf[t + L * j]);
        fft<M, L, +1, 0, 1>(v, buf, twM, t);
        cf* out = dst + ((size_t)vq * span + m) * lines + c;
#pragma unroll
        for (int j = 0; j < E; ++j) {
            const int k = t + L * j;
            if (live && k < R) out[(size_t)k * NS * lines] = DIR < 0 ? cmul(v[j], chirp[k]) : cmulc(v[j], chirp[k]);
        }
    }
}

// full transform; data starts in bufA, returns the buffer holding the result.  tw: the n
// twiddles followed by the plan's Bluestein tables (LDS); xbuf: pl.xslots exchange slots.
// BM: the plan's Bluestein size (a template parameter, so a kernel without Bluestein stages keeps
// its small register footprint; each BM is its own kernel instantiation).
template <int DIR, int BM, class C>
__device__ __forceinline__ C* gfft_lds(C* bufA, C* bufB, const GPlan& pl, int lines, const C* __restrict__ tw,
                       C* __restrict__ xbuf) {  // bufA is clobbered
    static_assert(BM == 0 || std::is_same<C, cf>::value, "Bluestein stages: fp32 only");
    C* src = bufA;
    C* dst = bufB;
    int NS = 1;
    for (int s = 0; s < pl.nst; ++s) {
        const int R = pl.rad[s];
        if (BM > 0 && pl.bst[s] > 0) {
            if constexpr (BM > 0 && std::is_same<C, cf>::value)
                gstage_blue<DIR, BM>(src, dst, pl.n, NS, R, lines, tw, tw + pl.boff[s], xbuf);
        } else if constexpr (std::is_same<C, cd>::value) {
            // fp64 plans: radices 4, 2, 3, 5 and the any-prime stage (make_plan_f64), which keeps the
            // double kernels' register footprint bounded
            switch (R) {
                case 2: gstage_r<DIR, 2>(src, dst, pl.n, NS, lines, tw); break;
                case 3: gstage_r<DIR, 3>(src, dst, pl.n, NS, lines, tw); break;
                case 4: gstage_r<DIR, 4>(src, dst, pl.n, NS, lines, tw); break;
                case 5: gstage_r<DIR, 5>(src, dst, pl.n, NS, lines, tw); break;
                default: gstage_any<DIR>(src, dst, pl.n, NS, R, lines, tw); break;
            }
        } else {
            switch (R) {
                case 2: gstage_r<DIR, 2>(src, dst, pl.n, NS, lines, tw); break;
                case 3: gstage_r<DIR, 3>(src, dst, pl.n, NS, lines, tw); break;
                case 4: gstage_r<DIR, 4>(src, dst, pl.n, NS, lines, tw); break;
                case 8: gstage_r<DIR, 8>(src, dst, pl.n, NS, lines, tw); break;
                case 16: gstage_r<DIR, 16>(src, dst, pl.n, NS, lines, tw); break;
                case 5: gstage_r<DIR, 5>(src, dst, pl.n, NS, lines, tw); break;
                case 7: gstage_r<DIR, 7>(src, dst, pl.n, NS, lines, tw); break;
                case 11: gstage_r<DIR, 11>(src, dst, pl.n, NS, lines, tw); break;
                case 13: gstage_r<DIR, 13>(src, dst, pl.n, NS, lines, tw); break;
                default: gstage_any<DIR>(src, dst, pl.n, NS, R, lines, tw); break;
            }
        }
        __syncthreads();
        C* t = src;
        src = dst;
        dst = t;
        NS *= R;
    }
    return src;
}

// Bluestein tables of a plan, written after the n twiddles of `tab` (fp64 arithmetic, fp32 store):
// per Bluestein stage s (R = rad[s], M = bst[s]) at tab + boff[s]: chirp[R], B[M], twM[M].
// One wave per table entry: the M-term sum of a B entry is split over the wave's lanes (a fixed
// lane-stride order and a fixed butterfly reduction, so the tables are deterministic); a thread
// per entry made the setup a 100-us serial chain of 2M fp64 sincospi per B entry.
static __global__ void k_blue_tables(cf* __restrict__ tab, GPlan pl) {
    const int lane = threadIdx.x & 63;
    const int i = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);  // wave-uniform
    for (int s = 0; s < pl.nst; ++s) {
        const int R = pl.rad[s], M = pl.bst[s];
        if (M == 0 || i >= R + 2 * M) continue;
        cf* o = tab + pl.boff[s];
        double re, im;
        if (i < R) {  // c_q = exp(-i pi q^2 / R)
            const long long q2 = ((long long)i * i) % (2LL * R);
            sincospi((double)q2 / R, &im, &re);
            if (lane == 0) o[i] = mkc((float)re, (float)-im);
        } else if (i < R + M) {  // B[k] = (1/M) sum_j bt_j exp(-2 pi i j k / M), bt = conj(c) even-extended
            const int k = i - R;
            double sr = 0.0, si = 0.0;
            for (int j = lane; j < M; j += 64) {
                const int jj = j < R ? j : (M - j < R ? M - j : -1);
                if (jj < 0) continue;
                const long long q2 = ((long long)jj * jj) % (2LL * R);
                double bs, bc;
                sincospi((double)q2 / R, &bs, &bc);  // bt_j = exp(+i pi jj^2 / R)
                double ws, wc;
                sincospi(2.0 * (double)(((long long)j * k) % M) / M, &ws, &wc);  // exp(-i ...) = wc - i ws
                sr += bc * wc + bs * ws;
                si += bs * wc - bc * ws;
            }
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) {
                sr += __shfl_xor(sr, d, 64);
                si += __shfl_xor(si, d, 64);
            }
            if (lane == 0) o[i] = mkc((float)(sr / M), (float)(si / M));
        } else {  // twM[j] = exp(-2 pi i j / M)
            const int j = i - R - M;
            sincospi(2.0 * (double)j / M, &im, &re);
            if (lane == 0) o[i] = mkc((float)re, (float)-im);
        }
    }
}

// ---------------------------------------------------------------------------
// row transforms: `lines` rows per block (contiguous rows of one image set)
// ---------------------------------------------------------------------------
template <class T> struct GRowArgsT {
    const T* img;        // fwd: input rows [rows][W];   inv: output rows
    cx_t<T>* spec;       // fwd: output [rows][Wh];       inv: input
    T* img_out;
    const cx_t<T>* tw;   // [W]
    GPlan plan;
    long long rows;
    int lines;           // rows per block
    cx_t<T>* gscr;       // plan.glb: the blocks' scratch slots, 2 W lines values each
    int ldw;             // spectrum row pitch in complex values (0: Wh = W / 2 + 1)
};

// the line buffers of a transform block: the LDS image after the twiddles (twl), or -- long lines
// (GLB) -- this block's slot of the global scratch.  Long-line blocks walk their work items
// grid-stride (one scratch slot per block, ADMM_GEN_ITEMS), every other block runs its one item.
template <bool GLB, class C>
__device__ __forceinline__ C* line_bufs(C* twl, int tw_slots, C* gscr, size_t slot) {
    if constexpr (GLB) return gscr + (size_t)blockIdx.x * slot;
    else return twl + tw_slots;
}
using GRowArgs = GRowArgsT<float>;

// Real rows are transformed two at a time: rows a, b as one complex row z = a + i b, whose
// spectrum Z gives A[k] = (Z[k] + conj Z[-k]) / 2 and B[k] = (Z[k] - conj Z[-k]) / 2i.  A block
// holds `lines` complex rows = 2 * lines real rows.
// TWG: twiddles / tables read from global memory (GPlan::twg; a template parameter, so the LDS
// variant keeps its LDS reads)
template <int BM, class T>
__device__ __forceinline__ void grow_fwd_item(const GRowArgsT<T>& a, cx_t<T>* A, cx_t<T>* B, cx_t<T>* X,
                                              const cx_t<T>* tw, long long r0) {
    using C = cx_t<T>;
    const int W = a.plan.n, Wh = W / 2 + 1, lines = a.lines;
    const int nl = (int)min((long long)2 * lines, a.rows - r0);  // real rows in this block
    for (int rr = 0; rr < 2 * lines; ++rr)  // coalesced along the row
        for (int i = threadIdx.x; i < W; i += blockDim.x) {
            const T v = rr < nl ? a.img[(r0 + rr) * W + i] : T(0);
            T* slot = reinterpret_cast<T*>(&A[i * lines + (rr >> 1)]);
            slot[rr & 1] = v;  // even row -> real part, odd row -> imaginary part
        }
    __syncthreads();
    const C* res = gfft_lds<-1, BM>(A, B, a.plan, lines, tw, X);
    const T half = T(0.5);
    const long long ld = a.ldw ? a.ldw : Wh;
    for (int c = 0; c < lines; ++c)
        for (int k = threadIdx.x; k < Wh; k += blockDim.x) {
            const C z = res[k * lines + c];
            const C m = res[(k == 0 ? 0 : W - k) * lines + c];
            const long long ra = r0 + 2 * c;
            if (2 * c < nl) a.spec[ra * ld + k] = mkx<T>(half * (z.x + m.x), half * (z.y - m.y));
            if (2 * c + 1 < nl) a.spec[(ra + 1) * ld + k] = mkx<T>(half * (z.y + m.y), half * (m.x - z.x));
        }
}

// GLB: long lines, the blocks' scratch slots walk the work items grid-stride (one slot per block)
#define ADMM_GEN_ITEMS(nitems, stride, call)                                                        \
    if constexpr (GLB) {                                                                            \
        for (long long u_ = blockIdx.x; u_ < (nitems); u_ += gridDim.x) {                          \
            call(u_ * (stride));                                                                    \
            __syncthreads(); /* the slot's next item overwrites what this one still reads */       \
        }                                                                                           \
    } else {                                                                                        \
        call((long long)blockIdx.x * (stride));                                                     \
    }

template <int BM, bool TWG, int NT = GNT, class T = float, bool GLB = false>
__global__ void __launch_bounds__(NT) k_grow_fwd(GRowArgsT<T> a) {
    using C = cx_t<T>;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int W = a.plan.n, lines = a.lines;
    C* twl = reinterpret_cast<C*>(smem);
    C* A = line_bufs<GLB>(twl, TWG ? 0 : W + a.plan.ntab, a.gscr, 2 * (size_t)W * lines);
    C* B = A + (size_t)W * lines;
    C* X = GLB ? nullptr : B + (size_t)W * lines;  // Bluestein exchange slots
    if constexpr (!TWG)
        for (int i = threadIdx.x; i < W + a.plan.ntab; i += blockDim.x) twl[i] = a.tw[i];
    const C* tw = TWG ? a.tw : twl;
#define ADMM_ITEM(r0) grow_fwd_item<BM>(a, A, B, X, tw, r0)
    ADMM_GEN_ITEMS((a.rows + 2 * lines - 1) / (2 * lines), 2 * lines, ADMM_ITEM)
#undef ADMM_ITEM
}

template <int BM, class T>
__device__ __forceinline__ void grow_inv_item(const GRowArgsT<T>& a, cx_t<T>* A, cx_t<T>* B, cx_t<T>* X,
                                              const cx_t<T>* tw, long long r0) {
    using C = cx_t<T>;
    const int W = a.plan.n, Wh = W / 2 + 1, lines = a.lines;
    const int nl = (int)min((long long)2 * lines, a.rows - r0);
    // Hermitian completion of a half spectrum: X[k] = conj X[W - k] for k >= Wh; the imaginary
    // parts of the self-conjugate bins (DC, and Nyquist for even W) are dropped, as irfft does
    const long long ld = a.ldw ? a.ldw : Wh;
    auto full = [&](long long row, int k) -> C {
        if (k < Wh) {
            C v = a.spec[row * ld + k];
            if (k == 0 || 2 * k == W) v.y = T(0);
            return v;
        }
        return cconj(a.spec[row * ld + (W - k)]);
    };
    for (int c = 0; c < lines; ++c)
        for (int k = threadIdx.x; k < W; k += blockDim.x) {
            const long long ra = r0 + 2 * c;
            const C xa = 2 * c < nl ? full(ra, k) : mkx<T>(0, 0);
            const C xb = 2 * c + 1 < nl ? full(ra + 1, k) : mkx<T>(0, 0);
            A[k * lines + c] = mkx<T>(xa.x - xb.y, xa.y + xb.x);  // Z = Xa + i Xb
        }
    __syncthreads();
    const C* res = gfft_lds<+1, BM>(A, B, a.plan, lines, tw, X);
    for (int rr = 0; rr < nl; ++rr)
        for (int i = threadIdx.x; i < W; i += blockDim.x) {
            const C z = res[i * lines + (rr >> 1)];
            a.img_out[(r0 + rr) * W + i] = (rr & 1) ? z.y : z.x;
        }
}

template <int BM, bool TWG, int NT = GNT, class T = float, bool GLB = false>
__global__ void __launch_bounds__(NT) k_grow_inv(GRowArgsT<T> a) {
    using C = cx_t<T>;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int W = a.plan.n, lines = a.lines;
    C* twl = reinterpret_cast<C*>(smem);
    C* A = line_bufs<GLB>(twl, TWG ? 0 : W + a.plan.ntab, a.gscr, 2 * (size_t)W * lines);
    C* B = A + (size_t)W * lines;
    C* X = GLB ? nullptr : B + (size_t)W * lines;
    if constexpr (!TWG)
        for (int i = threadIdx.x; i < W + a.plan.ntab; i += blockDim.x) twl[i] = a.tw[i];
    const C* tw = TWG ? a.tw : twl;
#define ADMM_ITEM(r0) grow_inv_item<BM>(a, A, B, X, tw, r0)
    ADMM_GEN_ITEMS((a.rows + 2 * lines - 1) / (2 * lines), 2 * lines, ADMM_ITEM)
#undef ADMM_ITEM
}

// ---------------------------------------------------------------------------
// column pass: per column kx of the half spectrum, FFT along H, multiply, inverse FFT.
// MODE 0: real factor fcT[kx][ky]; 1: mT[kx][ky]; 2: conj(mT); 3: transform only (dump the
// forward column spectrum to `dump` and stop; used for cross-spectra).  `dump` (MODE 0) also
// receives the forward spectrum before the multiply when non-null.
// ---------------------------------------------------------------------------
template <class T> struct GColArgsT {
    cx_t<T>* spec;        // [P][H][Wh], in place
    cx_t<T>* dump;        // optional [P][H][Wh]
    const T* fcT;
    const cx_t<T>* mT;
    const cx_t<T>* tw;    // [H]
    GPlan plan;           // n = H
    int Wh;
    int cols;             // columns per block
    int colblocks;
    long long P;
    cx_t<T>* gscr;        // plan.glb: the blocks' scratch slots, 2 H cols values each
};
using GColArgs = GColArgsT<float>;

// occupancy hint of the column pass with Bluestein stages of size 256 (waves per SIMD; A/B knob
// -DADMM_GCOL_MINW=4 caps its VGPRs at 128)
#ifndef ADMM_GCOL_MINW
#define ADMM_GCOL_MINW 1
#endif
constexpr int gcol_minw(int bm) { return bm == 256 ? ADMM_GCOL_MINW : 1; }

template <int MODE, int BM, class T>
__device__ __forceinline__ void gcol_item(const GColArgsT<T>& a, cx_t<T>* A, cx_t<T>* B, cx_t<T>* X,
                                          const cx_t<T>* tw, long long item) {
    using C = cx_t<T>;
    const int H = a.plan.n, Wh = a.Wh, cols = a.cols;
    const int lgc = __ffs(cols) - 1;  // cols is a power of two
    const long long p = item / a.colblocks;
    const int c0 = (int)(item % a.colblocks) * cols;
    const int nc = min(cols, Wh - c0);
    C* S = a.spec + (size_t)p * H * Wh + c0;
    for (int idx = threadIdx.x; idx < H * cols; idx += blockDim.x) {
        const int i = idx >> lgc, c = idx & (cols - 1);  // coalesced across the block's columns
        A[i * cols + c] = c < nc ? S[(size_t)i * Wh + c] : mkx<T>(0, 0);
    }
    __syncthreads();
    C* res = gfft_lds<-1, BM>(A, B, a.plan, cols, tw, X);
    C* other = (res == A) ? B : A;
    if (a.dump) {
        C* D = a.dump + (size_t)p * H * Wh + c0;
        for (int idx = threadIdx.x; idx < H * cols; idx += blockDim.x) {
            const int i = idx >> lgc, c = idx & (cols - 1);
            if (c < nc) D[(size_t)i * Wh + c] = res[i * cols + c];
        }
    }
    if constexpr (MODE == 3) return;
    for (int idx = threadIdx.x; idx < H * cols; idx += blockDim.x) {
        const int ky = idx >> lgc, c = idx & (cols - 1);
        if (c >= nc) continue;
        const size_t f = (size_t)(c0 + c) * H + ky;
        C v = res[ky * cols + c];
        if constexpr (MODE == 0) v = cscale(v, a.fcT[f]);
        else if constexpr (MODE == 1) v = cmul(v, a.mT[f]);
        else v = cmulc(v, a.mT[f]);
        res[ky * cols + c] = v;
    }
    __syncthreads();
    const C* out = gfft_lds<+1, BM>(res, other, a.plan, cols, tw, X);
    for (int idx = threadIdx.x; idx < H * cols; idx += blockDim.x) {
        const int i = idx >> lgc, c = idx & (cols - 1);
        if (c < nc) S[(size_t)i * Wh + c] = out[i * cols + c];
    }
}

template <int MODE, int BM, bool TWG, int NT = GNT, class T = float, bool GLB = false>
__global__ void __launch_bounds__(NT, gcol_minw(BM)) k_gcol(GColArgsT<T> a) {
    using C = cx_t<T>;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int H = a.plan.n, cols = a.cols;
    C* twl = reinterpret_cast<C*>(smem);
    C* A = line_bufs<GLB>(twl, TWG ? 0 : H + a.plan.ntab, a.gscr, 2 * (size_t)H * cols);
    C* B = A + (size_t)H * cols;
    C* X = GLB ? nullptr : B + (size_t)H * cols;
    if constexpr (!TWG)
        for (int i = threadIdx.x; i < H + a.plan.ntab; i += blockDim.x) twl[i] = a.tw[i];
    const C* tw = TWG ? a.tw : twl;
#define ADMM_ITEM(item) gcol_item<MODE, BM>(a, A, B, X, tw, item)
    ADMM_GEN_ITEMS(a.P * a.colblocks, 1, ADMM_ITEM)
#undef ADMM_ITEM
}

// ---------------------------------------------------------------------------
// per-pixel ADMM step (the generic pass A).  Thread per pixel; the w of the right and lower
// neighbours is recomputed from the same inputs by the same expressions, so every pixel
// sees exactly the values its neighbours compute for themselves.
// ---------------------------------------------------------------------------
template <class T> struct GStepArgsT {
    const T* x;          // x_k                                   [P][H][W]
    const T* b;          // H_t(xin)
    const T* uxi;        // u_{k-1} (a_{k-1} when HIST)
    const T* uyi;
    T* uxo;              // u_k (a_k when HIST)
    T* uyo;
    T* r;                // r_{k+1} = b + rho D^T w_k (may be null: training's last iteration)
    const T* nsq;        // iso: N_k  [2][H][W]
    const T* nsq_prev;   // iso + HIST: N_{k-1}
    const T* lam;
    const T* rho;
    int H, W;
    long long npx;       // P H W
};
using GStepArgs = GStepArgsT<float>;

template <bool ISO, bool FIRST, bool HIST, class T>
__device__ __forceinline__ T gprev_u(const T* __restrict__ src, const T* __restrict__ np, size_t i, size_t hw, T tau) {
    if constexpr (FIRST) {
        return T(0);
    } else {
        const T v = src[i];
        if constexpr (HIST) return v - shrink_z<ISO>(v, tau, ISO ? np[hw] : T(0));
        else return v;
    }
}

// one pixel (image row `row` of P H, column j) of the step: writes u_k and returns r_{k+1}
// (b + rho D^T w; unused when a.r is null in k_gstep)
// (the image pointers as __restrict__ parameters: after inlining the compiler may move one
// pixel's loads above another's stores, so a thread's pixels overlap their memory latency)
template <bool ISO, bool FIRST, bool HIST, class T>
__device__ __forceinline__ T gstep_pxr(const GStepArgsT<T>& a, const T* __restrict__ xs, const T* __restrict__ bs,
                                       const T* __restrict__ uxs, const T* __restrict__ uys, T* __restrict__ uxd,
                                       T* __restrict__ uyd, unsigned row, int j) {
    const int H = a.H, W = a.W;
    const int i = (int)(row % (unsigned)H);
    const long long pb = (long long)(row - (unsigned)i) * W;
    const long long idx = pb + (long long)i * W + j;
    const int rem = i * W + j;
    const long long HW = (long long)H * W;
    const int jm = j == 0 ? W - 1 : j - 1, jp = j == W - 1 ? 0 : j + 1;
    const int im = i == 0 ? H - 1 : i - 1, ip = i == H - 1 ? 0 : i + 1;
    const size_t P0 = (size_t)idx, PR = (size_t)(pb + (long long)i * W + jp), PD = (size_t)(pb + (long long)ip * W + j);
    const size_t h0 = (size_t)rem, hR = (size_t)i * W + jp, hD = (size_t)ip * W + j;
    const T rho = a.rho[0];
    const T tau = a.lam[0] / rho;
    const T x = xs[P0];
    const T xl = xs[pb + (long long)i * W + jm], xr = xs[PR];
    const T xu = xs[pb + (long long)im * W + j], xd = xs[PD];
    const T* npx = a.nsq_prev;
    const T* npy = a.nsq_prev ? a.nsq_prev + HW : nullptr;
    const T ux0 = gprev_u<ISO, FIRST, HIST>(uxs, npx, P0, h0, tau);
    const T uxR = gprev_u<ISO, FIRST, HIST>(uxs, npx, PR, hR, tau);
    const T uy0 = gprev_u<ISO, FIRST, HIST>(uys, npy, P0, h0, tau);
    const T uyD = gprev_u<ISO, FIRST, HIST>(uys, npy, PD, hD, tau);
    T nx0 = 0, nxR = 0, ny0 = 0, nyD = 0;
    if constexpr (ISO) {
        nx0 = a.nsq[h0];
        nxR = a.nsq[hR];
        ny0 = a.nsq[HW + h0];
        nyD = a.nsq[HW + hD];
    }
    // own pixel
    const T ax = (x - xl) + ux0, ay = (x - xu) + uy0;
    const T zx = shrink_z<ISO>(ax, tau, nx0), zy = shrink_z<ISO>(ay, tau, ny0);
    const T nux = ax - zx, nuy = ay - zy;
    const T wx = zx - nux, wy = zy - nuy;
    // right neighbour's w_x and lower neighbour's w_y
    const T axR = (xr - x) + uxR, ayD = (xd - x) + uyD;
    const T zxR = shrink_z<ISO>(axR, tau, nxR), zyD = shrink_z<ISO>(ayD, tau, nyD);
    const T wxR = zxR - (axR - zxR), wyD = zyD - (ayD - zyD);
    uxd[P0] = HIST ? ax : nux;
    uyd[P0] = HIST ? ay : nuy;
    const T v = (wx - wxR) + (wy - wyD);
    return fmat(rho, v, bs[P0]);
}

template <bool ISO, bool FIRST, bool HIST, class T>
__device__ __forceinline__ T gstep_px(const GStepArgsT<T>& a, unsigned row, int j) {
    return gstep_pxr<ISO, FIRST, HIST>(a, a.x, a.b, a.uxi, a.uyi, a.uxo, a.uyo, row, j);
}

template <bool ISO, bool FIRST, bool HIST, class T = float>
__global__ void __launch_bounds__(256) k_gstep(GStepArgsT<T> a) {
    // grid (rows P H, column chunks): one 32-bit division per thread instead of 64-bit ones
    const int j = (int)(blockIdx.y * blockDim.x + threadIdx.x);
    if (j >= a.W) return;
    const T r = gstep_px<ISO, FIRST, HIST>(a, blockIdx.x, j);
    if (a.r) a.r[(size_t)blockIdx.x * a.W + j] = r;
}

// the step fused into the next row transform (inference): a block computes r_{k+1} for its
// 2 lines rows pixel by pixel (gstep_px, writing u_k) straight into the LDS image of k_grow_fwd,
// so r never goes through HBM (-8 B/px and one launch per iteration)
template <int BM, bool ISO, bool FIRST, class T>
__device__ __forceinline__ void grow_fwd_step_item(const GRowArgsT<T>& a, const GStepArgsT<T>& g, cx_t<T>* A,
                                                   cx_t<T>* B, cx_t<T>* X, const cx_t<T>* tw, long long r0) {
    using C = cx_t<T>;
    const int W = a.plan.n, Wh = W / 2 + 1, lines = a.lines;
    const int nl = (int)min((long long)2 * lines, a.rows - r0);
    // both rows of a complex line per step: two pixels' loads in flight together
    for (int c = 0; c < lines; ++c)
        for (int i = threadIdx.x; i < W; i += blockDim.x) {
            const int rr = 2 * c;
            T v0 = 0, v1 = 0;
            if (rr + 1 < nl) {
                v0 = gstep_pxr<ISO, FIRST, false>(g, g.x, g.b, g.uxi, g.uyi, g.uxo, g.uyo, (unsigned)(r0 + rr), i);
                v1 = gstep_pxr<ISO, FIRST, false>(g, g.x, g.b, g.uxi, g.uyi, g.uxo, g.uyo, (unsigned)(r0 + rr + 1), i);
            } else if (rr < nl) {
                v0 = gstep_pxr<ISO, FIRST, false>(g, g.x, g.b, g.uxi, g.uyi, g.uxo, g.uyo, (unsigned)(r0 + rr), i);
            }
            A[i * lines + c] = mkx<T>(v0, v1);  // even row -> real part, odd row -> imaginary part
        }
    __syncthreads();
    const C* res = gfft_lds<-1, BM>(A, B, a.plan, lines, tw, X);
    const T half = T(0.5);
    const long long ld = a.ldw ? a.ldw : Wh;
    for (int c = 0; c < lines; ++c)
        for (int k = threadIdx.x; k < Wh; k += blockDim.x) {
            const C z = res[k * lines + c];
            const C m = res[(k == 0 ? 0 : W - k) * lines + c];
            const long long ra = r0 + 2 * c;
            if (2 * c < nl) a.spec[ra * ld + k] = mkx<T>(half * (z.x + m.x), half * (z.y - m.y));
            if (2 * c + 1 < nl) a.spec[(ra + 1) * ld + k] = mkx<T>(half * (z.y + m.y), half * (m.x - z.x));
        }
}

template <int BM, bool TWG, bool ISO, bool FIRST, int NT = GNT, class T = float, bool GLB = false>
__global__ void __launch_bounds__(NT) k_grow_fwd_step(GRowArgsT<T> a, GStepArgsT<T> g) {
    using C = cx_t<T>;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int W = a.plan.n, lines = a.lines;
    C* twl = reinterpret_cast<C*>(smem);
    C* A = line_bufs<GLB>(twl, TWG ? 0 : W + a.plan.ntab, a.gscr, 2 * (size_t)W * lines);
    C* B = A + (size_t)W * lines;
    C* X = GLB ? nullptr : B + (size_t)W * lines;
    if constexpr (!TWG)
        for (int i = threadIdx.x; i < W + a.plan.ntab; i += blockDim.x) twl[i] = a.tw[i];
    const C* tw = TWG ? a.tw : twl;
#define ADMM_ITEM(r0) grow_fwd_step_item<BM, ISO, FIRST>(a, g, A, B, X, tw, r0)
    ADMM_GEN_ITEMS((a.rows + 2 * lines - 1) / (2 * lines), 2 * lines, ADMM_ITEM)
#undef ADMM_ITEM
}

// iso: N_k[pixel] = sum over planes of a_x^2, a_y^2 with a = D x_k + u_{k-1}
template <bool FIRST, bool HIST, class T = float>
__global__ void __launch_bounds__(256) k_giso_norm(const T* __restrict__ x, const T* __restrict__ uxi,
                                                   const T* __restrict__ uyi, const T* __restrict__ nprev,
                                                   const T* __restrict__ lam, const T* __restrict__ rho,
                                                   T* __restrict__ nsq, int H, int W, long long P) {
    const long long HW = (long long)H * W;
    const long long hw = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (hw >= HW) return;
    const int i = (int)(hw / W), j = (int)(hw % W);
    const int jm = j == 0 ? W - 1 : j - 1, im = i == 0 ? H - 1 : i - 1;
    const T tau = lam[0] / rho[0];
    T sx = 0, sy = 0;
    for (long long p = 0; p < P; ++p) {
        const long long o = p * HW;
        const T xc = x[o + hw];
        const T ux = gprev_u<true, FIRST, HIST>(uxi, nprev, (size_t)(o + hw), (size_t)hw, tau);
        const T uy = gprev_u<true, FIRST, HIST>(uyi, nprev ? nprev + HW : nullptr, (size_t)(o + hw), (size_t)hw, tau);
        const T ax = (xc - x[o + (long long)i * W + jm]) + ux;
        const T ay = (xc - x[o + (long long)im * W + j]) + uy;
        sx = fmat(ax, ax, sx);
        sy = fmat(ay, ay, sy);
    }
    nsq[hw] = sx;
    nsq[HW + hw] = sy;
}

// ---------------------------------------------------------------------------
// backward: per-pixel reverse step (the generic k_bwd_pass_a)
// ---------------------------------------------------------------------------
template <class T> struct GBwdArgsT {
    const T* rb;          // r^_k                               [P][H][W]
    T* xb;                // x^_{k-1} (k >= 2)
    T* bbar;              // b^ accumulator
    const T* abx_in;      // a^_k (k < K)
    const T* aby_in;
    T* abx_out;           // a^_{k-1} (k >= 2)
    T* aby_out;
    const T* akx;         // a_k
    const T* aky;
    const T* apx;         // a_{k-1} (k >= 2)
    const T* apy;
    const T* np;          // iso: N_{k-1}  [2][H][W]
    const T* qp;          // iso: Q_{k-1}  [2][H][W]
    const T* lam;
    const T* rho;
    double* part;         // per block {rho^, tau^}, fp64
    int H, W;
    long long npx;
};
using GBwdArgs = GBwdArgsT<float>;

template <bool ISO, bool LASTK, bool FIRSTK, class T>
__device__ __forceinline__ T gabar(T d, T ap, T ub, T tau, T rho, T n, T q) {
    const T wb = rho * d;
    const T zb = T(2) * wb - ub;
    return ub - wb + shrink_vjp<ISO>(ap, zb, tau, n, q);
}

template <bool ISO, bool LASTK, bool FIRSTK, class T = float>
__global__ void __launch_bounds__(256) k_gbwd(GBwdArgsT<T> a) {
    __shared__ double red[2][256];  // the lambda / rho partials reduce in fp64
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    double rho_acc = 0.0, tau_acc = 0.0;
    if (idx < a.npx) {
        const int H = a.H, W = a.W;
        const long long HW = (long long)H * W;
        const long long pb = idx - idx % HW;
        const int rem = (int)(idx % HW), i = rem / W, j = rem % W;
        const int jm = j == 0 ? W - 1 : j - 1, jp = j == W - 1 ? 0 : j + 1;
        const int im = i == 0 ? H - 1 : i - 1, ip = i == H - 1 ? 0 : i + 1;
        const size_t P0 = (size_t)idx, PR = (size_t)(pb + (long long)i * W + jp), PD = (size_t)(pb + (long long)ip * W + j);
        const size_t h0 = (size_t)rem, hR = (size_t)i * W + jp, hD = (size_t)ip * W + j;
        const T rho = a.rho[0];
        const T tau = a.lam[0] / rho;
        const T r0 = a.rb[P0];
        const T rl = a.rb[pb + (long long)i * W + jm], rr = a.rb[PR];
        const T ru = a.rb[pb + (long long)im * W + j], rd = a.rb[PD];
        const T dx0 = r0 - rl, dy0 = r0 - ru;  // D r^ at the pixel
        // rho^ partial: D r^ . (w_{k-1} - D x_k), w = 2z - a, D x_k = a_k - a_{k-1} + z_{k-1}
        T apx0 = 0, apy0 = 0, nx0 = 0, ny0 = 0;
        if constexpr (!FIRSTK) {
            apx0 = a.apx[P0];
            apy0 = a.apy[P0];
            if constexpr (ISO) {
                nx0 = a.np[h0];
                ny0 = a.np[HW + h0];
            }
        }
        const T zpx = FIRSTK ? T(0) : shrink_z<ISO>(apx0, tau, nx0);
        const T zpy = FIRSTK ? T(0) : shrink_z<ISO>(apy0, tau, ny0);
        {
            const T ex = (T(2) * zpx - apx0) - (a.akx[P0] - apx0 + zpx);
            const T ey = (T(2) * zpy - apy0) - (a.aky[P0] - apy0 + zpy);
            rho_acc = fma((double)dx0, (double)ex, (double)dy0 * (double)ey);
        }
        // b^ += r^
        a.bbar[P0] = LASTK ? r0 : a.bbar[P0] + r0;
        if constexpr (!FIRSTK) {
            T qx0 = 0, qy0 = 0, qxR = 0, qyD = 0, nxR = 0, nyD = 0;
            if constexpr (ISO) {
                qx0 = a.qp[h0];
                qy0 = a.qp[HW + h0];
                qxR = a.qp[hR];
                qyD = a.qp[HW + hD];
                nxR = a.np[hR];
                nyD = a.np[HW + hD];
            }
            const T ubx0 = LASTK ? T(0) : a.abx_in[P0], uby0 = LASTK ? T(0) : a.aby_in[P0];
            const T ubxR = LASTK ? T(0) : a.abx_in[PR], ubyD = LASTK ? T(0) : a.aby_in[PD];
            const T abx0 = gabar<ISO, LASTK, FIRSTK>(dx0, apx0, ubx0, tau, rho, nx0, qx0);
            const T aby0 = gabar<ISO, LASTK, FIRSTK>(dy0, apy0, uby0, tau, rho, ny0, qy0);
            // a^_x at the right neighbour, a^_y at the lower one
            const T abxR = gabar<ISO, LASTK, FIRSTK>(rr - r0, a.apx[PR], ubxR, tau, rho, nxR, qxR);
            const T abyD = gabar<ISO, LASTK, FIRSTK>(rd - r0, a.apy[PD], ubyD, tau, rho, nyD, qyD);
            a.abx_out[P0] = abx0;
            a.aby_out[P0] = aby0;
            a.xb[P0] = (abx0 - abxR) + (aby0 - abyD);
            if constexpr (!ISO) {
                const T wbx = rho * dx0, wby = rho * dy0;
                tau_acc = (double)soft_dtau(apx0, T(2) * wbx - ubx0, tau) + (double)soft_dtau(apy0, T(2) * wby - uby0, tau);
            }
        }
    }
    red[0][threadIdx.x] = rho_acc;
    red[1][threadIdx.x] = tau_acc;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            red[0][threadIdx.x] += red[0][threadIdx.x + o];
            red[1][threadIdx.x] += red[1][threadIdx.x + o];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        a.part[2 * blockIdx.x + 0] = red[0][0];
        a.part[2 * blockIdx.x + 1] = red[1][0];
    }
}

// iso backward: Q_{k-1}[pixel] = sum over planes of a_{k-1} z^_{k-1}, z^ = 2 rho D r^_k - a^_k
template <bool LASTK, class T = float>
__global__ void __launch_bounds__(256) k_giso_q(const T* __restrict__ rb, const T* __restrict__ abx,
                                                const T* __restrict__ aby, const T* __restrict__ apx,
                                                const T* __restrict__ apy, const T* __restrict__ rho_p,
                                                T* __restrict__ q, int H, int W, long long P) {
    const long long HW = (long long)H * W;
    const long long hw = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (hw >= HW) return;
    const int i = (int)(hw / W), j = (int)(hw % W);
    const int jm = j == 0 ? W - 1 : j - 1, im = i == 0 ? H - 1 : i - 1;
    const T rho = rho_p[0];
    T qx = 0, qy = 0;
    for (long long p = 0; p < P; ++p) {
        const long long o = p * HW;
        const T r0 = rb[o + hw];
        const T zx = T(2) * rho * (r0 - rb[o + (long long)i * W + jm]) - (LASTK ? T(0) : abx[o + hw]);
        const T zy = T(2) * rho * (r0 - rb[o + (long long)im * W + j]) - (LASTK ? T(0) : aby[o + hw]);
        qx = fmat(apx[o + hw], zx, qx);
        qy = fmat(apy[o + hw], zy, qy);
    }
    q[hw] = qx;
    q[HW + hw] = qy;
}

// PSF gradient on the generic path: acc[kx][ky] += sum_p conj(U_p) V_p at every half-plane
// frequency, U, V 2-D spectra [P][H][Wh] (column-pass dumps).  With fcT: only
// fc^2 Re(conj(U) V) is kept (the Wiener-factor path); without: the complex sum (Z).
template <class T = float>
__global__ void k_gxspec_acc(const cx_t<T>* __restrict__ U, const cx_t<T>* __restrict__ V, long long P, int H,
                             int Wh, const T* __restrict__ fcT, double2* __restrict__ acc) {
    const long long nf = (long long)H * Wh;
    const long long f = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= nf) return;
    const int ky = (int)(f / Wh), kx = (int)(f % Wh);
    double re = 0.0, im = 0.0;
    for (long long p = 0; p < P; ++p) {
        const cx_t<T> u = U[p * nf + f], v = V[p * nf + f];
        re += (double)u.x * v.x + (double)u.y * v.y;
        im += (double)u.x * v.y - (double)u.y * v.x;
    }
    const size_t i = (size_t)kx * H + ky;
    if (fcT) {
        const double c = fcT[i];
        acc[i].x += c * c * re;
    } else {
        acc[i].x += re;
        acc[i].y += im;
    }
}

}  // namespace admm

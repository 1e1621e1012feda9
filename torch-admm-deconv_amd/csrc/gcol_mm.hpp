// gcol_mm.hpp -- the generic column pass on the matrix cores, for column lengths H = S * R with an
// odd R in [17, 127] that carries H's large prime factor (BSD: 321 = 3 * 107), S <= 8.
//
// What it computes is k_gcol MODE 0 (generic_kernels.hpp): per half-spectrum column kx, the H-point
// DFT along the column, the real Wiener factor, the inverse DFT (both unnormalised; 1/(H W) is in the
// factor).  The reference's x-update, deconv.py:104-106, restricted to one column frequency.
//
// Decomposition (Cooley-Tukey, n = n2 + S n1 in, k = k1 + R k2 out):
//   1. R-point DFTs of the S decimated sequences x[n2 + S n1]            -> matrix cores
//   2. twiddle W_H^{n2 k1}, S-point DFT over n2, factor, inverse S-point
//      DFT, conjugate twiddle -- per (column, k1) in registers            -> VALU
//   3. inverse R-point DFTs                                               -> matrix cores
// The R-point DFT of a complex sequence x_q is taken on input sums and differences
// s_q = x_q + x_{R-q}, d_q = x_q - x_{R-q} (q = 1..h, h = (R-1)/2; s_0 = x_0, d_0 = 0):
//   P_k = sum_q cos(2 pi k q / R) s_q,  Q_k = sum_q sin(2 pi k q / R) d_q   (k = 0..h)
//   forward  Y_k = P_k - i Q_k,  Y_{R-k} = P_k + i Q_k   (inverse: the signs of Q swap)
// so both directions are two real (h+1) x (h+1) matrix products -- the cosine and sine matrices, the
// same for every column, plane and direction -- applied to the real and imaginary parts of every
// sequence of the block as separate matrix columns: a quarter of the multiplies of the plain complex
// DFT matrix.  They run as v_mfma_f32_16x16x4_f32 (exact fp32 products, one rounding each, the f32
// rate = the VALU peak): the matrices' fragments stay in registers for the whole block (a wave owns a
// 16-row tile of both), the s / d operands come from LDS.  The old column pass spent most of its time
// in the dependent exchange chains of its 107-point Bluestein stage (SQ counters).
//
// LDS image F (floats), one row per q (or k) in [0, 4 KS): element (q, j, slot) at q RP + 2 j + slot,
// real matrix column j = 2 seq + c (c: 0 real, 1 imaginary part; seq = n2 NL + L for column L of the
// block), slot 0: s_q (later Y_q, x_q), slot 1: d_q (later Y_{R-q}, x_{R-q}).  Every phase reads and
// writes the (q, seq) quadruple it owns in place, so one image serves the whole chain.  RP = 32 mod 64
// floats: the 16-lane groups of an operand read (8 B per lane, rows q .. q+3) hit disjoint banks.
#pragma once
#include "generic_kernels.hpp"

namespace admm {

struct GColMMArgs {
    cf* spec;          // [P][H][Wh], in place
    cf* dump;          // optional [P][H][Wh]: the forward column spectrum (before the factor)
    const float* fcN;  // Wiener factor, [H][Wh] (k_fc_transpose of fcT)
    const cf* tw;      // [H] exp(-2 pi i m / H)
    int H, R, h, KS, MT, NL, lgNL, RP, Wh, colblocks;
    long long P;
    int dbg;  // timing experiments only (ADMM_MM_DBG): phases to skip, results invalid when set
    int ldw;  // spectrum row pitch in complex values (>= Wh; the factor and the dump keep Wh)
};

typedef float mm_f32x4 __attribute__((ext_vector_type(4)));

// the value of the lane next to this one (lane ^ 1): DPP quad_perm [1, 0, 3, 2]
__device__ __forceinline__ float mm_pair_swap(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));
}

// both R-point transforms of the block: acc1 = C S1, acc2 = S S2 over this wave's NTW n-tiles
// (NTW compile-time: the wave's loads of a k-step are issued together, the MFMAs follow unguarded)
template <int NTW>
__device__ __forceinline__ void mm_products(const float* __restrict__ F, const float (&a1)[16], const float (&a2)[16],
                                            mm_f32x4 (&acc1)[8], mm_f32x4 (&acc2)[8], int KS, int RP, int tile0,
                                            int tstep, int g, int jl) {
    static_for<0, NTW>([&](auto tc) {
        constexpr int t = decltype(tc)::value;
        acc1[t] = mm_f32x4{0.f, 0.f, 0.f, 0.f};
        acc2[t] = mm_f32x4{0.f, 0.f, 0.f, 0.f};
    });
    const float2* F2 = reinterpret_cast<const float2*>(F) + g * (RP / 2) + 16 * tile0 + jl;
    // compile-time k-step / tile indices (static_for): the fragment and accumulator arrays must stay in
    // registers
    static_for<0, 16>([&](auto kc) {
        constexpr int ks = decltype(kc)::value;
        if (ks < KS) {  // KS is uniform: a scalar branch
            const float2* row = F2 + 4 * ks * (RP / 2);
            float2 b[NTW];
            static_for<0, NTW>([&](auto tc) {
                constexpr int t = decltype(tc)::value;
                b[t] = row[16 * t * tstep];
            });
            static_for<0, NTW>([&](auto tc) {
                constexpr int t = decltype(tc)::value;
                acc1[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[ks], b[t].x, acc1[t], 0, 0, 0);
                acc2[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a2[ks], b[t].y, acc2[t], 0, 0, 0);
            });
        }
    });
}

// combine P (acc1) and Q (acc2) into the two outputs of each row k and store them at (k, j):
// forward (DIR < 0) Y_k = P - i Q, Y_{R-k} = P + i Q; inverse the conjugate signs
template <int DIR, int NTW>
__device__ __forceinline__ void mm_store(float* __restrict__ F, const mm_f32x4 (&acc1)[8], const mm_f32x4 (&acc2)[8],
                                         int h, int RP, int tile0, int tstep, int mt, int g, int jl) {
    const int c = jl & 1;
    // a lane holds the real (c = 0) or imaginary (c = 1) part; its partner lane ^ 1 the other part of Q
    // forward, c = 0: Re Y_k = Pr + Qi;  c = 1: Im Y_k = Pi - Qr   (inverse: the opposite signs)
    const bool plus = (c == 0) == (DIR < 0);
    float2* F2 = reinterpret_cast<float2*>(F);
    static_for<0, NTW>([&](auto tc) {
        constexpr int t = decltype(tc)::value;
        const int j = 16 * (tile0 + t * tstep) + jl;
        static_for<0, 4>([&](auto rc) {
            constexpr int r = decltype(rc)::value;
            const float P = acc1[t][r], Qo = mm_pair_swap(acc2[t][r]);
            const int k = 16 * mt + 4 * g + r;
            const float yk = plus ? P + Qo : P - Qo, yr = plus ? P - Qo : P + Qo;
            if (k <= h) F2[k * (RP / 2) + j] = make_float2(yk, yr);
        });
    });
}

// runs f(integral_constant NTW) for the wave's tile count (wave-uniform, 0: no call); instances up to
// MAXT (the accumulator registers of the largest instance are reserved for all)
template <int MAXT = 8, class Fn> __device__ __forceinline__ void mm_ntw(int ntw, Fn&& f) {
    switch (ntw) {
        case 1: f(std::integral_constant<int, 1>{}); break;
        case 2: f(std::integral_constant<int, 2>{}); break;
        case 3: if constexpr (MAXT >= 3) f(std::integral_constant<int, 3>{}); break;
        case 4: if constexpr (MAXT >= 4) f(std::integral_constant<int, 4>{}); break;
        case 5: if constexpr (MAXT >= 5) f(std::integral_constant<int, 5>{}); break;
        case 6: if constexpr (MAXT >= 6) f(std::integral_constant<int, 6>{}); break;
        case 7: if constexpr (MAXT >= 7) f(std::integral_constant<int, 7>{}); break;
        case 8: if constexpr (MAXT >= 8) f(std::integral_constant<int, 8>{}); break;
        default: break;
    }
}

// per (column, k1): twiddle, S-point DFT, factor (and dump), inverse S-point DFT, conjugate twiddle
template <int S>
__device__ __forceinline__ void mm_column_mid(cf (&v)[S], const float (&f)[S], int kk, int kx, bool valid,
                                              const GColMMArgs& a, const cf* __restrict__ tw, cf* __restrict__ dump) {
    cf w[S];
#pragma unroll
    for (int n2 = 1; n2 < S; ++n2) {
        w[n2] = tw[n2 * kk];
        v[n2] = cmul(v[n2], w[n2]);
    }
    small_dft<-1, S>(v, tw, a.H);
#pragma unroll
    for (int k2 = 0; k2 < S; ++k2) {
        if (dump && valid) dump[(size_t)(kk + a.R * k2) * a.Wh + kx] = v[k2];
        v[k2] = cscale(v[k2], f[k2]);
    }
    small_dft<+1, S>(v, tw, a.H);
#pragma unroll
    for (int n2 = 1; n2 < S; ++n2) v[n2] = cmulc(v[n2], w[n2]);
}

// items per thread of the load / store loops whose global accesses are issued together
constexpr int kMMU = 4;

// NTH threads per block (256 or 512, ADMM_GCOL_MM_NT): with 512 the waves of a row tile split its n-tiles
// (fewer accumulators per wave) and more waves per CU are resident
template <int S, int NTH = 256>
__global__ void __launch_bounds__(NTH) __attribute__((amdgpu_waves_per_eu(NTH == 512 ? 4 : (S <= 3 ? 3 : 2))))
k_gcol_mm(GColMMArgs a) {
    extern __shared__ __attribute__((aligned(16))) float F[];
    const int H = a.H, R = a.R, h = a.h, NL = a.NL, RP = a.RP, KS = a.KS, MT = a.MT, Wh = a.Wh;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar branches below
    const int jl = lane & 15, g = lane >> 4;
    const long long item = blockIdx.x;
    const long long p = item / a.colblocks;
    const int c0 = (int)(item % a.colblocks) * NL;
    const int ld = a.ldw;
    cf* Sp = a.spec + (size_t)p * H * ld + c0;
    cf* Dp = a.dump ? a.dump + (size_t)p * H * Wh : nullptr;  // indexed by the absolute column kx
    cf* twl = reinterpret_cast<cf*>(F + 4 * KS * RP);       // the H twiddles, after the image

    // wave -> (row tile mt, n-tiles tile0, tile0 + tstep, ...): MT row tiles of 16, G waves per tile
    const int NT = (NL * S + 7) / 8;  // n-tiles of 16 real columns (the last one padded)
    const int G = (NTH / 64) / MT;  // waves per row tile
    const bool gw = wv < MT * G;
    const int mt = wv % MT, tile0 = wv / MT, tstep = G;
    const int ntw = gw ? (NT - tile0 + G - 1) / G : 0;

    // load: s_q, d_q of every sequence (L, n2), straight from the spectrum (rows of NL columns); a
    // thread's kMMU items issue their loads together
    const int nload = NL * S * (h + 1);
    for (int base = tid; base < nload; base += NTH * kMMU) {
        cf x0[kMMU], x1[kMMU];
        static_for<0, kMMU>([&](auto uc) {
            constexpr int u = decltype(uc)::value;
            const int it = base + NTH * u;
            const int L = it & (NL - 1), rest = it >> a.lgNL;
            const int n2 = rest % S, q = rest / S;
            x0[u] = x1[u] = mkc(0.f, 0.f);
            if (!(a.dbg & 8) && it < nload && c0 + L < Wh) {
                x0[u] = Sp[(size_t)(n2 + S * q) * ld + L];
                if (q) x1[u] = Sp[(size_t)(n2 + S * (R - q)) * ld + L];
            }
        });
        static_for<0, kMMU>([&](auto uc) {
            constexpr int u = decltype(uc)::value;
            const int it = base + NTH * u;
            const int L = it & (NL - 1), rest = it >> a.lgNL;
            const int n2 = rest % S, q = rest / S;
            if (it < nload)
                *reinterpret_cast<float4*>(&F[q * RP + 4 * (n2 * NL + L)]) =
                    q ? make_float4(x0[u].x + x1[u].x, x0[u].x - x1[u].x, x0[u].y + x1[u].y, x0[u].y - x1[u].y)
                      : make_float4(x0[u].x, 0.f, x0[u].y, 0.f);
        });
    }
    for (int i = tid; i < H; i += NTH) twl[i] = a.tw[i];
    // rows h+1 .. 4 KS - 1 are the k-steps' padding: zero (their matrix entries are zero too)
    for (int idx = tid; idx < (4 * KS - h - 1) * RP; idx += NTH) F[(h + 1) * RP + idx] = 0.f;

    __syncthreads();

    // this lane's fragments of the cosine / sine matrices: A[i = lane & 15][q = lane >> 4] of each
    // 16 x 4 k-step; cos / sin(2 pi m / R) = Re / -Im tw[m S], m = i q mod R stepped by 4 i mod R
    float a1[16], a2[16];
    {
        const int i = 16 * mt + jl;
        const int step = (4 * i) % R;
        int m = (i * g) % R;
        static_for<0, 16>([&](auto kc) {
            constexpr int ks = decltype(kc)::value;
            const int q = 4 * ks + g;
            const bool ok = gw && ks < KS && i <= h && q <= h;
            const cf w = ok ? twl[m * S] : mkc(0.f, 0.f);
            a1[ks] = w.x;
            a2[ks] = -w.y;
            m += step;
            m -= (m >= R) ? R : 0;
        });
    }
    mm_f32x4 acc1[8], acc2[8];  // (the entries a wave's tile count uses)
    if (!(a.dbg & 1)) mm_ntw<NTH == 512 ? 4 : (2 * S < 8 ? 2 * S : 8)>(ntw, [&](auto nc) { mm_products<decltype(nc)::value>(F, a1, a2, acc1, acc2, KS, RP, tile0, tstep, g, jl); });
    __syncthreads();  // every operand read before the outputs overwrite them
    mm_ntw<NTH == 512 ? 4 : (2 * S < 8 ? 2 * S : 8)>(ntw, [&](auto nc) { mm_store<-1, decltype(nc)::value>(F, acc1, acc2, h, RP, tile0, tstep, mt, g, jl); });

    // per (column L, k1 <= h): outputs k1 and R - k1 of all S sequences -> factor -> inverse
    // inputs, stored as the sums / differences the inverse R-point transforms take.  A thread has at
    // most MAXI such items (NL (h + 1) <= 1,024); their factors are loaded before the barrier.
    const int nmid = NL * (h + 1);
    constexpr int MAXI = 1024 / NTH;                    // items per thread at most
    constexpr int MI = S <= 4 ? MAXI : (MAXI < 2 ? MAXI : 2);  // items whose factors are prefetched
    float fk[MAXI][S], fr[MAXI][S];
    auto load_f = [&](auto uc) {
        constexpr int u = decltype(uc)::value;
        const int it = tid + NTH * u;
        const int L = it & (NL - 1), k1 = it >> a.lgNL;
        const int kx = c0 + L;
        const bool ok = it < nmid && kx < Wh;
#pragma unroll
        for (int k2 = 0; k2 < S; ++k2) {
            fk[u][k2] = ok ? a.fcN[(size_t)(k1 + R * k2) * Wh + kx] : 0.f;
            fr[u][k2] = ok && k1 ? a.fcN[(size_t)(R - k1 + R * k2) * Wh + kx] : 0.f;
        }
    };
    static_for<0, MI>(load_f);
    __syncthreads();
    static_for<0, MAXI>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        const int it = tid + NTH * u;
        if (!(a.dbg & 4) && it < nmid) {
            if constexpr (u >= MI) load_f(uc);
            const int L = it & (NL - 1), k1 = it >> a.lgNL;
            const int kx = c0 + L;
            const bool valid = kx < Wh;
            cf yk[S], yr[S];
#pragma unroll
            for (int n2 = 0; n2 < S; ++n2) {
                const float4 v = *reinterpret_cast<const float4*>(&F[k1 * RP + 4 * (n2 * NL + L)]);
                yk[n2] = mkc(v.x, v.z);
                yr[n2] = mkc(v.y, v.w);
            }
            mm_column_mid<S>(yk, fk[u], k1, kx, valid, a, twl, Dp);
            if (k1) mm_column_mid<S>(yr, fr[u], R - k1, kx, valid, a, twl, Dp);
#pragma unroll
            for (int n2 = 0; n2 < S; ++n2) {
                const cf x = yk[n2], y = yr[n2];
                const float4 v = k1 ? make_float4(x.x + y.x, x.x - y.x, x.y + y.y, x.y - y.y)
                                    : make_float4(x.x, 0.f, x.y, 0.f);
                *reinterpret_cast<float4*>(&F[k1 * RP + 4 * (n2 * NL + L)]) = v;
            }
        }
    });
    __syncthreads();

    if (!(a.dbg & 2)) mm_ntw<NTH == 512 ? 4 : (2 * S < 8 ? 2 * S : 8)>(ntw, [&](auto nc) { mm_products<decltype(nc)::value>(F, a1, a2, acc1, acc2, KS, RP, tile0, tstep, g, jl); });
    __syncthreads();
    mm_ntw<NTH == 512 ? 4 : (2 * S < 8 ? 2 * S : 8)>(ntw, [&](auto nc) { mm_store<+1, decltype(nc)::value>(F, acc1, acc2, h, RP, tile0, tstep, mt, g, jl); });
    __syncthreads();

    // store: x[n2 + S n1] and x[n2 + S (R - n1)] of every sequence
    const int nout = NL * S * (h + 1);
    for (int it = tid; it < nout; it += NTH) {
        const int L = it & (NL - 1), rest = it >> a.lgNL;
        const int n2 = rest % S, n1 = rest / S;
        if (c0 + L >= Wh || (a.dbg & 16)) continue;
        const float4 v = *reinterpret_cast<const float4*>(&F[n1 * RP + 4 * (n2 * NL + L)]);
        Sp[(size_t)(n2 + S * n1) * ld + L] = mkc(v.x, v.z);
        if (n1) Sp[(size_t)(n2 + S * (R - n1)) * ld + L] = mkc(v.y, v.w);
    }
}

// ---------------------------------------------------------------------------------------------
// Row inverse on the matrix cores (k_grow_inv_mm): half spectra -> real rows for row lengths
// W = S R (BSD: 481 = 13 * 37), the k_grow_inv contract (generic_kernels.hpp): two real rows a, b of
// a line as one complex sequence Z = Xa + i Xb with Hermitian completion (the imaginary parts of the
// self-conjugate bins dropped, as irfft does), its inverse DFT z = xa + i xb.
// Input index k = k1 + R k2, output n = n2 + S n1:
//   1. per (line, k1 <= h): Z[k1 + R k2] and Z[R - k1 + R k2] (k2 < S) from the staged half
//      spectra, inverse S-point DFT over k2, conjugate twiddle W_W^{-n2 k}, sums / differences
//   2. inverse R-point transforms as the cosine / sine matrix products (as k_gcol_mm)
//   3. rows a and b of every line written along n (coalesced)
// LDS: the block's 2 NL spectrum rows, then (aliased) the matrix image, columns seq = l S + n2.
// ---------------------------------------------------------------------------------------------
struct GRowInvMMArgs {
    const cf* spec;  // [rows][Wh]
    float* img;      // [rows][W]
    const cf* tw;    // [W] exp(-2 pi i m / W)
    long long rows;
    int W, R, h, KS, MT, NL, RP, Wh;
    int stage;       // floats of the staged spectrum rows (the image region starts at 0 too)
    int ldw;         // spectrum row pitch in complex values (>= Wh)
};

// occupancy target of the 256-thread row inverse (waves per SIMD; A/B build knob ADMM_GROW_INV_MM_W: 4 caps
// its VGPRs at 128 so four blocks share a CU instead of three)
#ifndef ADMM_GROW_INV_MM_W
#define ADMM_GROW_INV_MM_W 3
#endif
template <int S, int NTH = 256>
__global__ void __launch_bounds__(NTH) __attribute__((amdgpu_waves_per_eu(NTH == 512 ? 4 : ADMM_GROW_INV_MM_W)))
k_grow_inv_mm(GRowInvMMArgs a) {
    extern __shared__ __attribute__((aligned(16))) float F[];
    const int W = a.W, R = a.R, h = a.h, NL = a.NL, RP = a.RP, KS = a.KS, MT = a.MT, Wh = a.Wh;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int jl = lane & 15, g = lane >> 4;
    const long long r0 = (long long)blockIdx.x * 2 * NL;
    const int nrows = (int)min((long long)2 * NL, a.rows - r0);
    const int regn = max(a.stage, 4 * KS * RP);
    cf* Xs = reinterpret_cast<cf*>(F);        // staged spectrum rows [2 NL][Wh]
    cf* twl = reinterpret_cast<cf*>(F + regn);

    const int NT = (NL * S + 7) / 8;  // n-tiles of 16 real columns (the last one padded)
    const int G = (NTH / 64) / MT;
    const bool gw = wv < MT * G;
    const int mt = wv % MT, tile0 = wv / MT, tstep = G;
    const int ntw = gw ? (NT - tile0 + G - 1) / G : 0;

    {   // stage: the block's rows (contiguous in the spectrum when the pitch is Wh)
        const cf* src = a.spec + r0 * a.ldw;
        if (a.ldw == Wh) {
            const int n = nrows * Wh;
            for (int i = tid; i < n; i += NTH) Xs[i] = src[i];
        } else {
            for (int r = 0; r < nrows; ++r)
                for (int i = tid; i < Wh; i += NTH) Xs[r * Wh + i] = src[(size_t)r * a.ldw + i];
        }
        for (int i = nrows * Wh + tid; i < 2 * NL * Wh; i += NTH) Xs[i] = mkc(0.f, 0.f);
        for (int i = tid; i < W; i += NTH) twl[i] = a.tw[i];
    }
    __syncthreads();

    // Z[k] of line l from its two staged rows (Hermitian completion)
    auto zval = [&](int l, int k) -> cf {
        const bool lo = k < Wh;
        const int kk = lo ? k : W - k;
        cf xa = Xs[(2 * l) * Wh + kk], xb = Xs[(2 * l + 1) * Wh + kk];
        if (kk == 0 || 2 * kk == W) xa.y = xb.y = 0.f;
        if (!lo) xa.y = -xa.y, xb.y = -xb.y;
        return mkc(xa.x - xb.y, xa.y + xb.x);
    };
    // phase 1: one item (l, k1) per thread (NL (h + 1) <= NTH), kept in registers until the image may
    // overwrite the staged rows
    const int nmid = NL * (h + 1);
    float4 sd[S];
    const int l1 = tid % NL, k1 = tid / NL;
    if (tid < nmid) {
        cf v[S], vr[S];
#pragma unroll
        for (int k2 = 0; k2 < S; ++k2) {
            v[k2] = zval(l1, k1 + R * k2);
            vr[k2] = k1 ? zval(l1, R - k1 + R * k2) : mkc(0.f, 0.f);
        }
        small_dft<+1, S>(v, twl, W);
        small_dft<+1, S>(vr, twl, W);
#pragma unroll
        for (int n2 = 1; n2 < S; ++n2) {
            v[n2] = cmulc(v[n2], twl[n2 * k1]);
            if (k1) vr[n2] = cmulc(vr[n2], twl[n2 * (R - k1)]);
        }
#pragma unroll
        for (int n2 = 0; n2 < S; ++n2) {
            const cf x = v[n2], y = vr[n2];
            sd[n2] = k1 ? make_float4(x.x + y.x, x.x - y.x, x.y + y.y, x.y - y.y) : make_float4(x.x, 0.f, x.y, 0.f);
        }
    }
    __syncthreads();
    if (tid < nmid) {
#pragma unroll
        for (int n2 = 0; n2 < S; ++n2) *reinterpret_cast<float4*>(&F[k1 * RP + 4 * (l1 * S + n2)]) = sd[n2];
    }
    for (int idx = tid; idx < (4 * KS - h - 1) * RP; idx += NTH) F[(h + 1) * RP + idx] = 0.f;
    __syncthreads();

    float a1[16], a2[16];
    {
        const int i = 16 * mt + jl;
        const int step = (4 * i) % R;
        int m = (i * g) % R;
        static_for<0, 16>([&](auto kc) {
            constexpr int ks = decltype(kc)::value;
            const int q = 4 * ks + g;
            const bool ok = gw && ks < KS && i <= h && q <= h;
            const cf w = ok ? twl[m * S] : mkc(0.f, 0.f);
            a1[ks] = w.x;
            a2[ks] = -w.y;
            m += step;
            m -= (m >= R) ? R : 0;
        });
    }
    mm_f32x4 acc1[8], acc2[8];
    mm_ntw<NTH == 512 ? 4 : 8>(ntw, [&](auto nc) { mm_products<decltype(nc)::value>(F, a1, a2, acc1, acc2, KS, RP, tile0, tstep, g, jl); });
    __syncthreads();
    mm_ntw<NTH == 512 ? 4 : 8>(ntw, [&](auto nc) { mm_store<+1, decltype(nc)::value>(F, acc1, acc2, h, RP, tile0, tstep, mt, g, jl); });
    __syncthreads();

    // phase 3: z[n] of line l at n = n2 + S n1: (n1 <= h) slot 0 of row n1, else slot 1 of row R - n1
    for (int l = 0; l < NL && 2 * l < nrows; ++l) {
        float* dst = a.img + (r0 + 2 * l) * W;
        const bool two = 2 * l + 1 < nrows;
        for (int n = tid; n < W; n += NTH) {
            const int n1 = n / S, n2 = n - n1 * S;
            const bool lo = n1 <= h;
            const float* e = &F[(lo ? n1 : R - n1) * RP + 4 * (l * S + n2) + (lo ? 0 : 1)];
            dst[n] = e[0];
            if (two) dst[W + n] = e[2];
        }
    }
}

// the Wiener factor in the spectra's [H][Wh] order (fcN[ky][kx] = fcT[kx][ky]): the matrix-core column
// pass reads it along kx, the block's columns
__global__ void k_fc_transpose(const float* __restrict__ fcT, float* __restrict__ fcN, int H, int Wh) {
    const long long n = (long long)H * Wh;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < n;
         idx += (long long)gridDim.x * blockDim.x) {
        const int ky = (int)(idx / Wh), kx = (int)(idx % Wh);
        fcN[idx] = fcT[(size_t)kx * H + ky];
    }
}

}  // namespace admm

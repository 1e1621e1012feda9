// odd_kernels.hpp -- the fused row pass (pass A) of the two-launch iteration for ODD row lengths
// W = W1 W2 (W1, W2 odd and coprime, e.g. BSD's 481 = 13 * 37), gfx950.
//
// The generic path (generic_kernels.hpp) runs such sizes as three launches per iteration: the column
// pass, the row inverse (half spectra -> x image) and the step fused into the row forward (x image, u,
// b -> half spectra): 44 B/px.  Here the row inverse, the step and the row forward are ONE launch, so x
// never goes through HBM: pass A reads the x half spectra (4), u (8), b (4) and writes u (8) and the r
// half spectra (4) -- 28 B/px, the fused path's bytes; with the unchanged column pass (8) the iteration
// moves 36 B/px in two launches, as on the power-of-two and smooth-size paths.
//
// Work unit: one wave = one strip of RS = 2 NLD rows of a plane, walked independently of every other
// wave (no block barrier anywhere: a block is only a launch granule, so the waves of a CU are in
// different phases -- loads, transforms, the step -- and overlap one another; round 4's fused generic row
// pass, whose blocks went through ten barrier-separated phases together, lost to three launches).
//   1. the strip's half-spectrum rows in LDS as complex lines: rows (r0 + 2m, r0 + 2m + 1) as
//      Z = Xa + i Xb (line 1 + m, Hermitian completion as irfft does), and the two halo rows r0 - 1 and
//      r0 + nr (the rows above and below the strip) as line 0 -- one inverse for both halos;
//   2. inverse W-point DFTs of all the lines at once;
//   3. the step row by row (Dx, Dy from the x rows in LDS, shrink, dual update, w, then
//      r = b + rho D^T w one row behind, written over the x row it replaces);
//   4. forward W-point DFTs of the data lines, split into the rows' half spectra, stored.
// The W-point DFT is a prime-factor (Good-Thomas) transform on a W1 x W2 array, so it has no twiddle
// multiplications: element n of a line sits at (n A mod W1, n B mod W2) (A = W2^-1 mod W1,
// B = W1^-1 mod W2), frequency k at (k mod W1, k mod W2), and the transform is W1-point DFTs along the
// first axis and W2-point DFTs along the second, in place.  Batching every line of the strip into each
// stage keeps the lanes busy: the 37-point stage runs 13 DFTs per line, 52 over the wave's 4 lines.
// The odd-point DFTs run on input sums and differences with fp64-derived constants (OddTw, as
// small_dft), each output pair written to LDS as it is formed (the 37 inputs stay in registers, no
// output array).  Arithmetic is the generic kernels' operation for operation where they share a step
// (the Hermitian completion and split, the step's expressions), so the results agree to fp32 rounding
// of the transforms; every rounding is explicit (-ffp-contract=off).
#pragma once
#include "generic_kernels.hpp"
#include "odd_capi.hpp"

namespace admm {

// cos / sin(2 pi m / R), m <= (R - 1) / 2, for the larger odd radices of the fused odd-length rows
// (Python math.cos / math.sin in fp64, rounded to fp32 at use)
template <> struct OddTw<17> {
    static constexpr double C[9] = {1.0, 0.9324722294043558, 0.7390089172206591, 0.4457383557765383,
                                    0.09226835946330202, -0.2736629900720829, -0.6026346363792563,
                                    -0.850217135729614, -0.9829730996839018};
    static constexpr double S[9] = {0.0, 0.3612416661871529, 0.6736956436465572, 0.8951632913550623,
                                    0.9957341762950345, 0.961825643172819, 0.7980172272802396,
                                    0.5264321628773561, 0.18374951781657037};
};
template <> struct OddTw<19> {
    static constexpr double C[10] = {1.0, 0.9458172417006346, 0.7891405093963936, 0.5469481581224269,
                                     0.24548548714079924, -0.08257934547233227, -0.4016954246529694,
                                     -0.6772815716257409, -0.879473751206489, -0.9863613034027223};
    static constexpr double S[10] = {0.0, 0.32469946920468346, 0.6142127126896678, 0.8371664782625285,
                                     0.9694002659393304, 0.9965844930066698, 0.9157733266550574,
                                     0.7357239106731318, 0.4759473930370737, 0.16459459028073403};
};
template <> struct OddTw<37> {
    static constexpr double C[19] = {1.0, 0.9856159103477085, 0.9428774454610842, 0.8730141131611882,
                                     0.7780357543184395, 0.6606747233900815, 0.5243072835572317,
                                     0.3728564777803086, 0.21067926999572642, 0.04244120319614846,
                                     -0.12701781974687876, -0.2928227712765501, -0.4502037448176734,
                                     -0.5946331763042866, -0.7219560939545244, -0.8285096492438421,
                                     -0.9112284903881356, -0.9677329469334989, -0.9963974885425265};
    static constexpr double S[19] = {0.0, 0.16900082032184907, 0.33313979474205757, 0.48769494381363454,
                                     0.6282199972956423, 0.7506723052527243, 0.8515291377333113,
                                     0.9278890272965093, 0.9775552389476861, 0.9990989662046814,
                                     0.9919004352588768, 0.9561667347392511, 0.8929258581495685,
                                     0.8039971303669405, 0.6919388689775462, 0.5599747861375954,
                                     0.4119012482439928, 0.251978061385125, 0.0848059244755095};
};

// R-point DFT (R odd) of the R values at base[e * ES], in place in LDS: inputs into registers, input
// sums / differences s_q, d_q (q = 1 .. h), then each output pair k, R - k formed and stored
//   y_k, y_{R-k} = x_0 + sum_q s_q cos(2 pi qk / R)  -+ DIR i sum_q d_q sin(2 pi qk / R)
// (small_dft's odd branch, operation for operation)
template <int DIR, int R, int ES>
__device__ __forceinline__ void odd_dft_lds(cf* __restrict__ base) {
    constexpr int h = (R - 1) / 2;
    cf v[R];
#pragma unroll
    for (int e = 0; e < R; ++e) v[e] = base[e * ES];
    cf y0 = v[0];
    static_for<1, h + 1>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        const cf s = cadd(v[q], v[R - q]), d = csub(v[q], v[R - q]);
        v[q] = s;
        v[R - q] = d;
        y0 = cadd(y0, s);
    });
    static_for<1, h + 1>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        cf a = v[0], b = mkc(0.f, 0.f);
        static_for<1, h + 1>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            constexpr float c = odd_cos<R, float>((q * k) % R), sn = odd_sin<R, float>((q * k) % R);
            a.x = fmaf(v[q].x, c, a.x);
            a.y = fmaf(v[q].y, c, a.y);
            b.x = fmaf(v[R - q].x, sn, b.x);
            b.y = fmaf(v[R - q].y, sn, b.y);
        });
        const cf ib = mkc(-b.y, b.x);  // i b
        base[k * ES] = DIR < 0 ? csub(a, ib) : cadd(a, ib);
        base[(R - k) * ES] = DIR < 0 ? cadd(a, ib) : csub(a, ib);
    });
    base[0] = y0;
}

// one DFT stage over lines [l0, l0 + nl) of a wave's LDS image: per line NPER independent R-point DFTs,
// DFT i of line l on the elements l LS + i IS + e ES (e < R); the wave's lanes take the DFTs in turn
template <int DIR, int R, int NPER, int IS, int ES, int LS, int MAXL>
__device__ __forceinline__ void odd_stage(cf* __restrict__ X, int l0, int nl, int lane) {
    const int items = nl * NPER;
#pragma unroll 1
    for (int q = 0; q < (MAXL * NPER + 63) / 64; ++q) {
        const int it = lane + 64 * q;
        if (it < items) {
            const int l = it / NPER, i = it - l * NPER;
            odd_dft_lds<DIR, R, ES>(X + (l0 + l) * LS + i * IS);
        }
    }
}

// a^-1 mod m (a, m coprime)
__host__ __device__ constexpr int odd_inv_mod(int a, int m) {
    for (int i = 1; i < m; ++i)
        if ((a * i) % m == 1) return i;
    return 1;
}
// positions in the W1 x W2 prime-factor image of a line: frequency k at (k mod W1, k mod W2), pixel n at
// (n A mod W1, n B mod W2), A = W2^-1 mod W1, B = W1^-1 mod W2
template <int W1, int W2> __device__ __forceinline__ int odd_kpos(int k) { return (k % W1) * W2 + k % W2; }
template <int W1, int W2> __device__ __forceinline__ int odd_npos(int n) {
    constexpr int A = odd_inv_mod(W2 % W1, W1), B = odd_inv_mod(W1 % W2, W2);
    return ((n * A) % W1) * W2 + (n * B) % W2;
}


// LDS bytes of one wave: NLD + 1 lines of W complex values, then the w_x row (W floats)
template <int W, int NLD> __host__ __device__ constexpr int odd_wave_lds() {
    return (NLD + 1) * W * 8 + ((W * 4 + 15) / 16) * 16;
}

// threads per block (whole waves, each on its own strip; A/B builds: -DADMM_ODD_NT) and an optional
// occupancy target in waves per SIMD (-DADMM_ODD_MINW; 0: the compiler's choice).  Two-wave blocks
// (34.6 KB of LDS) measured best at BSD size, interleaved on one box (profiles/r06_ab_odd_launch.txt):
// 5,703-5,719 it/s against 5,487-5,530 with four-wave blocks (a CU then holds 2 of them, 8 waves, and
// no column-pass block beside them), 5,563-5,625 with one-wave blocks, 5,504-5,542 with three; strips of
// 4 rows (NLD 2, 13.5 KB per wave) 5,466-5,582; a 168-VGPR cap (3 waves per SIMD, 16 B spill) 5,658-5,669.
#ifndef ADMM_ODD_NT
#define ADMM_ODD_NT 128
#endif
#ifndef ADMM_ODD_MINW
#define ADMM_ODD_MINW 0
#endif
template <int W1, int W2, int NLD, bool FIRST>
__global__ void __launch_bounds__(ADMM_ODD_NT) __attribute__((amdgpu_waves_per_eu(ADMM_ODD_MINW > 0 ? ADMM_ODD_MINW : 1)))
k_pass_a_odd(OddPassAArgs a) {
    constexpr int W = W1 * W2, Wh = (W + 1) / 2, NL = NLD + 1, LS = W, RS = 2 * NLD;
    constexpr int JP = (W + 63) / 64;   // pixel slots of a lane (pixel n = lane + 64 j)
    constexpr int JK = (Wh + 63) / 64;  // half-spectrum slots of a lane (bin k = lane + 64 j)
    static_assert(W % 2 == 1 && W1 > 1 && W2 > 1, "odd coprime factors");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const long long s = (long long)blockIdx.x * (blockDim.x >> 6) + wv;  // this wave's strip
    if (s >= a.nstrips) return;  // whole waves only: nothing below synchronises across waves
    cf* X = reinterpret_cast<cf*>(smem + (size_t)wv * odd_wave_lds<W, NLD>());
    float* wxb = reinterpret_cast<float*>(X + NL * LS);
    const int H = a.H;
    const long long p = s / a.ns;
    const int r0 = (int)(s - p * a.ns) * RS;
    const int nr = min(RS, H - r0), nlf = (nr + 1) >> 1;  // rows of the strip, its data lines
    const long long pb = p * H;
    auto grow = [&](int ro) -> long long {  // global row of strip row ro (ro in [-1, nr]), circular in H
        int r = r0 + ro;
        r += r < 0 ? H : 0;
        r -= r >= H ? H : 0;
        return pb + r;
    };
    auto kpos = [](int k) { return odd_kpos<W1, W2>(k); };  // frequency k
    auto npos = [](int n) { return odd_npos<W1, W2>(n); };  // pixel n

    // 1. half spectra -> complex lines (line 0: rows r0 - 1 / r0 + nr; line 1 + m: rows r0 + 2m, + 1)
    {
        const size_t ld = (size_t)a.ld;
        cf xa[NL][JK], xb[NL][JK];
        static_for<0, NL>([&](auto lc) {
            constexpr int l = decltype(lc)::value;
            if (l <= nlf) {
                const long long ra = l == 0 ? grow(-1) : grow(2 * l - 2);
                const long long rb = l == 0 ? grow(nr) : grow(2 * l - 1);
                const bool vb = l == 0 || 2 * l - 1 < nr;
#pragma unroll
                for (int j = 0; j < JK; ++j) {
                    const int k = lane + 64 * j;
                    xa[l][j] = xb[l][j] = mkc(0.f, 0.f);
                    if (k < Wh) {
                        xa[l][j] = a.sin[(size_t)ra * ld + k];
                        if (vb) xb[l][j] = a.sin[(size_t)rb * ld + k];
                    }
                }
            }
        });
        static_for<0, NL>([&](auto lc) {
            constexpr int l = decltype(lc)::value;
            if (l <= nlf) {
                cf* Z = X + l * LS;
#pragma unroll
                for (int j = 0; j < JK; ++j) {
                    const int k = lane + 64 * j;
                    if (k < Wh) {
                        cf ca = xa[l][j], cb = xb[l][j];
                        if (k == 0) ca.y = cb.y = 0.f;  // irfft drops the DC bin's imaginary part
                        Z[kpos(k)] = mkc(ca.x - cb.y, ca.y + cb.x);              // Xa + i Xb
                        if (k) Z[kpos(W - k)] = mkc(ca.x + cb.y, cb.x - ca.y);   // conj(Xa) + i conj(Xb)
                    }
                }
            }
        });
    }
    // The step's u / b rows are loaded one row ahead of their use (row 0's are in flight during the
    // inverse transforms), and a row's u stores are issued one row later, after the next prefetch: the
    // strip walk is sequential, and gfx9's vmcnt counts stores too, so waiting for a prefetch would
    // otherwise also wait for the stores just issued.  Every load is unconditional (lanes past the row
    // end read its last pixel), so each iteration issues the same operations and the waits stay exact.
    // The row streams go through buffer resources of one row each (W floats): a lane past the row end has
    // an out-of-range offset, so its load returns 0 and its store is dropped by the hardware -- no per-lane
    // branch around a memory instruction (an exec-skip branch there made the compiler's waits conservative).
    constexpr int kNT = 2;  // cache policy of the streams: non-temporal (as the fused pass A, ADMM_NT)
    auto rowbuf = [&](const float* base, int ro) {
        return make_rsrc(base + (size_t)grow(ro) * W, (unsigned)(W * sizeof(float)));
    };
    // two register sets of prefetched rows, used alternately (the loop below is unrolled by two, so no
    // register copy forces an early wait): pf[s][0..2] = u_x, u_y, b
    float pf[2][3][JP];
    auto load_row = [&](int ro, auto sc) {
        constexpr int S = decltype(sc)::value;
        const rsrc_t rx = rowbuf(a.uxi, ro), ry = rowbuf(a.uyi, ro), rb = rowbuf(a.b, ro);
#pragma unroll
        for (int j = 0; j < JP; ++j) {
            const int off = (lane + 64 * j) * (int)sizeof(float);
            pf[S][0][j] = pf[S][1][j] = 0.f;
            if constexpr (!FIRST) {
                pf[S][0][j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rx, off, 0, kNT));
                pf[S][1][j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ry, off, 0, kNT));
            }
            // (the row below the strip: loaded for a uniform stream, unused)
            pf[S][2][j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rb, off, 0, kNT));
        }
    };
    load_row(0, std::integral_constant<int, 0>{});
    xsync<0>();
    // 2. inverse DFTs of lines 0 .. nlf: W1-point along the first axis, W2-point along the second
    odd_stage<+1, W1, W2, 1, W2, LS, NL>(X, 0, nlf + 1, lane);
    xsync<0>();
    odd_stage<+1, W2, W1, W2, 1, LS, NL>(X, 0, nlf + 1, lane);
    xsync<0>();

    // 3. the step, row by row (generic_kernels.hpp gstep_pxr's expressions)
    const float rho = a.rho[0];
    const float tau = a.lam[0] / rho;
    int pn[JP], pl[JP];
#pragma unroll
    for (int j = 0; j < JP; ++j) {
        const int n = lane + 64 * j;
        pn[j] = npos(n < W ? n : 0);
        pl[j] = npos(n == 0 ? W - 1 : (n < W ? n - 1 : 0));
    }
    // x of strip row ro: line and real / imaginary part
    auto xrow = [&](int ro) -> float* {
        const int l = (ro < 0 || ro >= nr) ? 0 : 1 + (ro >> 1);
        const int c = ro < 0 ? 0 : (ro >= nr ? 1 : (ro & 1));
        return reinterpret_cast<float*>(X + l * LS) + c;
    };
    float wxp[JP], wyp[JP], bp[JP], sux[JP], suy[JP];
    auto store_u = [&](int ro) {  // u of strip row ro (computed one iteration earlier)
        const rsrc_t rx = rowbuf(a.uxo, ro), ry = rowbuf(a.uyo, ro);
#pragma unroll
        for (int j = 0; j < JP; ++j) {
            const int off = (lane + 64 * j) * (int)sizeof(float);
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, sux[j]), rx, off, 0, kNT);
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, suy[j]), ry, off, 0, kNT);
        }
    };
    // one row: w (and, for the strip's own rows, u) of row ro, then r of row ro - 1
    auto step_row = [&](int ro, auto ownc, auto sc) {
        constexpr bool OWN = decltype(ownc)::value;  // false: the row below the strip (its w only)
        constexpr int S = decltype(sc)::value;       // the register set holding this row's u / b
        const float(&ux)[JP] = pf[S][0];
        const float(&uy)[JP] = pf[S][1];
        const float(&bb)[JP] = pf[S][2];
        if constexpr (OWN) load_row(ro + 1, std::integral_constant<int, 1 - S>{});  // in flight meanwhile
        if (ro > 0) store_u(ro - 1);
        const float* xc = xrow(ro);
        const float* xu = xrow(ro - 1);
        float wx[JP], wy[JP];
#pragma unroll
        for (int j = 0; j < JP; ++j) {
            const int n = lane + 64 * j;
            wx[j] = wy[j] = 0.f;
            if (n < W) {
                const float x = xc[2 * pn[j]], xl = xc[2 * pl[j]], xup = xu[2 * pn[j]];
                const float ax = (x - xl) + ux[j], ay = (x - xup) + uy[j];
                const float zx = soft(ax, tau), zy = soft(ay, tau);
                const float nux = ax - zx, nuy = ay - zy;
                wx[j] = zx - nux;
                wy[j] = zy - nuy;
                sux[j] = nux;
                suy[j] = nuy;
            }
        }
        if (ro > 0) {  // r of the row above: b + rho ((w_x - w_x right) + (w_y - w_y below))
            float* xr = xrow(ro - 1);
#pragma unroll
            for (int j = 0; j < JP; ++j) {
                const int n = lane + 64 * j;
                if (n < W) {
                    const float wxr = wxb[n == W - 1 ? 0 : n + 1];
                    const float v = (wxp[j] - wxr) + (wyp[j] - wy[j]);
                    xr[2 * pn[j]] = fmaf(rho, v, bp[j]);
                }
            }
        }
        if constexpr (OWN) {
            xsync<0>();  // every lane has read the previous row's w_x
#pragma unroll
            for (int j = 0; j < JP; ++j) {
                const int n = lane + 64 * j;
                if (n < W) wxb[n] = wx[j];
                wxp[j] = wx[j];
                wyp[j] = wy[j];
                bp[j] = bb[j];
            }
            xsync<0>();
        }
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
#pragma unroll 1
    for (int ro = 0; ro < nr; ro += 2) {
        step_row(ro, std::true_type{}, I0{});
        if (ro + 1 < nr) step_row(ro + 1, std::true_type{}, I1{});
    }
    if (nr & 1) step_row(nr, std::false_type{}, I1{});
    else step_row(nr, std::false_type{}, I0{});
    if (nr & 1) {  // the last data line's second row does not exist: zero it before the forward DFT
        float* xz = xrow(nr - 1) + 1;
#pragma unroll
        for (int j = 0; j < JP; ++j)
            if (lane + 64 * j < W) xz[2 * pn[j]] = 0.f;
    }
    xsync<0>();

    // 4. forward DFTs of the data lines, split into the two rows' half spectra (k_grow_fwd's split)
    odd_stage<-1, W2, W1, W2, 1, LS, NLD>(X, 1, nlf, lane);
    xsync<0>();
    odd_stage<-1, W1, W2, 1, W2, LS, NLD>(X, 1, nlf, lane);
    xsync<0>();
    const size_t ld = (size_t)a.ld;
#pragma unroll 1
    for (int m = 0; m < nlf; ++m) {
        const cf* Z = X + (1 + m) * LS;
        const long long ra = grow(2 * m);
        const bool vb = 2 * m + 1 < nr;
#pragma unroll
        for (int j = 0; j < JK; ++j) {
            const int k = lane + 64 * j;
            if (k < Wh) {
                const cf z = Z[kpos(k)];
                const cf mz = Z[kpos(k == 0 ? 0 : W - k)];
                st_pol<(ADMM_NT & 1) != 0>(&a.sout[(size_t)ra * ld + k], mkc(0.5f * (z.x + mz.x), 0.5f * (z.y - mz.y)));
                if (vb) st_pol<(ADMM_NT & 1) != 0>(&a.sout[(size_t)(ra + 1) * ld + k], mkc(0.5f * (z.y + mz.y), 0.5f * (mz.x - z.x)));
            }
        }
    }
}

}  // namespace admm

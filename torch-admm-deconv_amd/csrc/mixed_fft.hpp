// mixed_fft.hpp -- register/LDS FFTs of smooth (2^a 3^b 5^c) lengths for the fused two-pass
// iteration at non-power-of-two image sizes (gfx950).
//
// fft_core.hpp's transforms keep E values per lane with every radix dividing E, so every stage runs
// E/R butterflies per lane and the data stay in "natural layout" between stages.  A smooth length
// such as 960 = 16*4*15 has no small E that all its radices divide, so here a stage of radix R runs
// its N/R butterflies over the L lanes of the transform as Q = ceil(N/(R L)) per lane, the lanes past
// the last butterfly idle ("guarded" stages).  The stages still exchange through LDS only between
// them, and the first and last stage of a schedule read / write registers directly:
//   edge layout of a radix-R stage: lane t, register k  <->  element t + (N/R) k   (k < R, t < N/R)
// so a schedule (Ra, ..., Rb) reads layout(Ra) and writes layout(Rb), and the reversed schedule
// (Rb, ..., Ra) maps layout(Rb) back to layout(Ra).  The row pass uses that to keep its pixels in
// layout(Rb) with N/Rb lanes (a natural layout: E = Rb values per lane) and its spectra in layout(Ra).
//
// Butterflies: radix 2/4/8/16 from fft_core.hpp; radix 3 and 5 with exact-constant rotations;
// 6 = 2x3, 10 = 2x5, 12 = 4x3, 15 = 3x5 as prime-factor (Good-Thomas) butterflies (no twiddles);
// 9 = 3x3 Cooley-Tukey with constant twiddles.  Every rounding is an explicit operation (the library
// builds with -ffp-contract=off), as in fft_core.hpp.
#pragma once
#include "fft_core.hpp"

namespace admm {

// ---------------------------------------------------------------------------------------------
// small DFTs on a register array x[R] (in place): y_k = sum_n x_n exp(DIR 2 pi i n k / R)
// ---------------------------------------------------------------------------------------------
template <int R, int DIR> struct SDFT;

template <int DIR> struct SDFT<1, DIR> {
    __device__ __forceinline__ static void run(cf (&)[1]) {}
};
template <int DIR> struct SDFT<2, DIR> {
    __device__ __forceinline__ static void run(cf (&x)[2]) { DFT<2, DIR>::template run<1, 0>(x); }
};
template <int DIR> struct SDFT<4, DIR> {
    __device__ __forceinline__ static void run(cf (&x)[4]) { DFT<4, DIR>::template run<1, 0>(x); }
};
template <int DIR> struct SDFT<8, DIR> {
    __device__ __forceinline__ static void run(cf (&x)[8]) { DFT<8, DIR>::template run<1, 0>(x); }
};
template <int DIR> struct SDFT<16, DIR> {
    __device__ __forceinline__ static void run(cf (&x)[16]) { DFT<16, DIR>::template run<1, 0>(x); }
};

// radix 3: y1,2 = x0 - (x1 + x2)/2 +- DIR i (sqrt3/2)(x1 - x2)
template <int DIR> struct SDFT<3, DIR> {
    __device__ __forceinline__ static void run(cf (&x)[3]) {
        constexpr float s3 = 0.86602540378443865f;
        const cf b = cadd(x[1], x[2]), d = csub(x[1], x[2]);
        const cf m = mkc(fmaf(-0.5f, b.x, x[0].x), fmaf(-0.5f, b.y, x[0].y));
        const cf r = mul_i<DIR>(mkc(s3 * d.x, s3 * d.y));
        x[0] = cadd(x[0], b);
        x[1] = cadd(m, r);
        x[2] = csub(m, r);
    }
};

// radix 5 on input sums / differences (cos / sin of 2pi/5, 4pi/5)
template <int DIR> struct SDFT<5, DIR> {
    __device__ __forceinline__ static void run(cf (&x)[5]) {
        constexpr float c1 = 0.30901699437494742f, c2 = -0.80901699437494742f;
        constexpr float s1 = 0.95105651629515357f, s2 = 0.58778525229247313f;
        const cf b1 = cadd(x[1], x[4]), b2 = cadd(x[2], x[3]);
        const cf d1 = csub(x[1], x[4]), d2 = csub(x[2], x[3]);
        const cf r1 = mkc(fmaf(c2, b2.x, fmaf(c1, b1.x, x[0].x)), fmaf(c2, b2.y, fmaf(c1, b1.y, x[0].y)));
        const cf r2 = mkc(fmaf(c1, b2.x, fmaf(c2, b1.x, x[0].x)), fmaf(c1, b2.y, fmaf(c2, b1.y, x[0].y)));
        const cf i1 = mul_i<DIR>(mkc(fmaf(s1, d1.x, s2 * d2.x), fmaf(s1, d1.y, s2 * d2.y)));
        const cf i2 = mul_i<DIR>(mkc(fmaf(s2, d1.x, -(s1 * d2.x)), fmaf(s2, d1.y, -(s1 * d2.y))));
        x[0] = cadd(x[0], cadd(b1, b2));
        x[1] = cadd(r1, i1);
        x[4] = csub(r1, i1);
        x[2] = cadd(r2, i2);
        x[3] = csub(r2, i2);
    }
};

// prime-factor butterfly N = N1 N2 (coprime): input n = (N2 n1 + N1 n2) mod N, output
// k = (N2 (N2^-1 mod N1) k1 + N1 (N1^-1 mod N2) k2) mod N; N2-point DFTs over n2, then N1-point over n1
__host__ __device__ constexpr int inv_mod(int a, int m) {
    for (int i = 1; i < m; ++i)
        if ((a * i) % m == 1) return i;
    return 1;
}
template <int N1, int N2, int DIR> struct PFA {
    static constexpr int N = N1 * N2;
    __device__ __forceinline__ static void run(cf (&x)[N]) {
        cf t[N1][N2];
#pragma unroll
        for (int n1 = 0; n1 < N1; ++n1) {
#pragma unroll
            for (int n2 = 0; n2 < N2; ++n2) t[n1][n2] = x[(N2 * n1 + N1 * n2) % N];
            SDFT<N2, DIR>::run(t[n1]);
        }
#pragma unroll
        for (int k2 = 0; k2 < N2; ++k2) {
            cf u[N1];
#pragma unroll
            for (int n1 = 0; n1 < N1; ++n1) u[n1] = t[n1][k2];
            SDFT<N1, DIR>::run(u);
#pragma unroll
            for (int k1 = 0; k1 < N1; ++k1)
                x[(N2 * inv_mod(N2 % N1, N1) * k1 + N1 * inv_mod(N1 % N2, N2) * k2) % N] = u[k1];
        }
    }
};
template <int DIR> struct SDFT<6, DIR> {
    __device__ __forceinline__ static void run(cf (&x)[6]) { PFA<2, 3, DIR>::run(x); }
};
template <int DIR> struct SDFT<10, DIR> {
    __device__ __forceinline__ static void run(cf (&x)[10]) { PFA<2, 5, DIR>::run(x); }
};
template <int DIR> struct SDFT<12, DIR> {
    __device__ __forceinline__ static void run(cf (&x)[12]) { PFA<4, 3, DIR>::run(x); }
};
template <int DIR> struct SDFT<15, DIR> {
    __device__ __forceinline__ static void run(cf (&x)[15]) { PFA<3, 5, DIR>::run(x); }
};

// radix 9 = 3 x 3 (Cooley-Tukey): x[3 n1 + n2] -> 3-point DFTs over n1, twiddles W9^(n2 k1), 3-point
// DFTs over n2, y[k1 + 3 k2]
template <int DIR> struct SDFT<9, DIR> {
    __device__ __forceinline__ static void run(cf (&x)[9]) {
        // exp(DIR 2 pi i m / 9), m = 1, 2, 4
        constexpr float c1 = 0.76604444311897804f, s1 = 0.64278760968653933f;
        constexpr float c2 = 0.17364817766693035f, s2 = 0.98480775301220806f;
        constexpr float c4 = -0.93969262078590838f, s4 = 0.34202014332566873f;
        cf a[3][3];
#pragma unroll
        for (int n2 = 0; n2 < 3; ++n2) {
            cf u[3] = {x[n2], x[3 + n2], x[6 + n2]};
            SDFT<3, DIR>::run(u);
#pragma unroll
            for (int k1 = 0; k1 < 3; ++k1) a[k1][n2] = u[k1];
        }
        a[1][1] = cmul(a[1][1], mkc(c1, DIR * s1));
        a[2][1] = cmul(a[2][1], mkc(c2, DIR * s2));
        a[1][2] = cmul(a[1][2], mkc(c2, DIR * s2));
        a[2][2] = cmul(a[2][2], mkc(c4, DIR * s4));
#pragma unroll
        for (int k1 = 0; k1 < 3; ++k1) {
            SDFT<3, DIR>::run(a[k1]);
#pragma unroll
            for (int k2 = 0; k2 < 3; ++k2) x[k1 + 3 * k2] = a[k1][k2];
        }
    }
};

// ---------------------------------------------------------------------------------------------
// one guarded Stockham stage: radix R at span NS of an N-point transform over L lanes; lane t runs
// butterflies vt = t + L q (q < Q, vt < N / R), its inputs in registers v[q + Q k] (k < R)
// ---------------------------------------------------------------------------------------------
template <int N, int R> struct StageGeom {
    static constexpr int NB = N / R;
};

template <int N, int L, int EM, int R, int NS, int DIR, bool FIRST, bool LAST, int SYNC, int TWMUL, class Buf>
__device__ __forceinline__ void mstage(cf (&v)[EM], const Buf& buf, const cf* __restrict__ tw, int t) {
    constexpr int NB = N / R;
    constexpr int Q = (NB + L - 1) / L;
    constexpr bool FULL = NB % L == 0;
    static_assert(Q * R <= EM, "register array too small for this stage");
    if constexpr (!FIRST) {
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int vt = t + L * q;
            if (FULL || vt < NB) {
#pragma unroll
                for (int k = 0; k < R; ++k) v[q + Q * k] = buf.at(vt + k * NB);
            }
        }
    }
    static_for<0, Q>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        const int vt = t + L * q;
        if constexpr (NS > 1) {
            const int m = vt % NS;
#pragma unroll
            for (int k = 1; k < R; ++k) {
                const cf w = tw[(m * k) * (N / (NS * R)) * TWMUL];
                v[q + Q * k] = DIR < 0 ? cmul(v[q + Q * k], w) : cmulc(v[q + Q * k], w);
            }
        }
        cf y[R];
#pragma unroll
        for (int k = 0; k < R; ++k) y[k] = v[q + Q * k];
        SDFT<R, DIR>::run(y);
#pragma unroll
        for (int k = 0; k < R; ++k) v[q + Q * k] = y[k];
    });
    if constexpr (!LAST) {
        xsync<SYNC>();  // everyone has read before anyone overwrites
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int vt = t + L * q;
            if (FULL || vt < NB) {
                const int base = (vt / NS) * NS * R + vt % NS;
#pragma unroll
                for (int k = 0; k < R; ++k) buf.at(base + k * NS) = v[q + Q * k];
            }
        }
        xsync<SYNC>();
    }
}

template <int N, int L, int EM, int NS, int DIR, bool FIRST, int SYNC, int TWMUL, class Buf, int R, int... Rest>
__device__ __forceinline__ void mrun(cf (&v)[EM], const Buf& buf, const cf* __restrict__ tw, int t) {
    constexpr bool LAST = sizeof...(Rest) == 0;
    mstage<N, L, EM, R, NS, DIR, FIRST, LAST, SYNC, TWMUL>(v, buf, tw, t);
    if constexpr (!LAST) mrun<N, L, EM, NS * R, DIR, false, SYNC, TWMUL, Buf, Rest...>(v, buf, tw, t);
}

// N-point transform over L lanes with schedule Sched<Rs...>: reads layout(first radix), writes
// layout(last radix) (see the header comment); unnormalised
template <int N, int L, int EM, int DIR, int SYNC, int TWMUL, class Buf, int... Rs>
__device__ __forceinline__ void mfft(cf (&v)[EM], const Buf& buf, const cf* __restrict__ tw, int t, Sched<Rs...>) {
    mrun<N, L, EM, 1, DIR, true, SYNC, TWMUL, Buf, Rs...>(v, buf, tw, t);
}

// registers a schedule needs: max over its stages of R ceil(N / (R L))
template <int N, int L> __host__ __device__ constexpr int stage_regs(int R) { return R * ((N / R + L - 1) / L); }
template <int N, int L, int... Rs> __host__ __device__ constexpr int sched_regs(Sched<Rs...>) {
    int m = 0;
    for (int r : {Rs...}) m = stage_regs<N, L>(r) > m ? stage_regs<N, L>(r) : m;
    return m;
}
template <int... Rs> __host__ __device__ constexpr int sched_first(Sched<Rs...>) {
    constexpr int a[] = {Rs...};
    return a[0];
}
template <int... Rs> __host__ __device__ constexpr int sched_last(Sched<Rs...>) {
    constexpr int a[] = {Rs...};
    return a[sizeof...(Rs) - 1];
}
template <int... Rs> __host__ __device__ constexpr long long sched_prod(Sched<Rs...>) {
    long long p = 1;
    for (int r : {Rs...}) p *= r;
    return p;
}

}  // namespace admm

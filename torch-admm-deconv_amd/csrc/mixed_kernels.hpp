// mixed_kernels.hpp -- the fused two-pass ADMM iteration (admm_kernels.hpp) at smooth image sizes
// (H, W with factors 2, 3, 5 only, W even), e.g. 1080 x 1920, 720 x 1280, 480 x 640 (gfx950).
//
// Same algorithm, data layout and bytes as the power-of-two path: pass B is the
// column FFT -> Wiener factor -> column IFFT in place, pass A the row pass that inverts the row
// spectra of a strip of R rows (+ one halo row), forms Dx, Dy, the shrink, the dual update, D^T w,
// r = b + rho v and the r row spectra -- 36 B/px per iteration (48 iso), against the generic path's
// three transform launches per iteration (~44-60 B/px, §7a).  The transforms are mixed_fft.hpp's
// guarded Stockham schedules; a plan per length fixes the lanes and the edge layouts:
//   rows (MRow<N>, N = W/2 complex points):  a row group of Lg lanes (power of two <= 64, within one
//     wave); pixels in layout(Ep) over Lp = N/Ep lanes (Ep pixel pairs per lane: pair t + Lp j), row
//     spectra in layout(Es) over Ls = N/Es lanes (element t + Ls j); the inverse schedule runs
//     Es ... Ep, the forward one Ep ... Es.
//   columns (MCol<H>): Lc threads per column, C columns per block (ColBuf interleave); column values in
//     layout(Ec) (element t + Lc j, as the spectrum rows are loaded), the forward schedule Ec ... Rz
//     leaves the frequencies in layout(Rz), where the Wiener factor is applied; the inverse schedule
//     Rz ... Ec returns them.
// Power-of-two lengths get the plans of fft_core.hpp's RowCfg (natural layout, same arithmetic), so
// a power-of-two W with a smooth H (or the reverse) runs here too.
// Training too: the forward with history (HIST variants) and the reverse passes (k_bwd_pass_a_m,
// k_bwd_iso_q_m, at the end of this file); with a PSF gradient the generic kernels train.
#pragma once
#include <type_traits>

#include "admm_backward.hpp"
#include "admm_kernels.hpp"
#include "mixed_fft.hpp"

namespace admm {

// ---------------------------------------------------------------------------------------------
// plans
// ---------------------------------------------------------------------------------------------
// The edge stage of radix R over L lanes leaves element t + L q + (N/R) k in register q + Q k
// (Q = ceil(N/(R L))): that is the natural layout over Lx lanes (element t + Lx j in register j) when
// it runs one butterfly per lane over exactly Lx = N/R lanes, or full rows of butterflies over all L
// lanes (the power-of-two plans: Q = E / R).
template <int N, int L> __host__ __device__ constexpr bool edge_ok(int R, int Lx) {
    return ((N / R + L - 1) / L == 1 && N / R == Lx) || (L == Lx && (N / R) % L == 0);
}
template <int N> struct MRow;
// power-of-two rows: fft_core's configuration
template <int N> struct MRowPow2 {
    static constexpr int Lg = N / RowCfg<N>::E, Lp = Lg, Ls = Lg, Ep = RowCfg<N>::E, Es = Ep;
    using Inv = typename RowCfg<N>::S;
    using Fwd = typename RowCfg<N>::S;
};
template <> struct MRow<16> : MRowPow2<16> {};
template <> struct MRow<32> : MRowPow2<32> {};
template <> struct MRow<64> : MRowPow2<64> {};
template <> struct MRow<128> : MRowPow2<128> {};
template <> struct MRow<256> : MRowPow2<256> {};
template <> struct MRow<512> : MRowPow2<512> {};
template <> struct MRow<1024> {  // W = 2048 beside a smooth H: 128 lanes x 8 (2 waves)
    static constexpr int Lg = 128, Lp = 128, Ep = 8, Ls = 128, Es = 8;
    using Inv = Sched<8, 16, 8>;
    using Fwd = Sched<8, 16, 8>;
};
// smooth rows.  Rows whose pixel state would exceed ~8 pairs per lane at 64 lanes run "wide": a row
// group of 128 or 256 lanes (2 or 4 waves of the block) exchanging through LDS with block barriers, so
// each lane keeps 8 pixel pairs (15 per lane at 64 lanes measured ~320 VGPRs: 1 wave per SIMD).
// (measured slower for 960: 8 * 3 * 5 * 8, pass A 0.304 -> 0.327 ms, profiles/r04_ab_hd_m960v1.txt; 4-wave
// groups of 4 pairs per lane as 4 * 15 * 4 * 4)
template <> struct MRow<960> {  // W = 1920 (HD): 960 = 8 * 15 * 8 over 120 of 128 lanes
    static constexpr int Lg = 128, Lp = 120, Ep = 8, Ls = 120, Es = 8;
    using Inv = Sched<8, 15, 8>;
    using Fwd = Sched<8, 15, 8>;
};
template <> struct MRow<1920> {  // W = 3840 (4K UHD): spectra and pixels 240 x 8 (4 waves), 8 * 6 * 5 * 8
    static constexpr int Lg = 256, Lp = 240, Ep = 8, Ls = 240, Es = 8;
    using Inv = Sched<8, 6, 5, 8>;
    using Fwd = Sched<8, 5, 6, 8>;
};
template <> struct MRow<2048> {  // W = 4096: 256 lanes x 8 (4 waves)
    static constexpr int Lg = 256, Lp = 256, Ep = 8, Ls = 256, Es = 8;
    using Inv = Sched<8, 4, 8, 8>;
    using Fwd = Sched<8, 8, 4, 8>;
};
// 720p / VGA rows with fewer values per stage (640: 10 * 8 * 8 over 64 / 80 lanes, 320: 8 * 5 * 8 over 40
// lanes) than 5 * 16 * 8 / 16 * 4 * 5: VGA pass A 0.201 -> 0.182 ms, 720p 0.333 -> 0.326
// (profiles/r04_ab_vga_rows.txt, r04_ab_p720_rows.txt)
template <> struct MRow<640> {  // W = 1280 (720p): spectra 64 x 10, pixels 80 x 8 (2 waves)
    static constexpr int Lg = 128, Lp = 80, Ep = 8, Ls = 64, Es = 10;
    using Inv = Sched<10, 8, 8>;
    using Fwd = Sched<8, 8, 10>;
};
template <> struct MRow<480> {  // W = 960: spectra 40 x 12, pixels 60 x 8
    static constexpr int Lg = 64, Lp = 60, Ep = 8, Ls = 40, Es = 12;
    using Inv = Sched<12, 5, 8>;
    using Fwd = Sched<8, 5, 12>;
};
template <> struct MRow<320> {  // W = 640 (VGA): spectra 40 x 8, pixels 40 x 8
    static constexpr int Lg = 64, Lp = 40, Ep = 8, Ls = 40, Es = 8;
    using Inv = Sched<8, 5, 8>;
    using Fwd = Sched<8, 5, 8>;
};
template <> struct MRow<240> {  // W = 480: spectra 16 x 15, pixels 30 x 8
    static constexpr int Lg = 32, Lp = 30, Ep = 8, Ls = 16, Es = 15;
    using Inv = Sched<15, 2, 8>;
    using Fwd = Sched<8, 2, 15>;
};
template <> struct MRow<360> {  // W = 720: spectra 40 x 9, pixels 45 x 8
    static constexpr int Lg = 64, Lp = 45, Ep = 8, Ls = 40, Es = 9;
    using Inv = Sched<9, 5, 8>;
    using Fwd = Sched<8, 5, 9>;
};
template <> struct MRow<540> {  // W = 1080: spectra 45 x 12, pixels 60 x 9
    static constexpr int Lg = 64, Lp = 60, Ep = 9, Ls = 45, Es = 12;
    using Inv = Sched<12, 5, 9>;
    using Fwd = Sched<9, 5, 12>;
};
// common photo / display widths (plans from tools/mixed_plans.py, each simulated to ~1e-15)
template <> struct MRow<400> {  // W = 800 (SVGA): spectra 40 x 10, pixels 50 x 8
    static constexpr int Lg = 64, Lp = 50, Ep = 8, Ls = 40, Es = 10;
    using Inv = Sched<10, 5, 8>;
    using Fwd = Sched<8, 5, 10>;
};
template <> struct MRow<720> {  // W = 1440: spectra 60 x 12, pixels 120 x 6 (2 waves)
    static constexpr int Lg = 128, Lp = 120, Ep = 6, Ls = 60, Es = 12;
    using Inv = Sched<12, 10, 6>;
    using Fwd = Sched<6, 10, 12>;
};
template <> struct MRow<800> {  // W = 1600: spectra 100 x 8, pixels 160 x 5 (4 waves)
    static constexpr int Lg = 256, Lp = 160, Ep = 5, Ls = 100, Es = 8;
    using Inv = Sched<8, 4, 5, 5>;
    using Fwd = Sched<5, 5, 4, 8>;
};
template <> struct MRow<1280> {  // W = 2560: spectra 160 x 8, pixels 256 x 5 (4 waves)
    static constexpr int Lg = 256, Lp = 256, Ep = 5, Ls = 160, Es = 8;
    using Inv = Sched<8, 4, 8, 5>;
    using Fwd = Sched<5, 8, 4, 8>;
};

// Row plans of the training backward (the reverse row pass and the iso Q pass): their lanes carry five
// row states besides the transform (admm_backward.hpp), so these plans keep 3-5 pixel pairs per lane over
// up to 256 lanes and small transform stages (EM 5-8 values), where the inference plans above keep 8 pairs
// and up to 15-value stages (tools/mixed_plans.py search with Ep <= 5, each plan simulated on the CPU,
// tests/test_mixed_plans.py).  Lengths without one use the inference plan.
template <int N> struct MRowT : MRow<N> {};
template <> struct MRowT<240> {
    static constexpr int Lg = 64, Lp = 60, Ep = 4, Ls = 40, Es = 6;
    using Inv = Sched<6, 2, 5, 4>;
    using Fwd = Sched<4, 5, 2, 6>;
};
// 320 points (VGA rows): 5 pairs per lane over the inference plan's 64 lanes, so inference takes it too
// (infer_tplan): VGA pass A 0.1825 -> 0.1552 ms, 3,800 -> 4,215 it/s (profiles/r05_ab_vga_tplan320.txt)
#ifndef ADMM_TPLAN_320  // compile-time A/B knob: 0 = no training plan for 320 points (VGA rows)
#define ADMM_TPLAN_320 1
#endif
#if ADMM_TPLAN_320
template <> struct MRowT<320> {
    static constexpr int Lg = 64, Lp = 64, Ep = 5, Ls = 40, Es = 8;
    using Inv = Sched<8, 8, 5>;
    using Fwd = Sched<5, 8, 8>;
};
#endif
template <> struct MRowT<360> {
    static constexpr int Lg = 128, Lp = 120, Ep = 3, Ls = 60, Es = 6;
    using Inv = Sched<6, 4, 5, 3>;
    using Fwd = Sched<3, 5, 4, 6>;
};
template <> struct MRowT<400> {
    static constexpr int Lg = 128, Lp = 100, Ep = 4, Ls = 80, Es = 5;
    using Inv = Sched<5, 4, 5, 4>;
    using Fwd = Sched<4, 5, 4, 5>;
};
template <> struct MRowT<480> {
    static constexpr int Lg = 128, Lp = 120, Ep = 4, Ls = 80, Es = 6;
    using Inv = Sched<6, 4, 5, 4>;
    using Fwd = Sched<4, 5, 4, 6>;
};
template <> struct MRowT<540> {
    static constexpr int Lg = 128, Lp = 108, Ep = 5, Ls = 90, Es = 6;
    using Inv = Sched<6, 3, 6, 5>;
    using Fwd = Sched<5, 6, 3, 6>;
};
template <> struct MRowT<640> {
    // one 2-wave group per 128-thread block (its LDS barriers wait only for its own two waves): 720p inference
    // 2,206-2,211 -> 2,338-2,339 it/s, pass A 0.310 -> 0.283 ms, interleaved (profiles/r06_ab_p720_wide_nt.txt);
    // HD's 8-pair 960-point plan lost 1.5 % that way (profiles/r06_ab_hd_wide_nt.txt) and keeps 256 threads
    static constexpr int NT = 128;
    static constexpr int Lg = 128, Lp = 128, Ep = 5, Ls = 80, Es = 8;
    using Inv = Sched<8, 2, 8, 5>;
    using Fwd = Sched<5, 8, 2, 8>;
};
template <> struct MRowT<720> {
    static constexpr int Lg = 256, Lp = 240, Ep = 3, Ls = 90, Es = 8;
    using Inv = Sched<8, 5, 6, 3>;
    using Fwd = Sched<3, 6, 5, 8>;
};
template <> struct MRowT<800> {
    static constexpr int Lg = 256, Lp = 200, Ep = 4, Ls = 100, Es = 8;
    using Inv = Sched<8, 5, 5, 4>;
    using Fwd = Sched<4, 5, 5, 8>;
};
template <> struct MRowT<960> {
    static constexpr int Lg = 256, Lp = 240, Ep = 4, Ls = 120, Es = 8;
    using Inv = Sched<8, 5, 6, 4>;
    using Fwd = Sched<4, 6, 5, 8>;
};
template <> struct MRowT<1280> {
    static constexpr int Lg = 256, Lp = 256, Ep = 5, Ls = 160, Es = 8;
    using Inv = Sched<8, 4, 8, 5>;
    using Fwd = Sched<5, 8, 4, 8>;
};

#ifndef ADMM_MROW_WIDE_NT
#define ADMM_MROW_WIDE_NT 256
#endif
// threads per block of a row plan: its NT member where it has one, else 256
template <class PL, class = void> struct PlanNT : std::integral_constant<int, 256> {};
template <class PL> struct PlanNT<PL, std::void_t<decltype(PL::NT)>> : std::integral_constant<int, PL::NT> {};
template <int N, class PL = MRow<N>> struct MRowG {
    using P = PL;
    static constexpr int Lg = P::Lg, Lp = P::Lp, Ep = P::Ep, Ls = P::Ls, Es = P::Es, W = 2 * N;
    static constexpr int a = sched_regs<N, Lg>(typename P::Inv{}), b = sched_regs<N, Lg>(typename P::Fwd{});
    static constexpr int EM = a > b ? a : b;
    // threads per block: the plan's (PlanNT); every 2-wave group alone, A/B: -DADMM_MROW_WIDE_NT=128 (one group
    // per block, so a group's block barriers wait only for its own waves)
    static constexpr int NT =
        (Lg > 64 && ADMM_MROW_WIDE_NT < 256 && Lg <= ADMM_MROW_WIDE_NT) ? ADMM_MROW_WIDE_NT : PlanNT<PL>::value;
    static constexpr int SG = NT / Lg;
    static constexpr bool WIDE = Lg > 64;  // the row group spans several waves: LDS exchanges, block barriers
    // wide groups synchronise their LDS exchanges with LDS-only block barriers (fft_core xsync<2>): a
    // __syncthreads would also drain the wave's outstanding global loads and stores at every exchange
    static constexpr int SYNC = WIDE ? 2 : 0;
    static_assert(Lp * Ep == N && Ls * Es == N && Lp <= Lg && Ls <= Lg && Lg <= 256 && (Lg & (Lg - 1)) == 0,
                  "row plan");
    static_assert(sched_prod(typename P::Inv{}) == N && sched_prod(typename P::Fwd{}) == N, "row schedule");
    static_assert(edge_ok<N, Lg>(sched_first(typename P::Inv{}), Ls) && edge_ok<N, Lg>(sched_last(typename P::Inv{}), Lp),
                  "inverse edges");
    static_assert(edge_ok<N, Lg>(sched_first(typename P::Fwd{}), Lp) && edge_ok<N, Lg>(sched_last(typename P::Fwd{}), Ls),
                  "forward edges");
    // one exchange buffer per sub-group (ping-pong buffers for the wide groups measured within +-0.5 %)
    static constexpr size_t lds_bytes() { return sizeof(cf) * (W + SG * RowBuf::slots(N)); }
};

template <int H> struct MCol;
template <int H> struct MColPow2 {
    // up to 512 threads per block (1,024 would cap the transform at 128 VGPRs: it spills at H >= 2048)
    static constexpr int Lc = H / RowCfg<H>::E, Ec = RowCfg<H>::E, C = Lc <= 64 ? 8 : 512 / Lc;
    using Fwd = typename RowCfg<H>::S;
    using Inv = typename RowCfg<H>::S;
};
template <> struct MCol<16> : MColPow2<16> {};
template <> struct MCol<32> : MColPow2<32> {};
template <> struct MCol<64> : MColPow2<64> {};
template <> struct MCol<128> : MColPow2<128> {};
template <> struct MCol<256> : MColPow2<256> {};
template <> struct MCol<512> : MColPow2<512> {};
template <> struct MCol<1024> : MColPow2<1024> {};
template <> struct MCol<2048> : MColPow2<2048> {};
template <> struct MCol<4096> : MColPow2<4096> {};
// columns per block of the smooth column plans: 8 (64-byte row segments, pairs of blocks sharing each
// 128-byte line, as k_pass_b) wherever 8 Lc <= 1024 threads
// 1080: 120 threads x 9 values per column, schedule 9 * 12 * 10 -- lanes busy 100 / 75 / 90 % per stage
// (9 * 15 * 8: 100 / 60 / 56 %), 12 values: HD pass B 0.160 -> 0.120 ms, 62 VGPRs
// (profiles/r04_ab_hd_m1080s.txt; 60 threads x 18 values measured 6 % slower)
template <> struct MCol<1080> {
    static constexpr int Lc = 120, Ec = 9, C = 8;
    using Fwd = Sched<9, 12, 10>;
    using Inv = Sched<10, 12, 9>;
};
// schedules that keep more lanes busy per guarded stage: 2160 as 9 * 2 * 12 * 10 (lanes 100 / 90 / 75 /
// 90 %, 12 values, one more exchange) instead of 9 * 16 * 15 (100 / 56 / 60 %, 16 values): 4K UHD pass B
// 0.2345 -> 0.214 ms (profiles/r04_ab_uhd_cols.txt); 360 as 9 * 10 * 4 instead of 9 * 8 * 5: 0.0566 ->
// 0.0545 ms (profiles/r04_ab_sd_cols.txt)
template <> struct MCol<2160> {
    static constexpr int Lc = 240, Ec = 9, C = 2;
    using Fwd = Sched<9, 2, 12, 10>;
    using Inv = Sched<10, 12, 2, 9>;
};
template <> struct MCol<720> {
    static constexpr int Lc = 80, Ec = 9, C = 8;
    using Fwd = Sched<9, 16, 5>;
    using Inv = Sched<5, 16, 9>;
};
template <> struct MCol<960> {
    static constexpr int Lc = 64, Ec = 15, C = 8;
    using Fwd = Sched<15, 16, 4>;
    using Inv = Sched<4, 16, 15>;
};
template <> struct MCol<540> {
    static constexpr int Lc = 60, Ec = 9, C = 8;
    using Fwd = Sched<9, 12, 5>;
    using Inv = Sched<5, 12, 9>;
};
template <> struct MCol<480> {
    static constexpr int Lc = 32, Ec = 15, C = 8;
    using Fwd = Sched<15, 16, 2>;
    using Inv = Sched<2, 16, 15>;
};
template <> struct MCol<360> {
    static constexpr int Lc = 40, Ec = 9, C = 8;
    using Fwd = Sched<9, 10, 4>;
    using Inv = Sched<4, 10, 9>;
};
template <> struct MCol<240> {
    static constexpr int Lc = 16, Ec = 15, C = 8;
    using Fwd = Sched<15, 16>;
    using Inv = Sched<16, 15>;
};
// common photo / display heights (tools/mixed_plans.py)
template <> struct MCol<600> {
    static constexpr int Lc = 100, Ec = 6, C = 8;
    using Fwd = Sched<6, 10, 10>;
    using Inv = Sched<10, 10, 6>;
};
template <> struct MCol<768> {
    static constexpr int Lc = 128, Ec = 6, C = 8;
    using Fwd = Sched<6, 2, 8, 8>;
    using Inv = Sched<8, 8, 2, 6>;
};
template <> struct MCol<800> {
    static constexpr int Lc = 100, Ec = 8, C = 8;
    using Fwd = Sched<8, 10, 10>;
    using Inv = Sched<10, 10, 8>;
};
template <> struct MCol<1200> {
    static constexpr int Lc = 120, Ec = 10, C = 8;
    using Fwd = Sched<10, 10, 12>;
    using Inv = Sched<12, 10, 10>;
};
template <> struct MCol<1440> {
    static constexpr int Lc = 120, Ec = 12, C = 8;
    using Fwd = Sched<12, 8, 15>;
    using Inv = Sched<15, 8, 12>;
};
template <> struct MCol<1536> {
    static constexpr int Lc = 256, Ec = 6, C = 4;
    using Fwd = Sched<6, 4, 8, 8>;
    using Inv = Sched<8, 8, 4, 6>;
};

// CC: columns per block of this instance -- the plan's C, or fewer when the row spectrum's N = W / 2
// columns are not a multiple of it (mixed_capi.hip pass_b: C, 4 or 2)
template <int H, int CC = MCol<H>::C> struct MColG {
    using P = MCol<H>;
    static constexpr int Lc = P::Lc, Ec = P::Ec, C = CC, NT = C * Lc;
    static constexpr int Rz = sched_last(typename P::Fwd{});
    static constexpr int NBz = H / Rz, Qz = (NBz + Lc - 1) / Lc;
    static constexpr int a = sched_regs<H, Lc>(typename P::Fwd{}), b = sched_regs<H, Lc>(typename P::Inv{});
    static constexpr int EM = a > b ? a : b;
    static_assert(Lc * Ec == H && NT <= 1024, "column plan");
    static_assert(sched_prod(typename P::Fwd{}) == H && sched_prod(typename P::Inv{}) == H, "column schedule");
    static_assert(edge_ok<H, Lc>(sched_first(typename P::Fwd{}), Lc) && edge_ok<H, Lc>(sched_last(typename P::Inv{}), Lc),
                  "column edges");
    // the inverse starts from the layout the forward ends in (the same radix, or both natural)
    static_assert(sched_first(typename P::Inv{}) == Rz ||
                      (NBz % Lc == 0 && (H / sched_first(typename P::Inv{})) % Lc == 0), "column frequency layout");
    static constexpr size_t lds_bytes() { return sizeof(cf) * (H + (size_t)H * C); }
};

// ---------------------------------------------------------------------------------------------
// packed real-row transforms over one row group (as RowXf<N>, admm_kernels.hpp, in the plan's layouts)
// ---------------------------------------------------------------------------------------------
template <int N, class PL = MRow<N>> struct RowXfM {
    using G = MRowG<N, PL>;
    static constexpr int Lg = G::Lg, Lp = G::Lp, Ep = G::Ep, Ls = G::Ls, Es = G::Es, EM = G::EM;
    static constexpr bool WIDE = G::WIDE;
    static constexpr int SYNC = G::SYNC;

    template <bool INV> __device__ __forceinline__ static cf one(int k, cf x, cf pp, const cf* __restrict__ tw) {
        const cf w = tw[k < N ? k : 0];
        const cf pc = cconj(pp);
        if (INV) {  // c2r: e + i o, o = (x - conj p) exp(+2 pi i k / W)
            const cf e = cadd(x, pc);
            const cf o = cmulc(csub(x, pc), w);
            return mkc(e.x - o.y, e.y + o.x);
        } else {    // r2c: s - i d, d = (x - conj p) exp(-2 pi i k / W)
            const cf sm = cadd(x, pc);
            const cf d = cmul(csub(x, pc), w);
            return mkc(sm.x + d.y, sm.y - d.x);
        }
    }
    // the row group's LDS exchange buffer
    struct Lds {
        cf* base;
        __device__ __forceinline__ RowBuf cur() const { return RowBuf{base}; }
    };
    __device__ __forceinline__ static Lds lds_of(cf* base) { return Lds{base}; }
    // wide row groups: the partners through the LDS exchange buffer (every lane of the block takes part)
    template <bool INV>
    __device__ __forceinline__ static void combine_lds(cf (&v)[EM], Lds& l, const cf* __restrict__ tw, int t) {
        const RowBuf buf = l.cur();
        lds_barrier();  // its previous readers are done
        if (t < Ls) {
#pragma unroll
            for (int j = 0; j < Es; ++j) buf.at(t + Ls * j) = v[j];
        }
        lds_barrier();
#pragma unroll
        for (int j = 0; j < Es; ++j) {
            const int k = t + Ls * j;
            const cf x = v[j];
            if (k == 0) {
                v[j] = INV ? mkc(x.x + x.y, x.x - x.y) : mkc(2.f * (x.x + x.y), 2.f * (x.x - x.y));
            } else {
                const int kp = N - k;
                v[j] = one<INV>(k, x, buf.at(kp >= 0 ? kp : 0), tw);
            }
        }
    }
    // The Hermitian combine of element k = t + Ls j with its partner N - k, which sits in lane
    // Ls - t, register Es - 1 - j (t = 0: this lane, register Es - j).  Registers j and Es - 1 - j are
    // each other's partner registers, so they are combined as a pair from one pair of shuffles (no
    // partner array held across the loop).
    template <bool INV>
    __device__ __forceinline__ static void combine(cf (&v)[EM], const cf* __restrict__ tw, int t) {
        const int src = (t == 0 || t >= Ls) ? 0 : Ls - t;
        auto one = [&](int j, cf x, cf pp) -> cf { return RowXfM::one<INV>(t + Ls * j, x, pp, tw); };
        // Lane 0's partners are its own registers Es - j, which the loop has already rewritten (as the
        // previous iteration's jp) by the time it needs them: their original values are carried in prev.
        const cf v0 = v[0];
        cf prev = v0;
#pragma unroll
        for (int j = 0; j < (Es + 1) / 2; ++j) {
            const int jp = Es - 1 - j;
            const cf a = mkc(__shfl(v[jp].x, src, Lg), __shfl(v[jp].y, src, Lg));  // partner of j
            const cf b = mkc(__shfl(v[j].x, src, Lg), __shfl(v[j].y, src, Lg));    // partner of jp
            const cf xj = v[j], xp = v[jp];
            // lane 0: partner of register j is its register Es - j (j = 0: itself), of jp register j + 1
            const cf pa = t == 0 ? (j == 0 ? v0 : prev) : a;
            const cf pb = t == 0 ? v[(j + 1) % Es] : b;
            cf nj = one(j, xj, pa);
            const cf np = one(jp, xp, pb);
            if (j == 0 && t == 0)
                nj = INV ? mkc(v0.x + v0.y, v0.x - v0.y) : mkc(2.f * (v0.x + v0.y), 2.f * (v0.x - v0.y));
            prev = xp;
            v[j] = nj;
            if (jp != j) v[jp] = np;
        }
    }
    // row spectrum in layout(Es) (v[j], j < Es) -> pixel pairs in layout(Ep) (v[j], j < Ep), x 2W
    __device__ __forceinline__ static void c2r(cf (&v)[EM], Lds& l, const cf* __restrict__ tw, int t) {
        if constexpr (WIDE) {
            combine_lds<true>(v, l, tw, t);
            mfft<N, Lg, EM, +1, SYNC, 2>(v, RowBuf{l.base}, tw, t, typename PL::Inv{});
        } else {
            combine<true>(v, tw, t);
            mfft<N, Lg, EM, +1, 0, 2>(v, RowBuf{l.base}, tw, t, typename PL::Inv{});
        }
    }
    // pixel pairs in layout(Ep) -> packed spectrum (2 rfft) in layout(Es)
    __device__ __forceinline__ static void r2c(cf (&v)[EM], Lds& l, const cf* __restrict__ tw, int t) {
        if constexpr (WIDE) {
            mfft<N, Lg, EM, -1, SYNC, 2>(v, RowBuf{l.base}, tw, t, typename PL::Fwd{});
            combine_lds<false>(v, l, tw, t);
        } else {
            mfft<N, Lg, EM, -1, 0, 2>(v, RowBuf{l.base}, tw, t, typename PL::Fwd{});
            combine<false>(v, tw, t);
        }
    }
    // the value of pixel-pair neighbour k + SHIFT (SHIFT = -1 / +1, circular) of every pair this lane
    // holds: lane shuffles within a wave, the LDS buffer across the waves of a wide row group
    template <int SHIFT>
    __device__ __forceinline__ static void neighbour(const float (&val)[Ep], float (&out)[Ep], Lds& l, int t) {
        if constexpr (WIDE) {
            const RowBuf buf = l.cur();
            lds_barrier();
            if (t < Lp) {
#pragma unroll
                for (int j = 0; j < Ep; ++j) buf.at(t + Lp * j).x = val[j];
            }
            lds_barrier();
#pragma unroll
            for (int j = 0; j < Ep; ++j) {
                int k = t + Lp * j + SHIFT;
                k = k < 0 ? N - 1 : k >= N ? 0 : k;
                out[j] = buf.at(k).x;
            }
        } else {
            const int src = SHIFT < 0 ? (t == 0 ? Lp - 1 : t - 1) : (t + 1 >= Lp ? 0 : t + 1);
            float sh[Ep];
#pragma unroll
            for (int j = 0; j < Ep; ++j) sh[j] = __shfl(val[j], src, Lg);
#pragma unroll
            for (int j = 0; j < Ep; ++j) {
                if (SHIFT < 0) out[j] = (t == 0) ? sh[(j + Ep - 1) % Ep] : sh[j];
                else out[j] = (t == Lp - 1) ? sh[(j + 1) % Ep] : sh[j];
            }
        }
    }
};

// real rows (pixel order) -> packed row spectra
template <int N>
__global__ void __launch_bounds__(256) k_row_r2c_m(const float* __restrict__ img, cf* __restrict__ spec,
                                                   const cf* __restrict__ twW_g, long long rows) {
    using G = MRowG<N>;
    constexpr int Lg = G::Lg, Lp = G::Lp, Ep = G::Ep, Ls = G::Ls, Es = G::Es, EM = G::EM;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    cf* tw = reinterpret_cast<cf*>(smem);
    load_tw(tw, twW_g, G::W);
    __syncthreads();
    const int sgl = threadIdx.x / Lg, t = threadIdx.x % Lg;
    long long row = (long long)blockIdx.x * G::SG + sgl;
    const bool ok = row < rows;
    if (!G::WIDE && !ok) return;  // (a wide row group keeps every lane for the block barriers)
    if (!ok) row = rows - 1;
    auto lx = RowXfM<N>::lds_of(tw + G::W + sgl * RowBuf::slots(N));
    const cf* src = reinterpret_cast<const cf*>(img + row * G::W);
    cf v[EM];
    if (t < Lp) {
#pragma unroll
        for (int j = 0; j < Ep; ++j) v[j] = src[t + Lp * j];
    }
    RowXfM<N>::r2c(v, lx, tw, t);
    if (ok && t < Ls) {
        cf* dst = spec + row * N;
#pragma unroll
        for (int j = 0; j < Es; ++j) dst[t + Ls * j] = v[j];
    }
}

// packed row spectra -> real rows (pixel order)
template <int N>
__global__ void __launch_bounds__(256) k_row_c2r_m(const cf* __restrict__ spec, float* __restrict__ img,
                                                   const cf* __restrict__ twW_g, long long rows) {
    using G = MRowG<N>;
    constexpr int Lg = G::Lg, Lp = G::Lp, Ep = G::Ep, Ls = G::Ls, Es = G::Es, EM = G::EM;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    cf* tw = reinterpret_cast<cf*>(smem);
    load_tw(tw, twW_g, G::W);
    __syncthreads();
    const int sgl = threadIdx.x / Lg, t = threadIdx.x % Lg;
    long long row = (long long)blockIdx.x * G::SG + sgl;
    const bool ok = row < rows;
    if (!G::WIDE && !ok) return;
    if (!ok) row = rows - 1;
    auto lx = RowXfM<N>::lds_of(tw + G::W + sgl * RowBuf::slots(N));
    const cf* src = spec + row * N;
    cf v[EM];
    if (t < Ls) {
#pragma unroll
        for (int j = 0; j < Es; ++j) v[j] = src[t + Ls * j];
    }
    RowXfM<N>::c2r(v, lx, tw, t);
    if (ok && t < Lp) {
        cf* dst = reinterpret_cast<cf*>(img + row * G::W);
#pragma unroll
        for (int j = 0; j < Ep; ++j) dst[t + Lp * j] = v[j];
    }
}

// Wiener factor for the mixed column pass: fcM[ky][kx] = fcT[kx][ky] / 2 (kx in [0, N], row-major so a
// block's C adjacent columns read adjacent factors; the / 2 turns the generic path's 1/(HW) scale into
// the packed row transforms' 1/(2HW), exactly), followed by the column-block-packed copy
// fcP[cb][ky][c] = fcM[ky][cb C + c] (kx < N): a block's factors are one contiguous C H run, so a wave
// reads whole lines and no line is shared with the neighbouring column blocks (which may run on other XCDs)
static __global__ void k_fc_mixed(const float* __restrict__ fcT, float* __restrict__ fcM, int H, int N, int C) {
    const long long n = (long long)H * (N + 1), np = (long long)H * N;
    float* fcP = fcM + n;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n + np; i += (long long)gridDim.x * blockDim.x) {
        if (i < n) {
            const int ky = (int)(i / (N + 1)), kx = (int)(i % (N + 1));
            fcM[i] = 0.5f * fcT[(size_t)kx * H + ky];
        } else {
            const long long j = i - n;  // (cb, ky, c)
            const int c = (int)(j % C), ky = (int)((j / C) % H), cb = (int)(j / ((long long)C * H));
            fcP[j] = 0.5f * fcT[(size_t)(cb * C + c) * H + ky];
        }
    }
}

// the PSF multiplier for the mixed column pass: mM[ky][kx] = mT[kx][ky] / 2 (kx in [0, N]; the / 2 as for
// k_fc_mixed)
static __global__ void k_mt_mixed(const cf* __restrict__ mT, cf* __restrict__ mM, int H, int N) {
    const long long n = (long long)H * (N + 1);
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        const int ky = (int)(i / (N + 1)), kx = (int)(i % (N + 1));
        const cf v = mT[(size_t)kx * H + ky];
        mM[i] = mkc(0.5f * v.x, 0.5f * v.y);
    }
}

// ---------------------------------------------------------------------------------------------
// pass B: column FFT -> Wiener factor -> column IFFT, in place, C columns per block
// ---------------------------------------------------------------------------------------------
// Measured and not kept (profiles/r04_ab_hd_passb_gp.txt): blocks walking 2-8 planes of their column
// block with the next plane streamed into LDS (global_load_lds) during the inverse transform and
// LDS-only barriers -- HD pass B 0.258-0.267 ms against 0.160 for one tile per block; an occupancy
// target for the smooth column plans (capped registers spill and lose 4-21 %).
// CM: a complex multiplier instead of the real Wiener factor -- b = H_t(xin) once per solve (the PSF
// multiplier mT, pre-halved and row-major: mM[ky][kx], kx in [0, N]; k_mt_mixed), in place of the generic
// transforms' three launches.  The packed (DC, Nyquist) column then takes complex a, b (as the
// power-of-two pass B's MODE 1).
template <int H, int CC, bool CM = false>
__global__ void __launch_bounds__((MColG<H, CC>::NT))
k_pass_b_m(cf* spec, const float* __restrict__ fcM, const cf* __restrict__ twH_g, int N, int colblocks, int order,
           int fpack, const cf* __restrict__ mM = nullptr) {
    using G = MColG<H, CC>;
    constexpr int Lc = G::Lc, Ec = G::Ec, C = G::C, EM = G::EM, NBz = G::NBz, Qz = G::Qz;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    cf* tw = reinterpret_cast<cf*>(smem);
    cf* data = tw + H;
    load_tw(tw, twH_g, H);
    const int tid = threadIdx.x;
    const int c = tid % C, t = tid / C;
    int p, cb;
    pb_tile(xcd_remap(blockIdx.x, gridDim.x), colblocks, order, true, p, cb);
    const int col = cb * C + c;
    const rsrc_t rs = make_rsrc(spec + (size_t)p * H * N, (unsigned)((size_t)H * N * sizeof(cf)));
    const int voff = (t * N + col) * (int)sizeof(cf);
    const int sstep = Lc * N * (int)sizeof(cf);
    ColBuf<C> buf{data + c};
    cf v[EM];
#pragma unroll
    for (int j = 0; j < Ec; ++j) v[j] = bload_cf(rs, voff, j * sstep);
    // frequencies in layout(Rz): v[q + Qz k] <-> ky = t + Lc q + NBz k (valid for t + Lc q < NBz)
    typename std::conditional<CM, cf, float>::type m[EM];
    // the factors of this thread's column: from the column-block-packed copy (k_fc_mixed) or the
    // row-major table (CM: the row-major complex multiplier)
    const float* fcP = CM ? nullptr : fcM + (size_t)H * (N + 1) + (size_t)cb * H * C + c;
    auto load_m = [&]() {
#pragma unroll
        for (int q = 0; q < Qz; ++q) {
            const int vt = t + Lc * q;
#pragma unroll
            for (int k = 0; k < G::Rz; ++k) {
                if constexpr (CM)
                    m[q + Qz * k] = (vt < NBz) ? mM[(size_t)(vt + NBz * k) * (N + 1) + col] : mkc(0.f, 0.f);
                else
                    m[q + Qz * k] = (vt < NBz) ? (fpack ? fcP[(size_t)(vt + NBz * k) * C]
                                                        : fcM[(size_t)(vt + NBz * k) * (N + 1) + col]) : 0.f;
            }
        }
    };
    __syncthreads();  // twiddles in LDS
    mfft<H, Lc, EM, -1, 1, 1>(v, buf, tw, t, typename MCol<H>::Fwd{});
    // the factors are loaded after the forward transform (fewer live registers through it) rather than
    // with the data: HD pass B 0.183 -> 0.160 ms (profiles/r04_ab_hd_latef.txt)
    load_m();
    if (cb == 0) {  // block-uniform: column 0 carries (DC, Nyquist) packed -> needs F[H - ky]
        __syncthreads();
#pragma unroll
        for (int q = 0; q < Qz; ++q) {
            const int vt = t + Lc * q;
            if (vt < NBz) {
#pragma unroll
                for (int k = 0; k < G::Rz; ++k) buf.at(vt + NBz * k) = v[q + Qz * k];
            }
        }
        __syncthreads();
        if (col == 0) {
#pragma unroll
            for (int q = 0; q < Qz; ++q) {
                const int vt = t + Lc * q;
                if (vt < NBz) {
#pragma unroll
                    for (int k = 0; k < G::Rz; ++k) {
                        const int ky = vt + NBz * k;
                        const cf qv = cconj(buf.at(ky == 0 ? 0 : H - ky));
                        const cf x = v[q + Qz * k];
                        if constexpr (CM) {
                            const cf m0 = m[q + Qz * k], mn = mM[(size_t)ky * (N + 1) + N];
                            const cf a = mkc(0.5f * (m0.x + mn.x), 0.5f * (m0.y + mn.y));
                            const cf b = mkc(0.5f * (m0.x - mn.x), 0.5f * (m0.y - mn.y));
                            v[q + Qz * k] = cadd(cmul(x, a), cmul(qv, b));
                        } else {
                            const float f0 = m[q + Qz * k], fn = fcM[(size_t)ky * (N + 1) + N];
                            const float a = 0.5f * (f0 + fn), b = 0.5f * (f0 - fn);
                            v[q + Qz * k] = mkc(fmaf(a, x.x, b * qv.x), fmaf(a, x.y, b * qv.y));
                        }
                    }
                }
            }
        }
        __syncthreads();  // the partner reads are done before the inverse transform reuses buf
    }
    if (col != 0) {
#pragma unroll
        for (int i = 0; i < Qz * G::Rz; ++i) {
            if constexpr (CM) v[i] = cmul(v[i], m[i]);
            else v[i] = cscale(v[i], m[i]);
        }
    }
    mfft<H, Lc, EM, +1, 1, 1>(v, buf, tw, t, typename MCol<H>::Inv{});
#pragma unroll
    for (int j = 0; j < Ec; ++j) bstore_cf(rs, voff, j * sstep, v[j]);
}

// ---------------------------------------------------------------------------------------------
// pass A: the fused row pass (k_pass_a, pixel-order images), one row group per strip of R rows
// ---------------------------------------------------------------------------------------------
// occupancy target of the mixed row pass (waves per SIMD): the plans keep <= 9 pixel pairs per lane
// (wide row groups where a wave would need more), ~150-170 VGPRs: 2 guaranteed, 3 when they fit
#ifdef ADMM_PASSA_M_W  // compile-time A/B knob (tools/build_mixed_variant.sh): one target for every row plan
#define PASSA_M_MINW(ep) (ADMM_PASSA_M_W)
#else
#define PASSA_M_MINW(ep) ((ep) > 9 ? 1 : 2)
#endif
// HIST (the training forward): uxi / uyi hold a_{k-1} (u_{k-1} is rebuilt from it with the norms N_{k-1},
// admm_kernels.hpp prev_u) and a_k is written instead of u_k -- the history the backward reads.
// The history store and the u rebuild add live state that the inference plans carry at up to 256 VGPRs, so
// the training forward runs on the training row plans (MRowT) where they keep the inference plan's
// row-group width: 640 points (10 8 8 over 128 lanes -> 5 pairs per lane) 11.4 -> 6.3 ms per 20 iterations
// at 720p, while a wider group (960: 2 -> 4 waves, 360: 1 -> 2) costs more in exchanges than the registers
// return (HD 10.1 -> 11.6 ms, 360x720 5.6 -> 6.0 ms; profiles/r05_ab_train_fwd_plans.txt).  Compile-time
// A/B knob ADMM_TRAIN_FWD_PLAN (tools/build_mixed_variant.sh): 0 = inference plans, 2 = training plans for
// every length.
#ifndef ADMM_TRAIN_FWD_PLAN
#define ADMM_TRAIN_FWD_PLAN 1
#endif
template <int N> constexpr bool train_fwd_plan() {
    return ADMM_TRAIN_FWD_PLAN == 2 || (ADMM_TRAIN_FWD_PLAN == 1 && MRowT<N>::Lg == MRow<N>::Lg);
}
// Inference (TRAIN = false) takes the training plans at equal group width too: 720p pass A (640 points,
// 10 8 8 -> 5 pairs per lane over the same 128 lanes) 0.327 -> 0.309 ms, 2,130 -> 2,215 it/s
// (profiles/r05_ab_p720_infer_tplan.txt; 800 and 1280 points follow the same rule).  Compile-time A/B knob
// ADMM_INFER_TPLAN=0: the inference plans.
#ifndef ADMM_INFER_TPLAN
#define ADMM_INFER_TPLAN 1
#endif
template <int N> constexpr bool infer_tplan() { return ADMM_INFER_TPLAN != 0 && MRowT<N>::Lg == MRow<N>::Lg; }
template <int N, bool TRAIN>
using MPlan = typename std::conditional<TRAIN ? train_fwd_plan<N>() : infer_tplan<N>(), MRowT<N>, MRow<N>>::type;
template <int N, bool ISO, bool FIRST, bool HIST>
__global__ void __launch_bounds__(256, PASSA_M_MINW((MPlan<N, HIST>::Ep))) k_pass_a_m(PassAArgs a) {
    using G = MRowG<N, MPlan<N, HIST>>;
    using Xf = RowXfM<N, MPlan<N, HIST>>;
    constexpr int Lg = G::Lg, Lp = G::Lp, Ep = G::Ep, Ls = G::Ls, Es = G::Es, EM = G::EM, W = G::W;
    constexpr bool kSpecNT = (ADMM_NT & 2) != 0 || ((ADMM_NT & 32) != 0 && N >= 512);
    constexpr bool kUNT = (ADMM_NT & 16) != 0;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    cf* tw = reinterpret_cast<cf*>(smem);
    load_tw(tw, a.twW, W);
    __syncthreads();
    const int sgl = threadIdx.x / Lg, t = threadIdx.x % Lg;
    long long strip = (long long)blockIdx.x * G::SG + sgl;
    const bool ok = strip < a.nstrips;  // a wide row group past the last strip redoes it without storing
    if (!G::WIDE && !ok) return;
    if (!ok) strip = a.nstrips - 1;
    const int H = a.H, R = a.R;
    const int spp = H / R;
    const long long p = strip / spp;
    const int i0 = (int)(strip % spp) * R;
    auto lx = Xf::lds_of(tw + W + sgl * RowBuf::slots(N));
    const float rho = a.rho[0];
    const float tau = a.lam[0] / rho;
    const bool pa = t < Lp, sa = t < Ls;  // lane holds pixels / spectrum elements
    const bool pst = ok && pa, sst = ok && sa;  // ... and stores them

    const cf* sp = a.sin + (size_t)p * H * N;
    cf* so = a.sout + (size_t)p * H * N;
    const size_t poff = (size_t)p * H * W;
    const cf* bimg = reinterpret_cast<const cf*>(a.b + poff);
    const cf* uxi = reinterpret_cast<const cf*>(a.uxi + poff);
    const cf* uyi = reinterpret_cast<const cf*>(a.uyi + poff);
    cf* uxo = reinterpret_cast<cf*>(a.uxo + poff);
    cf* uyo = reinterpret_cast<cf*>(a.uyo + poff);
    const cf* nsx = reinterpret_cast<const cf*>(a.nsq);
    const cf* nsy = reinterpret_cast<const cf*>(a.nsq + (size_t)H * W);
    const cf* npx = reinterpret_cast<const cf*>(a.nsq_prev);
    const cf* npy = reinterpret_cast<const cf*>(a.nsq_prev + (size_t)H * W);

    // row g's x in pixel layout (spectrum row -> c2r)
    auto xrow = [&](int g, cf (&x)[Ep]) {
        cf v[EM];
        if (sa) {
#pragma unroll
            for (int j = 0; j < Es; ++j) v[j] = ld_pol<kSpecNT>(&sp[(size_t)g * N + t + Ls * j]);
        }
        Xf::c2r(v, lx, tw, t);
#pragma unroll
        for (int j = 0; j < Ep; ++j) x[j] = v[j];
    };
    cf xprev[Ep], xcur[Ep], wxp[Ep], wyp[Ep];
    xrow(i0 == 0 ? H - 1 : i0 - 1, xprev);
    for (int rr = 0; rr <= R; ++rr) {
        const int g = i0 + rr >= H ? i0 + rr - H : i0 + rr;
        const size_t ro = (size_t)g * N;  // row offset in cf units (spectrum and pixel pairs alike)
        xrow(g, xcur);

        // ---- y direction: a_y = x[g] - x[g-1] + u_y; z_y, u_y, w_y of row g
        cf wyc[Ep];
        {
            cf uy[Ep], fy[Ep];
#pragma unroll
            for (int j = 0; j < Ep; ++j) {
                if constexpr (HIST) uy[j] = pa ? prev_u<ISO, FIRST, true>(uyi, npy, ro + t + Lp * j, tau) : mkc(0.f, 0.f);
                else uy[j] = (FIRST || !pa) ? mkc(0.f, 0.f) : ld_pol<kUNT>(&uyi[ro + t + Lp * j]);
                if constexpr (ISO) fy[j] = pa ? nsy[ro + t + Lp * j] : mkc(0.f, 0.f);
            }
#pragma unroll
            for (int j = 0; j < Ep; ++j) {
                const float a0 = (xcur[j].x - xprev[j].x) + uy[j].x;
                const float a1 = (xcur[j].y - xprev[j].y) + uy[j].y;
                const float z0 = shrink_z<ISO>(a0, tau, ISO ? fy[j].x : 0.f);
                const float z1 = shrink_z<ISO>(a1, tau, ISO ? fy[j].y : 0.f);
                const float n0 = a0 - z0, n1 = a1 - z1;  // u_y(new)
                uy[j] = HIST ? mkc(a0, a1) : mkc(n0, n1);
                wyc[j] = mkc(z0 - n0, z1 - n1);
            }
            if (rr < R && pst) {
#pragma unroll
                for (int j = 0; j < Ep; ++j) sta(&uyo[ro + t + Lp * j], uy[j]);
            }
        }

        // ---- finalize row g-1: v = Dx^T w_x + Dy^T w_y, r = b + rho v, row FFT
        if (rr >= 1) {
            const int gm = g == 0 ? H - 1 : g - 1;
            const size_t rm = (size_t)gm * N;
            float wxs[Ep], wrs[Ep];
#pragma unroll
            for (int j = 0; j < Ep; ++j) wxs[j] = wxp[j].x;
            Xf::template neighbour<+1>(wxs, wrs, lx, t);  // w_x at pixel q1+1
            cf r[EM];
#pragma unroll
            for (int j = 0; j < Ep; ++j) {
                const float wr = wrs[j];
                const cf bb = pa ? lda<16>(&bimg[rm + t + Lp * j]) : mkc(0.f, 0.f);
                const float v0 = (wxp[j].x - wxp[j].y) + (wyp[j].x - wyc[j].x);
                const float v1 = (wxp[j].y - wr) + (wyp[j].y - wyc[j].y);
                r[j] = mkc(fmaf(rho, v0, bb.x), fmaf(rho, v1, bb.y));
            }
            Xf::r2c(r, lx, tw, t);
            if (sst) {
#pragma unroll
                for (int j = 0; j < Es; ++j) sta(&so[rm + t + Ls * j], r[j]);
            }
        }

        // ---- x direction: a_x = x[g][j] - x[g][j-1] + u_x; z_x, u_x, w_x of row g
        if (rr < R) {
            cf ux[Ep], fx[Ep];
            float xys[Ep], xls[Ep];
#pragma unroll
            for (int j = 0; j < Ep; ++j) {
                if constexpr (HIST) ux[j] = pa ? prev_u<ISO, FIRST, true>(uxi, npx, ro + t + Lp * j, tau) : mkc(0.f, 0.f);
                else ux[j] = (FIRST || !pa) ? mkc(0.f, 0.f) : ld_pol<kUNT>(&uxi[ro + t + Lp * j]);
                if constexpr (ISO) fx[j] = pa ? nsx[ro + t + Lp * j] : mkc(0.f, 0.f);
                xys[j] = xcur[j].y;
            }
            Xf::template neighbour<-1>(xys, xls, lx, t);  // x at pixel q0-1
#pragma unroll
            for (int j = 0; j < Ep; ++j) {
                const float xl = xls[j];
                const float a0 = (xcur[j].x - xl) + ux[j].x;
                const float a1 = (xcur[j].y - xcur[j].x) + ux[j].y;
                const float z0 = shrink_z<ISO>(a0, tau, ISO ? fx[j].x : 0.f);
                const float z1 = shrink_z<ISO>(a1, tau, ISO ? fx[j].y : 0.f);
                const float n0 = a0 - z0, n1 = a1 - z1;
                ux[j] = HIST ? mkc(a0, a1) : mkc(n0, n1);
                wxp[j] = mkc(z0 - n0, z1 - n1);
            }
            if (pst) {
#pragma unroll
                for (int j = 0; j < Ep; ++j) sta(&uxo[ro + t + Lp * j], ux[j]);
            }
        }
#pragma unroll
        for (int j = 0; j < Ep; ++j) {
            wyp[j] = wyc[j];
            xprev[j] = xcur[j];
        }
    }
}

// ---------------------------------------------------------------------------------------------
// iso pass A1 (k_iso_norm): per-pixel partial sums over a group of planes of a_x^2, a_y^2
// ---------------------------------------------------------------------------------------------
template <int N, bool FIRST, bool HIST>
__global__ void __launch_bounds__(256) k_iso_norm_m(IsoArgs a) {
    using G = MRowG<N, MPlan<N, HIST>>;
    using Xf = RowXfM<N, MPlan<N, HIST>>;
    constexpr int Lg = G::Lg, Lp = G::Lp, Ep = G::Ep, Ls = G::Ls, Es = G::Es, EM = G::EM, W = G::W;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    cf* tw = reinterpret_cast<cf*>(smem);
    load_tw(tw, a.twW, W);
    __syncthreads();
    const int sgl = threadIdx.x / Lg, t = threadIdx.x % Lg;
    long long item = (long long)blockIdx.x * G::SG + sgl;
    const bool ok = item < a.nitems;
    if (!G::WIDE && !ok) return;
    if (!ok) item = a.nitems - 1;
    const int H = a.H;
    const int g = (int)(item % H);
    const int grp = (int)(item / H);
    const int gm = g == 0 ? H - 1 : g - 1;
    auto lx = Xf::lds_of(tw + W + sgl * RowBuf::slots(N));
    const bool pa = t < Lp, sa = t < Ls;
    const float tau = HIST ? a.lam[0] / a.rho[0] : 0.f;
    const cf* npx = reinterpret_cast<const cf*>(a.nsq_prev);
    const cf* npy = reinterpret_cast<const cf*>(a.nsq_prev + (size_t)H * W);
    cf sx[Ep], sy[Ep];
#pragma unroll
    for (int j = 0; j < Ep; ++j) sx[j] = sy[j] = mkc(0.f, 0.f);
    const int p1 = min(a.P, (grp + 1) * a.ppg);
    for (int p = grp * a.ppg; p < p1; ++p) {
        const cf* sp = a.sin + (size_t)p * H * N;
        cf vp[EM], vc[EM];
        if (sa) {
#pragma unroll
            for (int j = 0; j < Es; ++j) {
                vp[j] = sp[(size_t)gm * N + t + Ls * j];
                vc[j] = sp[(size_t)g * N + t + Ls * j];
            }
        }
        Xf::c2r(vp, lx, tw, t);
        Xf::c2r(vc, lx, tw, t);
        const size_t ro = (size_t)p * H * N + (size_t)g * N;  // cf units == pixel pairs
        const cf* uxi = reinterpret_cast<const cf*>(a.uxi);
        const cf* uyi = reinterpret_cast<const cf*>(a.uyi);
        float xys[Ep], xls[Ep];
#pragma unroll
        for (int j = 0; j < Ep; ++j) xys[j] = vc[j].y;
        Xf::template neighbour<-1>(xys, xls, lx, t);
#pragma unroll
        for (int j = 0; j < Ep; ++j) {
            cf ux = (FIRST || !pa) ? mkc(0.f, 0.f) : uxi[ro + t + Lp * j];
            cf uy = (FIRST || !pa) ? mkc(0.f, 0.f) : uyi[ro + t + Lp * j];
            if constexpr (HIST && !FIRST) {  // ux / uy hold a_{k-1}: u_{k-1} = a - f(N_{k-1}) a
                const size_t rn = (size_t)g * N + t + Lp * j;
                const cf nx = pa ? npx[rn] : mkc(0.f, 0.f), ny = pa ? npy[rn] : mkc(0.f, 0.f);
                ux = mkc(ux.x - block_factor(nx.x, tau) * ux.x, ux.y - block_factor(nx.y, tau) * ux.y);
                uy = mkc(uy.x - block_factor(ny.x, tau) * uy.x, uy.y - block_factor(ny.y, tau) * uy.y);
            }
            const float xl = xls[j];
            const float ax0 = (vc[j].x - xl) + ux.x, ax1 = (vc[j].y - vc[j].x) + ux.y;
            const float ay0 = (vc[j].x - vp[j].x) + uy.x, ay1 = (vc[j].y - vp[j].y) + uy.y;
            sx[j].x = fmaf(ax0, ax0, sx[j].x);
            sx[j].y = fmaf(ax1, ax1, sx[j].y);
            sy[j].x = fmaf(ay0, ay0, sy[j].x);
            sy[j].y = fmaf(ay1, ay1, sy[j].y);
        }
    }
    if (ok && pa) {
        cf* px = reinterpret_cast<cf*>(a.partial + ((size_t)grp * 2 + 0) * H * W) + (size_t)g * N;
        cf* py = reinterpret_cast<cf*>(a.partial + ((size_t)grp * 2 + 1) * H * W) + (size_t)g * N;
#pragma unroll
        for (int j = 0; j < Ep; ++j) {
            px[t + Lp * j] = sx[j];
            py[t + Lp * j] = sy[j];
        }
    }
}

// row plan of the reverse passes: the training plans, except where they would widen the row group to 4
// waves (960, 720): HD reverse row pass 16.55 -> 15.3 ms per 20 iterations on the inference plan, while
// 360 points keep the training plan's 2-wave group over the 1-wave inference one (8.97 -> 8.55 ms) and
// 640 its equal-width one (22.6 -> 15.9 ms; profiles/r05_ab_train_bwd_plans.txt).  A/B knob
// ADMM_TRAIN_BWD_PLAN: 2 = training plans everywhere, 1 = only at equal group width.
#ifndef ADMM_TRAIN_BWD_PLAN
#define ADMM_TRAIN_BWD_PLAN 3
#endif
template <int N> constexpr bool train_bwd_plan() {
    constexpr int a = MRow<N>::Lg, b = MRowT<N>::Lg;
    return ADMM_TRAIN_BWD_PLAN == 2 || (ADMM_TRAIN_BWD_PLAN == 1 && a == b) ||
           (ADMM_TRAIN_BWD_PLAN == 3 && (b < 256 || a == 256));
}
template <int N> using BPlan = typename std::conditional<train_bwd_plan<N>(), MRowT<N>, MRow<N>>::type;
// occupancy target of the reverse row pass on the training plans (waves per SIMD)
#ifndef BWD_M_MINW
#define BWD_M_MINW 2
#endif
// ---------------------------------------------------------------------------------------------
// training backward at smooth sizes: the reverse row pass and the iso Q pass of admm_backward.hpp
// (k_bwd_pass_a, k_bwd_iso_q) on the mixed row transforms.  Same algebra (admm_backward.hpp header),
// same history layout (pixel-order a_k images, the norms N_k), same per-strip fp64 partials; the
// column side of a reverse step is the inference pass B (M is self-adjoint).  Lanes past the pixel
// layout (t >= Lp) load nothing, store nothing and add nothing to the partials.
// ---------------------------------------------------------------------------------------------
template <int N, bool ISO, bool LASTK, bool FIRSTK>
__global__ void __launch_bounds__(256, BWD_M_MINW) k_bwd_pass_a_m(BwdArgs a) {
    using G = MRowG<N, BPlan<N>>;
    using Xf = RowXfM<N, BPlan<N>>;
    constexpr int Lg = G::Lg, Lp = G::Lp, Ep = G::Ep, Ls = G::Ls, Es = G::Es, EM = G::EM, W = G::W;
    constexpr bool kNT = ADMM_NT_BWD != 0;
    constexpr bool kSpecNT = kNT && ((ADMM_NT & 2) != 0 || ((ADMM_NT & 32) != 0 && N >= 512));
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    cf* tw = reinterpret_cast<cf*>(smem);
    load_tw(tw, a.twW, W);
    __syncthreads();
    const int sgl = threadIdx.x / Lg, t = threadIdx.x % Lg;
    long long strip = (long long)blockIdx.x * G::SG + sgl;
    const bool ok = strip < a.nstrips;  // a wide row group past the last strip redoes it without storing
    if (!G::WIDE && !ok) return;
    if (!ok) strip = a.nstrips - 1;
    const int H = a.H, R = a.R;
    const int spp = H / R;
    const long long p = strip / spp;
    const int i0 = (int)(strip % spp) * R;
    auto lx = Xf::lds_of(tw + W + sgl * RowBuf::slots(N));
    const float rho = a.rho[0];
    const float tau = a.lam[0] / rho;
    const bool pa = t < Lp, sa = t < Ls;
    const bool pst = ok && pa, sst = ok && sa;

    const cf* sp = a.sin + (size_t)p * H * N;
    cf* so = a.sout + (size_t)p * H * N;
    const size_t poff = (size_t)p * H * W;
    auto img = [&](const float* base) { return reinterpret_cast<const cf*>(base + poff); };
    cf* bb = reinterpret_cast<cf*>(a.bbar + poff);
    const cf* abxi = LASTK ? nullptr : img(a.abx_in);
    const cf* abyi = LASTK ? nullptr : img(a.aby_in);
    cf* abxo = FIRSTK ? nullptr : reinterpret_cast<cf*>(a.abx_out + poff);
    cf* abyo = FIRSTK ? nullptr : reinterpret_cast<cf*>(a.aby_out + poff);
    const cf* akx = img(a.akx);
    const cf* aky = img(a.aky);
    const cf* apx = FIRSTK ? nullptr : img(a.apx);
    const cf* apy = FIRSTK ? nullptr : img(a.apy);
    const cf* npx = reinterpret_cast<const cf*>(a.np);
    const cf* npy = reinterpret_cast<const cf*>(a.np + (size_t)H * W);
    const cf* qpx = reinterpret_cast<const cf*>(a.qp);
    const cf* qpy = reinterpret_cast<const cf*>(a.qp + (size_t)H * W);
    const cf z2 = mkc(0.f, 0.f);

    auto rrow = [&](int g, cf (&x)[Ep]) {  // r^ row g in pixel layout
        cf v[EM];
        if (sa) {
#pragma unroll
            for (int j = 0; j < Es; ++j) v[j] = ld_pol<kSpecNT>(&sp[(size_t)g * N + t + Ls * j]);
        }
        Xf::c2r(v, lx, tw, t);
#pragma unroll
        for (int j = 0; j < Ep; ++j) x[j] = v[j];
    };
    double rho_acc = 0.0, tau_acc = 0.0;
    cf rprev[Ep], rcur[Ep], abxp[Ep], abyp[Ep];
    rrow(i0 == 0 ? H - 1 : i0 - 1, rprev);
    for (int rr = 0; rr <= R; ++rr) {
        const int g = i0 + rr >= H ? i0 + rr - H : i0 + rr;
        const size_t ro = (size_t)g * N;
        rrow(g, rcur);

        // ---- y direction at row g
        cf abyc[Ep];
#pragma unroll
        for (int j = 0; j < Ep; ++j) {
            const size_t i = ro + t + Lp * j;
            const float d0 = rcur[j].x - rprev[j].x, d1 = rcur[j].y - rprev[j].y;  // Dy r^
            cf ap = z2, npv = z2;
            if constexpr (!FIRSTK) {
                if (pa) {
                    ap = ld_pol<kNT>(&apy[i]);
                    if constexpr (ISO) npv = npy[i];
                }
            }
            const float zp0 = FIRSTK ? 0.f : shrink_z<ISO>(ap.x, tau, npv.x);
            const float zp1 = FIRSTK ? 0.f : shrink_z<ISO>(ap.y, tau, npv.y);
            if (rr < R && pa) {
                // rho^ += Dy r^ . (w_{k-1} - Dy x_k),  w = 2z - a,  Dy x_k = a_k - a_p + z_p
                const cf ak = ld_pol<kNT>(&aky[i]);
                const float e0 = (2.f * zp0 - ap.x) - (ak.x - ap.x + zp0);
                const float e1 = (2.f * zp1 - ap.y) - (ak.y - ap.y + zp1);
                rho_acc = fma((double)d0, (double)e0, fma((double)d1, (double)e1, rho_acc));
            }
            if constexpr (!FIRSTK) {
                const cf ub = (LASTK || !pa) ? z2 : ld_pol<kNT>(&abyi[i]);
                const float wb0 = rho * d0, wb1 = rho * d1;
                const float zb0 = 2.f * wb0 - ub.x, zb1 = 2.f * wb1 - ub.y;
                cf q = z2;
                if constexpr (ISO) q = pa ? qpy[i] : z2;
                abyc[j] = mkc(ub.x - wb0 + shrink_vjp<ISO>(ap.x, zb0, tau, npv.x, q.x),
                              ub.y - wb1 + shrink_vjp<ISO>(ap.y, zb1, tau, npv.y, q.y));
                if constexpr (!ISO) {
                    if (rr < R && pa) tau_acc += (double)soft_dtau(ap.x, zb0, tau) + (double)soft_dtau(ap.y, zb1, tau);
                }
            }
        }
        if constexpr (!FIRSTK) {
            if (rr < R && pst) {
#pragma unroll
                for (int j = 0; j < Ep; ++j) st_pol<kNT>(&abyo[ro + t + Lp * j], abyc[j]);
            }
        }
        // ---- b^ += r^ (row g)
        if (rr < R && pst) {
#pragma unroll
            for (int j = 0; j < Ep; ++j) {
                cf v = rcur[j];
                if constexpr (!LASTK) {
                    const cf o = ld_pol<kNT>(&bb[ro + t + Lp * j]);
                    v = mkc(o.x + v.x, o.y + v.y);
                }
                st_pol<kNT>(&bb[ro + t + Lp * j], v);
            }
        }
        // ---- finalize x^_{k-1} at row g-1: D^T a^ = (a^x[q] - a^x[q+1]) + (a^y[g-1] - a^y[g])
        if constexpr (!FIRSTK) {
            if (rr >= 1) {
                const int gm = g == 0 ? H - 1 : g - 1;
                const size_t rm = (size_t)gm * N;
                float axs[Ep], ars[Ep];
#pragma unroll
                for (int j = 0; j < Ep; ++j) axs[j] = abxp[j].x;
                Xf::template neighbour<+1>(axs, ars, lx, t);  // a^_x at pixel q1+1
                cf r[EM];
#pragma unroll
                for (int j = 0; j < Ep; ++j)
                    r[j] = mkc((abxp[j].x - abxp[j].y) + (abyp[j].x - abyc[j].x),
                               (abxp[j].y - ars[j]) + (abyp[j].y - abyc[j].y));
                Xf::r2c(r, lx, tw, t);
                if (sst) {
#pragma unroll
                    for (int j = 0; j < Es; ++j) st_pol<kNT>(&so[rm + t + Ls * j], r[j]);
                }
            }
        }
        // ---- x direction at row g
        if (rr < R) {
            float rys[Ep], rls[Ep];
#pragma unroll
            for (int j = 0; j < Ep; ++j) rys[j] = rcur[j].y;
            Xf::template neighbour<-1>(rys, rls, lx, t);  // r^ at pixel q0-1
#pragma unroll
            for (int j = 0; j < Ep; ++j) {
                const size_t i = ro + t + Lp * j;
                const float d0 = rcur[j].x - rls[j], d1 = rcur[j].y - rcur[j].x;  // Dx r^
                cf ap = z2, npv = z2;
                if constexpr (!FIRSTK) {
                    if (pa) {
                        ap = ld_pol<kNT>(&apx[i]);
                        if constexpr (ISO) npv = npx[i];
                    }
                }
                const float zp0 = FIRSTK ? 0.f : shrink_z<ISO>(ap.x, tau, npv.x);
                const float zp1 = FIRSTK ? 0.f : shrink_z<ISO>(ap.y, tau, npv.y);
                if (pa) {
                    const cf ak = ld_pol<kNT>(&akx[i]);
                    const float e0 = (2.f * zp0 - ap.x) - (ak.x - ap.x + zp0);
                    const float e1 = (2.f * zp1 - ap.y) - (ak.y - ap.y + zp1);
                    rho_acc = fma((double)d0, (double)e0, fma((double)d1, (double)e1, rho_acc));
                }
                if constexpr (!FIRSTK) {
                    const cf ub = (LASTK || !pa) ? z2 : ld_pol<kNT>(&abxi[i]);
                    const float wb0 = rho * d0, wb1 = rho * d1;
                    const float zb0 = 2.f * wb0 - ub.x, zb1 = 2.f * wb1 - ub.y;
                    cf q = z2;
                    if constexpr (ISO) q = pa ? qpx[i] : z2;
                    abxp[j] = mkc(ub.x - wb0 + shrink_vjp<ISO>(ap.x, zb0, tau, npv.x, q.x),
                                  ub.y - wb1 + shrink_vjp<ISO>(ap.y, zb1, tau, npv.y, q.y));
                    if constexpr (!ISO) {
                        if (pa) tau_acc += (double)soft_dtau(ap.x, zb0, tau) + (double)soft_dtau(ap.y, zb1, tau);
                    }
                }
            }
            if constexpr (!FIRSTK) {
                if (pst) {
#pragma unroll
                    for (int j = 0; j < Ep; ++j) st_pol<kNT>(&abxo[ro + t + Lp * j], abxp[j]);
                }
            }
        }
#pragma unroll
        for (int j = 0; j < Ep; ++j) {
            if constexpr (!FIRSTK) abyp[j] = abyc[j];
            rprev[j] = rcur[j];
        }
    }
    // per-strip partial sums, fixed order: a butterfly over each wave's lanes of the row group, then
    // (wide groups) the waves' sums in wave order through the group's LDS buffer
    constexpr int WL = Lg < 64 ? Lg : 64;
#pragma unroll
    for (int o = WL / 2; o >= 1; o >>= 1) {
        rho_acc += __shfl_xor(rho_acc, o, WL);
        tau_acc += __shfl_xor(tau_acc, o, WL);
    }
    if constexpr (G::WIDE) {
        double* red = reinterpret_cast<double*>(lx.base);  // the group's exchange buffer, no longer read
        lds_barrier();
        if (t % 64 == 0) {
            red[2 * (t / 64)] = rho_acc;
            red[2 * (t / 64) + 1] = tau_acc;
        }
        lds_barrier();
        if (t == 0) {
            rho_acc = red[0];
            tau_acc = red[1];
#pragma unroll
            for (int w = 1; w < Lg / 64; ++w) {
                rho_acc += red[2 * w];
                tau_acc += red[2 * w + 1];
            }
        }
    }
    if (ok && t == 0) {
        a.part[2 * strip + 0] = rho_acc;
        a.part[2 * strip + 1] = tau_acc;
    }
}

// iso: Q_{k-1} = sum over planes of a_{k-1} z^_{k-1} (k_bwd_iso_q) on the mixed row transforms
template <int N, bool LASTK>
__global__ void __launch_bounds__(256) k_bwd_iso_q_m(BwdIsoArgs a) {
    using G = MRowG<N, BPlan<N>>;
    using Xf = RowXfM<N, BPlan<N>>;
    constexpr int Lg = G::Lg, Lp = G::Lp, Ep = G::Ep, Ls = G::Ls, Es = G::Es, EM = G::EM, W = G::W;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    cf* tw = reinterpret_cast<cf*>(smem);
    load_tw(tw, a.twW, W);
    __syncthreads();
    const int sgl = threadIdx.x / Lg, t = threadIdx.x % Lg;
    long long item = (long long)blockIdx.x * G::SG + sgl;
    const bool ok = item < a.nitems;
    if (!G::WIDE && !ok) return;
    if (!ok) item = a.nitems - 1;
    const int H = a.H;
    const int g = (int)(item % H);
    const int grp = (int)(item / H);
    const int gm = g == 0 ? H - 1 : g - 1;
    auto lx = Xf::lds_of(tw + W + sgl * RowBuf::slots(N));
    const bool pa = t < Lp, sa = t < Ls;
    const float rho = a.rho[0];
    const cf z2 = mkc(0.f, 0.f);
    cf qx[Ep], qy[Ep];
#pragma unroll
    for (int j = 0; j < Ep; ++j) qx[j] = qy[j] = z2;
    const int p1 = min(a.P, (grp + 1) * a.ppg);
    for (int p = grp * a.ppg; p < p1; ++p) {
        const cf* sp = a.sin + (size_t)p * H * N;
        cf rp[EM], rc[EM];
        if (sa) {
#pragma unroll
            for (int j = 0; j < Es; ++j) {
                rp[j] = sp[(size_t)gm * N + t + Ls * j];
                rc[j] = sp[(size_t)g * N + t + Ls * j];
            }
        }
        Xf::c2r(rp, lx, tw, t);
        Xf::c2r(rc, lx, tw, t);
        const size_t ro = (size_t)p * H * N + (size_t)g * N;
        const cf* abx = reinterpret_cast<const cf*>(a.abx_in);
        const cf* aby = reinterpret_cast<const cf*>(a.aby_in);
        const cf* apx = reinterpret_cast<const cf*>(a.apx);
        const cf* apy = reinterpret_cast<const cf*>(a.apy);
        float rys[Ep], rls[Ep];
#pragma unroll
        for (int j = 0; j < Ep; ++j) rys[j] = rc[j].y;
        Xf::template neighbour<-1>(rys, rls, lx, t);
        if (pa) {
#pragma unroll
            for (int j = 0; j < Ep; ++j) {
                const size_t i = ro + t + Lp * j;
                const cf ubx = LASTK ? z2 : abx[i];
                const cf uby = LASTK ? z2 : aby[i];
                const cf ax = apx[i], ay = apy[i];
                const float zx0 = 2.f * rho * (rc[j].x - rls[j]) - ubx.x, zx1 = 2.f * rho * (rc[j].y - rc[j].x) - ubx.y;
                const float zy0 = 2.f * rho * (rc[j].x - rp[j].x) - uby.x, zy1 = 2.f * rho * (rc[j].y - rp[j].y) - uby.y;
                qx[j].x = fmaf(ax.x, zx0, qx[j].x);
                qx[j].y = fmaf(ax.y, zx1, qx[j].y);
                qy[j].x = fmaf(ay.x, zy0, qy[j].x);
                qy[j].y = fmaf(ay.y, zy1, qy[j].y);
            }
        }
    }
    if (ok && pa) {
        cf* px = reinterpret_cast<cf*>(a.partial + ((size_t)grp * 2 + 0) * H * W) + (size_t)g * N;
        cf* py = reinterpret_cast<cf*>(a.partial + ((size_t)grp * 2 + 1) * H * W) + (size_t)g * N;
#pragma unroll
        for (int j = 0; j < Ep; ++j) {
            px[t + Lp * j] = qx[j];
            py[t + Lp * j] = qy[j];
        }
    }
}

}  // namespace admm

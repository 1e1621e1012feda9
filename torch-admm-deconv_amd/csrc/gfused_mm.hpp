// gfused_mm.hpp -- the generic-size row pass of an aniso inference iteration as ONE kernel on the matrix
// cores: row inverse (half spectra -> x), the ADMM step (u update, r = b + rho D^T w) and the row
// forward transform of r (r -> half spectra), for row lengths W = S R with an odd R in [17, 127] that
// carries W's large prime factor (BSD: 481 = 13 * 37).  The power-of-two path's pass A restated for
// generic sizes: x never goes through HBM, so an iteration moves 28 + 8 B/px
// (this pass + the column pass) instead of 28 + 8 + 8 (the step pass, the column pass and a separate
// row inverse).  The reference's loop body, deconv.py:104-115 (x-update, Dx/Dy, shrinkage, dual update).
//
// A block owns one strip of nr <= 2 NLf consecutive rows of one plane (strips never cross planes; the
// vertical neighbours wrap inside the plane as the reference's circular differences do):
//   1. stage the spectra of the strip's rows and its two halo rows (i0 - 1, i1, mod H)     -> LDS
//   2. inverse transform of those nr + 2 rows, two rows per complex line (k_grow_inv_mm's
//      decomposition: S-point DFTs + twiddles per (line, k1), then the R-point DFTs as
//      cosine / sine matrix products, v_mfma_f32_16x16x4_f32)                               -> x image
//   3. the step for every pixel of the strip (u_k out, r_{k+1} in registers), written straight as the
//      s / d operands of the forward R-point transforms (pixel pairs n2 + S q, n2 + S (R - q))
//   4. forward R-point DFTs (matrix products), twiddles, S-point DFTs, Hermitian split of the two
//      rows of each line -> the strip's half spectra (LDS), stored row by row (coalesced)
// The step reproduces k_gstep's expressions (generic_kernels.hpp gstep_pxr, ISO = false, HIST = false)
// operation for operation, so the unfused and fused passes differ only in the transforms' rounding.
#pragma once
#include "gcol_mm.hpp"

namespace admm {

struct GFusedArgs {
    const cf* spec_in;  // [P][H][ld]: the column pass's output (x_k's half spectra)
    cf* spec_out;       // [P][H][ld]: r_{k+1}'s half spectra (another buffer: neighbours read halos)
    const float* b;     // [P][H][W]
    const float* uxi;   // u_{k-1} (unused when FIRST)
    const float* uyi;
    float* uxo;         // u_k
    float* uyo;
    const float* lam;
    const float* rho;
    const cf* tw;       // [W] exp(-2 pi i m / W)
    long long P;
    int H, W, Wh, ld;
    int R, h, KS, MT;
    int NLi, RPi;       // inverse: lines (nr + 2 rows) and the matrix image's row pitch (floats)
    int NLf, RPf;       // forward: lines (nr rows)
    int nstrip;         // strips per plane
    int regA, offX, offT;  // LDS regions (floats): [0, regA) staging / matrix images, X, twiddles
};

template <int S, int NTH = 512>
__global__ void __launch_bounds__(NTH) __attribute__((amdgpu_waves_per_eu(NTH == 512 ? 4 : 3)))
k_grow_fused_mm(GFusedArgs a) {
    extern __shared__ __attribute__((aligned(16))) float F[];
    constexpr int MAXT = NTH == 512 ? 4 : 8;
    const int H = a.H, W = a.W, Wh = a.Wh, R = a.R, h = a.h, KS = a.KS, MT = a.MT;
    const int NLi = a.NLi, NLf = a.NLf, RPi = a.RPi, RPf = a.RPf;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int jl = lane & 15, g = lane >> 4;
    const long long p = blockIdx.x / a.nstrip;
    const int s = (int)(blockIdx.x - p * a.nstrip);
    const int i0 = (int)((long long)s * H / a.nstrip), i1 = (int)((long long)(s + 1) * H / a.nstrip);
    const int nr = i1 - i0, nri = nr + 2;
    const long long prow = p * H;  // first image row of the plane
    cf* Xs = reinterpret_cast<cf*>(F);                  // staged spectrum rows [2 NLi][Wh] (region A)
    float* X = F + a.offX;                               // x rows [nri][W]: row m = image row i0 - 1 + m
    cf* twl = reinterpret_cast<cf*>(F + a.offT);
    // image row of inverse row m (the halos wrap inside the plane)
    auto irow = [&](int m) -> int {
        int i = i0 - 1 + m;
        i += (i < 0) ? H : 0;
        i -= (i >= H) ? H : 0;
        return i;
    };

    // --- 1. stage (a thread's kMMU loads issued together)
    {
        const int nst = 2 * NLi * Wh;
        for (int base = tid; base < nst; base += kMMU * NTH) {
            cf v[kMMU];
            static_for<0, kMMU>([&](auto uc) {
                constexpr int u = decltype(uc)::value;
                const int idx = base + u * NTH;
                const int m = idx / Wh, k = idx - m * Wh;
                v[u] = (idx < nst && m < nri) ? a.spec_in[(prow + irow(m)) * a.ld + k] : mkc(0.f, 0.f);
            });
            static_for<0, kMMU>([&](auto uc) {
                constexpr int u = decltype(uc)::value;
                if (base + u * NTH < nst) Xs[base + u * NTH] = v[u];
            });
        }
    }
    for (int i = tid; i < W; i += NTH) twl[i] = a.tw[i];
    __syncthreads();

    // the cosine / sine matrix fragments (the same for both directions; k_grow_inv_mm's), loaded from
    // the twiddles right before each product phase (not held through the VALU phases: registers)
    const int G = (NTH / 64) / MT;
    const bool gw = wv < MT * G;
    const int mt = wv % MT, tile0 = wv / MT, tstep = G;
    float a1[16], a2[16];
    auto fragments = [&]() {
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
    };
    mm_f32x4 acc1[8], acc2[8];

    // --- 2. inverse: per (line l, k1 <= h) the S-point inverse DFTs + conjugate twiddles (registers)
    {
        auto zval = [&](int l, int k) -> cf {  // Z[k] of line l (Hermitian completion of both rows)
            const bool lo = k < Wh;
            const int kk = lo ? k : W - k;
            cf xa = Xs[(2 * l) * Wh + kk], xb = Xs[(2 * l + 1) * Wh + kk];
            if (kk == 0 || 2 * kk == W) xa.y = xb.y = 0.f;
            if (!lo) xa.y = -xa.y, xb.y = -xb.y;
            return mkc(xa.x - xb.y, xa.y + xb.x);
        };
        const int nmid = NLi * (h + 1);
        float4 sd[S];
        const int l1 = tid % NLi, k1 = tid / NLi;
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
        __syncthreads();  // the staged rows are read; the matrix image overwrites them
        if (tid < nmid) {
#pragma unroll
            for (int n2 = 0; n2 < S; ++n2) *reinterpret_cast<float4*>(&F[k1 * RPi + 4 * (l1 * S + n2)]) = sd[n2];
        }
        for (int idx = tid; idx < (4 * KS - h - 1) * RPi; idx += NTH) F[(h + 1) * RPi + idx] = 0.f;
    }
    __syncthreads();
    const int NTi = (NLi * S + 7) / 8, NTf = (NLf * S + 7) / 8;
    const int ntwi = gw ? (NTi - tile0 + G - 1) / G : 0, ntwf = gw ? (NTf - tile0 + G - 1) / G : 0;
    fragments();
    mm_ntw<MAXT>(ntwi, [&](auto nc) { mm_products<decltype(nc)::value>(F, a1, a2, acc1, acc2, KS, RPi, tile0, tstep, g, jl); });
    __syncthreads();
    mm_ntw<MAXT>(ntwi, [&](auto nc) { mm_store<+1, decltype(nc)::value>(F, acc1, acc2, h, RPi, tile0, tstep, mt, g, jl); });
    __syncthreads();
    // x[n] of inverse row m at n = n2 + S n1: (n1 <= h) slot 0 of row n1, else slot 1 of row R - n1;
    // real part = even row of the line, imaginary part = odd row
    for (int idx = tid; idx < nri * W; idx += NTH) {
        const int m = idx / W, n = idx - m * W;
        const int n1 = n / S, n2 = n - n1 * S;
        const bool lo = n1 <= h;
        X[idx] = F[(lo ? n1 : R - n1) * RPi + 4 * ((m >> 1) * S + n2) + (lo ? 0 : 1) + 2 * (m & 1)];
    }
    __syncthreads();

    // --- 3. the step, straight into the forward matrix image: item (line l, q <= h, n2) owns the pixel
    // pair n2 + S q, n2 + S (R - q) of the strip rows 2 l, 2 l + 1
    {
        const float rho = a.rho[0];
        const float tau = a.lam[0] / rho;
        const int per_line = (h + 1) * S;
        const int nitem = NLf * per_line;
        // r at (strip row r, column j); writes u_k
        auto step = [&](int r, int j) -> float {
            const int i = i0 + r;
            const int jm = j == 0 ? W - 1 : j - 1, jp = j == W - 1 ? 0 : j + 1;
            const int ip = i == H - 1 ? 0 : i + 1;
            const size_t P0 = (size_t)(prow + i) * W + j, PR = (size_t)(prow + i) * W + jp,
                         PD = (size_t)(prow + ip) * W + j;
            const float* xr0 = X + (r + 1) * W;
            const float x = xr0[j], xl = xr0[jm], xr = xr0[jp];
            const float xu = X[r * W + j], xd = X[(r + 2) * W + j];
            const float ux0 = a.uxi ? a.uxi[P0] : 0.f, uxR = a.uxi ? a.uxi[PR] : 0.f;
            const float uy0 = a.uyi ? a.uyi[P0] : 0.f, uyD = a.uyi ? a.uyi[PD] : 0.f;
            const float ax = (x - xl) + ux0, ay = (x - xu) + uy0;
            const float zx = shrink_z<false>(ax, tau, 0.f), zy = shrink_z<false>(ay, tau, 0.f);
            const float nux = ax - zx, nuy = ay - zy;
            const float wx = zx - nux, wy = zy - nuy;
            const float axR = (xr - x) + uxR, ayD = (xd - x) + uyD;
            const float zxR = shrink_z<false>(axR, tau, 0.f), zyD = shrink_z<false>(ayD, tau, 0.f);
            const float wxR = zxR - (axR - zxR), wyD = zyD - (ayD - zyD);
            a.uxo[P0] = nux;
            a.uyo[P0] = nuy;
            const float v = (wx - wxR) + (wy - wyD);
            return fmat(rho, v, a.b[P0]);
        };
        for (int it = tid; it < nitem; it += NTH) {
            const int l = it / per_line, rest = it - l * per_line;
            const int q = rest / S, n2 = rest - q * S;
            const int ra = 2 * l, rb = 2 * l + 1;
            const int j0 = n2 + S * q, j1 = n2 + S * (R - q);
            float a0 = 0.f, b0 = 0.f, a1v = 0.f, b1v = 0.f;
            if (ra < nr) {
                a0 = step(ra, j0);
                if (q) a1v = step(ra, j1);
            }
            if (rb < nr) {
                b0 = step(rb, j0);
                if (q) b1v = step(rb, j1);
            }
            // z = r_a + i r_b at j0 and j1 -> s / d of the R-point transform's operands
            *reinterpret_cast<float4*>(&F[q * RPf + 4 * (l * S + n2)]) =
                q ? make_float4(a0 + a1v, a0 - a1v, b0 + b1v, b0 - b1v) : make_float4(a0, 0.f, b0, 0.f);
        }
        for (int idx = tid; idx < (4 * KS - h - 1) * RPf; idx += NTH) F[(h + 1) * RPf + idx] = 0.f;
    }
    __syncthreads();

    // --- 4. forward transforms of r
    fragments();
    mm_ntw<MAXT>(ntwf, [&](auto nc) { mm_products<decltype(nc)::value>(F, a1, a2, acc1, acc2, KS, RPf, tile0, tstep, g, jl); });
    __syncthreads();
    mm_ntw<MAXT>(ntwf, [&](auto nc) { mm_store<-1, decltype(nc)::value>(F, acc1, acc2, h, RPf, tile0, tstep, mt, g, jl); });
    __syncthreads();
    // per (line l, k1 <= h): twiddles, S-point DFTs -> Z[k1 + R k2], Z[R - k1 + R k2]; the two real rows'
    // spectra A = (Z[k] + conj Z[W - k]) / 2, B = (Z[k] - conj Z[W - k]) / 2i into the output staging
    // (the x image's region: x is no longer read)
    {
        cf* Os = reinterpret_cast<cf*>(X);  // [2 NLf][Wh]
        const int nmid = NLf * (h + 1);
        for (int it = tid; it < nmid; it += NTH) {
            const int l = it % NLf, k1 = it / NLf;
            cf v[S], vr[S];
#pragma unroll
            for (int n2 = 0; n2 < S; ++n2) {
                const float4 y = *reinterpret_cast<const float4*>(&F[k1 * RPf + 4 * (l * S + n2)]);
                v[n2] = mkc(y.x, y.z);
                vr[n2] = mkc(y.y, y.w);
            }
#pragma unroll
            for (int n2 = 1; n2 < S; ++n2) {
                v[n2] = cmul(v[n2], twl[n2 * k1]);
                if (k1) vr[n2] = cmul(vr[n2], twl[n2 * (R - k1)]);
            }
            small_dft<-1, S>(v, twl, W);
            if (k1) small_dft<-1, S>(vr, twl, W);
            const int ra = 2 * l;
            auto put = [&](int k, cf z, cf m) {
                if (k < Wh) {
                    Os[ra * Wh + k] = mkc(0.5f * (z.x + m.x), 0.5f * (z.y - m.y));
                    Os[(ra + 1) * Wh + k] = mkc(0.5f * (z.y + m.y), 0.5f * (m.x - z.x));
                }
            };
#pragma unroll
            for (int k2 = 0; k2 < S; ++k2) {
                if (k1 == 0) {
                    put(R * k2, v[k2], v[(S - k2) % S]);
                } else {
                    put(k1 + R * k2, v[k2], vr[S - 1 - k2]);
                    put(R - k1 + R * k2, vr[k2], v[S - 1 - k2]);
                }
            }
        }
        __syncthreads();
        const int nout = nr * Wh;
        for (int idx = tid; idx < nout; idx += NTH) {
            const int r = idx / Wh, k = idx - r * Wh;
            a.spec_out[(prow + i0 + r) * a.ld + k] = Os[idx];
        }
    }
}

}  // namespace admm

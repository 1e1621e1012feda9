// admm_backward.hpp -- reverse pass of the unrolled ADMM-TV iteration (gfx950).
//
// Forward iteration k = 1..K (training mode keeps a_k for every k, see pass A):
//   r_k = b + rho D^T w_{k-1}            w_{k-1} = z_{k-1} - u_{k-1}   (w_0 = u_0 = 0)
//   x_k = M r_k,  M = F^-1 diag(fc) F    (self-adjoint)
//   a_k = D x_k + u_{k-1};  z_k = S(a_k; tau);  u_k = a_k - z_k;  w_k = 2 z_k - a_k
// Reverse step k = K..1, given the adjoints u^_k, w^_k of iteration k's outputs
// (zero at k = K) and x^_K = dL/dx_K:
//   r^_k   = M x^_k                                  (pass B, unchanged)
//   b^    += r^_k
//   w^_{k-1} = rho D r^_k
//   rho^  += <D r^_k, w_{k-1}> - <D r^_k, D x_k>     (second term: dM/drho = -M D^T D M)
//   z^_{k-1} = 2 w^_{k-1} - u^_{k-1},  u^_{k-1} = a^_k
//   a^_{k-1} = u^_{k-1} - w^_{k-1} + J_S(a_{k-1})^T z^_{k-1};  tau^ += dS/dtau . z^_{k-1}
//   x^_{k-1} = D^T a^_{k-1}
// with D x_k = a_k - u_{k-1}.  The spatial stencils and shrink Jacobians are fused into
// one row pass (k_bwd_pass_a), the same strip/halo structure as the forward pass A.
// iso: J_S couples planes through the per-pixel norm; Q = sum_{b,c} a z^ is formed by
// k_bwd_iso_q first (like the forward norm pass).
#pragma once
#include "admm_kernels.hpp"

namespace admm {

struct BwdArgs {
    const cf* sin;        // r^_k row spectra (pass B output)                  [P][H][N]
    cf* sout;             // x^_{k-1} row spectra (k >= 2)                      [P][H][N]
    float* bbar;          // b^ accumulator                                    [P][H][W]
    const float* abx_in;  // a^_k = u^_{k-1}  (k < K)                           [P][H][W]
    const float* aby_in;
    float* abx_out;       // a^_{k-1} (k >= 2)
    float* aby_out;
    const float* akx;     // a_k      (history slot k-1)
    const float* aky;
    const float* apx;     // a_{k-1}  (history slot k-2, k >= 2)
    const float* apy;
    const float* np;      // iso: N_{k-1}                                       [2][H][W]
    const float* qp;      // iso: Q_{k-1} = sum_{b,c} a_{k-1} z^_{k-1}          [2][H][W]
    const float* lam;
    const float* rho;
    double* part;         // per strip: {rho^ partial, tau^ partial}, fp64      [nstrips][2]
    const cf* twW;
    int H, R;
    long long nstrips;
    long long ppm;        // planes per module (PassAArgs): lam/rho[m], np/qp + m 2HW
};

// S'(a) contracted with z^: aniso mask, iso block Jacobian (f z^ + 2 a f'(N) Q)
template <bool ISO>
__device__ __forceinline__ float shrink_vjp(float a, float zb, float tau, float n, float q) {
    if constexpr (ISO) {
        const float s = sqrtf(n + 1e-15f);
        const float d = s + 1e-15f;
        const float f = 1.f - tau / d;
        if (!(f > 0.f)) return 0.f;
        const float fp = tau / (d * d) * (0.5f / s);  // df/dN
        return fmaf(f, zb, 2.f * a * fp * q);
    } else {
        return (fabsf(a) > tau) ? zb : 0.f;
    }
}
// dS/dtau . z^ (aniso only; iso's tau term is summed per pixel in k_bwd_iso_q)
__device__ __forceinline__ float soft_dtau(float a, float zb, float tau) {
    return (fabsf(a) > tau) ? (a > 0.f ? -zb : zb) : 0.f;  // -sign(a) z^ on the active set
}
// fp64 (the generic kernels' double instantiation)
template <bool ISO>
__device__ __forceinline__ double shrink_vjp(double a, double zb, double tau, double n, double q) {
    if constexpr (ISO) {
        const double s = sqrt(n + 1e-15);
        const double d = s + 1e-15;
        const double f = 1.0 - tau / d;
        if (!(f > 0.0)) return 0.0;
        const double fp = tau / (d * d) * (0.5 / s);
        return fma(f, zb, 2.0 * a * fp * q);
    } else {
        return (fabs(a) > tau) ? zb : 0.0;
    }
}
__device__ __forceinline__ double soft_dtau(double a, double zb, double tau) {
    return (fabs(a) > tau) ? (a > 0.0 ? -zb : zb) : 0.0;
}

// Row transform configuration of the reverse row pass.  Its lanes carry five row states (r^ of two
// rows, a^_x of the previous row, a^_y of two rows) besides the transform, so at the forward's E values
// per lane the 256-point rows (W = 512: config 5) needed 229 VGPRs iso -- two waves per SIMD, and the
// latency-bound pass ran at 0.33 of the HBM peak (SQ: an instruction in flight 26 % of the cycles).
// 256-point rows run here with 4 values per lane over a full wave (4 * 4 * 4 * 4: one more LDS exchange
// per transform), which halves the state registers.
template <int N> struct BwdCfg : RowCfg<N> {};
template <> struct BwdCfg<256> {
    static constexpr int E = 4;
    using S = Sched<4, 4, 4, 4>;
};
template <int N> struct BwdGeom {
    static constexpr int E = BwdCfg<N>::E, L = N / E, W = 2 * N;
    static constexpr int NT = 256, SG = NT / L;
    static constexpr size_t lds_bytes() { return sizeof(cf) * (W + SG * RowBuf::slots(N)); }
};

// occupancy target of the reverse row pass (waves per SIMD), as PASSA_MINW for the forward:
// 3 for aniso (measured -2.4 % at C3 size; a few registers spill), 2 for iso, whose extra
// norm / Q operands would spill ~240 B at 3 (measured +4 %); the 4-value 256-point rows fit 3 iso
#define BWDA_MINW(n, iso) ((n) >= 1024 ? 1 : (n) == 256 ? 3 : (iso) ? 2 : 3)

template <int N, bool ISO, bool LASTK, bool FIRSTK>
__global__ void __launch_bounds__(256, BWDA_MINW(N, ISO)) k_bwd_pass_a(BwdArgs a) {
    using G = BwdGeom<N>;
    using Xf = RowXf<N, BwdCfg<N>>;
    constexpr int E = G::E, L = G::L, W = G::W;
    // streaming history / adjoint images and the spectra non-temporal, as the forward's pass A;
    // the per-module norm and Q maps (re-read by every plane) stay cacheable
    constexpr bool kNT = ADMM_NT_BWD != 0;
    constexpr bool kSpecNT = kNT && ((ADMM_NT & 2) != 0 || ((ADMM_NT & 32) != 0 && N >= 512));
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    cf* tw = reinterpret_cast<cf*>(smem);
    load_tw(tw, a.twW, W);
    __syncthreads();
    const int sgl = threadIdx.x / L, t = threadIdx.x % L;
    const long long strip = (long long)blockIdx.x * G::SG + sgl;
    if (strip >= a.nstrips) return;
    const int H = a.H, R = a.R;
    const int spp = H / R;
    const long long p = strip / spp;
    const int i0 = (int)(strip % spp) * R;
    RowBuf buf{tw + W + sgl * RowBuf::slots(N)};
    const int mod = (int)(p / a.ppm);
    const float rho = a.rho[mod];
    const float tau = a.lam[mod] / rho;
    const size_t moff = (size_t)mod * 2 * H * W;

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
    const cf* npx = reinterpret_cast<const cf*>(a.np + moff);
    const cf* npy = reinterpret_cast<const cf*>(a.np + moff + (size_t)H * W);
    const cf* qpx = reinterpret_cast<const cf*>(a.qp + moff);
    const cf* qpy = reinterpret_cast<const cf*>(a.qp + moff + (size_t)H * W);

    // the lambda / rho gradient partials accumulate in fp64 from the first product on (per lane,
    // then over the sub-group, the strips and the iterations: k_bwd_scalars)
    double rho_acc = 0.0, tau_acc = 0.0;
    cf rprev[E], rcur[E], abxp[E], abyp[E];
    {
        const int g = (i0 - 1 + H) & (H - 1);
#pragma unroll
        for (int j = 0; j < E; ++j) rprev[j] = ld_pol<kSpecNT>(&sp[(size_t)g * N + t + L * j]);
        Xf::c2r(rprev, buf, tw, t);
    }
    for (int rr = 0; rr <= R; ++rr) {
        const int g = (i0 + rr) & (H - 1);
        const size_t ro = (size_t)g * N;
#pragma unroll
        for (int j = 0; j < E; ++j) rcur[j] = ld_pol<kSpecNT>(&sp[ro + t + L * j]);
        Xf::c2r(rcur, buf, tw, t);

        // ---- y direction at row g
        cf abyc[E];
        {
#pragma unroll
            for (int j = 0; j < E; ++j) {
                const int i = (int)ro + t + L * j;
                const float d0 = rcur[j].x - rprev[j].x, d1 = rcur[j].y - rprev[j].y;  // Dy r^
                cf ap = mkc(0.f, 0.f), npv = mkc(0.f, 0.f);
                if constexpr (!FIRSTK) {
                    ap = ld_pol<kNT>(&apy[i]);
                    if constexpr (ISO) npv = npy[i];
                }
                const float zp0 = FIRSTK ? 0.f : shrink_z<ISO>(ap.x, tau, npv.x);
                const float zp1 = FIRSTK ? 0.f : shrink_z<ISO>(ap.y, tau, npv.y);
                if (rr < R) {
                    // rho^ += Dy r^ . (w_{k-1} - Dy x_k),  w = 2z - a,  Dy x_k = a_k - u_{k-1} = a_k - a_p + z_p
                    const cf ak = ld_pol<kNT>(&aky[i]);
                    const float e0 = (2.f * zp0 - ap.x) - (ak.x - ap.x + zp0);
                    const float e1 = (2.f * zp1 - ap.y) - (ak.y - ap.y + zp1);
                    rho_acc = fma((double)d0, (double)e0, fma((double)d1, (double)e1, rho_acc));
                }
                if constexpr (!FIRSTK) {
                    const cf ub = LASTK ? mkc(0.f, 0.f) : ld_pol<kNT>(&abyi[i]);
                    const float wb0 = rho * d0, wb1 = rho * d1;
                    const float zb0 = 2.f * wb0 - ub.x, zb1 = 2.f * wb1 - ub.y;
                    cf q = mkc(0.f, 0.f);
                    if constexpr (ISO) q = qpy[i];
                    abyc[j] = mkc(ub.x - wb0 + shrink_vjp<ISO>(ap.x, zb0, tau, npv.x, q.x),
                                  ub.y - wb1 + shrink_vjp<ISO>(ap.y, zb1, tau, npv.y, q.y));
                    if constexpr (!ISO) {
                        if (rr < R) tau_acc += (double)soft_dtau(ap.x, zb0, tau) + (double)soft_dtau(ap.y, zb1, tau);
                    }
                }
            }
            if constexpr (!FIRSTK) {
                if (rr < R) {
#pragma unroll
                    for (int j = 0; j < E; ++j) st_pol<kNT>(&abyo[ro + t + L * j], abyc[j]);
                }
            }
        }
        // ---- b^ += r^ (row g)
        if (rr < R) {
#pragma unroll
            for (int j = 0; j < E; ++j) {
                cf v = rcur[j];
                if constexpr (!LASTK) {
                    const cf o = ld_pol<kNT>(&bb[ro + t + L * j]);
                    v = mkc(o.x + v.x, o.y + v.y);
                }
                st_pol<kNT>(&bb[ro + t + L * j], v);
            }
        }
        // ---- finalize x^_{k-1} at row g-1: D^T a^ = (a^x[j] - a^x[j+1]) + (a^y[g-1] - a^y[g])
        if constexpr (!FIRSTK) {
            if (rr >= 1) {
                const int gm = (g - 1 + H) & (H - 1);
                const size_t rm = (size_t)gm * N;
                cf r[E], sh[E];
#pragma unroll
                for (int j = 0; j < E; ++j) sh[j].x = __shfl(abxp[j].x, (t + 1) & (L - 1), L);
#pragma unroll
                for (int j = 0; j < E; ++j) {
                    const float ar = (t == L - 1) ? sh[(j + 1) & (E - 1)].x : sh[j].x;
                    r[j] = mkc((abxp[j].x - abxp[j].y) + (abyp[j].x - abyc[j].x),
                               (abxp[j].y - ar) + (abyp[j].y - abyc[j].y));
                }
                Xf::r2c(r, buf, tw, t);
#pragma unroll
                for (int j = 0; j < E; ++j) st_pol<kNT>(&so[rm + t + L * j], r[j]);
            }
        }
        // ---- x direction at row g
        if (rr < R) {
            cf sh[E];
#pragma unroll
            for (int j = 0; j < E; ++j) sh[j].x = __shfl(rcur[j].y, (t - 1) & (L - 1), L);
#pragma unroll
            for (int j = 0; j < E; ++j) {
                const int i = (int)ro + t + L * j;
                const float rl = (t == 0) ? sh[(j - 1) & (E - 1)].x : sh[j].x;
                const float d0 = rcur[j].x - rl, d1 = rcur[j].y - rcur[j].x;  // Dx r^
                cf ap = mkc(0.f, 0.f), npv = mkc(0.f, 0.f);
                if constexpr (!FIRSTK) {
                    ap = ld_pol<kNT>(&apx[i]);
                    if constexpr (ISO) npv = npx[i];
                }
                const float zp0 = FIRSTK ? 0.f : shrink_z<ISO>(ap.x, tau, npv.x);
                const float zp1 = FIRSTK ? 0.f : shrink_z<ISO>(ap.y, tau, npv.y);
                const cf ak = ld_pol<kNT>(&akx[i]);
                const float e0 = (2.f * zp0 - ap.x) - (ak.x - ap.x + zp0);
                const float e1 = (2.f * zp1 - ap.y) - (ak.y - ap.y + zp1);
                rho_acc = fma((double)d0, (double)e0, fma((double)d1, (double)e1, rho_acc));
                if constexpr (!FIRSTK) {
                    const cf ub = LASTK ? mkc(0.f, 0.f) : ld_pol<kNT>(&abxi[i]);
                    const float wb0 = rho * d0, wb1 = rho * d1;
                    const float zb0 = 2.f * wb0 - ub.x, zb1 = 2.f * wb1 - ub.y;
                    cf q = mkc(0.f, 0.f);
                    if constexpr (ISO) q = qpx[i];
                    abxp[j] = mkc(ub.x - wb0 + shrink_vjp<ISO>(ap.x, zb0, tau, npv.x, q.x),
                                  ub.y - wb1 + shrink_vjp<ISO>(ap.y, zb1, tau, npv.y, q.y));
                    if constexpr (!ISO) tau_acc += (double)soft_dtau(ap.x, zb0, tau) + (double)soft_dtau(ap.y, zb1, tau);
                }
            }
            if constexpr (!FIRSTK) {
#pragma unroll
                for (int j = 0; j < E; ++j) st_pol<kNT>(&abxo[ro + t + L * j], abxp[j]);
            }
        }
#pragma unroll
        for (int j = 0; j < E; ++j) {
            if constexpr (!FIRSTK) abyp[j] = abyc[j];
            rprev[j] = rcur[j];
        }
    }
    // per-strip partial sums (fixed-order butterfly over the sub-group's lanes)
#pragma unroll
    for (int o = L / 2; o >= 1; o >>= 1) {
        rho_acc += __shfl_xor(rho_acc, o, L);
        tau_acc += __shfl_xor(tau_acc, o, L);
    }
    if (t == 0) {
        a.part[2 * strip + 0] = rho_acc;
        a.part[2 * strip + 1] = tau_acc;
    }
}

// iso: Q_{k-1}[pixel] = sum over planes of a_{k-1} z^_{k-1}, z^ = 2 rho D r^_k - a^_k;
// per (plane group, row) partial sums, reduced by k_iso_reduce.
struct BwdIsoArgs {
    const cf* sin;       // r^_k row spectra
    const float* abx_in; // a^_k (k < K)
    const float* aby_in;
    const float* apx;    // a_{k-1}
    const float* apy;
    const float* rho;
    float* partial;      // [ngroups][2][H][W]
    const cf* twW;
    int P, H, ppg;
    long long nitems;
    long long ppm;       // planes per module
};

template <int N, bool LASTK>
__global__ void __launch_bounds__(256) k_bwd_iso_q(BwdIsoArgs a) {
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
    const float rho = a.rho[(long long)grp * a.ppg / a.ppm];
    cf qx[E], qy[E];
#pragma unroll
    for (int j = 0; j < E; ++j) qx[j] = qy[j] = mkc(0.f, 0.f);
    const int p1 = min(a.P, (grp + 1) * a.ppg);
    for (int p = grp * a.ppg; p < p1; ++p) {
        const cf* sp = a.sin + (size_t)p * H * N;
        cf rp[E], rc[E];
#pragma unroll
        for (int j = 0; j < E; ++j) {
            rp[j] = sp[(size_t)gm * N + t + L * j];
            rc[j] = sp[(size_t)g * N + t + L * j];
        }
        RowXf<N>::c2r(rp, buf, tw, t);
        RowXf<N>::c2r(rc, buf, tw, t);
        const size_t ro = (size_t)p * H * N + (size_t)g * N;
        const cf* abx = reinterpret_cast<const cf*>(a.abx_in);
        const cf* aby = reinterpret_cast<const cf*>(a.aby_in);
        const cf* apx = reinterpret_cast<const cf*>(a.apx);
        const cf* apy = reinterpret_cast<const cf*>(a.apy);
        cf sh[E];
#pragma unroll
        for (int j = 0; j < E; ++j) sh[j].x = __shfl(rc[j].y, (t - 1) & (L - 1), L);
#pragma unroll
        for (int j = 0; j < E; ++j) {
            const float rl = (t == 0) ? sh[(j - 1) & (E - 1)].x : sh[j].x;
            const cf ubx = LASTK ? mkc(0.f, 0.f) : abx[ro + t + L * j];
            const cf uby = LASTK ? mkc(0.f, 0.f) : aby[ro + t + L * j];
            const cf ax = apx[ro + t + L * j], ay = apy[ro + t + L * j];
            const float zx0 = 2.f * rho * (rc[j].x - rl) - ubx.x, zx1 = 2.f * rho * (rc[j].y - rc[j].x) - ubx.y;
            const float zy0 = 2.f * rho * (rc[j].x - rp[j].x) - uby.x, zy1 = 2.f * rho * (rc[j].y - rp[j].y) - uby.y;
            qx[j].x = fmaf(ax.x, zx0, qx[j].x);
            qx[j].y = fmaf(ax.y, zx1, qx[j].y);
            qy[j].x = fmaf(ay.x, zy0, qy[j].x);
            qy[j].y = fmaf(ay.y, zy1, qy[j].y);
        }
    }
    cf* px = reinterpret_cast<cf*>(a.partial + ((size_t)grp * 2 + 0) * H * W) + (size_t)g * N;
    cf* py = reinterpret_cast<cf*>(a.partial + ((size_t)grp * 2 + 1) * H * W) + (size_t)g * N;
#pragma unroll
    for (int j = 0; j < E; ++j) {
        px[t + L * j] = qx[j];
        py[t + L * j] = qy[j];
    }
}

// iso tau^: sum over pixels of -Q / (s + eps) where f > 0 (dz/dtau = -a / (s + eps));
// one partial per block, fixed order.
template <class T = float>
__global__ void k_iso_tau_partial(const T* __restrict__ q, const T* __restrict__ n, const T* __restrict__ lam,
                                  const T* __restrict__ rho, double* __restrict__ part, long long count) {
    __shared__ double red[256];
    const T tau = lam[0] / rho[0];
    double acc = 0.0;  // fp64 from the first term (each term is the solve's precision)
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < count;
         i += (long long)gridDim.x * blockDim.x) {
        const T s = sqrt(n[i] + eps15<T>()), d = s + eps15<T>();
        if (T(1) - tau / d > T(0)) acc += (double)(-q[i] / d);
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

// per-iteration sums of one module's partials, in place: block `it` sums the module's strips
// [soff, soff + spm) of iteration it (and its tau^ partials, iso) in a fixed order and writes the two
// sums over its first strip's pair, which k_bwd_scalars (spm = 1, no tpart) then adds up over the
// iterations.  (One block over all K x spm pairs took 1.1 ms at the C5 shape.)
static __global__ void k_bwd_iter_sums(double* __restrict__ part, long long nstrips, long long spm, long long soff,
                                       const double* __restrict__ tpart, int ntp, int G, int g) {
    __shared__ double r1[256], r2[256];
    const int it = blockIdx.x;
    double* pp = part + ((size_t)it * nstrips + soff) * 2;
    double sr = 0.0, st = 0.0;
    for (long long i = threadIdx.x; i < spm; i += blockDim.x) {
        sr += pp[2 * i + 0];
        st += pp[2 * i + 1];
    }
    if (tpart) {
        const double* tp = tpart + ((size_t)it * G + g) * ntp;
        for (int i = threadIdx.x; i < ntp; i += blockDim.x) st += tp[i];
    }
    r1[threadIdx.x] = sr;
    r2[threadIdx.x] = st;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            r1[threadIdx.x] += r1[threadIdx.x + o];
            r2[threadIdx.x] += r2[threadIdx.x + o];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        pp[0] = r1[0];
        pp[1] = r2[0];
    }
}

// iso, fused-path backward: Q = sum of the plane-group partials (k_iso_reduce) and, in the same pass,
// this block's tau^ partial of k_iso_tau_partial (-Q / (s + eps) where the shrink is active) -- one launch
// and no re-read of Q and N.  tpart[blockIdx.x]; the launch has (n4 + 255) / 256 blocks = ntp.
static __global__ void k_iso_reduce_tau(const float4* __restrict__ partial, float4* __restrict__ q, int ngroups,
                                        long long n4, const float4* __restrict__ n, const float* __restrict__ lam,
                                        const float* __restrict__ rho, double* __restrict__ tpart) {
    __shared__ double red[256];
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    double acc = 0.0;
    if (i < n4) {
        float4 s = partial[i];
        for (int g = 1; g < ngroups; ++g) {
            const float4 v = partial[(size_t)g * n4 + i];
            s.x += v.x;
            s.y += v.y;
            s.z += v.z;
            s.w += v.w;
        }
        q[i] = s;
        const float4 nn = n[i];
        const float tau = lam[0] / rho[0];
        auto term = [&](float qv, float nv) {
            const float sq = sqrtf(nv + eps15<float>()), d = sq + eps15<float>();
            if (1.f - tau / d > 0.f) acc += (double)(-qv / d);
        };
        term(s.x, nn.x);
        term(s.y, nn.y);
        term(s.z, nn.z);
        term(s.w, nn.w);
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) tpart[blockIdx.x] = red[0];
}

// final scalars of one module: tau^ = sum of its partials, rho^ = sum + tau^ * (-lam / rho^2),
// lam^ = tau^ / rho.  part: [K][nstrips][2], the module's strips at [soff, soff + spm) of every
// iteration; tpart (iso, or null): [K][G][ntp].  Single block, fixed order -> deterministic.
template <class T = float>
__global__ void k_bwd_scalars(const double* __restrict__ part, int K, long long nstrips, long long spm, long long soff,
                              const double* __restrict__ tpart, int ntp, int G, int g, const T* __restrict__ lam,
                              const T* __restrict__ rho, T* __restrict__ glam, T* __restrict__ grho) {
    __shared__ double r1[256], r2[256];
    double sr = 0.0, st = 0.0;
    for (int it = 0; it < K; ++it) {
        const double* pp = part + ((size_t)it * nstrips + soff) * 2;
        for (long long i = threadIdx.x; i < spm; i += blockDim.x) {
            sr += pp[2 * i + 0];
            st += pp[2 * i + 1];
        }
        if (tpart) {
            const double* tp = tpart + ((size_t)it * G + g) * ntp;
            for (int i = threadIdx.x; i < ntp; i += blockDim.x) st += tp[i];
        }
    }
    r1[threadIdx.x] = sr;
    r2[threadIdx.x] = st;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            r1[threadIdx.x] += r1[threadIdx.x + o];
            r2[threadIdx.x] += r2[threadIdx.x + o];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const double l = lam[0], r = rho[0];
        const double tb = r2[0];
        glam[0] = (T)(tb / r);
        grho[0] = (T)(r1[0] - tb * l / (r * r));
    }
}

// sum of the modules' b^ images: out[i] = sum_g in[g n + i] (fixed order)
static __global__ void k_sum_modules(const float4* __restrict__ in, float4* __restrict__ out, int G, long long n4) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n4) return;
    float4 s = in[i];
    for (int g = 1; g < G; ++g) {
        const float4 q = in[(size_t)g * n4 + i];
        s.x += q.x;
        s.y += q.y;
        s.z += q.z;
        s.w += q.w;
    }
    out[i] = s;
}

}  // namespace admm

namespace admm {

// ---------------------------------------------------------------------------
// PSF gradient.  The PSF k enters through b = H_t(xin) (centred circular
// convolution, anchor c) and through s2 = |sigma|^2 in the Wiener factor.  With G = K^T K
// (spectrum s2), dM = -M dG M, so dL = -sum_k <r^_k, dG x_k>; in Fourier (half plane,
// c(kx) = 2 for 0 < kx < N else 1):
//   dL/ds2(f)  = -(1/HW) c(kx) sum_k sum_p fc(f)^2 Re(conj(X^_k(f)) R_k(f))
//   kbar2[a,b] = sum_f dL/ds2(f) 2 Re(conj(sigma(f)) exp(-2 pi i (a ky/H + b kx/W)))
//   kbar1[a,b] = (1/HW) sum_f c(kx) Re(Z(f) exp(-2 pi i (ky (a-c)/H + kx (b-c)/W))),
//                Z(f) = sum_p conj(Bbar_p(f)) Xin_p(f)
// k_xspec forms sum_p conj(colFFT(U_p)) colFFT(V_p) per frequency from two sets of row
// spectra, plane-group partials, with the packed column 0 split into kx = 0 and kx = N.
// ---------------------------------------------------------------------------
template <int H, int C, bool COL0>
__global__ void __launch_bounds__(C * (H / RowCfg<H>::E), 1)
    k_xspec(const cf* __restrict__ U, const cf* __restrict__ V, cf* __restrict__ part, const cf* __restrict__ twH_g,
            int N, int colblocks, int P, int ppg) {
    using G = ColGeom<H, C>;
    constexpr int E = G::E, L = G::L;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    cf* tw = reinterpret_cast<cf*>(smem);
    cf* data = tw + H;
    load_tw(tw, twH_g, H);
    const int tid = threadIdx.x;
    const int c = tid % C, t = tid / C;
    const int ncb = COL0 ? 1 : colblocks - 1;
    const int grp = blockIdx.x / ncb;
    const int cb = COL0 ? 0 : 1 + (int)(blockIdx.x % ncb);
    const int col = cb * C + c;
    ColBuf<C> buf{data + c};
    cf acc[E], accn[COL0 ? E : 1];
#pragma unroll
    for (int j = 0; j < E; ++j) acc[j] = mkc(0.f, 0.f);
    if constexpr (COL0) {
#pragma unroll
        for (int j = 0; j < E; ++j) accn[j] = mkc(0.f, 0.f);
    }
    __syncthreads();
    const int p1 = min(P, (grp + 1) * ppg);
    for (int p = grp * ppg; p < p1; ++p) {
        const cf* up = U + (size_t)p * H * N + col;
        const cf* vp = V + (size_t)p * H * N + col;
        cf u[E], v[E];
#pragma unroll
        for (int j = 0; j < E; ++j) u[j] = up[(size_t)(t + L * j) * N];
#pragma unroll
        for (int j = 0; j < E; ++j) v[j] = vp[(size_t)(t + L * j) * N];
        __syncthreads();  // previous plane's LDS reads are done
        fft<H, L, -1, 1, 1>(u, buf, tw, t);
        __syncthreads();
        fft<H, L, -1, 1, 1>(v, buf, tw, t);
        if constexpr (COL0) {
            // split the packed (DC, Nyquist) column: A = (F + conj F~)/2, B = (F - conj F~)/(2i)
            cf ua[E], ub[E];
            __syncthreads();
#pragma unroll
            for (int j = 0; j < E; ++j) buf.at(t + L * j) = u[j];
            __syncthreads();
#pragma unroll
            for (int j = 0; j < E; ++j) {
                const cf q = cconj(buf.at((H - (t + L * j)) & (H - 1)));
                ua[j] = mkc(0.5f * (u[j].x + q.x), 0.5f * (u[j].y + q.y));
                ub[j] = mkc(0.5f * (u[j].y - q.y), -0.5f * (u[j].x - q.x));
            }
            __syncthreads();
#pragma unroll
            for (int j = 0; j < E; ++j) buf.at(t + L * j) = v[j];
            __syncthreads();
#pragma unroll
            for (int j = 0; j < E; ++j) {
                const cf q = cconj(buf.at((H - (t + L * j)) & (H - 1)));
                const cf va = mkc(0.5f * (v[j].x + q.x), 0.5f * (v[j].y + q.y));
                const cf vb = mkc(0.5f * (v[j].y - q.y), -0.5f * (v[j].x - q.x));
                if (col == 0) {
                    acc[j] = cadd(acc[j], cmulc(va, ua[j]));    // conj(uA) vA
                    accn[j] = cadd(accn[j], cmulc(vb, ub[j]));  // conj(uB) vB
                } else {
                    acc[j] = cadd(acc[j], cmulc(v[j], u[j]));
                }
            }
        } else {
#pragma unroll
            for (int j = 0; j < E; ++j) acc[j] = cadd(acc[j], cmulc(v[j], u[j]));
        }
    }
    cf* out = part + (size_t)grp * (N + 1) * H;
#pragma unroll
    for (int j = 0; j < E; ++j) out[(size_t)col * H + t + L * j] = acc[j];
    if constexpr (COL0) {
        if (col == 0) {
#pragma unroll
            for (int j = 0; j < E; ++j) out[(size_t)N * H + t + L * j] = accn[j];
        }
    }
}

// acc[f] += sum_g part[g][f] * (fcT ? fcT[f]^2 real part : complex), in fp64 (f over (N+1)*H)
static __global__ void k_xspec_reduce(const cf* __restrict__ part, int ngroups, long long nf, const float* __restrict__ fcT,
                               double2* __restrict__ acc) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nf) return;
    double re = 0.0, im = 0.0;
    for (int g = 0; g < ngroups; ++g) {
        const cf v = part[(size_t)g * nf + i];
        re += v.x;
        im += v.y;
    }
    if (fcT) {
        const double f = fcT[i];
        acc[i].x += f * f * re;  // only Re(conj(X^) R) enters dL/ds2
    } else {
        acc[i].x += re;
        acc[i].y += im;
    }
}

// kbar[a][b] (one block per tap) from A (fc^2-weighted, scaled sums), Z (scaled) and sigma.
// Scalings: fast path -- row spectra carry a factor 2, fc is stored / (2HW):
//   A_true = (HW)^2 A,  Z_true = Z / 4  (zscale 0.25);
// generic path -- plain rfft spectra, fc stored / (HW): A_true = (HW)^2 A, Z_true = Z (zscale 1).
template <class T = float>
__global__ void k_psf_grad(const double2* __restrict__ A, const double2* __restrict__ Z,
                           const double2* __restrict__ sigma, int k, int H, int W, T* __restrict__ gk,
                           double zscale) {
    __shared__ double red[256];
    const int tap = blockIdx.x;
    const int a = tap / k, b = tap % k, c = k / 2;
    const int N = W / 2;
    const double HW = (double)H * W;
    const long long nf = (long long)(N + 1) * H;
    double acc = 0.0;
    for (long long i = threadIdx.x; i < nf; i += blockDim.x) {
        const int kx = (int)(i / H), ky = (int)(i % H);
        const double cw = (kx == 0 || 2 * kx == W) ? 1.0 : 2.0;  // self-conjugate columns once
        double s, co;
        // through fc: dL/ds2 * 2 Re(conj(sigma) e^{-2 pi i (a ky/H + b kx/W)})
        const long long ph2 = ((long long)a * ky % H) * W + ((long long)b * kx % W) * H;  // units 1/(HW)
        sincospi(2.0 * (double)(ph2 % (long long)HW) / HW, &s, &co);  // e^{-i t} = co - i s
        const double2 sg = sigma[i];
        const double dls2 = -HW * cw * A[i].x;
        acc += dls2 * 2.0 * (sg.x * co - sg.y * s);  // Re(conj(sg) (co - i s)) = sg.x co - sg.y s
        // through b = H_t(xin): (1/HW) c Re(Z_true e^{-2 pi i (ky (a-c)/H + kx (b-c)/W)})
        long long ph1 = ((long long)(a - c) * ky) % H;
        if (ph1 < 0) ph1 += H;
        long long ph1x = ((long long)(b - c) * kx) % W;
        if (ph1x < 0) ph1x += W;
        const long long p1 = (ph1 * W + ph1x * H) % (long long)HW;
        sincospi(2.0 * (double)p1 / HW, &s, &co);
        const double2 z = Z[i];
        acc += cw / HW * zscale * (z.x * co + z.y * s);  // Re((zx + i zy)(co - i s))
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) gk[tap] = (T)red[0];
}

}  // namespace admm

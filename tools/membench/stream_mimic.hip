// Memory-system ceiling for pass A's access pattern (no FFT work): each wave walks a strip of
// R rows of P planes x H x W floats, per row reading 4 row streams (spectrum, u_x, u_y, b) and
// writing 3 (u_x, u_y, spectrum out), 8-byte accesses in the kernels' natural layout
// (lane t, register j -> element t + 64 j).  Variants change only the stream structure.
//   hipcc -O3 --offload-arch=gfx950 -o stream_mimic stream_mimic.hip && ./stream_mimic
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

typedef float2 cf;
constexpr int W = 1024, N = 512, E = 8, L = 64;

// 4 reads + 3 writes per row, pass A's layout
template <class T> __device__ __forceinline__ void st(T* p, T v, bool nt) {
    typedef float V __attribute__((ext_vector_type(sizeof(T) / 4)));
    if (nt) __builtin_nontemporal_store(__builtin_bit_cast(V, v), reinterpret_cast<V*>(p)); else *p = v;
}

template <class T> __device__ __forceinline__ T ld(const T* p, bool nt) {
    typedef float V __attribute__((ext_vector_type(sizeof(T) / 4)));
    if (nt) return __builtin_bit_cast(T, __builtin_nontemporal_load(reinterpret_cast<const V*>(p)));
    return *p;
}

template <int R, bool NT = false, bool NTL = false>
__global__ void __launch_bounds__(256) k_mimic(const cf* __restrict__ sp, const cf* __restrict__ uxi,
                                               const cf* __restrict__ uyi, const cf* __restrict__ b,
                                               cf* __restrict__ uxo, cf* __restrict__ uyo, cf* __restrict__ so,
                                               int H, long long nstrips) {
    const int t = threadIdx.x % L;
    const long long strip = (long long)blockIdx.x * 4 + threadIdx.x / L;
    if (strip >= nstrips) return;
    const int spp = H / R;
    const long long p = strip / spp;
    const int i0 = (int)(strip % spp) * R;
    const size_t base = (size_t)p * H * N;
    cf acc[E];
    for (int j = 0; j < E; ++j) acc[j] = ld(&sp[base + (size_t)((i0 - 1 + H) & (H - 1)) * N + t + L * j], NTL);
    for (int rr = 0; rr <= R; ++rr) {
        const size_t ro = base + (size_t)((i0 + rr) & (H - 1)) * N;
        const size_t rm = base + (size_t)((i0 + rr - 1 + H) & (H - 1)) * N;
        cf x[E], uy[E];
        for (int j = 0; j < E; ++j) x[j] = ld(&sp[ro + t + L * j], NTL);
        for (int j = 0; j < E; ++j) { uy[j] = ld(&uyi[ro + t + L * j], NTL); uy[j].x += x[j].x; uy[j].y += acc[j].y; }
        if (rr < R) for (int j = 0; j < E; ++j) st(&uyo[ro + t + L * j], uy[j], NT);
        if (rr >= 1) {
            for (int j = 0; j < E; ++j) { cf bb = ld(&b[rm + t + L * j], NTL); acc[j].x += bb.x; acc[j].y -= bb.y; }
            for (int j = 0; j < E; ++j) st(&so[rm + t + L * j], acc[j], NT);
        }
        if (rr < R) {
            for (int j = 0; j < E; ++j) { cf u = ld(&uxi[ro + t + L * j], NTL); u.x -= x[j].y; u.y += x[j].x; st(&uxo[ro + t + L * j], u, NT); }
        }
        for (int j = 0; j < E; ++j) acc[j] = x[j];
    }
}

// strip-walking with only 1 read + 1 write stream (isolates the walk from the stream count)
template <int R>
__global__ void __launch_bounds__(256) k_walk11(const cf* __restrict__ sp, cf* __restrict__ so, int H, long long nstrips) {
    const int t = threadIdx.x % L;
    const long long strip = (long long)blockIdx.x * 4 + threadIdx.x / L;
    if (strip >= nstrips) return;
    const int spp = H / R;
    const long long p = strip / spp;
    const int i0 = (int)(strip % spp) * R;
    const size_t base = (size_t)p * H * N;
    for (int rr = 0; rr < R; ++rr) {
        const size_t ro = base + (size_t)(i0 + rr) * N;
        cf x[E];
        for (int j = 0; j < E; ++j) x[j] = sp[ro + t + L * j];
        for (int j = 0; j < E; ++j) { x[j].x *= 1.0001f; so[ro + t + L * j] = x[j]; }
    }
}

// walk variants: MODE 0 contiguous strips (pass A's mapping), 1 row-interleaved (wave w takes
// rows w, w + S, w + 2S ... so concurrent waves touch adjacent rows), 2 consecutive waves in
// different planes
template <int R, int MODE>
__global__ void __launch_bounds__(256) k_walkv(const cf* __restrict__ sp, cf* __restrict__ so, int H, long long nstrips,
                                               int P) {
    const int t = threadIdx.x % L;
    const long long w = (long long)blockIdx.x * 4 + threadIdx.x / L;
    if (w >= nstrips) return;
    for (int rr = 0; rr < R; ++rr) {
        size_t ro;
        if (MODE == 0) {
            ro = (size_t)(w * R + rr) * N;
        } else if (MODE == 1) {
            ro = (size_t)(rr * nstrips + w) * N;
        } else {
            const long long spp = H / R;
            const long long p = w % P, s = w / P;
            ro = ((size_t)p * H + s * R + rr) * N;
        }
        cf x[E];
        for (int j = 0; j < E; ++j) x[j] = sp[ro + t + L * j];
        for (int j = 0; j < E; ++j) { x[j].x *= 1.0001f; so[ro + t + L * j] = x[j]; }
    }
}

// 4R+3W, two rows per step (twice the bytes in flight per wave)
template <int R>
__global__ void __launch_bounds__(256) k_mimic2(const cf* __restrict__ sp, const cf* __restrict__ uxi,
                                                const cf* __restrict__ uyi, const cf* __restrict__ b,
                                                cf* __restrict__ uxo, cf* __restrict__ uyo, cf* __restrict__ so,
                                                int H, long long nstrips) {
    const int t = threadIdx.x % L;
    const long long strip = (long long)blockIdx.x * 4 + threadIdx.x / L;
    if (strip >= nstrips) return;
    const int spp = H / R;
    const long long p = strip / spp;
    const int i0 = (int)(strip % spp) * R;
    const size_t base = (size_t)p * H * N;
    for (int rr = 0; rr < R; rr += 2) {
        const size_t r0 = base + (size_t)(i0 + rr) * N, r1 = r0 + N;
        cf x0[E], x1[E], a0[E], a1[E], c0[E], c1[E], d0[E], d1[E];
        for (int j = 0; j < E; ++j) { x0[j] = sp[r0 + t + L * j]; x1[j] = sp[r1 + t + L * j]; }
        for (int j = 0; j < E; ++j) { a0[j] = uxi[r0 + t + L * j]; a1[j] = uxi[r1 + t + L * j]; }
        for (int j = 0; j < E; ++j) { c0[j] = uyi[r0 + t + L * j]; c1[j] = uyi[r1 + t + L * j]; }
        for (int j = 0; j < E; ++j) { d0[j] = b[r0 + t + L * j]; d1[j] = b[r1 + t + L * j]; }
        for (int j = 0; j < E; ++j) {
            uxo[r0 + t + L * j] = make_float2(a0[j].x + x0[j].x, a0[j].y); uxo[r1 + t + L * j] = make_float2(a1[j].x + x1[j].x, a1[j].y);
            uyo[r0 + t + L * j] = make_float2(c0[j].x - x0[j].y, c0[j].y); uyo[r1 + t + L * j] = make_float2(c1[j].x - x1[j].y, c1[j].y);
            so[r0 + t + L * j] = make_float2(d0[j].x * x0[j].x, d0[j].y); so[r1 + t + L * j] = make_float2(d1[j].x * x1[j].x, d1[j].y);
        }
    }
}

// pass A's 4R+3W walk over a row-permuted layout: logical row i of a plane is stored at
// position (i % R) * (H / R) + i / R, so at each step the waves of one plane touch adjacent rows
template <int R>
__global__ void __launch_bounds__(256) k_mimic_perm(const cf* __restrict__ sp, const cf* __restrict__ uxi,
                                                    const cf* __restrict__ uyi, const cf* __restrict__ b,
                                                    cf* __restrict__ uxo, cf* __restrict__ uyo, cf* __restrict__ so,
                                                    int H, long long nstrips) {
    const int t = threadIdx.x % L;
    const long long strip = (long long)blockIdx.x * 4 + threadIdx.x / L;
    if (strip >= nstrips) return;
    const int spp = H / R;
    const long long p = strip / spp;
    const int i0 = (int)(strip % spp) * R;
    const size_t base = (size_t)p * H * N;
    auto prow = [&](int i) { i &= (H - 1); return (size_t)((i % R) * spp + i / R) * N; };
    cf acc[E];
    for (int j = 0; j < E; ++j) acc[j] = sp[base + prow(i0 - 1) + t + L * j];
    for (int rr = 0; rr <= R; ++rr) {
        const size_t ro = base + prow(i0 + rr);
        const size_t rm = base + prow(i0 + rr - 1);
        cf x[E], uy[E];
        for (int j = 0; j < E; ++j) x[j] = sp[ro + t + L * j];
        for (int j = 0; j < E; ++j) { uy[j] = uyi[ro + t + L * j]; uy[j].x += x[j].x; uy[j].y += acc[j].y; }
        if (rr < R) for (int j = 0; j < E; ++j) uyo[ro + t + L * j] = uy[j];
        if (rr >= 1) {
            for (int j = 0; j < E; ++j) { cf bb = b[rm + t + L * j]; acc[j].x += bb.x; acc[j].y -= bb.y; }
            for (int j = 0; j < E; ++j) so[rm + t + L * j] = acc[j];
        }
        if (rr < R) {
            for (int j = 0; j < E; ++j) { cf u = uxi[ro + t + L * j]; u.x -= x[j].y; u.y += x[j].x; uxo[ro + t + L * j] = u; }
        }
        for (int j = 0; j < E; ++j) acc[j] = x[j];
    }
}

// pass B's access over the permuted layout: column block, logical row r at stored row perm(r)
template <int C, int TPB, int R>
__global__ void __launch_bounds__(TPB) k_colmimic_perm(cf* __restrict__ spec, int H, int colblocks) {
    constexpr int L = TPB / C;
    const int c = threadIdx.x % C, t = threadIdx.x / C;
    const int p = blockIdx.x / colblocks, cb = blockIdx.x % colblocks;
    cf* base = spec + (size_t)p * H * N + cb * C + c;
    const int E = H / L, spp = H / R;
    cf v[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) if (j < E) { const int r = t + L * j; v[j] = base[(size_t)((r % R) * spp + r / R) * N]; }
#pragma unroll
    for (int j = 0; j < 32; ++j) if (j < E) { const int r = t + L * j; v[j].x *= 1.0001f; base[(size_t)((r % R) * spp + r / R) * N] = v[j]; }
}

// row records: per row {spectrum, u_x, u_y} contiguous (3N cf), ping-pong in/out; b separate
template <int R>
__global__ void __launch_bounds__(256) k_mimic_rec(const cf* __restrict__ ri, const cf* __restrict__ b,
                                                   cf* __restrict__ ro_, int H, long long nstrips) {
    const int t = threadIdx.x % L;
    const long long strip = (long long)blockIdx.x * 4 + threadIdx.x / L;
    if (strip >= nstrips) return;
    const int spp = H / R;
    const long long p = strip / spp;
    const int i0 = (int)(strip % spp) * R;
    const size_t base = (size_t)p * H * N;
    auto rec = [&](int i) { return 3 * (base + (size_t)(i & (H - 1)) * N); };
    cf acc[E];
    for (int j = 0; j < E; ++j) acc[j] = ri[rec(i0 - 1) + t + L * j];
    for (int rr = 0; rr <= R; ++rr) {
        const size_t r0 = rec(i0 + rr), rm = rec(i0 + rr - 1);
        cf x[E], uy[E];
        for (int j = 0; j < E; ++j) x[j] = ri[r0 + t + L * j];
        for (int j = 0; j < E; ++j) { uy[j] = ri[r0 + 2 * N + t + L * j]; uy[j].x += x[j].x; uy[j].y += acc[j].y; }
        if (rr < R) for (int j = 0; j < E; ++j) ro_[r0 + 2 * N + t + L * j] = uy[j];
        if (rr >= 1) {
            const size_t bm = base + (size_t)((i0 + rr - 1) & (H - 1)) * N;
            for (int j = 0; j < E; ++j) { cf bb = b[bm + t + L * j]; acc[j].x += bb.x; acc[j].y -= bb.y; }
            for (int j = 0; j < E; ++j) ro_[rm + t + L * j] = acc[j];
        }
        if (rr < R) {
            for (int j = 0; j < E; ++j) { cf u = ri[r0 + N + t + L * j]; u.x -= x[j].y; u.y += x[j].x; ro_[r0 + N + t + L * j] = u; }
        }
        for (int j = 0; j < E; ++j) acc[j] = x[j];
    }
}

// u_x / u_y interleaved per row ([P][H][2][N] cf): 3 read + 2 write streams
template <int R>
__global__ void __launch_bounds__(256) k_mimic_il(const cf* __restrict__ sp, const cf* __restrict__ ui,
                                                  const cf* __restrict__ b, cf* __restrict__ uo,
                                                  cf* __restrict__ so, int H, long long nstrips) {
    const int t = threadIdx.x % L;
    const long long strip = (long long)blockIdx.x * 4 + threadIdx.x / L;
    if (strip >= nstrips) return;
    const int spp = H / R;
    const long long p = strip / spp;
    const int i0 = (int)(strip % spp) * R;
    const size_t base = (size_t)p * H * N;
    cf acc[E];
    for (int j = 0; j < E; ++j) acc[j] = sp[base + (size_t)((i0 - 1 + H) & (H - 1)) * N + t + L * j];
    for (int rr = 0; rr <= R; ++rr) {
        const size_t ro = base + (size_t)((i0 + rr) & (H - 1)) * N;
        const size_t rm = base + (size_t)((i0 + rr - 1 + H) & (H - 1)) * N;
        cf x[E], uy[E];
        for (int j = 0; j < E; ++j) x[j] = sp[ro + t + L * j];
        for (int j = 0; j < E; ++j) { uy[j] = ui[2 * ro + N + t + L * j]; uy[j].x += x[j].x; uy[j].y += acc[j].y; }
        if (rr < R) for (int j = 0; j < E; ++j) uo[2 * ro + N + t + L * j] = uy[j];
        if (rr >= 1) {
            for (int j = 0; j < E; ++j) { cf bb = b[rm + t + L * j]; acc[j].x += bb.x; acc[j].y -= bb.y; }
            for (int j = 0; j < E; ++j) so[rm + t + L * j] = acc[j];
        }
        if (rr < R) {
            for (int j = 0; j < E; ++j) { cf u = ui[2 * ro + t + L * j]; u.x -= x[j].y; u.y += x[j].x; uo[2 * ro + t + L * j] = u; }
        }
        for (int j = 0; j < E; ++j) acc[j] = x[j];
    }
}

template <bool NT>
__global__ void __launch_bounds__(256) k_copy(const float4* __restrict__ a, float4* __restrict__ o, size_t n) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) st(&o[i], a[i], NT);
}
// one float2 per thread, no loop (many blocks)
template <bool NT>
__global__ void __launch_bounds__(256) k_copy2(const float2* __restrict__ a, float2* __restrict__ o) {
    const size_t i = blockIdx.x * 256ull + threadIdx.x;
    st(&o[i], a[i], NT);
}
__global__ void __launch_bounds__(256) k_read(const float4* __restrict__ a, float* __restrict__ o, size_t n) {
    float s = 0.f;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) { float4 v = a[i]; s += v.x + v.y + v.z + v.w; }
    if (s == 12345.f) o[0] = s;
}

// pass B's access pattern: a block owns C adjacent columns of one plane (all H rows), thread
// (c = tid % C, t = tid / C) moves element (t + L j, c), L = threads / C rows per step.
template <int C, int TPB>
__global__ void __launch_bounds__(TPB) k_colmimic(cf* __restrict__ spec, int H, int colblocks) {
    constexpr int L = TPB / C;
    const int c = threadIdx.x % C, t = threadIdx.x / C;
    const int p = blockIdx.x / colblocks, cb = blockIdx.x % colblocks;
    cf* base = spec + (size_t)p * H * N + cb * C + c;
    const int E = H / L;
    cf v[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) if (j < E) v[j] = base[(size_t)(t + L * j) * N];
#pragma unroll
    for (int j = 0; j < 32; ++j) if (j < E) { v[j].x *= 1.0001f; base[(size_t)(t + L * j) * N] = v[j]; }
}


// column-tiled spectrum layout [P][H/T][N/8][T][8] (u, b stay row-major): offset of (row, col) in cf units
template <int T> __device__ __forceinline__ size_t toff(int row, int col) {
    return ((size_t)(row / T) * (N / 8) + (col >> 3)) * (T * 8) + (row % T) * 8 + (col & 7);
}
// pass A mimic with the spectrum streams (sp in, so out) in the tiled layout
template <int R, int T>
__global__ void __launch_bounds__(256) k_mimic_t(const cf* __restrict__ sp, const cf* __restrict__ uxi,
                                                 const cf* __restrict__ uyi, const cf* __restrict__ b,
                                                 cf* __restrict__ uxo, cf* __restrict__ uyo, cf* __restrict__ so,
                                                 int H, long long nstrips) {
    const int t = threadIdx.x % L;
    const long long strip = (long long)blockIdx.x * 4 + threadIdx.x / L;
    if (strip >= nstrips) return;
    const int spp = H / R;
    const long long p = strip / spp;
    const int i0 = (int)(strip % spp) * R;
    const size_t base = (size_t)p * H * N;
    cf acc[E];
    for (int j = 0; j < E; ++j) acc[j] = sp[base + toff<T>((i0 - 1 + H) & (H - 1), t + L * j)];
    for (int rr = 0; rr <= R; ++rr) {
        const int gi = (i0 + rr) & (H - 1), gm = (i0 + rr - 1 + H) & (H - 1);
        const size_t ro = base + (size_t)gi * N;
        const size_t rm = base + (size_t)gm * N;
        cf x[E], uy[E];
        for (int j = 0; j < E; ++j) x[j] = sp[base + toff<T>(gi, t + L * j)];
        for (int j = 0; j < E; ++j) { uy[j] = uyi[ro + t + L * j]; uy[j].x += x[j].x; uy[j].y += acc[j].y; }
        if (rr < R) for (int j = 0; j < E; ++j) uyo[ro + t + L * j] = uy[j];
        if (rr >= 1) {
            for (int j = 0; j < E; ++j) { cf bb = b[rm + t + L * j]; acc[j].x += bb.x; acc[j].y -= bb.y; }
            for (int j = 0; j < E; ++j) so[base + toff<T>(gm, t + L * j)] = acc[j];
        }
        if (rr < R) {
            for (int j = 0; j < E; ++j) { cf u = uxi[ro + t + L * j]; u.x -= x[j].y; u.y += x[j].x; uxo[ro + t + L * j] = u; }
        }
        for (int j = 0; j < E; ++j) acc[j] = x[j];
    }
}
// pass B mimic on the tiled layout: a block owns 8 adjacent columns (one tile column), all H rows
template <int TPB, int T>
__global__ void __launch_bounds__(TPB) k_colmimic_t(cf* __restrict__ spec, int H, int colblocks) {
    constexpr int C = 8, LL = TPB / C;
    const int c = threadIdx.x % C, t = threadIdx.x / C;
    const int p = blockIdx.x / colblocks, cb = blockIdx.x % colblocks;
    cf* base = spec + (size_t)p * H * N;
    const int EE = H / LL;
    cf v[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) if (j < EE) v[j] = base[toff<T>(t + LL * j, cb * 8 + c)];
#pragma unroll
    for (int j = 0; j < 32; ++j) if (j < EE) { v[j].x *= 1.0001f; base[toff<T>(t + LL * j, cb * 8 + c)] = v[j]; }
}


// --- mixed layouts (round 2): pass A reads the x spectrum row-major and writes the r spectrum
// column-tiled [P][H/T][N/8][T][8]; pass B reads tiled and writes row-major (out of place).
__device__ __forceinline__ unsigned xcd_remap(unsigned b, unsigned nb) {
    const unsigned x = b & 7u, i = b >> 3, q = nb >> 3, r = nb & 7u;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}
template <int R, int T, bool SO_NT = true, bool IN_T = false>
__global__ void __launch_bounds__(256) k_mimic_ot(const cf* __restrict__ sp, const cf* __restrict__ uxi,
                                                  const cf* __restrict__ uyi, const cf* __restrict__ b,
                                                  cf* __restrict__ uxo, cf* __restrict__ uyo, cf* __restrict__ so,
                                                  int H, long long nstrips) {
    const int t = threadIdx.x % L;
    const long long strip = (long long)blockIdx.x * 4 + threadIdx.x / L;
    if (strip >= nstrips) return;
    const int spp = H / R;
    const long long p = strip / spp;
    const int i0 = (int)(strip % spp) * R;
    const size_t base = (size_t)p * H * N;
    cf acc[E];
    {
        const int gp = (i0 - 1 + H) & (H - 1);
        for (int j = 0; j < E; ++j) acc[j] = ld(&sp[base + (IN_T ? toff<T>(gp, t + L * j) : (size_t)gp * N + t + L * j)], !IN_T);
    }
    for (int rr = 0; rr <= R; ++rr) {
        const int gi = (i0 + rr) & (H - 1), gm = (i0 + rr - 1 + H) & (H - 1);
        const size_t ro = base + (size_t)gi * N;
        const size_t rm = base + (size_t)gm * N;
        cf x[E], uy[E];
        for (int j = 0; j < E; ++j) x[j] = ld(&sp[base + (IN_T ? toff<T>(gi, t + L * j) : (size_t)gi * N + t + L * j)], !IN_T);
        for (int j = 0; j < E; ++j) { uy[j] = ld(&uyi[ro + t + L * j], true); uy[j].x += x[j].x; uy[j].y += acc[j].y; }
        if (rr < R) for (int j = 0; j < E; ++j) st(&uyo[ro + t + L * j], uy[j], true);
        if (rr >= 1) {
            for (int j = 0; j < E; ++j) { cf bb = ld(&b[rm + t + L * j], true); acc[j].x += bb.x; acc[j].y -= bb.y; }
            for (int j = 0; j < E; ++j) st(&so[base + toff<T>(gm, t + L * j)], acc[j], SO_NT);
        }
        if (rr < R) {
            for (int j = 0; j < E; ++j) { cf u = ld(&uxi[ro + t + L * j], true); u.x -= x[j].y; u.y += x[j].x; st(&uxo[ro + t + L * j], u, true); }
        }
        for (int j = 0; j < E; ++j) acc[j] = x[j];
    }
}
// pass B: 8 columns x all H rows per block; IN_T / OUT_T: tiled (T) or row-major input / output
template <int TPB, int T, bool IN_T, bool OUT_T, bool REMAP>
__global__ void __launch_bounds__(TPB) k_colmimic_mix(const cf* __restrict__ si, cf* __restrict__ so, int H, int colblocks) {
    constexpr int C = 8, LL = TPB / C;
    const int c = threadIdx.x % C, t = threadIdx.x / C;
    const unsigned lb = REMAP ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
    const int p = lb / colblocks, cb = lb % colblocks;
    const size_t base = (size_t)p * H * N;
    const int EE = H / LL;
    cf v[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) if (j < EE) {
        const int r = t + LL * j, col = cb * 8 + c;
        v[j] = si[base + (IN_T ? toff<T>(r, col) : (size_t)r * N + col)];
    }
#pragma unroll
    for (int j = 0; j < 32; ++j) if (j < EE) {
        const int r = t + LL * j, col = cb * 8 + c;
        v[j].x *= 1.0001f;
        so[base + (OUT_T ? toff<T>(r, col) : (size_t)r * N + col)] = v[j];
    }
}


// pass A mimic with the u_x, u_y, b streams moved as 16-byte accesses (lane t holds pixel pairs
// 2t, 2t+1 + 128 j): half the load/store instructions for those streams
template <int R>
__global__ void __launch_bounds__(256) k_mimic_u4(const cf* __restrict__ sp, const cf* __restrict__ uxi,
                                                  const cf* __restrict__ uyi, const cf* __restrict__ b,
                                                  cf* __restrict__ uxo, cf* __restrict__ uyo, cf* __restrict__ so,
                                                  int H, long long nstrips) {
    const int t = threadIdx.x % L;
    const long long strip = (long long)blockIdx.x * 4 + threadIdx.x / L;
    if (strip >= nstrips) return;
    const int spp = H / R;
    const long long p = strip / spp;
    const int i0 = (int)(strip % spp) * R;
    const size_t base = (size_t)p * H * N;
    typedef float f4 __attribute__((ext_vector_type(4)));
    cf acc[E];
    for (int j = 0; j < E; ++j) acc[j] = ld(&sp[base + (size_t)((i0 - 1 + H) & (H - 1)) * N + t + L * j], true);
    for (int rr = 0; rr <= R; ++rr) {
        const size_t ro = base + (size_t)((i0 + rr) & (H - 1)) * N;
        const size_t rm = base + (size_t)((i0 + rr - 1 + H) & (H - 1)) * N;
        cf x[E];
        for (int j = 0; j < E; ++j) x[j] = ld(&sp[ro + t + L * j], true);
        const f4* uy4 = reinterpret_cast<const f4*>(uyi + ro);
        f4* uyo4 = reinterpret_cast<f4*>(uyo + ro);
        const f4* ux4 = reinterpret_cast<const f4*>(uxi + ro);
        f4* uxo4 = reinterpret_cast<f4*>(uxo + ro);
        const f4* b4 = reinterpret_cast<const f4*>(b + rm);
        for (int j = 0; j < E / 2; ++j) {
            f4 u = __builtin_nontemporal_load(&uy4[t + L * j]);
            u.x += x[2 * j].x; u.y += acc[2 * j].y; u.z += x[2 * j + 1].x; u.w += acc[2 * j + 1].y;
            if (rr < R) __builtin_nontemporal_store(u, &uyo4[t + L * j]);
        }
        if (rr >= 1) {
            for (int j = 0; j < E / 2; ++j) {
                f4 bb = __builtin_nontemporal_load(&b4[t + L * j]);
                acc[2 * j].x += bb.x; acc[2 * j].y -= bb.y; acc[2 * j + 1].x += bb.z; acc[2 * j + 1].y -= bb.w;
            }
            for (int j = 0; j < E; ++j) st(&so[rm + t + L * j], acc[j], true);
        }
        if (rr < R) {
            for (int j = 0; j < E / 2; ++j) {
                f4 u = __builtin_nontemporal_load(&ux4[t + L * j]);
                u.x -= x[2 * j].y; u.y += x[2 * j].x; u.z -= x[2 * j + 1].y; u.w += x[2 * j + 1].x;
                __builtin_nontemporal_store(u, &uxo4[t + L * j]);
            }
        }
        for (int j = 0; j < E; ++j) acc[j] = x[j];
    }
}


// all seven streams of pass A at 16 bytes per lane (spectrum too): lane t holds pairs 2t, 2t+1 + 128 j
template <int R>
__global__ void __launch_bounds__(256) k_mimic_all16(const cf* __restrict__ sp, const cf* __restrict__ uxi,
                                                     const cf* __restrict__ uyi, const cf* __restrict__ b,
                                                     cf* __restrict__ uxo, cf* __restrict__ uyo, cf* __restrict__ so,
                                                     int H, long long nstrips) {
    const int t = threadIdx.x % L;
    const long long strip = (long long)blockIdx.x * 4 + threadIdx.x / L;
    if (strip >= nstrips) return;
    const int spp = H / R;
    const long long p = strip / spp;
    const int i0 = (int)(strip % spp) * R;
    const size_t base = (size_t)p * H * N;
    typedef float f4 __attribute__((ext_vector_type(4)));
    f4 acc[E / 2];
    {
        const f4* s4 = reinterpret_cast<const f4*>(sp + base + (size_t)((i0 - 1 + H) & (H - 1)) * N);
        for (int j = 0; j < E / 2; ++j) acc[j] = __builtin_nontemporal_load(&s4[t + L * j]);
    }
    for (int rr = 0; rr <= R; ++rr) {
        const size_t ro = base + (size_t)((i0 + rr) & (H - 1)) * N;
        const size_t rm = base + (size_t)((i0 + rr - 1 + H) & (H - 1)) * N;
        f4 x[E / 2];
        const f4* s4 = reinterpret_cast<const f4*>(sp + ro);
        for (int j = 0; j < E / 2; ++j) x[j] = __builtin_nontemporal_load(&s4[t + L * j]);
        const f4* uy4 = reinterpret_cast<const f4*>(uyi + ro);
        f4* uyo4 = reinterpret_cast<f4*>(uyo + ro);
        const f4* ux4 = reinterpret_cast<const f4*>(uxi + ro);
        f4* uxo4 = reinterpret_cast<f4*>(uxo + ro);
        const f4* b4 = reinterpret_cast<const f4*>(b + rm);
        f4* so4 = reinterpret_cast<f4*>(so + rm);
        for (int j = 0; j < E / 2; ++j) {
            f4 u = __builtin_nontemporal_load(&uy4[t + L * j]);
            u += x[j] - acc[j];
            if (rr < R) __builtin_nontemporal_store(u, &uyo4[t + L * j]);
        }
        if (rr >= 1) {
            for (int j = 0; j < E / 2; ++j) {
                f4 bb = __builtin_nontemporal_load(&b4[t + L * j]);
                acc[j] += bb;
                __builtin_nontemporal_store(acc[j], &so4[t + L * j]);
            }
        }
        if (rr < R) {
            for (int j = 0; j < E / 2; ++j) {
                f4 u = __builtin_nontemporal_load(&ux4[t + L * j]);
                u -= x[j];
                __builtin_nontemporal_store(u, &uxo4[t + L * j]);
            }
        }
        for (int j = 0; j < E / 2; ++j) acc[j] = x[j];
    }
}

// column-strip spectrum layout [P][N/S][H][S] (S columns per strip, full height; u and b row-major):
// pass A's row reads are N/S pieces of 8S bytes, pass B's column blocks read contiguous strips
template <int S> __device__ __forceinline__ size_t soff(int H, int row, int col) {
    return ((size_t)(col / S) * H + row) * S + (col % S);
}
template <int R, int S>
__global__ void __launch_bounds__(256) k_mimic_s(const cf* __restrict__ sp, const cf* __restrict__ uxi,
                                                 const cf* __restrict__ uyi, const cf* __restrict__ b,
                                                 cf* __restrict__ uxo, cf* __restrict__ uyo, cf* __restrict__ so,
                                                 int H, long long nstrips) {
    const int t = threadIdx.x % L;
    const long long strip = (long long)blockIdx.x * 4 + threadIdx.x / L;
    if (strip >= nstrips) return;
    const int spp = H / R;
    const long long p = strip / spp;
    const int i0 = (int)(strip % spp) * R;
    const size_t base = (size_t)p * H * N;
    cf acc[E];
    for (int j = 0; j < E; ++j) acc[j] = ld(&sp[base + soff<S>(H, (i0 - 1 + H) & (H - 1), t + L * j)], true);
    for (int rr = 0; rr <= R; ++rr) {
        const int gi = (i0 + rr) & (H - 1), gm = (i0 + rr - 1 + H) & (H - 1);
        const size_t ro = base + (size_t)gi * N;
        const size_t rm = base + (size_t)gm * N;
        cf x[E], uy[E];
        for (int j = 0; j < E; ++j) x[j] = ld(&sp[base + soff<S>(H, gi, t + L * j)], true);
        for (int j = 0; j < E; ++j) { uy[j] = ld(&uyi[ro + t + L * j], true); uy[j].x += x[j].x; uy[j].y += acc[j].y; }
        if (rr < R) for (int j = 0; j < E; ++j) st(&uyo[ro + t + L * j], uy[j], true);
        if (rr >= 1) {
            for (int j = 0; j < E; ++j) { cf bb = ld(&b[rm + t + L * j], true); acc[j].x += bb.x; acc[j].y -= bb.y; }
            for (int j = 0; j < E; ++j) st(&so[base + soff<S>(H, gm, t + L * j)], acc[j], true);
        }
        if (rr < R) {
            for (int j = 0; j < E; ++j) { cf u = ld(&uxi[ro + t + L * j], true); u.x -= x[j].y; u.y += x[j].x; st(&uxo[ro + t + L * j], u, true); }
        }
        for (int j = 0; j < E; ++j) acc[j] = x[j];
    }
}
// pass B on the strip layout: C columns x all H rows per block (C <= S), in place, optional XCD remap
template <int C, int TPB, int S, bool REMAP>
__global__ void __launch_bounds__(TPB) k_colmimic_s(cf* __restrict__ spec, int H, int colblocks) {
    constexpr int LL = TPB / C;
    const int c = threadIdx.x % C, t = threadIdx.x / C;
    const unsigned lb = REMAP ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
    const int p = lb / colblocks, cb = lb % colblocks;
    cf* base = spec + (size_t)p * H * N;
    const int EE = H / LL;
    cf v[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) if (j < EE) v[j] = base[soff<S>(H, t + LL * j, cb * C + c)];
#pragma unroll
    for (int j = 0; j < 32; ++j) if (j < EE) { v[j].x *= 1.0001f; base[soff<S>(H, t + LL * j, cb * C + c)] = v[j]; }
}

int main() {
    const int P = 192, H = 1024;
    const size_t n = (size_t)P * H * N;  // cf per array
    std::vector<cf*> buf(8);
    for (auto& p : buf) { CK(hipMalloc(&p, n * sizeof(cf))); CK(hipMemset(p, 0, n * sizeof(cf))); }
    cf *ui, *uo;
    CK(hipMalloc(&ui, 2 * n * sizeof(cf))); CK(hipMalloc(&uo, 2 * n * sizeof(cf)));
    CK(hipMemset(ui, 0, 2 * n * sizeof(cf)));
    cf *reci, *reco;
    CK(hipMalloc(&reci, 3 * n * sizeof(cf))); CK(hipMalloc(&reco, 3 * n * sizeof(cf)));
    CK(hipMemset(reci, 0, 3 * n * sizeof(cf)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, double bytes, auto launch) {
        for (int i = 0; i < 3; ++i) launch();
        hipEventRecord(e0);
        const int reps = 20;
        for (int i = 0; i < reps; ++i) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        ms /= reps;
        printf("%-40s %8.4f ms  %7.0f GB/s\n", name, ms, bytes / (ms * 1e-3) / 1e9);
    };
    const double arr = (double)n * sizeof(cf);
    if (getenv("STRIP_SWEEP")) {
        const long long ns = (long long)P * H / 8;
        const int cb8 = N / 8;
        for (int rep = 0; rep < 3; ++rep) {
            timeit("A row-major nt (prod) R=8", 7 * arr, [&] { k_mimic<8, true, true><<<(unsigned)((ns + 3) / 4), 256>>>(buf[0], buf[1], buf[2], buf[3], buf[4], buf[5], buf[6], H, ns); });
            timeit("A strips S=16 nt R=8", 7 * arr, [&] { k_mimic_s<8, 16><<<(unsigned)((ns + 3) / 4), 256>>>(buf[0], buf[1], buf[2], buf[3], buf[4], buf[5], buf[6], H, ns); });
            timeit("A strips S=32 nt R=8", 7 * arr, [&] { k_mimic_s<8, 32><<<(unsigned)((ns + 3) / 4), 256>>>(buf[0], buf[1], buf[2], buf[3], buf[4], buf[5], buf[6], H, ns); });
            timeit("A strips S=64 nt R=8", 7 * arr, [&] { k_mimic_s<8, 64><<<(unsigned)((ns + 3) / 4), 256>>>(buf[0], buf[1], buf[2], buf[3], buf[4], buf[5], buf[6], H, ns); });
            timeit("B row-major C=8 remap (prod)", 2 * arr, [&] { k_colmimic_mix<512, 8, false, false, true><<<(unsigned)(P * cb8), 512>>>(buf[6], buf[6], H, cb8); });
            timeit("B strips16 C=8 remap", 2 * arr, [&] { k_colmimic_s<8, 512, 16, true><<<(unsigned)(P * cb8), 512>>>(buf[6], H, cb8); });
            timeit("B strips16 C=8 noremap", 2 * arr, [&] { k_colmimic_s<8, 512, 16, false><<<(unsigned)(P * cb8), 512>>>(buf[6], H, cb8); });
            timeit("B strips32 C=8 remap", 2 * arr, [&] { k_colmimic_s<8, 512, 32, true><<<(unsigned)(P * cb8), 512>>>(buf[6], H, cb8); });
            timeit("B strips64 C=8 remap", 2 * arr, [&] { k_colmimic_s<8, 512, 64, true><<<(unsigned)(P * cb8), 512>>>(buf[6], H, cb8); });
            timeit("B strips16 C=16 1024thr remap", 2 * arr, [&] { k_colmimic_s<16, 1024, 16, true><<<(unsigned)(P * cb8 / 2), 1024>>>(buf[6], H, cb8 / 2); });
            timeit("copy float4", 2 * arr, [&] { k_copy<false><<<16384, 256>>>((const float4*)buf[0], (float4*)buf[1], arr / 16); });
        }
        return 0;
    }
    if (getenv("U4_SWEEP")) {
        const long long ns = (long long)P * H / 8;
        for (int rep = 0; rep < 3; ++rep) {
            timeit("A row-major nt (prod) R=8", 7 * arr, [&] { k_mimic<8, true, true><<<(unsigned)((ns + 3) / 4), 256>>>(buf[0], buf[1], buf[2], buf[3], buf[4], buf[5], buf[6], H, ns); });
            timeit("A u/b streams 16 B/lane R=8", 7 * arr, [&] { k_mimic_u4<8><<<(unsigned)((ns + 3) / 4), 256>>>(buf[0], buf[1], buf[2], buf[3], buf[4], buf[5], buf[6], H, ns); });
            timeit("A all streams 16 B/lane R=8", 7 * arr, [&] { k_mimic_all16<8><<<(unsigned)((ns + 3) / 4), 256>>>(buf[0], buf[1], buf[2], buf[3], buf[4], buf[5], buf[6], H, ns); });
        }
        return 0;
    }
    if (getenv("MIXED_SWEEP3")) {  // T = 2 row-pair tiles: pass B reads whole 128-B lines
        const long long ns = (long long)P * H / 8;
        const int colblocks = N / 8;
        const int reps = getenv("ONCE") ? 1 : 3;
        for (int rep = 0; rep < reps; ++rep) {
            timeit("A row-major nt (prod) R=8", 7 * arr, [&] { k_mimic<8, true, true><<<(unsigned)((ns + 3) / 4), 256>>>(buf[0], buf[1], buf[2], buf[3], buf[4], buf[5], buf[6], H, ns); });
            timeit("A out-tiled T=2 nt st", 7 * arr, [&] { k_mimic_ot<8, 2, true><<<(unsigned)((ns + 3) / 4), 256>>>(buf[0], buf[1], buf[2], buf[3], buf[4], buf[5], buf[6], H, ns); });
            timeit("A out-tiled T=2 plain st", 7 * arr, [&] { k_mimic_ot<8, 2, false><<<(unsigned)((ns + 3) / 4), 256>>>(buf[0], buf[1], buf[2], buf[3], buf[4], buf[5], buf[6], H, ns); });
            timeit("B row->row remap in place (prod)", 2 * arr, [&] { k_colmimic_mix<512, 8, false, false, true><<<(unsigned)(P * colblocks), 512>>>(buf[6], buf[6], H, colblocks); });
            timeit("B tiled2->row remap oop", 2 * arr, [&] { k_colmimic_mix<512, 2, true, false, true><<<(unsigned)(P * colblocks), 512>>>(buf[6], buf[0], H, colblocks); });
            timeit("B tiled2->tiled2 remap in place", 2 * arr, [&] { k_colmimic_mix<512, 2, true, true, true><<<(unsigned)(P * colblocks), 512>>>(buf[6], buf[6], H, colblocks); });
            timeit("B row->row remap oop", 2 * arr, [&] { k_colmimic_mix<512, 8, false, false, true><<<(unsigned)(P * colblocks), 512>>>(buf[6], buf[0], H, colblocks); });
        }
        return 0;
    }
    if (getenv("STAGGER_SWEEP")) {
        // pass A's 7 streams carved from one allocation with a stagger between arrays: do the
        // same (plane, row) offsets of different arrays collide in HBM channels when the arrays
        // start at multiples of 768 MiB?
        const long long ns = (long long)P * H / 8;
        const size_t stg_max = 1 << 20;
        char* big;
        CK(hipMalloc(&big, 7 * ((size_t)arr + stg_max) + 4096));
        CK(hipMemset(big, 0, 7 * ((size_t)arr + stg_max) + 4096));
        const size_t strides[] = {0, 256, 2048, 4096 + 256, 16384 + 512, 65536 + 4096, 262144 + 8192, 1048576};
        for (int rep = 0; rep < 2; ++rep)
            for (size_t sg : strides) {
                cf* a[7];
                for (int i = 0; i < 7; ++i) a[i] = reinterpret_cast<cf*>(big + (size_t)i * ((size_t)arr + sg));
                char name[64];
                snprintf(name, sizeof name, "A nt stagger %zu B", sg);
                timeit(name, 7 * arr, [&] { k_mimic<8, true, true><<<(unsigned)((ns + 3) / 4), 256>>>(a[0], a[1], a[2], a[3], a[4], a[5], a[6], H, ns); });
                snprintf(name, sizeof name, "B remap in place stagger %zu B", sg);
                timeit(name, 2 * arr, [&] { k_colmimic_mix<512, 8, false, false, true><<<(unsigned)(P * (N / 8)), 512>>>(a[6], a[6], H, N / 8); });
            }
        return 0;
    }
    if (getenv("MIXED_SWEEP2")) {
        const long long ns = (long long)P * H / 8;
        const int colblocks = N / 8;
        for (int rep = 0; rep < 3; ++rep) {
            timeit("A row-major nt (prod) R=8", 7 * arr, [&] { k_mimic<8, true, true><<<(unsigned)((ns + 3) / 4), 256>>>(buf[0], buf[1], buf[2], buf[3], buf[4], buf[5], buf[6], H, ns); });
            timeit("A out-tiled T=8 plain st", 7 * arr, [&] { k_mimic_ot<8, 8, false><<<(unsigned)((ns + 3) / 4), 256>>>(buf[0], buf[1], buf[2], buf[3], buf[4], buf[5], buf[6], H, ns); });
            timeit("A in+out tiled T=8 nt st", 7 * arr, [&] { k_mimic_ot<8, 8, true, true><<<(unsigned)((ns + 3) / 4), 256>>>(buf[0], buf[1], buf[2], buf[3], buf[4], buf[5], buf[6], H, ns); });
            timeit("A in+out tiled T=8 plain st", 7 * arr, [&] { k_mimic_ot<8, 8, false, true><<<(unsigned)((ns + 3) / 4), 256>>>(buf[0], buf[1], buf[2], buf[3], buf[4], buf[5], buf[6], H, ns); });
            timeit("A in-tiled T=8 only", 7 * arr, [&] { k_mimic_ot<8, 8, true, true><<<(unsigned)((ns + 3) / 4), 256>>>(buf[0], buf[1], buf[2], buf[3], buf[4], buf[5], buf[6], H, ns); });
            timeit("B row->row remap in place", 2 * arr, [&] { k_colmimic_mix<512, 8, false, false, true><<<(unsigned)(P * colblocks), 512>>>(buf[0], buf[0], H, colblocks); });
            timeit("B row->row remap oop", 2 * arr, [&] { k_colmimic_mix<512, 8, false, false, true><<<(unsigned)(P * colblocks), 512>>>(buf[6], buf[0], H, colblocks); });
            timeit("B row->row noremap in place", 2 * arr, [&] { k_colmimic_mix<512, 8, false, false, false><<<(unsigned)(P * colblocks), 512>>>(buf[0], buf[0], H, colblocks); });
            timeit("B tiled->tiled remap in place", 2 * arr, [&] { k_colmimic_mix<512, 8, true, true, true><<<(unsigned)(P * colblocks), 512>>>(buf[0], buf[0], H, colblocks); });
            timeit("B C=16 1024thr row in place", 2 * arr, [&] { k_colmimic<16, 1024><<<(unsigned)(P * colblocks / 2), 1024>>>(buf[0], H, colblocks / 2); });
            timeit("copy float4", 2 * arr, [&] { k_copy<false><<<16384, 256>>>((const float4*)buf[0], (float4*)buf[1], arr / 16); });
            timeit("copy float2 1/thread nt", 2 * arr, [&] { k_copy2<true><<<(unsigned)(n / 256), 256>>>((const float2*)buf[0], (float2*)buf[1]); });
        }
        return 0;
    }
    if (getenv("MIXED_SWEEP")) {
        const long long ns = (long long)P * H / 8;
        const int colblocks = N / 8;
        for (int rep = 0; rep < 3; ++rep) {
            timeit("A row-major nt (prod) R=8", 7 * arr, [&] { k_mimic<8, true, true><<<(unsigned)((ns + 3) / 4), 256>>>(buf[0], buf[1], buf[2], buf[3], buf[4], buf[5], buf[6], H, ns); });
            timeit("A out-tiled T=8 R=8", 7 * arr, [&] { k_mimic_ot<8, 8><<<(unsigned)((ns + 3) / 4), 256>>>(buf[0], buf[1], buf[2], buf[3], buf[4], buf[5], buf[6], H, ns); });
            timeit("A out-tiled T=16 R=8", 7 * arr, [&] { k_mimic_ot<8, 16><<<(unsigned)((ns + 3) / 4), 256>>>(buf[0], buf[1], buf[2], buf[3], buf[4], buf[5], buf[6], H, ns); });
            timeit("A out-tiled T=4 R=8", 7 * arr, [&] { k_mimic_ot<8, 4><<<(unsigned)((ns + 3) / 4), 256>>>(buf[0], buf[1], buf[2], buf[3], buf[4], buf[5], buf[6], H, ns); });
            timeit("B row->row remap (prod, oop)", 2 * arr, [&] { k_colmimic_mix<512, 8, false, false, true><<<(unsigned)(P * colblocks), 512>>>(buf[6], buf[0], H, colblocks); });
            timeit("B tiled8->row remap", 2 * arr, [&] { k_colmimic_mix<512, 8, true, false, true><<<(unsigned)(P * colblocks), 512>>>(buf[6], buf[0], H, colblocks); });
            timeit("B tiled8->row noremap", 2 * arr, [&] { k_colmimic_mix<512, 8, true, false, false><<<(unsigned)(P * colblocks), 512>>>(buf[6], buf[0], H, colblocks); });
            timeit("B tiled16->row remap", 2 * arr, [&] { k_colmimic_mix<512, 16, true, false, true><<<(unsigned)(P * colblocks), 512>>>(buf[6], buf[0], H, colblocks); });
            timeit("B tiled4->row remap", 2 * arr, [&] { k_colmimic_mix<512, 4, true, false, true><<<(unsigned)(P * colblocks), 512>>>(buf[6], buf[0], H, colblocks); });
            timeit("B tiled8->tiled8 remap", 2 * arr, [&] { k_colmimic_mix<512, 8, true, true, true><<<(unsigned)(P * colblocks), 512>>>(buf[6], buf[0], H, colblocks); });
            timeit("copy float4", 2 * arr, [&] { k_copy<false><<<16384, 256>>>((const float4*)buf[0], (float4*)buf[1], arr / 16); });
        }
        return 0;
    }
    if (getenv("TILE_SWEEP")) {
        const long long ns = (long long)P * H / 8;
        for (int rep = 0; rep < 2; ++rep) {
            timeit("A row-major 4R+3W R=8", 7 * arr, [&] { k_mimic<8><<<(unsigned)((ns + 3) / 4), 256>>>(buf[0], buf[1], buf[2], buf[3], buf[4], buf[5], buf[6], H, ns); });
            timeit("A tiled T=8 4R+3W R=8", 7 * arr, [&] { k_mimic_t<8, 8><<<(unsigned)((ns + 3) / 4), 256>>>(buf[0], buf[1], buf[2], buf[3], buf[4], buf[5], buf[6], H, ns); });
            timeit("A tiled T=16 4R+3W R=8", 7 * arr, [&] { k_mimic_t<8, 16><<<(unsigned)((ns + 3) / 4), 256>>>(buf[0], buf[1], buf[2], buf[3], buf[4], buf[5], buf[6], H, ns); });
            timeit("A tiled T=4 4R+3W R=8", 7 * arr, [&] { k_mimic_t<8, 4><<<(unsigned)((ns + 3) / 4), 256>>>(buf[0], buf[1], buf[2], buf[3], buf[4], buf[5], buf[6], H, ns); });
            timeit("A tiled T=2 4R+3W R=8", 7 * arr, [&] { k_mimic_t<8, 2><<<(unsigned)((ns + 3) / 4), 256>>>(buf[0], buf[1], buf[2], buf[3], buf[4], buf[5], buf[6], H, ns); });
            const int colblocks = N / 8;
            timeit("B row-major C=8 512thr", 2 * arr, [&] { k_colmimic<8, 512><<<(unsigned)(P * colblocks), 512>>>(buf[0], H, colblocks); });
            timeit("B row-major C=16 1024thr", 2 * arr, [&] { k_colmimic<16, 1024><<<(unsigned)(P * colblocks / 2), 1024>>>(buf[0], H, colblocks / 2); });
            timeit("B tiled T=8 C=8 512thr", 2 * arr, [&] { k_colmimic_t<512, 8><<<(unsigned)(P * colblocks), 512>>>(buf[0], H, colblocks); });
            timeit("B tiled T=16 C=8 512thr", 2 * arr, [&] { k_colmimic_t<512, 16><<<(unsigned)(P * colblocks), 512>>>(buf[0], H, colblocks); });
            timeit("B tiled T=4 C=8 512thr", 2 * arr, [&] { k_colmimic_t<512, 4><<<(unsigned)(P * colblocks), 512>>>(buf[0], H, colblocks); });
            timeit("B tiled T=2 C=8 512thr", 2 * arr, [&] { k_colmimic_t<512, 2><<<(unsigned)(P * colblocks), 512>>>(buf[0], H, colblocks); });
            timeit("copy float4", 2 * arr, [&] { k_copy<false><<<16384, 256>>>((const float4*)buf[0], (float4*)buf[1], arr / 16); });
        }
        return 0;
    }
    if (getenv("MALL_SWEEP")) {
        // one ADMM iteration's traffic pattern (pass A mimic + pass B mimic, ping-ponged spectrum and u)
        // run ITERS times on a chunk of Pc planes before moving to the next chunk: does a chunk
        // whose working set fits the 256 MiB Infinity Cache stream faster than HBM?
        const int ITERS = 50;
        const int chunks[] = {1, 2, 3, 4, 6, 8, 12, 16, 24, 48, 192};
        for (int rep = 0; rep < 2; ++rep)
        for (int Pc : chunks) {
            const size_t pn = (size_t)H * N;  // cf per plane
            auto run = [&] {
                for (int p0 = 0; p0 < P; p0 += Pc) {
                    const int pc = (P - p0 < Pc) ? P - p0 : Pc;
                    const size_t off = (size_t)p0 * pn;
                    const long long ns = (long long)pc * H / 8;
                    for (int it = 0; it < ITERS; ++it) {
                        cf* si = buf[it & 1 ? 6 : 0] + off; cf* so = buf[it & 1 ? 0 : 6] + off;
                        cf* xi = buf[it & 1 ? 4 : 1] + off; cf* xo = buf[it & 1 ? 1 : 4] + off;
                        cf* yi = buf[it & 1 ? 5 : 2] + off; cf* yo = buf[it & 1 ? 2 : 5] + off;
                        k_mimic<8><<<(unsigned)((ns + 3) / 4), 256>>>(si, xi, yi, buf[3] + off, xo, yo, so, H, ns);
                        k_colmimic<8, 512><<<(unsigned)(pc * (N / 8)), 512>>>(so, H, N / 8);
                    }
                }
            };
            run();
            hipEventRecord(e0);
            run();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            const double bytes = 9.0 * arr * ITERS;  // 36 B/px per iteration = 9 cf-arrays of 8 B per 2 px
            printf("chunk %3d planes (%6.1f MiB live): %8.2f ms for %d it  -> %6.0f GB/s algorithmic, %6.1f it/s\n",
                   Pc, Pc * pn * sizeof(cf) * 7 / 1048576.0, ms, ITERS, bytes / (ms * 1e-3) / 1e9, ITERS / (ms * 1e-3));
        }
        return 0;
    }
    if (getenv("NT_ONLY")) {  // cache-policy ceilings of pass A's pattern
        const long long ns = (long long)P * H / 8;
        auto m = [&](auto kern, const char* name) {
            timeit(name, 7 * arr, [&] { kern<<<(unsigned)((ns + 3) / 4), 256>>>(buf[0], buf[1], buf[2], buf[3], buf[4], buf[5], buf[6], H, ns); });
        };
        for (int rep = 0; rep < 2; ++rep) {
            timeit("copy float2 1/thread", 2 * arr, [&] { k_copy2<false><<<(unsigned)(n / 256), 256>>>((const float2*)buf[0], (float2*)buf[1]); });
            timeit("copy float2 1/thread nt", 2 * arr, [&] { k_copy2<true><<<(unsigned)(n / 256), 256>>>((const float2*)buf[0], (float2*)buf[1]); });
            m(k_mimic<8, false, false>, "mimic R=8 plain");
            m(k_mimic<8, true, false>, "mimic R=8 nt stores");
            m(k_mimic<8, true, true>, "mimic R=8 nt stores + loads");
        }
        return 0;
    }
    if (getenv("AB_ONLY")) {
        const long long ns = (long long)P * H / 8;
        for (int rep = 0; rep < 4; ++rep) {
            timeit("A  separate u 4R+3W R=8", 7 * arr, [&] { k_mimic<8><<<(unsigned)((ns + 3) / 4), 256>>>(buf[0], buf[1], buf[2], buf[3], buf[4], buf[5], buf[6], H, ns); });
            timeit("B  interleaved u 3R+2W R=8", 7 * arr, [&] { k_mimic_il<8><<<(unsigned)((ns + 3) / 4), 256>>>(buf[0], ui, buf[3], uo, buf[6], H, ns); });
            timeit("C  row records 2R+1W R=8", 7 * arr, [&] { k_mimic_rec<8><<<(unsigned)((ns + 3) / 4), 256>>>(reci, buf[3], reco, H, ns); });
            timeit("D  interleaved u R=4", 7 * arr, [&] { k_mimic_il<4><<<(unsigned)((2 * ns + 3) / 4), 256>>>(buf[0], ui, buf[3], uo, buf[6], H, 2 * ns); });
        }
        return 0;
    }
    timeit("copy 1R+1W (float4, grid-stride 4096 blk)", 2 * arr, [&] { k_copy<false><<<4096, 256>>>((const float4*)buf[0], (float4*)buf[1], arr / 16); });
    timeit("copy nt-store (float4, 4096 blk)", 2 * arr, [&] { k_copy<true><<<4096, 256>>>((const float4*)buf[0], (float4*)buf[1], arr / 16); });
    timeit("copy (float4, 16384 blk)", 2 * arr, [&] { k_copy<false><<<16384, 256>>>((const float4*)buf[0], (float4*)buf[1], arr / 16); });
    timeit("copy float2 1/thread", 2 * arr, [&] { k_copy2<false><<<(unsigned)(n / 256), 256>>>((const float2*)buf[0], (float2*)buf[1]); });
    timeit("copy float2 1/thread nt", 2 * arr, [&] { k_copy2<true><<<(unsigned)(n / 256), 256>>>((const float2*)buf[0], (float2*)buf[1]); });
    timeit("read only (float4)", arr, [&] { k_read<<<4096, 256>>>((const float4*)buf[0], (float*)buf[7], arr / 16); });
    auto mimic = [&](auto kern, int R, const char* name) {
        const long long ns = (long long)P * H / R;
        const double bytes = 7 * arr;  // algorithmic: 4 reads + 3 writes
        timeit(name, bytes, [&] { kern<<<(unsigned)((ns + 3) / 4), 256>>>(buf[0], buf[1], buf[2], buf[3], buf[4], buf[5], buf[6], H, ns); });
    };
    mimic(k_mimic<8>, 8, "mimic 4R+3W R=8");
    mimic(k_mimic<16>, 16, "mimic 4R+3W R=16");
    mimic(k_mimic<4>, 4, "mimic 4R+3W R=4");
    mimic(k_mimic<8, true>, 8, "mimic 4R+3W R=8 nt stores");
    mimic(k_mimic2<8>, 8, "mimic2 4R+3W R=8, 2 rows/step");
    mimic(k_mimic_perm<8>, 8, "mimic PERMUTED 4R+3W R=8");
    mimic(k_mimic_perm<16>, 16, "mimic PERMUTED 4R+3W R=16");
    mimic(k_mimic_perm<4>, 4, "mimic PERMUTED 4R+3W R=4");
    mimic(k_mimic<8>, 8, "mimic 4R+3W R=8 (again)");
    {
        const long long ns = (long long)P * H / 8;
        timeit("walk 1R+1W R=8", 2 * arr, [&] { k_walk11<8><<<(unsigned)((ns + 3) / 4), 256>>>(buf[0], buf[1], H, ns); });
        timeit("walkv contiguous R=8", 2 * arr, [&] { k_walkv<8, 0><<<(unsigned)((ns + 3) / 4), 256>>>(buf[0], buf[1], H, ns, P); });
        timeit("walkv row-interleaved R=8", 2 * arr, [&] { k_walkv<8, 1><<<(unsigned)((ns + 3) / 4), 256>>>(buf[0], buf[1], H, ns, P); });
        timeit("walkv plane-interleaved R=8", 2 * arr, [&] { k_walkv<8, 2><<<(unsigned)((ns + 3) / 4), 256>>>(buf[0], buf[1], H, ns, P); });
        const long long n1 = (long long)P * H;
        timeit("walkv R=1", 2 * arr, [&] { k_walkv<1, 0><<<(unsigned)((n1 + 3) / 4), 256>>>(buf[0], buf[1], H, n1, P); });
        const long long n32 = (long long)P * H / 32;
        timeit("walkv contiguous R=32", 2 * arr, [&] { k_walkv<32, 0><<<(unsigned)((n32 + 3) / 4), 256>>>(buf[0], buf[1], H, n32, P); });
    }
    mimic(k_mimic<4, true>, 4, "mimic 4R+3W R=4 nt stores");
    auto colm = [&](auto kern, int C, int tpb, const char* name) {
        const int colblocks = N / C;
        timeit(name, 2 * arr, [&] { kern<<<(unsigned)(P * colblocks), tpb>>>(buf[0], H, colblocks); });
    };
    colm(k_colmimic<8, 512>, 8, 512, "colmimic C=8  512 thr (E=16)");
    colm(k_colmimic<16, 1024>, 16, 1024, "colmimic C=16 1024 thr (E=16)");
    colm(k_colmimic<16, 512>, 16, 512, "colmimic C=16 512 thr (E=32)");
    colm(k_colmimic<32, 1024>, 32, 1024, "colmimic C=32 1024 thr (E=32)");
    colm(k_colmimic<8, 256>, 8, 256, "colmimic C=8  256 thr (E=32)");
    colm(k_colmimic_perm<8, 512, 8>, 8, 512, "colmimic PERMUTED C=8 512 thr");
    colm(k_colmimic<8, 512>, 8, 512, "colmimic C=8  512 thr (again)");
    {
        const long long ns = (long long)P * H / 8;
        timeit("mimic interleaved u 3R+2W R=8", 7 * arr, [&] { k_mimic_il<8><<<(unsigned)((ns + 3) / 4), 256>>>(buf[0], ui, buf[3], uo, buf[6], H, ns); });
    }
    return 0;
}

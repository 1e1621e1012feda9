// plane_stats.hip -- median and mode over whole planes (16-bit types): the C ABI of the
// admm_planestat_* entry points in include/admm_chanstat.h.  Replaces the reference's
// ChannelWiseAttention statistics amedian / amodes (/root/reference/src/admmtor/elayers/cwa.py:
// 8-27: x.view(B, C, -1).median(-1) / .mode(-1)), which PyTorch runs per slice through thrust
// sorts (thousands of launches per config-5 step).
//
// One workgroup (1024 threads) per plane of N elements:
//  * k_plane_hist: 16-bit order-preserving codes counted in an LDS histogram, one half of the
//    code space per pass (32768 x u32 = 128 KB); gives the median's code and its rank within its
//    run of equal values, and the mode (smallest most frequent code).
//  * k_plane_median_idx: the r-th occurrence of the median's code in flat order (torch.median's
//    stable rank), by block-wide prefix counts over steps of 8192 elements.
//  * k_plane_mode_idx: the index torch.mode (CPU) reports is where libstdc++ std::sort leaves the
//    last element of the mode's run.  Only the rightmost partition range still holding a
//    mode-valued element matters, and only while it holds two or more (ranges keep their order,
//    the final insertion sort is stable), so the kernel replays the partitions along that one
//    path: each Hoare partition as four passes over the range (stop counts, stop ranks and the
//    swap count S, swapped elements into slots, swapped positions updated in place).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "admm_chanstat.h"
#include "admm_tv.h"

namespace {

constexpr int NT = 1024;  // threads per workgroup (16 waves)
constexpr int NW = NT / 64;
constexpr int KR = 8;      // elements per thread per block-scan step of the partition replay

__device__ __forceinline__ uint32_t ord16_bf16(uint32_t u) {
    if ((u & 0x7F80u) == 0x7F80u && (u & 0x7Fu)) return 0xFFFFu;  // NaN above +inf
    if ((u & 0x7FFFu) == 0) u = 0;                                // -0 == +0
    return (u & 0x8000u) ? (~u & 0xFFFFu) : (u | 0x8000u);
}
__device__ __forceinline__ uint32_t ord16_f16(uint32_t u) {
    if ((u & 0x7C00u) == 0x7C00u && (u & 0x3FFu)) return 0xFFFFu;
    if ((u & 0x7FFFu) == 0) u = 0;
    return (u & 0x8000u) ? (~u & 0xFFFFu) : (u | 0x8000u);
}
__device__ __forceinline__ uint32_t ord32_f32(uint32_t u) {
    if ((u & 0x7FFFFFFFu) > 0x7F800000u) return 0xFFFFFFFFu;
    if ((u & 0x7FFFFFFFu) == 0) u = 0;
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
template <int DT> struct Elem { using type = uint16_t; };
template <> struct Elem<ADMM_CHANSTAT_F32> { using type = uint32_t; };
template <int DT> __device__ __forceinline__ uint32_t code_of(typename Elem<DT>::type raw) {
    if constexpr (DT == ADMM_CHANSTAT_F32) return ord32_f32(raw);
    else if constexpr (DT == ADMM_CHANSTAT_BF16) return ord16_bf16(raw);
    else return ord16_f16(raw);
}

// block-wide exclusive prefix sums of two per-thread counts (thread order); row totals.  Two
// barriers; `sh` holds 2 * NW ints.
__device__ __forceinline__ void block_scan2(int a, int b, int* sh, int& ea, int& eb, int& ta, int& tb) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int ia = a, ib = b;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int ua = __shfl_up(ia, o), ub = __shfl_up(ib, o);
        if (lane >= o) {
            ia += ua;
            ib += ub;
        }
    }
    if (lane == 63) {
        sh[w] = ia;
        sh[NW + w] = ib;
    }
    __syncthreads();
    int oa = 0, ob = 0;
    ta = 0;
    tb = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        const int ca = sh[i], cb = sh[NW + i];
        if (i < w) {
            oa += ca;
            ob += cb;
        }
        ta += ca;
        tb += cb;
    }
    __syncthreads();
    ea = oa + ia - a;
    eb = ob + ib - b;
}

__device__ __forceinline__ int block_sum(int v, int* sh) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (lane == 0) sh[w] = v;
    __syncthreads();
    int t = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) t += sh[i];
    __syncthreads();
    return t;
}

struct PlaneStat {
    int mode_code, mode_count, med_code, med_r;
};

// ------------------------------------------------------------------------------- histogram
template <int DT>
__global__ void __launch_bounds__(NT) k_plane_hist(const uint16_t* __restrict__ x, long long N,
                                                  PlaneStat* __restrict__ st) {
    extern __shared__ __align__(16) unsigned char smem[];
    uint32_t* hist = reinterpret_cast<uint32_t*>(smem);  // [32768]
    __shared__ int sh_i[2 * NW];
    __shared__ unsigned long long sh_best;
    __shared__ int sh_nan;
    const int t = threadIdx.x;
    const uint16_t* xp = x + (size_t)blockIdx.x * N;
    const long long mpos = (N - 1) >> 1;
    long long below = 0;                    // elements in lower halves already counted
    int best_code = 0, best_count = 0;      // mode so far (ties keep the smaller code)
    int med_code = -1, med_r = 0;
    if (t == 0) sh_best = 0;
    for (int half = 0; half < 2; ++half) {
        for (int i = t; i < 32768; i += NT) hist[i] = 0u;
        __syncthreads();
#pragma unroll 8
        for (long long i = t; i < N; i += NT) {
            const uint32_t c = code_of<DT>(xp[i]);
            if ((int)(c >> 15) == half) atomicAdd(&hist[c & 0x7FFFu], 1u);
        }
        __syncthreads();
        // each thread owns 32 consecutive bins
        const int b0 = t * 32;
        uint32_t sum = 0, mx = 0;
        int mxb = 0;
#pragma unroll 8
        for (int i = 0; i < 32; ++i) {
            const uint32_t h = hist[b0 + i];
            sum += h;
            if (h > mx) {
                mx = h;
                mxb = b0 + i;
            }
        }
        // mode: the largest count, the smallest code among equal counts (64-bit key)
        const unsigned long long key = ((unsigned long long)mx << 32) | (0xFFFFFFFFu - (uint32_t)mxb);
        atomicMax(&sh_best, key);
        // median: exclusive prefix of the per-thread sums (sequential over waves via shared)
        int rs, tot;
        {
            // prefix over threads: in-wave inclusive scan then wave offsets
            uint32_t v = sum;
            const int lane = t & 63, w = t >> 6;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t u = (uint32_t)__shfl_up((int)v, o);
                if (lane >= o) v += u;
            }
            if (lane == 63) sh_i[w] = (int)v;
            __syncthreads();
            int off = 0;
            tot = 0;
#pragma unroll
            for (int i = 0; i < NW; ++i) {
                if (i < w) off += sh_i[i];
                tot += sh_i[i];
            }
            __syncthreads();
            rs = off + (int)v - (int)sum;  // exclusive
        }
        if (half == 1 && t == NT - 1) sh_nan = (int)hist[0x7FFF];  // code 0xFFFF: NaN
        const long long lo = below + rs, hi = lo + sum;
        if (med_code < 0 && mpos >= lo && mpos < hi) {  // exactly one thread of the block
            long long acc = lo;
            for (int i = 0; i < 32; ++i) {
                const uint32_t h = hist[b0 + i];
                if (mpos < acc + h) {
                    sh_i[0] = (half << 15) | (b0 + i);
                    sh_i[1] = (int)(mpos - acc);
                    break;
                }
                acc += h;
            }
        }
        __syncthreads();
        if (med_code < 0 && mpos >= below && mpos < below + tot) {
            med_code = sh_i[0];
            med_r = sh_i[1];
        }
        const unsigned long long kb = sh_best;
        const int cnt = (int)(kb >> 32), code = (half << 15) | (int)(0xFFFFFFFFu - (uint32_t)kb);
        if (cnt > best_count) {  // strictly more: a lower half's mode keeps ties
            best_count = cnt;
            best_code = code;
        }
        below += tot;
        __syncthreads();
        if (t == 0) sh_best = 0;
        __syncthreads();
    }
    if (sh_nan > 0) {  // torch.median: a plane holding NaN gives its first NaN
        med_code = 0xFFFF;
        med_r = 0;
    }
    if (t == 0) st[blockIdx.x] = PlaneStat{best_code, best_count, med_code, med_r};
}

// ---------------------------------------------------------------- fp32 median (radix select)
// Rank `target` among the 16-bit keys (c >> shift) & 0xFFFF of the codes c of a plane (only
// codes whose high half equals `hi` when `filter`): LDS histogram, half the key space per
// pass, the second half skipped once the target is found.  Returns the key and the target's
// rank among the elements with that key.
__device__ void hist_rank16(const uint32_t* __restrict__ xp, long long N, int shift, bool filter, uint32_t hi,
                            long long target, uint32_t* hist, int* sh_i, int* sh_nan, int& key, int& rank) {
    const int t = threadIdx.x;
    long long below = 0;
    for (int half = 0; half < 2; ++half) {
        for (int i = t; i < 32768; i += NT) hist[i] = 0u;
        __syncthreads();
        bool nan = false;
#pragma unroll 8
        for (long long i = t; i < N; i += NT) {
            const uint32_t c = ord32_f32(xp[i]);
            const uint32_t k = (c >> shift) & 0xFFFFu;
            nan |= c == 0xFFFFFFFFu;
            if ((!filter || (c >> 16) == hi) && (int)(k >> 15) == half) atomicAdd(&hist[k & 0x7FFFu], 1u);
        }
        if (nan) *sh_nan = 1;
        __syncthreads();
        const int b0 = t * 32;
        uint32_t sum = 0;
#pragma unroll 8
        for (int i = 0; i < 32; ++i) sum += hist[b0 + i];
        uint32_t v = sum;
        const int lane = t & 63, w = t >> 6;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t u = (uint32_t)__shfl_up((int)v, o);
            if (lane >= o) v += u;
        }
        if (lane == 63) sh_i[w] = (int)v;
        __syncthreads();
        long long off = 0, tot = 0;
#pragma unroll
        for (int i = 0; i < NW; ++i) {
            if (i < w) off += sh_i[i];
            tot += sh_i[i];
        }
        __syncthreads();
        const long long lo = below + off + (long long)v - sum;
        if (target >= lo && target < lo + sum) {  // exactly one thread of the block
            long long acc = lo;
            for (int i = 0; i < 32; ++i) {
                const uint32_t h = hist[b0 + i];
                if (target < acc + h) {
                    sh_i[0] = (half << 15) | (b0 + i);
                    sh_i[1] = (int)(target - acc);
                    break;
                }
                acc += h;
            }
        }
        __syncthreads();
        if (target < below + tot) {  // uniform
            key = sh_i[0];
            rank = sh_i[1];
            __syncthreads();
            return;
        }
        below += tot;
    }
    key = 0xFFFF;  // not reached: target < N
    rank = 0;
}

// {median code, rank in its run} of each fp32 plane: the high 16 bits of the median's code by
// one histogram pass, the low 16 bits by a second over the elements of that high key
__global__ void __launch_bounds__(NT) k_plane_median32(const uint32_t* __restrict__ x, long long N,
                                                      PlaneStat* __restrict__ st) {
    extern __shared__ __align__(16) unsigned char smem[];
    uint32_t* hist = reinterpret_cast<uint32_t*>(smem);  // [32768]
    __shared__ int sh_i[2 * NW];
    __shared__ int sh_nan;
    const int t = threadIdx.x;
    const uint32_t* xp = x + (size_t)blockIdx.x * N;
    if (t == 0) sh_nan = 0;
    __syncthreads();
    const long long mpos = (N - 1) >> 1;
    int khi, rhi, klo = 0, rlo = 0;
    hist_rank16(xp, N, 16, false, 0u, mpos, hist, sh_i, &sh_nan, khi, rhi);
    int code, r;
    if (sh_nan) {  // torch.median: a plane holding NaN gives its first NaN (uniform branch)
        code = (int)0xFFFFFFFFu;
        r = 0;
    } else {
        hist_rank16(xp, N, 0, true, (uint32_t)khi, rhi, hist, sh_i, &sh_nan, klo, rlo);
        code = (int)(((uint32_t)khi << 16) | (uint32_t)klo);
        r = rlo;
    }
    if (t == 0) st[blockIdx.x] = PlaneStat{0, 0, code, r};
}

// --------------------------------------------------------------------------- median index
template <int DT>
__global__ void __launch_bounds__(NT) k_plane_median_idx(const typename Elem<DT>::type* __restrict__ x, long long N,
                                                        const PlaneStat* __restrict__ st, int64_t* __restrict__ idx) {
    __shared__ int sh[2 * NW];
    __shared__ long long found;
    const int t = threadIdx.x;
    const typename Elem<DT>::type* xp = x + (size_t)blockIdx.x * N;
    const uint32_t mc = (uint32_t)st[blockIdx.x].med_code;
    int r = st[blockIdx.x].med_r;
    if (t == 0) found = -1;
    __syncthreads();
    for (long long base = 0; base < N; base += (long long)NT * KR) {
        const long long i0 = base + (long long)t * KR;
        bool f[KR];
        int n = 0;
#pragma unroll
        for (int j = 0; j < KR; ++j) {
            f[j] = i0 + j < N && code_of<DT>(xp[i0 + j]) == mc;
            n += f[j] ? 1 : 0;
        }
        int ex, d0, tot, d1;
        block_scan2(n, 0, sh, ex, d0, tot, d1);
        if (r >= ex && r < ex + n) {  // this thread holds the r-th occurrence
            int k = r - ex;
#pragma unroll
            for (int j = 0; j < KR; ++j) {
                if (f[j]) {
                    if (k == 0) found = i0 + j;
                    --k;
                }
            }
        }
        r -= tot;
        if (r < 0) break;  // uniform
    }
    __syncthreads();
    if (t == 0) idx[blockIdx.x] = found;
}

// ------------------------------------------------------------------------------ mode index
// elements: (code << 32) | flat index
__device__ __forceinline__ uint32_t ecode(unsigned long long e) { return (uint32_t)(e >> 32); }

__device__ void heap_adjust(unsigned long long* A, long long f, long long hole, long long len, unsigned long long v) {
    const long long top = hole;
    long long sc = hole;
    while (sc < (len - 1) / 2) {
        sc = 2 * (sc + 1);
        if (ecode(A[f + sc]) < ecode(A[f + sc - 1])) --sc;
        A[f + hole] = A[f + sc];
        hole = sc;
    }
    if ((len & 1) == 0 && sc == (len - 2) / 2) {
        sc = 2 * (sc + 1);
        A[f + hole] = A[f + sc - 1];
        hole = sc - 1;
    }
    long long parent = (hole - 1) / 2;
    while (hole > top && ecode(A[f + parent]) < ecode(v)) {
        A[f + hole] = A[f + parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    A[f + hole] = v;
}
__device__ void heap_sort_serial(unsigned long long* A, long long f, long long l) {
    const long long len = l - f;
    if (len >= 2) {
        for (long long parent = (len - 2) / 2;; --parent) {
            heap_adjust(A, f, parent, len, A[f + parent]);
            if (parent == 0) break;
        }
    }
    for (long long last = l; last - f > 1;) {
        --last;
        const unsigned long long v = A[last];
        A[last] = A[f];
        heap_adjust(A, f, 0, last - f, v);
    }
}

template <int DT>
__global__ void __launch_bounds__(NT) k_plane_mode_idx(const typename Elem<DT>::type* __restrict__ x, long long N,
                                                      const PlaneStat* __restrict__ st, unsigned long long* ws,
                                                      int64_t* __restrict__ idx, int depth_limit) {
    __shared__ int sh[2 * NW];
    __shared__ long long sh_l[4];
    __shared__ unsigned long long sh_e[4];
    __shared__ unsigned long long sh_u[2];
    const int t = threadIdx.x;
    const typename Elem<DT>::type* xp = x + (size_t)blockIdx.x * N;
    const PlaneStat s = st[blockIdx.x];
    const uint32_t m = (uint32_t)s.mode_code;
    // per plane: the working array and the swap slots (L then R) as u64 [N] each, ranks int2 [N]
    unsigned long long* cur = ws + (size_t)blockIdx.x * 3 * N;
    unsigned long long* slotL = cur + N;
    unsigned long long* slotR = slotL + (N + 1) / 2;
    int2* rk = reinterpret_cast<int2*>(slotL + N);

    if (s.mode_count <= 1 || N <= 16) {
        // a unique value, or no partition (stable insertion sort only): the last occurrence in
        // flat order of the mode's code
        __shared__ unsigned long long lastp1;  // last position + 1
        if (t == 0) lastp1 = 0;
        __syncthreads();
        for (long long i = t; i < N; i += NT)
            if (code_of<DT>(xp[i]) == m) atomicMax(&lastp1, (unsigned long long)(i + 1));
        __syncthreads();
        if (t == 0) idx[blockIdx.x] = (long long)lastp1 - 1;
        return;
    }
#pragma unroll 8
    for (long long i = t; i < N; i += NT) cur[i] = ((unsigned long long)code_of<DT>(xp[i]) << 32) | (unsigned long long)i;
    __syncthreads();

    const int lg = 63 - __builtin_clzll((unsigned long long)N);
    long long f = 0, l = N;
    int depth = depth_limit < 0 ? 2 * lg : depth_limit;
    long long answer = -1;
    for (;;) {
        // mode-valued elements in [f, l): count and last position
        if (t == 0) sh_u[0] = 0;  // last position + 1
        __syncthreads();
        int cnt = 0;
#pragma unroll 8
        for (long long p = f + t; p < l; p += NT) {
            if (ecode(cur[p]) == m) {
                ++cnt;
                atomicMax(&sh_u[0], (unsigned long long)(p + 1));
            }
        }
        const int cntm = block_sum(cnt, sh);
        const long long lastp = (long long)sh_u[0] - 1;
        if (cntm == 1 || l - f <= 16) {
            answer = (long long)(cur[lastp] & 0xFFFFFFFFull);
            break;
        }
        if (depth == 0) {
            if (t == 0) heap_sort_serial(cur, f, l);
            __threadfence_block();
            __syncthreads();
            if (t == 0) sh_u[0] = 0;
            __syncthreads();
    #pragma unroll 8
        for (long long p = f + t; p < l; p += NT)
                if (ecode(cur[p]) == m) atomicMax(&sh_u[0], (unsigned long long)(p + 1));
            __syncthreads();
            answer = (long long)(cur[(long long)sh_u[0] - 1] & 0xFFFFFFFFull);
            break;
        }
        --depth;
        // median of three moved to f (__move_median_to_first(f, f + 1, mid, l - 1))
        if (t == 0) {
            const long long mid = f + (l - f) / 2;
            const uint32_t va = ecode(cur[f + 1]), vb = ecode(cur[mid]), vc = ecode(cur[l - 1]);
            long long sel;
            if (va < vb) sel = vb < vc ? mid : (va < vc ? l - 1 : f + 1);
            else sel = va < vc ? f + 1 : (vb < vc ? l - 1 : mid);
            const unsigned long long ef = cur[f], es = cur[sel];
            cur[f] = es;
            cur[sel] = ef;
            sh_e[0] = es;
        }
        __threadfence_block();
        __syncthreads();
        const uint32_t pv = ecode(sh_e[0]);
        // pass 1: right-stop count over [f + 1, l)
        int cl = 0;
#pragma unroll 8
        for (long long p = f + 1 + t; p < l; p += NT) cl += ecode(cur[p]) <= pv;
        const int TL = block_sum(cl, sh);
        // pass 2: ranks (left stops from the left, right stops from the right) and the swap count;
        // each thread takes KR consecutive elements per step (one block scan per NT * KR elements)
        int sw = 0;
        {
            int gb = 0, lb = 0;
            for (long long base = f + 1; base < l; base += (long long)NT * KR) {
                const long long p0 = base + (long long)t * KR;
                uint32_t c[KR];
                int ng = 0, nl = 0;
#pragma unroll
                for (int j = 0; j < KR; ++j) {
                    const bool in = p0 + j < l;
                    c[j] = in ? ecode(cur[p0 + j]) : 0u;
                    ng += (in && c[j] >= pv) ? 1 : 0;
                    nl += (in && c[j] <= pv) ? 1 : 0;
                }
                int eg, el, tg, tl;
                block_scan2(ng, nl, sh, eg, el, tg, tl);
                int rg = gb + eg, rl = lb + el;
#pragma unroll
                for (int j = 0; j < KR; ++j) {
                    const long long p = p0 + j;
                    if (p < l) {
                        const bool ge = c[j] >= pv, le = c[j] <= pv;
                        const int lrank = rg;
                        const int rrank = TL - (rl + (le ? 1 : 0));  // right stops after p
                        rk[p] = make_int2(ge ? lrank : -1, le ? rrank : -1);
                        sw += (ge && lrank < rrank) ? 1 : 0;
                        rg += ge ? 1 : 0;
                        rl += le ? 1 : 0;
                    }
                }
                gb += tg;
                lb += tl;
            }
        }
        const int S = block_sum(sw, sh);
        // pass 3: swapped elements into their slots; the cut
        if (t == 0) {
            sh_l[1] = 1LL << 62;  // L_{S+1}
            sh_l[2] = l;          // R_S (l when S == 0)
        }
        __syncthreads();
#pragma unroll 8
        for (long long p = f + 1 + t; p < l; p += NT) {
            const int2 r = rk[p];
            if (r.x >= 0 && r.x < S) slotL[r.x] = cur[p];
            if (r.y >= 0 && r.y < S) slotR[r.y] = cur[p];
            if (r.x == S) sh_l[1] = p;
            if (S > 0 && r.y == S - 1) sh_l[2] = p;
        }
        __threadfence_block();
        __syncthreads();
        const long long cut = min(sh_l[1], sh_l[2]);
        // pass 4: the swapped positions take their partners (in place: every other position keeps
        // its element); mode-valued elements right of the cut?
        int mr = 0;
#pragma unroll 8
        for (long long p = f + 1 + t; p < l; p += NT) {
            const int2 r = rk[p];
            unsigned long long e;
            if (r.x >= 0 && r.x < S) {
                e = slotR[r.x];
                cur[p] = e;
            } else if (r.y >= 0 && r.y < S) {
                e = slotL[r.y];
                cur[p] = e;
            } else {
                e = cur[p];
            }
            mr += (p >= cut && ecode(e) == m) ? 1 : 0;
        }
        const int mright = block_sum(mr, sh);
        __threadfence_block();
        if (mright > 0) f = cut;
        else l = cut;
    }
    if (t == 0) idx[blockIdx.x] = answer;
}

}  // namespace

extern "C" {

int admm_planestat_workspace_size(int64_t P, int64_t N, size_t* bytes) {
    if (!bytes || P < 0 || N < 0) return ADMM_TV_EINVAL;
    *bytes = (size_t)P * (sizeof(PlaneStat) + (size_t)3 * N * sizeof(unsigned long long)) + 256;
    return 0;
}

int admm_planestat_median_mode(int dtype, const void* x, int64_t P, int64_t N, int64_t* median_idx,
                               int64_t* mode_idx, void* ws, size_t ws_bytes, int depth_limit, void* stream) {
    if (!x || P < 0 || N < 1 || depth_limit > 62) return ADMM_TV_EINVAL;
    if (dtype != ADMM_CHANSTAT_BF16 && dtype != ADMM_CHANSTAT_F16 && !(dtype == ADMM_CHANSTAT_F32 && !mode_idx))
        return ADMM_TV_EUNSUPPORTED;
    if (N > (1LL << 31) - 2) return ADMM_TV_EUNSUPPORTED;
    if (P == 0) return 0;
    size_t need = 0;
    admm_planestat_workspace_size(P, N, &need);
    if (!ws || ws_bytes < need) return ADMM_TV_EWORKSPACE;
    const hipStream_t s = static_cast<hipStream_t>(stream);
    PlaneStat* st = reinterpret_cast<PlaneStat*>(ws);
    if (dtype == ADMM_CHANSTAT_F32) {  // median only (radix select over the 32-bit codes)
        if (!median_idx) return 0;
        const size_t lds = 32768 * sizeof(uint32_t);
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_plane_median32),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
            return ADMM_TV_EHIP;
        const uint32_t* xp = static_cast<const uint32_t*>(x);
        hipLaunchKernelGGL(k_plane_median32, dim3((unsigned)P), dim3(NT), lds, s, xp, (long long)N, st);
        hipLaunchKernelGGL(k_plane_median_idx<ADMM_CHANSTAT_F32>, dim3((unsigned)P), dim3(NT), 0, s, xp, (long long)N,
                           st, median_idx);
        return hipGetLastError() == hipSuccess ? 0 : ADMM_TV_EHIP;
    }
    auto* buf = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(ws) +
                                                      ((P * sizeof(PlaneStat) + 255) / 256) * 256);
    const uint16_t* xp = static_cast<const uint16_t*>(x);
    const size_t lds = 32768 * sizeof(uint32_t);
    const dim3 grid((unsigned)P), block(NT);
    if (dtype == ADMM_CHANSTAT_BF16) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_plane_hist<ADMM_CHANSTAT_BF16>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
            return ADMM_TV_EHIP;
        hipLaunchKernelGGL(k_plane_hist<ADMM_CHANSTAT_BF16>, grid, block, lds, s, xp, (long long)N, st);
        if (median_idx)
            hipLaunchKernelGGL(k_plane_median_idx<ADMM_CHANSTAT_BF16>, grid, block, 0, s, xp, (long long)N, st,
                               median_idx);
        if (mode_idx)
            hipLaunchKernelGGL(k_plane_mode_idx<ADMM_CHANSTAT_BF16>, grid, block, 0, s, xp, (long long)N, st, buf,
                               mode_idx, depth_limit);
    } else {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_plane_hist<ADMM_CHANSTAT_F16>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
            return ADMM_TV_EHIP;
        hipLaunchKernelGGL(k_plane_hist<ADMM_CHANSTAT_F16>, grid, block, lds, s, xp, (long long)N, st);
        if (median_idx)
            hipLaunchKernelGGL(k_plane_median_idx<ADMM_CHANSTAT_F16>, grid, block, 0, s, xp, (long long)N, st,
                               median_idx);
        if (mode_idx)
            hipLaunchKernelGGL(k_plane_mode_idx<ADMM_CHANSTAT_F16>, grid, block, 0, s, xp, (long long)N, st, buf,
                               mode_idx, depth_limit);
    }
    return hipGetLastError() == hipSuccess ? 0 : ADMM_TV_EHIP;
}

int admm_planestat_select(int dtype, const void* x, int64_t P, int64_t N, const int32_t* stats, int64_t* median_idx,
                          int64_t* mode_idx, void* ws, size_t ws_bytes, int depth_limit, void* stream) {
    if (!x || !stats || P < 0 || N < 1 || depth_limit > 62) return ADMM_TV_EINVAL;
    if (N > (1LL << 31) - 2) return ADMM_TV_EUNSUPPORTED;
    if (P == 0) return 0;
    size_t need = 0;
    admm_planestat_workspace_size(P, N, &need);
    if (mode_idx && (!ws || ws_bytes < need)) return ADMM_TV_EWORKSPACE;
    const hipStream_t s = static_cast<hipStream_t>(stream);
    const PlaneStat* st = reinterpret_cast<const PlaneStat*>(stats);
    auto* buf = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(ws) +
                                                      ((P * sizeof(PlaneStat) + 255) / 256) * 256);
    const dim3 grid((unsigned)P), block(NT);
    auto run = [&](auto dt) {
        constexpr int DT = decltype(dt)::value;
        using E = typename Elem<DT>::type;
        const E* xp = static_cast<const E*>(x);
        if (median_idx) hipLaunchKernelGGL(k_plane_median_idx<DT>, grid, block, 0, s, xp, (long long)N, st, median_idx);
        if (mode_idx)
            hipLaunchKernelGGL(k_plane_mode_idx<DT>, grid, block, 0, s, xp, (long long)N, st, buf, mode_idx, depth_limit);
    };
    switch (dtype) {
        case ADMM_CHANSTAT_F32: run(std::integral_constant<int, ADMM_CHANSTAT_F32>{}); break;
        case ADMM_CHANSTAT_BF16: run(std::integral_constant<int, ADMM_CHANSTAT_BF16>{}); break;
        case ADMM_CHANSTAT_F16: run(std::integral_constant<int, ADMM_CHANSTAT_F16>{}); break;
        default: return ADMM_TV_EINVAL;
    }
    return hipGetLastError() == hipSuccess ? 0 : ADMM_TV_EHIP;
}

}  // extern "C"

// channel_stats.hip -- per-pixel channel statistics (std, median, mode) in one pass, and their
// backward: the C ABI of include/admm_chanstat.h.  Replaces the reference's ChannelPool
// (/root/reference/src/admmtor/elayers/attentions.py:36-47), which PyTorch runs as three
// sort/select reductions over the channel dim of an NCHW tensor.
//
// Layout: x [B][C][HW].  A workgroup stages a tile of 64 consecutive pixels x C channels in LDS
// (each load a contiguous 64-pixel row segment), then each of its 4 waves works on one pixel at a
// time with the C values spread over its 64 lanes, so every step is wave-uniform (no per-lane
// divergence in the data-dependent sort).  The values are "sorted" with the exact algorithm the
// reference's CPU torch.mode uses (libstdc++ std::sort on (value, index) pairs compared by value:
// introsort, median-of-three pivot, unguarded partition, heapsort at the depth limit, final
// insertion sort) -- that algorithm is not stable, and the order it leaves equal values in is
// what decides the index torch.mode returns (and so where its gradient goes).  The median's index
// follows torch.median's rule instead (the stable rank (C-1)/2: ties broken by channel index).
// HBM traffic is the compulsory C reads + 3 writes (+2 index writes) per pixel.
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

#include <cstdint>

#include "admm_chanstat.h"
#include "admm_tv.h"
#include "knobs.hpp"

namespace {

// ---------------------------------------------------------------- element types
struct BF16T {
    using store = uint16_t;
    using key = uint32_t;
    static constexpr int bits = 16;
    static constexpr uint32_t inf = 0x7F80u;
    __device__ static bool isnan(uint32_t u) { return (u & 0x7F80u) == 0x7F80u && (u & 0x7Fu); }
    __device__ static float to_f(uint32_t u) { return __uint_as_float(u << 16); }
    __device__ static uint16_t from_f(float f) {  // round to nearest even (PyTorch's float -> bf16)
        uint32_t u = __float_as_uint(f);
        if ((u & 0x7FFFFFFFu) > 0x7F800000u) return 0x7FC0;
        u += 0x7FFFu + ((u >> 16) & 1u);
        return (uint16_t)(u >> 16);
    }
};
struct F16T {
    using store = uint16_t;
    using key = uint32_t;
    static constexpr int bits = 16;
    static constexpr uint32_t inf = 0x7C00u;
    __device__ static bool isnan(uint32_t u) { return (u & 0x7C00u) == 0x7C00u && (u & 0x3FFu); }
    __device__ static float to_f(uint32_t u) { return __half2float(__ushort_as_half((unsigned short)u)); }
    __device__ static uint16_t from_f(float f) { return __half_as_ushort(__float2half_rn(f)); }
};
struct F32T {
    using store = uint32_t;
    using key = uint64_t;
    static constexpr int bits = 32;
    __device__ static bool isnan(uint32_t u) { return (u & 0x7FFFFFFFu) > 0x7F800000u; }
    __device__ static float to_f(uint32_t u) { return __uint_as_float(u); }
    __device__ static uint32_t from_f(float f) { return __float_as_uint(f); }
};

// order-preserving unsigned image of the value bits: -0 folds onto +0 (they compare equal, as the
// reference's `<` on floats), every NaN onto the all-ones image
template <class T> __device__ __forceinline__ uint32_t ord(uint32_t u) {
    constexpr uint32_t sign = 1u << (T::bits - 1);
    constexpr uint32_t all = T::bits == 32 ? 0xFFFFFFFFu : ((1u << T::bits) - 1u);
    if (T::isnan(u)) return all;
    if ((u & ~sign) == 0) u = 0;
    return (u & sign) ? (~u & all) : (u | sign);
}

// ------------------------------------------------------------------------------ wave helpers
__device__ __forceinline__ int mbcnt(uint64_t m) {  // set bits of m below this lane
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
// lane i <-> lane i ^ M within the wave, on VALU cross-lane paths only (DPP, v_permlane*_swap):
// no LDS round trip.  quad_perm for 1/2/3, row_half_mirror (i ^ 7), row_ror:8 (i ^ 8 in a
// 16-lane row), row_mirror (i ^ 15), permlane16/32_swap for 16/32; the rest compose.
template <int M> __device__ __forceinline__ uint32_t xor_lane(uint32_t v, int lane) {
    if constexpr (M == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
    else if constexpr (M == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
    else if constexpr (M == 3) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x1B, 0xF, 0xF, false);
    else if constexpr (M == 7) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false);
    else if constexpr (M == 4) return xor_lane<7>(xor_lane<3>(v, lane), lane);
    else if constexpr (M == 8) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, false);
    else if constexpr (M == 15) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, false);
    else if constexpr (M == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return (lane & 16) ? r[0] : r[1];
    } else if constexpr (M == 32) {
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (lane & 32) ? r[0] : r[1];
    } else if constexpr (M == 31) return xor_lane<15>(xor_lane<16>(v, lane), lane);
    else if constexpr (M == 63) return xor_lane<31>(xor_lane<32>(v, lane), lane);
    else static_assert(M == 0, "unsupported lane mask");
}
template <int M> __device__ __forceinline__ uint64_t xor_lane(uint64_t v, int lane) {
    return ((uint64_t)xor_lane<M>((uint32_t)(v >> 32), lane) << 32) | xor_lane<M>((uint32_t)v, lane);
}

__device__ __forceinline__ uint32_t wave_max(uint32_t v, int lane) {
    v = max(v, xor_lane<1>(v, lane));
    v = max(v, xor_lane<2>(v, lane));
    v = max(v, xor_lane<4>(v, lane));
    v = max(v, xor_lane<8>(v, lane));
    v = max(v, xor_lane<16>(v, lane));
    return max(v, xor_lane<32>(v, lane));
}

// LDS written by some lanes of this wave and read by others: order the accesses within the wave
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The wave's array of C elements lives in registers: position p = e * 64 + lane, e < E.
// Reads and writes at a wave-uniform position.
template <int E> __device__ __forceinline__ uint32_t rd(const uint32_t (&a)[E], int p) {
    const int e = p >> 6;
    uint32_t r = a[0];
#pragma unroll
    for (int k = 1; k < E; ++k)
        if (e == k) r = a[k];
    return (uint32_t)__builtin_amdgcn_readlane((int)r, p & 63);
}
template <class K, int E> __device__ __forceinline__ K rd_key(const K (&a)[E], int p) {
    const int e = p >> 6;
    K r = a[0];
#pragma unroll
    for (int k = 1; k < E; ++k)
        if (e == k) r = a[k];
    if constexpr (sizeof(K) == 8) {
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)r, p & 63);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(r >> 32), p & 63);
        return ((K)hi << 32) | lo;
    } else {
        return (K)__builtin_amdgcn_readlane((int)r, p & 63);
    }
}
template <int E>
__device__ __forceinline__ void wr(uint32_t (&v)[E], uint32_t (&c)[E], int p, uint32_t vv, uint32_t cc, int lane) {
    const int e = p >> 6;
    if (lane == (p & 63)) {
#pragma unroll
        for (int k = 0; k < E; ++k)
            if (e == k) {
                v[k] = vv;
                c[k] = cc;
            }
    }
}

// ------------------------------------------------ libstdc++ std::sort, restated (bits/stl_algo.h,
// bits/stl_heap.h) for the comparator `a.value < b.value`.
//
// __unguarded_partition (Hoare) on [f+1, l) with the pivot at f, done by the whole wave at once:
// the left scan stops at the positions holding a value >= pivot (L_1 < L_2 < ...), the right scan
// at those holding a value <= pivot (R_1 > R_2 > ...), both judged on the values before any swap
// (a scan never revisits a swapped position before the pointers cross), and the k-th stops swap
// while L_k < R_k.  With S such swaps the returned cut is min(L_{S+1}, R_S) (R_0 = l).  Each lane
// ranks its elements among the stops with ballots, the swapped pairs trade places through LDS.
template <int E>
__device__ int partition_wave(uint32_t (&val)[E], uint32_t (&chan)[E], int f, int l, int lane, uint64_t* sL,
                              uint64_t* sR) {
    const int mid = f + (l - f) / 2;
    const uint32_t va = rd(val, f + 1), vb = rd(val, mid), vc = rd(val, l - 1);
    int sel;  // __move_median_to_first(f, f + 1, mid, l - 1)
    if (va < vb) sel = vb < vc ? mid : (va < vc ? l - 1 : f + 1);
    else sel = va < vc ? f + 1 : (vb < vc ? l - 1 : mid);
    const uint32_t v0 = rd(val, f), c0 = rd(chan, f), pv = rd(val, sel), c1 = rd(chan, sel);
    wr(val, chan, f, pv, c1, lane);
    wr(val, chan, sel, v0, c0, lane);

    bool ge[E], le[E];
    uint64_t gm[E], lm[E];
    int totle = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int p = e * 64 + lane;
        const bool in = p > f && p < l;
        ge[e] = in && val[e] >= pv;
        le[e] = in && val[e] <= pv;
        gm[e] = __ballot(ge[e]);
        lm[e] = __ballot(le[e]);
        totle += __popcll(lm[e]);
    }
    int lrank[E], rrank[E];
    bool swl[E];
    int S = 0;
    {
        int gb = 0, lb = 0;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            lrank[e] = gb + mbcnt(gm[e]);                              // # left stops before p
            rrank[e] = totle - (lb + mbcnt(lm[e]) + (le[e] ? 1 : 0));  // # right stops after p
            swl[e] = ge[e] && lrank[e] < rrank[e];
            gb += __popcll(gm[e]);
            lb += __popcll(lm[e]);
            S += __popcll(__ballot(swl[e]));
        }
    }
    wave_sync();
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint64_t me = ((uint64_t)val[e] << 32) | chan[e];
        if (swl[e]) sL[lrank[e]] = me;
        else if (le[e] && rrank[e] < S) sR[rrank[e]] = me;
    }
    wave_sync();
#pragma unroll
    for (int e = 0; e < E; ++e) {
        uint64_t in = 0;
        bool take = false;
        if (swl[e]) {
            in = sR[lrank[e]];
            take = true;
        } else if (le[e] && rrank[e] < S) {
            in = sL[rrank[e]];
            take = true;
        }
        if (take) {
            val[e] = (uint32_t)(in >> 32);
            chan[e] = (uint32_t)in;
        }
    }
    int lp = 1 << 30, rp = l;
#pragma unroll
    for (int e = E - 1; e >= 0; --e) {
        const uint64_t m = __ballot(ge[e] && lrank[e] == S);
        if (m) lp = e * 64 + __builtin_ctzll(m);
        if (S > 0) {
            const uint64_t r = __ballot(le[e] && rrank[e] == S - 1);
            if (r) rp = e * 64 + __builtin_ctzll(r);
        }
    }
    return min(lp, rp);
}

// heapsort fallback at the depth limit (std::__partial_sort(f, l, l)), run by one lane on the
// wave's keys in LDS; reached only by adversarial orders
template <class K> __device__ void adjust_heap(K* A, int f, int hole, int len, K v) {
    constexpr int IB = sizeof(K) == 8 ? 32 : 16;
    const int top = hole;
    int sc = hole;
    while (sc < (len - 1) / 2) {
        sc = 2 * (sc + 1);
        if ((A[f + sc] >> IB) < (A[f + sc - 1] >> IB)) --sc;
        A[f + hole] = A[f + sc];
        hole = sc;
    }
    if ((len & 1) == 0 && sc == (len - 2) / 2) {
        sc = 2 * (sc + 1);
        A[f + hole] = A[f + sc - 1];
        hole = sc - 1;
    }
    int parent = (hole - 1) / 2;  // __push_heap
    while (hole > top && (A[f + parent] >> IB) < (v >> IB)) {
        A[f + hole] = A[f + parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    A[f + hole] = v;
}

template <class K> __device__ void heap_sort(K* A, int f, int l) {
    const int len = l - f;
    if (len >= 2) {
        for (int parent = (len - 2) / 2;; --parent) {
            adjust_heap(A, f, parent, len, A[f + parent]);
            if (parent == 0) break;
        }
    }
    for (int last = l; last - f > 1;) {
        --last;
        const K v = A[last];
        A[last] = A[f];
        adjust_heap(A, f, 0, last - f, v);
    }
}

constexpr int WSCRATCH = 2048;  // per wave: 2 x 128 u64 swap slots (aliased by the heap keys)

template <class T> constexpr int tile_row() { return sizeof(typename T::store) == 2 ? 66 : 65; }  // odd words: no bank conflicts

// One compare-exchange stage of the sort over the wave's E*64 keys (position p = e*64 + lane):
// p meets p ^ MASK, the lower position keeps the smaller key.  MASK's lane part moves through
// xor_lane, its register part (>= 64) is a register pair within the lane.
template <int MASK, class K, int E> __device__ __forceinline__ void cx_stage(K (&k)[E], int lane) {
    constexpr int ML = MASK & 63, ME = MASK >> 6;
    if constexpr (ME == 0) {
        constexpr int HB = 1 << (31 - __builtin_clz(ML));
        const bool low = (lane & HB) == 0;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const K o = xor_lane<ML>(k[e], lane);
            k[e] = (low == (k[e] < o)) ? k[e] : o;
        }
    } else {
        constexpr int HE = 1 << (31 - __builtin_clz(ME));
#pragma unroll
        for (int e = 0; e < E; ++e) {
            if ((e & HE) == 0 && (e ^ ME) < E) {
                const int e2 = e ^ ME;
                K o1, o2;
                if constexpr (ML == 0) {
                    o1 = k[e2];
                    o2 = k[e];
                } else {
                    o1 = xor_lane<ML>(k[e2], lane);
                    o2 = xor_lane<ML>(k[e], lane);
                }
                k[e] = k[e] < o1 ? k[e] : o1;
                k[e2] = k[e2] < o2 ? o2 : k[e2];
            }
        }
    }
}

// merge step of size N: the mirror stage (p ^ (N-1)) then half-cleaners p ^ N/4 ... p ^ 1
template <int N, class K, int E> __device__ __forceinline__ void merge_stages(K (&k)[E], int lane) {
    cx_stage<N - 1>(k, lane);
    if constexpr (N >= 256) cx_stage<64>(k, lane);
    if constexpr (N >= 128) cx_stage<32>(k, lane);
    if constexpr (N >= 64) cx_stage<16>(k, lane);
    if constexpr (N >= 32) cx_stage<8>(k, lane);
    if constexpr (N >= 16) cx_stage<4>(k, lane);
    if constexpr (N >= 8) cx_stage<2>(k, lane);
    if constexpr (N >= 4) cx_stage<1>(k, lane);
}

// ascending bitonic sort of the wave's E*64 keys, every exchange on VALU cross-lane paths
template <class K, int E> __device__ __forceinline__ void wave_bitonic(K (&k)[E], int lane) {
    merge_stages<2>(k, lane);
    merge_stages<4>(k, lane);
    merge_stages<8>(k, lane);
    merge_stages<16>(k, lane);
    merge_stages<32>(k, lane);
    merge_stages<64>(k, lane);
    if constexpr (E >= 2) merge_stages<128>(k, lane);
    if constexpr (E >= 4) merge_stages<256>(k, lane);
}

// One workgroup = 4 waves and a tile of 64 consecutive pixels.  The tile [C][64] is staged in LDS
// with coalesced row loads.  The std of each pixel is one lane's loop over its column; everything
// else is done by one wave per pixel, its 64 lanes holding the C values (E per lane):
//  * a wave-wide bitonic sort of (value, channel) keys gives the median (stable rank, as
//    torch.median) and the runs of equal values, so the mode value (first longest run);
//  * which channel torch.mode reports for it is decided by libstdc++'s introsort: the last of the
//    mode-valued elements after the partitions (the final insertion sort is stable).  Partitioned
//    ranges are independent and keep their order, so only the rightmost range still holding a
//    mode-valued element matters, and only while it holds two or more: the kernel follows that one
//    range (a few partitions per pixel instead of the whole introsort).
template <class T, int E>
__global__ void __launch_bounds__(256) k_chanpool(const typename T::store* __restrict__ x,
                                                  typename T::store* __restrict__ out, int16_t* __restrict__ idx,
                                                  int C, long long HW, long long npix, int depth_limit) {
    using S = typename T::store;
    using K = typename T::key;  // (value image << 8 | channel): 24 bits for 16-bit types, 40 for fp32
    constexpr int ROW = tile_row<T>();
    constexpr int IB = sizeof(K) == 8 ? 32 : 16;  // heap keys (value << IB | channel)
    extern __shared__ __align__(16) unsigned char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    unsigned char* wbase = smem + wid * WSCRATCH;
    uint64_t* sL = reinterpret_cast<uint64_t*>(wbase);              // [128]
    uint64_t* sR = sL + 128;                                         // [128]
    K* hk = reinterpret_cast<K*>(wbase);                             // [256] heap keys (aliases sL, sR)
    float* res_sd = reinterpret_cast<float*>(smem + 4 * WSCRATCH);  // [64]
    int16_t* res_mi = reinterpret_cast<int16_t*>(res_sd + 64);      // [64]
    int16_t* res_oi = res_mi + 64;                                  // [64]
    S* tile = reinterpret_cast<S*>(smem + 4 * WSCRATCH + 512);      // [C][ROW]

    const long long P0 = (long long)blockIdx.x * 64;
    const int npx = (int)min(64LL, npix - P0);
    {
        const long long gp = P0 + lane;
        if (lane < npx) {
            const long long b = gp / HW, hw = gp - b * HW;
            const S* xp = x + (size_t)b * C * HW + hw;
            for (int c = wid; c < C; c += 4) tile[c * ROW + lane] = xp[(size_t)c * HW];
        }
    }
    __syncthreads();

    // std: lane L of wave w owns pixel w + 4L; two-pass in fp64, channel order
    if (lane < 16 && wid + 4 * lane < npx) {
        const int px = wid + 4 * lane;
        double s = 0.0;
        for (int c = 0; c < C; ++c) s += (double)T::to_f((uint32_t)tile[c * ROW + px]);
        const double mean = s / (double)C;
        double m2 = 0.0;
        for (int c = 0; c < C; ++c) {
            const double d = (double)T::to_f((uint32_t)tile[c * ROW + px]) - mean;
            m2 += d * d;
        }
        res_sd[px] = (float)sqrt(m2 / (double)(C - 1));  // C == 1: NaN, as the reference
    }

    const int mpos = (C - 1) >> 1;
    for (int px = wid; px < npx; px += 4) {
        uint32_t val[E], chan[E];
        K key[E];
        bool valid[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const int p = e * 64 + lane;
            valid[e] = p < C;
            val[e] = valid[e] ? ord<T>((uint32_t)tile[p * ROW + px]) : 0xFFFFFFFFu;
            chan[e] = (uint32_t)p;
            key[e] = valid[e] ? (((K)val[e] << 8) | (K)p) : ~(K)0;
        }
        wave_bitonic(key, lane);

        // median: sorted position mpos of the (value, channel) order; a column holding NaN gives
        // its first NaN (torch.median)
        constexpr uint32_t kNaN = T::bits == 32 ? 0xFFFFFFFFu : ((1u << T::bits) - 1u);
        int mi = -1;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const uint64_t nb = __ballot(valid[e] && val[e] == kNaN);
            if (mi < 0 && nb) mi = e * 64 + __builtin_ctzll(nb);
        }
        if (mi < 0) mi = (int)(rd_key(key, mpos) & 0xFF);

        // runs of equal values in the sorted keys: starts, lengths, the first longest run
        uint32_t sv[E];
        bool start[E];
        uint64_t sm[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
            sv[e] = (uint32_t)(key[e] >> 8);
            const uint32_t carry = e > 0 ? (uint32_t)__builtin_amdgcn_readlane((int)sv[e > 0 ? e - 1 : 0], 63) : 0u;
            uint32_t prev = (uint32_t)__shfl_up((int)sv[e], 1);
            if (lane == 0) prev = e > 0 ? carry : ~sv[e];
            const int p = e * 64 + lane;
            start[e] = p < C && sv[e] != prev;
            sm[e] = __ballot(start[e]);
        }
        uint32_t len[E], lmax = 0;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const int p = e * 64 + lane;
            int next = C;
#pragma unroll
            for (int e2 = E - 1; e2 > e; --e2)
                if (sm[e2]) next = e2 * 64 + __builtin_ctzll(sm[e2]);
            const uint64_t above = lane < 63 ? sm[e] >> (lane + 1) : 0ull;
            if (above) next = p + 1 + __builtin_ctzll(above);
            len[e] = start[e] ? (uint32_t)(next - p) : 0u;
            lmax = max(lmax, len[e]);
        }
        lmax = wave_max(lmax, lane);
        int ms = -1;  // position of the mode run's first key
#pragma unroll
        for (int e = E - 1; e >= 0; --e) {
            const uint64_t m = __ballot(len[e] == lmax && start[e]);
            if (m) ms = e * 64 + __builtin_ctzll(m);
        }
        const uint32_t mvl = (uint32_t)(rd_key(key, ms) >> 8);

        int oi;
        if (lmax == 1 || C <= 16) {
            // a unique value, or no partition at all (only the stable insertion sort): the run's
            // last key in (value, channel) order
            oi = (int)(rd_key(key, ms + (int)lmax - 1) & 0xFF);
        } else {
            const int lg = 31 - __builtin_clz((unsigned)C);
            int f = 0, l = C, depth = depth_limit < 0 ? 2 * lg : depth_limit;
            for (;;) {
                // mode-valued elements in [f, l): how many, and the last one
                int cntm = 0, lastp = -1;
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const int p = e * 64 + lane;
                    const uint64_t m = __ballot(p >= f && p < l && val[e] == mvl);
                    cntm += __popcll(m);
                    if (m) lastp = e * 64 + 63 - __builtin_clzll(m);
                }
                if (cntm == 1 || l - f <= 16) {
                    oi = (int)rd(chan, lastp);
                    break;
                }
                if (depth == 0) {
                    wave_sync();
#pragma unroll
                    for (int e = 0; e < E; ++e)
                        if (valid[e]) hk[e * 64 + lane] = ((K)val[e] << IB) | (K)chan[e];
                    wave_sync();
                    if (lane == 0) heap_sort(hk, f, l);
                    wave_sync();
                    int best = -1;
#pragma unroll
                    for (int e = 0; e < E; ++e) {
                        const int p = e * 64 + lane;
                        if (p >= f && p < l) {
                            const K k = hk[p];
                            if ((uint32_t)(k >> IB) == mvl) best = p;
                        }
                    }
                    const int bp = (int)wave_max((uint32_t)(best + 1), lane) - 1;
                    oi = (int)(hk[bp] & (K)0xFFFF);
                    break;
                }
                --depth;
                const int cut = partition_wave(val, chan, f, l, lane, sL, sR);
                bool right = false;
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const int p = e * 64 + lane;
                    right |= __ballot(p >= cut && p < l && val[e] == mvl) != 0;
                }
                if (right) f = cut;
                else l = cut;
            }
        }
        if (lane == 0) {
            res_mi[px] = (int16_t)mi;
            res_oi[px] = (int16_t)oi;
        }
    }
    __syncthreads();
    {
        const int px = lane, k = wid;
        if (px < npx) {
            const long long gp = P0 + px;
            const long long b = gp / HW, hw = gp - b * HW;
            if (k < 3) {
                // the selected elements themselves (keeps -0.0 and NaN payloads)
                const S v = k == 0 ? (S)T::from_f(res_sd[px]) : tile[(k == 1 ? res_mi[px] : res_oi[px]) * ROW + px];
                out[((size_t)b * 3 + k) * HW + hw] = v;
            } else if (idx) {
                idx[(size_t)b * 2 * HW + hw] = res_mi[px];
                idx[((size_t)b * 2 + 1) * HW + hw] = res_oi[px];
            }
        }
    }
}

// ------------------------------------------------ one pixel per lane (16-bit types, C <= 128)
//
// The wave kernel above spends a whole wave on each pixel: every step of its sort and of the
// introsort trace is a cross-lane operation with ~2/3 of the lanes idle at C = 86 (config 5), about
// 1,500 instructions per pixel.  Here each lane owns one pixel: its C values are loaded straight
// into registers (one coalesced 64-pixel row segment per channel), their 16-bit value images sorted
// by a register bitonic network two to a register (v_pk_min_u16 / v_pk_max_u16 on static register
// indices: ~1,900 instructions sort 64 pixels of 128 values), and everything that needs channels --
// the median's stable rank among ties, the mode's channel, the introsort trace -- runs on the lane's
// own column of LDS in channel order (element p of lane L at word p * 64 + L: conflict-free).  No
// cross-lane traffic and no barrier: a block is one wave.  Same results as the wave kernel, rule for
// rule (median stable rank / first NaN, first longest run, the mode index libstdc++ leaves).
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// ascending bitonic sort of NP 16-bit keys packed two per register: position p sits in register
// p % (NP/2), in the low half for p < NP/2 and the high half above.  Stage (K, J) is the classic
// directional network's block size K, stride J.
template <int K, int J, int NP> __device__ __forceinline__ void pk_stage(u16x2 (&v)[NP / 2]) {
    constexpr int H = NP / 2;
    if constexpr (J == H) {  // the two halves of one register
#pragma unroll
        for (int r = 0; r < H; ++r) {
            const u16x2 s = v[r].yx;
            const u16x2 mn = __builtin_elementwise_min(v[r], s), mx = __builtin_elementwise_max(v[r], s);
            v[r] = u16x2{mn.x, mx.y};
        }
    } else {
#pragma unroll
        for (int r = 0; r < H; ++r) {
            if ((r ^ J) > r) {
                const u16x2 a = v[r], b = v[r ^ J];
                const u16x2 mn = __builtin_elementwise_min(a, b), mx = __builtin_elementwise_max(a, b);
                if constexpr (K == H) {  // low half ascending, high half descending
                    v[r] = u16x2{mn.x, mx.y};
                    v[r ^ J] = u16x2{mx.x, mn.y};
                } else {
                    const bool asc = (r & K) == 0;  // K == NP: always
                    v[r] = asc ? mn : mx;
                    v[r ^ J] = asc ? mx : mn;
                }
            }
        }
    }
}
template <int K, int J, int NP> __device__ __forceinline__ void pk_strides(u16x2 (&v)[NP / 2]) {
    pk_stage<K, J, NP>(v);
    if constexpr (J > 1) pk_strides<K, J / 2, NP>(v);
}
template <int K, int NP> __device__ __forceinline__ void pk_blocks(u16x2 (&v)[NP / 2]) {
    pk_strides<K, K / 2, NP>(v);
    if constexpr (K < NP) pk_blocks<K * 2, NP>(v);
}
template <int NP> __device__ __forceinline__ void pk_bitonic(u16x2 (&v)[NP / 2]) { pk_blocks<2, NP>(v); }

// std::__adjust_heap / __push_heap / heap sort on the lane's LDS column (keys value << 8 | channel,
// compared by value): the depth-limit fallback, reached only by adversarial orders
__device__ void adjust_heap_col(uint32_t* col, int f, int hole, int len, uint32_t v) {
    const int top = hole;
    int sc = hole;
    while (sc < (len - 1) / 2) {
        sc = 2 * (sc + 1);
        if ((col[(f + sc) * 64] >> 8) < (col[(f + sc - 1) * 64] >> 8)) --sc;
        col[(f + hole) * 64] = col[(f + sc) * 64];
        hole = sc;
    }
    if ((len & 1) == 0 && sc == (len - 2) / 2) {
        sc = 2 * (sc + 1);
        col[(f + hole) * 64] = col[(f + sc - 1) * 64];
        hole = sc - 1;
    }
    int parent = (hole - 1) / 2;
    while (hole > top && (col[(f + parent) * 64] >> 8) < (v >> 8)) {
        col[(f + hole) * 64] = col[(f + parent) * 64];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    col[(f + hole) * 64] = v;
}
__device__ void heap_sort_col(uint32_t* col, int f, int l) {
    const int len = l - f;
    if (len >= 2)
        for (int parent = (len - 2) / 2;; --parent) {
            adjust_heap_col(col, f, parent, len, col[(f + parent) * 64]);
            if (parent == 0) break;
        }
    for (int last = l; last - f > 1;) {
        --last;
        const uint32_t v = col[last * 64];
        col[last * 64] = col[f * 64];
        adjust_heap_col(col, f, 0, last - f, v);
    }
}

// fn(p, key) over the lane's LDS column, positions [f, l) in order, eight reads issued before any use
// (a plain loop waits out one LDS round trip per element)
template <class F> __device__ __forceinline__ void for_channels(const uint32_t* col, int f, int l, F&& fn) {
    int p = f;
    for (; p + 8 <= l; p += 8) {
        uint32_t e[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) e[k] = col[(p + k) * 64];
#pragma unroll
        for (int k = 0; k < 8; ++k) fn(p + k, e[k]);
    }
    for (; p < l; ++p) fn(p, col[p * 64]);
}

// the lane kernel's 16-bit value image in straight arithmetic (ternaries here became divergent
// branches): ord<T>'s order (-0 folds onto +0), every NaN onto 0xFFFE, so that 0xFFFF is free for
// padding and sorts after every value.  INF = the infinity's bits; NaN <=> (u & 0x7FFF) > INF.
template <uint32_t INF> __device__ __forceinline__ uint32_t ord16(uint32_t u) {
    const uint32_t t = u & 0x7FFFu;
    u &= ~(((t - 1u) >> 31) << 15);                  // -0 -> +0
    const uint32_t o = (u ^ ((0u - (u >> 15)) | 0x8000u)) & 0xFFFFu;
    const uint32_t m = 0u - ((INF - t) >> 31);       // all ones for NaN
    return (o & ~m) | (0xFFFEu & m);
}

template <class T, int NP>
__global__ void __launch_bounds__(64) k_chanpool_lane(const typename T::store* __restrict__ x,
                                                      typename T::store* __restrict__ out,
                                                      int16_t* __restrict__ idx, int C, long long HW,
                                                      long long npix, int depth_limit, int exp) {
    static_assert(T::bits == 16, "16-bit value images, channel-order keys value << 8 | channel");
    using S = typename T::store;
    constexpr int H = NP / 2;
    extern __shared__ __align__(16) uint32_t colmem[];
    const int lane = threadIdx.x;
    const long long gp = (long long)blockIdx.x * 64 + lane;
    if (gp >= npix) return;
    uint32_t* col = colmem + lane;
    const long long b = gp / HW, hw = gp - b * HW;
    const S* xp = x + (size_t)b * C * HW + hw;

    // loads in chunks of 32 channels, each chunk's loads issued before any use (a scheduling barrier
    // between chunks keeps 32, not NP, unpacked values in flight); channels past C re-read channel
    // C-1 and are replaced by 0 (the sum) and the all-ones image (the sort: after every value, tied
    // only with NaN, which the scans below stop short of by counting positions < C).  As a chunk
    // lands: the value images into the packed registers and the channel-order keys (image << 8 |
    // channel) into the lane's LDS column.  C goes through a VGPR copy (opaque to the compiler) so
    // that the per-channel padding tests are vector arithmetic: as scalar masks, all NP of them were
    // kept live at once and spilled.
    int Cv;
    asm volatile("v_mov_b32 %0, %1" : "=v"(Cv) : "s"(C));
    // one buffer resource from the wave's first image on: a per-lane 32-bit offset shared by every
    // load, the channel offset in an SGPR (64-bit addresses per load cost two VGPRs each)
    const long long b0 = ((long long)blockIdx.x * 64) / HW;
    const S* wbase = x + (size_t)b0 * C * HW;
    const size_t left = ((size_t)(npix / HW) - (size_t)b0) * C * HW * sizeof(S);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<S*>(wbase), 0, (int)(left < 0xFFFFFFFFull ? left : 0xFFFFFFFFull), 0x00020000);
    const int voff = (int)(((b - b0) * C * HW + hw) * (long long)sizeof(S));
    u16x2 v[H];
#pragma unroll
    for (int c0 = 0; c0 < NP; c0 += 32) {
        uint32_t raw[32];
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            raw[i] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(rs, voff, (int)(min(c0 + i, C - 1) * HW * (long long)sizeof(S)), 0);
        }
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            const int c = c0 + i;
            const uint32_t keep = ~(uint32_t)((Cv - 1 - c) >> 31);  // all ones for c < C
            const uint32_t u = raw[i] & keep;
            const uint32_t o = ord16<T::inf>(u) | (~keep & 0xFFFFu);
            col[min(c, Cv) * 64] = (o << 8) | (uint32_t)c;  // padding: into the spare word C
            if (c < H) v[c % H].x = (unsigned short)o;
            else v[c % H].y = (unsigned short)o;
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    // std: two passes in fp64, channel order (as the wave kernel), over the keys in LDS, 8 reads in
    // flight (in the load loop, the fp64 sum held that chunk's values and doubled the registers).  The
    // image inverts to the value bits but for -0 -> +0 (no effect on the sums) and one NaN for all: a
    // column holding NaN (its first one noted here, for the median rule) re-reads its values from
    // global memory instead, so the NaN that propagates is the one the wave kernel's sum carried.
    auto value = [](uint32_t e) {
        const uint32_t o = e >> 8;
        return (double)T::to_f((o & 0x8000u) ? (o ^ 0x8000u) : (~o & 0xFFFFu));
    };
    double s = 0.0;
    int nanc = -1;
    if (!(exp & 2)) for_channels(col, 0, C, [&](int c, uint32_t e) {
        s += value(e);
        nanc = (nanc < 0 && (e >> 8) == 0xFFFEu) ? c : nanc;
    });
    double m2 = 0.0;
    if (exp & 2) {
    } else if (nanc < 0) {
        const double mean = s / (double)C;
        for_channels(col, 0, C, [&](int, uint32_t e) {
            const double d = value(e) - mean;
            m2 += d * d;
        });
    } else {
        s = 0.0;
        for (int c = 0; c < C; ++c) s += (double)T::to_f((uint32_t)xp[(size_t)c * HW]);
        const double mean = s / (double)C;
        for (int c = 0; c < C; ++c) {
            const double d = (double)T::to_f((uint32_t)xp[(size_t)c * HW]) - mean;
            m2 += d * d;
        }
    }
    const float sd = (float)sqrt(m2 / (double)(C - 1));  // C == 1: NaN, as the reference
    if (!(exp & 8)) pk_bitonic<NP>(v);
    __builtin_amdgcn_sched_barrier(0);

    // sorted scan: the median image (position (C-1)/2) and where its run starts; the first longest run
    // of values (the padding's run of 0xFFFF images, after every value, never counts)
    const int mpos = (C - 1) >> 1;
    int mposv;  // a VGPR copy, as Cv above: the per-position tests stay vector compares
    asm volatile("v_mov_b32 %0, %1" : "=v"(mposv) : "s"(mpos));
    uint32_t prev = v[0].x, medv = prev, mvl = prev, run = 1, lmax = 1;
    int r0 = 0;
#pragma unroll
    for (int p = 1; p < NP; ++p) {
        const uint32_t sv = p < H ? v[p % H].x : v[p % H].y;
        const bool same = sv == prev;
        run = same ? run + 1 : 1;
        medv = p == mposv ? sv : medv;
        const bool better = run > lmax && sv != 0xFFFFu;
        lmax = better ? run : lmax;
        mvl = better ? sv : mvl;
        prev = sv;
    }
    // where the median's run starts: the count of smaller values (a separate pass: folded into the
    // scan above, its equality masks were kept for a second walk and spilled)
#pragma unroll
    for (int p = 0; p < NP; ++p) r0 += (p < H ? v[p % H].x : v[p % H].y) < medv ? 1 : 0;
    // channel order: the median is the (mpos - r0)-th occurrence of its value (ties by channel), a
    // column holding NaN gives its first NaN; the mode run's last key in (value, channel) order is
    // the last occurrence of its value
    int mi = -1, oi = 0, seen = 0;
    const int jm = mpos - r0;
    if (!(exp & 4)) for_channels(col, 0, C, [&](int c, uint32_t e) {
        e >>= 8;
        mi = (e == medv && seen == jm) ? c : mi;
        seen += e == medv ? 1 : 0;
        oi = e == mvl ? c : oi;
    });
    if (nanc >= 0) mi = nanc;

    // oi so far: a unique value, or C <= 16 (only the stable insertion sort)
    if (lmax > 1 && C > 16 && !(exp & 1)) {
        // follow the rightmost introsort range holding two or more mode-valued elements
        const int lg = 31 - __builtin_clz((unsigned)C);
        int f = 0, l = C, cnt = (int)lmax, depth = depth_limit < 0 ? 2 * lg : depth_limit;
        for (;;) {
            if (cnt == 1 || l - f <= 16 || depth == 0) {
                if (cnt != 1 && l - f > 16) heap_sort_col(col, f, l);
                int lastp = f;
                for_channels(col, f, l, [&](int p, uint32_t e) { lastp = (e >> 8) == mvl ? p : lastp; });
                oi = (int)(col[lastp * 64] & 0xFF);
                break;
            }
            --depth;
            // __move_median_to_first(f, f + 1, mid, l - 1)
            const int mid = f + (l - f) / 2;
            const uint32_t kf = col[f * 64], ka = col[(f + 1) * 64], kb = col[mid * 64], kc = col[(l - 1) * 64];
            const uint32_t va = ka >> 8, vb = kb >> 8, vc = kc >> 8;
            int sel;
            uint32_t ks;
            if (va < vb) {
                sel = vb < vc ? mid : (va < vc ? l - 1 : f + 1);
                ks = vb < vc ? kb : (va < vc ? kc : ka);
            } else {
                sel = va < vc ? f + 1 : (vb < vc ? l - 1 : mid);
                ks = va < vc ? ka : (vb < vc ? kc : kb);
            }
            col[f * 64] = ks;
            col[sel * 64] = kf;
            // __unguarded_partition(f + 1, l, pivot f) as one flat loop over chunks of four positions: a
            // step reads the next four of the left scan (state 0, ascending from i) or of the right scan
            // (state 1, descending from j) and takes the first stop among them, so one LDS round trip
            // covers up to four elements.  Reads past a stop are clamped into the column ([0, C]) and
            // never used: the median-of-three leaves a stop inside [f, l) for either scan.
            const uint32_t pv = ks >> 8;
            int i = f + 1, j = l - 1;
            bool rs = false;
            uint32_t ai = 0;
            for (;;) {
                uint32_t e[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) e[k] = col[(rs ? max(j - k, 0) : min(i + k, C)) * 64];
                if (!rs) {
                    int k = 4;
#pragma unroll
                    for (int q = 3; q >= 0; --q) k = (e[q] >> 8) >= pv ? q : k;
                    i += k;
                    if (k < 4) {
                        ai = e[0];
#pragma unroll
                        for (int q = 1; q < 4; ++q) ai = q == k ? e[q] : ai;
                        rs = true;
                    }
                } else {
                    int k = 4;
#pragma unroll
                    for (int q = 3; q >= 0; --q) k = (e[q] >> 8) <= pv ? q : k;
                    j -= k;
                    if (k < 4) {
                        if (!(i < j)) break;
                        uint32_t bj = e[0];
#pragma unroll
                        for (int q = 1; q < 4; ++q) bj = q == k ? e[q] : bj;
                        col[i * 64] = bj;
                        col[j * 64] = ai;
                        ++i;
                        --j;
                        rs = false;
                    }
                }
            }
            const int cut = i;
            int cr = 0;
            for_channels(col, cut, l, [&](int, uint32_t e) { cr += (e >> 8) == mvl ? 1 : 0; });
            if (cr > 0) {
                f = cut;
                cnt = cr;
            } else {
                l = cut;
            }
        }
    }

    const size_t o3 = (size_t)b * 3 * HW + hw;
    out[o3] = (S)T::from_f(sd);
    out[o3 + HW] = xp[(size_t)mi * HW];  // the selected elements themselves (-0.0, NaN payloads)
    out[o3 + 2 * HW] = xp[(size_t)oi * HW];
    if (idx) {
        idx[(size_t)b * 2 * HW + hw] = (int16_t)mi;
        idx[((size_t)b * 2 + 1) * HW + hw] = (int16_t)oi;
    }
}

// backward: gx_c = g_std (x_c - mean) / ((C-1) std) + [c == mi] g_med + [c == oi] g_mode, in fp32
// with the std the forward returned (the reference's std_backward uses its result)
template <class T>
__global__ void __launch_bounds__(256) k_chanpool_bwd(const typename T::store* __restrict__ x,
                                                      const typename T::store* __restrict__ out,
                                                      const int16_t* __restrict__ idx,
                                                      const typename T::store* __restrict__ gout,
                                                      typename T::store* __restrict__ gx, int C, long long HW,
                                                      long long npix) {
    const long long p = (long long)blockIdx.x * 256 + threadIdx.x;
    if (p >= npix) return;
    const long long b = p / HW, hw = p - b * HW;
    const typename T::store* xp = x + (size_t)b * C * HW + hw;
    typename T::store* gp = gx + (size_t)b * C * HW + hw;
    float s = 0.f;
    for (int c = 0; c < C; ++c) s += T::to_f(xp[(size_t)c * HW]);
    const float mean = s / (float)C;
    const size_t o3 = (size_t)b * 3 * HW + hw, o2 = (size_t)b * 2 * HW + hw;
    const float sd = T::to_f(out[o3]);
    const float gs = T::to_f(gout[o3]), gm = T::to_f(gout[o3 + HW]), go = T::to_f(gout[o3 + 2 * HW]);
    const int mi = idx[o2], oi = idx[o2 + HW];
    const float scale = sd == 0.f ? 0.f : gs / ((float)(C - 1) * sd);  // std_backward's masked_fill_(std == 0, 0)
    for (int c = 0; c < C; ++c) {
        float g = scale * (T::to_f(xp[(size_t)c * HW]) - mean);
        if (c == mi) g += gm;
        if (c == oi) g += go;
        gp[(size_t)c * HW] = T::from_f(g);
    }
}

size_t lds_bytes(int dtype, int64_t C) {
    const size_t row = dtype == ADMM_CHANSTAT_F32 ? 65 * 4 : 66 * 2;
    return 4 * WSCRATCH + 512 + (size_t)C * row;
}

template <class T, int E>
int launch_e(const void* x, int64_t B, int64_t C, int64_t HW, void* out, int16_t* idx, size_t lds, int depth,
             hipStream_t s) {
    const long long npix = (long long)B * HW;
    if (lds > 65536 && hipFuncSetAttribute(reinterpret_cast<const void*>(&k_chanpool<T, E>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
        return ADMM_TV_EHIP;
    hipLaunchKernelGGL((k_chanpool<T, E>), dim3((unsigned)((npix + 63) / 64)), dim3(256), lds, s,
                       static_cast<const typename T::store*>(x), static_cast<typename T::store*>(out), idx, (int)C,
                       (long long)HW, npix, depth);
    return hipGetLastError() == hipSuccess ? 0 : ADMM_TV_EHIP;
}

template <class T, int NP>
int launch_lane(const void* x, int64_t B, int64_t C, int64_t HW, void* out, int16_t* idx, int depth, hipStream_t s) {
    const long long npix = (long long)B * HW;
    hipLaunchKernelGGL((k_chanpool_lane<T, NP>), dim3((unsigned)((npix + 63) / 64)), dim3(64),
                       (size_t)(C + 1) * 64 * sizeof(uint32_t), s, static_cast<const typename T::store*>(x),
                       static_cast<typename T::store*>(out), idx, (int)C, (long long)HW, npix, depth,
                       env_int("ADMM_CHANPOOL_EXP", 0));  // A/B knob: phases skipped for timing (wrong results)
    return hipGetLastError() == hipSuccess ? 0 : ADMM_TV_EHIP;
}

template <class T>
int launch(const void* x, int64_t B, int64_t C, int64_t HW, void* out, int16_t* idx, size_t lds, int depth,
           hipStream_t s) {
    // one pixel per lane: 16-bit types up to 128 channels whose per-image bytes suit the 32-bit
    // buffer offsets (ADMM_CHANPOOL_WAVE=1 keeps the wave kernel: an A/B knob)
    const bool lane_ok = (long long)(C + 64) * HW * 4 < (1LL << 31) && !env_int("ADMM_CHANPOOL_WAVE", 0);
    if constexpr (sizeof(typename T::store) == 2) {
        if (lane_ok && C <= 64) return launch_lane<T, 64>(x, B, C, HW, out, idx, depth, s);
        if (lane_ok && C <= 128) return launch_lane<T, 128>(x, B, C, HW, out, idx, depth, s);
    }
    if (C <= 64) return launch_e<T, 1>(x, B, C, HW, out, idx, lds, depth, s);
    if (C <= 128) return launch_e<T, 2>(x, B, C, HW, out, idx, lds, depth, s);
    if constexpr (sizeof(typename T::store) == 2) return launch_e<T, 4>(x, B, C, HW, out, idx, lds, depth, s);
    return ADMM_TV_EUNSUPPORTED;
}

template <class T>
int launch_bwd(const void* x, const void* out, const int16_t* idx, const void* gout, void* gx, int64_t B, int64_t C,
               int64_t HW, hipStream_t s) {
    const long long npix = (long long)B * HW;
    hipLaunchKernelGGL((k_chanpool_bwd<T>), dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, s,
                       static_cast<const typename T::store*>(x), static_cast<const typename T::store*>(out), idx,
                       static_cast<const typename T::store*>(gout), static_cast<typename T::store*>(gx), (int)C,
                       (long long)HW, npix);
    return hipGetLastError() == hipSuccess ? 0 : ADMM_TV_EHIP;
}

}  // namespace

extern "C" {

int admm_chanstat_max_channels(int dtype) {
    return dtype == ADMM_CHANSTAT_F32 ? 128 : (dtype == ADMM_CHANSTAT_BF16 || dtype == ADMM_CHANSTAT_F16) ? 256 : 0;
}

int admm_chanstat_pool_depth(int dtype, const void* x, int64_t B, int64_t C, int64_t HW, void* out, int16_t* idx,
                             int depth_limit, void* stream) {
    if (depth_limit > 16) return ADMM_TV_EINVAL;
    if (!x || !out || B < 0 || C < 1 || HW < 0) return ADMM_TV_EINVAL;
    if (C > admm_chanstat_max_channels(dtype)) return ADMM_TV_EUNSUPPORTED;
    if (B == 0 || HW == 0) return 0;
    if (B * HW > 0x7FFFFFFFLL * 64) return ADMM_TV_EUNSUPPORTED;
    const hipStream_t s = static_cast<hipStream_t>(stream);
    const size_t lds = lds_bytes(dtype, C);
    switch (dtype) {
        case ADMM_CHANSTAT_BF16: return launch<BF16T>(x, B, C, HW, out, idx, lds, depth_limit, s);
        case ADMM_CHANSTAT_F16: return launch<F16T>(x, B, C, HW, out, idx, lds, depth_limit, s);
        case ADMM_CHANSTAT_F32: return launch<F32T>(x, B, C, HW, out, idx, lds, depth_limit, s);
        default: return ADMM_TV_EINVAL;
    }
}

int admm_chanstat_pool(int dtype, const void* x, int64_t B, int64_t C, int64_t HW, void* out, int16_t* idx,
                       void* stream) {
    return admm_chanstat_pool_depth(dtype, x, B, C, HW, out, idx, -1, stream);
}

int admm_chanstat_pool_backward(int dtype, const void* x, const void* out, const int16_t* idx, const void* gout,
                                int64_t B, int64_t C, int64_t HW, void* gx, void* stream) {
    if (!x || !out || !idx || !gout || !gx || B < 0 || C < 1 || HW < 0) return ADMM_TV_EINVAL;
    if (C > admm_chanstat_max_channels(dtype)) return ADMM_TV_EUNSUPPORTED;
    if (B == 0 || HW == 0) return 0;
    if (B * HW > 0x7FFFFFFFLL * 256) return ADMM_TV_EUNSUPPORTED;
    const hipStream_t s = static_cast<hipStream_t>(stream);
    switch (dtype) {
        case ADMM_CHANSTAT_BF16: return launch_bwd<BF16T>(x, out, idx, gout, gx, B, C, HW, s);
        case ADMM_CHANSTAT_F16: return launch_bwd<F16T>(x, out, idx, gout, gx, B, C, HW, s);
        case ADMM_CHANSTAT_F32: return launch_bwd<F32T>(x, out, idx, gout, gx, B, C, HW, s);
        default: return ADMM_TV_EINVAL;
    }
}

}  // extern "C"

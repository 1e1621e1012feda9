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

#include "chanpool_lane.hpp"  // the element types, their value images and the one-pixel-per-lane kernel


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

// device memory accessors of the lane kernel: one buffer resource from the wave's first image on,
// a per-lane 32-bit offset shared by every load and the channel offset in an SGPR (64-bit
// addresses per load cost two VGPRs each)
template <class S> struct LaneIo {
    __amdgpu_buffer_rsrc_t rs;
    int voff;
    long long HW;
    const S* xp;
    __device__ __forceinline__ uint32_t load(int c) const {
        return (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(rs, voff, (int)(c * HW * (long long)sizeof(S)), 0);
    }
    __device__ __forceinline__ uint32_t raw(int c) const { return (uint32_t)xp[(size_t)c * HW]; }
    __device__ __forceinline__ int opaque(int v) const {
        int r;
        asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "s"(v));
        return r;
    }
    // an opaque pack: as plain vector code the compiler sank every pack to the sort and kept all NP
    // images unpacked (one register each) until then
    __device__ __forceinline__ u16x2 pack(uint32_t lo, uint32_t hi) const {
        uint32_t r;
        asm volatile("v_lshl_or_b32 %0, %2, 16, %1" : "=v"(r) : "v"(lo), "v"(hi));
        return __builtin_bit_cast(u16x2, r);
    }
    __device__ __forceinline__ void barrier() const { __builtin_amdgcn_sched_barrier(0); }
};

template <class T, int NP>
__global__ void __launch_bounds__(64) k_chanpool_lane(const typename T::store* __restrict__ x,
                                                      typename T::store* __restrict__ out,
                                                      int16_t* __restrict__ idx, int C, long long HW,
                                                      long long npix, int depth_limit) {
    using S = typename T::store;
    extern __shared__ __align__(16) uint16_t colmem[];
    const int lane = threadIdx.x;
    const long long gp = (long long)blockIdx.x * 64 + lane;
    if (gp >= npix) return;
    const long long b = gp / HW, hw = gp - b * HW;
    const long long b0 = ((long long)blockIdx.x * 64) / HW;
    const size_t left = ((size_t)(npix / HW) - (size_t)b0) * C * HW * sizeof(S);
    LaneIo<S> io;
    io.rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<S*>(x + (size_t)b0 * C * HW), 0,
                                              (int)(left < 0xFFFFFFFFull ? left : 0xFFFFFFFFull), 0x00020000);
    io.voff = (int)(((b - b0) * C * HW + hw) * (long long)sizeof(S));
    io.HW = HW;
    io.xp = x + (size_t)b * C * HW + hw;
    float sd;
    int mi, oi;
    lane_pixel<T, NP>(io, colmem + 3 * 64 + lane, C, depth_limit, sd, mi, oi);  // positions -3 .. C + 3
    const size_t o3 = (size_t)b * 3 * HW + hw;
    out[o3] = (S)T::from_f(sd);
    // the selected elements themselves (-0.0, NaN payloads); the channels clamped into [0, C) for
    // the address only, so that a wrong index can never read outside x (the tests see the index)
    out[o3 + HW] = io.xp[(size_t)min(max(mi, 0), C - 1) * HW];
    out[o3 + 2 * HW] = io.xp[(size_t)min(max(oi, 0), C - 1) * HW];
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
                       (size_t)(C + 7) * 64 * sizeof(uint16_t), s, static_cast<const typename T::store*>(x),
                       static_cast<typename T::store*>(out), idx, (int)C, (long long)HW, npix, depth);
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

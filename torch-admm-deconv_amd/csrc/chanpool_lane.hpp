// chanpool_lane.hpp -- the one-pixel-per-lane ChannelPool forward (16-bit types, C <= 128), as
// device functions that also compile for the host (tests/native/chanpool_lane_host.cpp runs
// lane_pixel there against the oracle), and the element types both ChannelPool kernels use.
#pragma once

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

// // The wave kernel above spends a whole wave on each pixel: every step of its sort and of the
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

// One pixel of the lane kernel: C channel values of one pixel through Io (load(c): raw bits of
// channel c < C, the loads of a chunk issued before any use; raw(c): the same, re-read; opaque(v): v
// in a VGPR, hidden from the compiler's scalar analysis; barrier(): a scheduling barrier), the lane's
// LDS column col (C + 1 words at stride 64) -> the std, the median's and the mode's channels.  The
// kernel passes device memory accessors; tests/native/chanpool_lane_host.cpp runs this same function
// on the host against the oracle's restatement.
template <class T, int NP, class Io>
__device__ __forceinline__ void lane_pixel(Io& io, uint32_t* col, int C, int depth_limit, int exp, float& sd,
                                           int& mi, int& oi) {
    static_assert(T::bits == 16, "16-bit value images, channel-order keys value << 8 | channel");
    constexpr int H = NP / 2;
    // loads in chunks of 32 channels, each chunk's loads issued before any use (a scheduling barrier
    // between chunks keeps 32, not NP, unpacked values in flight); channels past C re-read channel
    // C-1 and are replaced by 0 (the sum) and the all-ones image (the sort: after every value, tied
    // only with NaN, which the scans below stop short of by counting positions < C).  As a chunk
    // lands: the value images into the packed registers and the channel-order keys (image << 8 |
    // channel) into the lane's LDS column.  C goes through a VGPR copy (opaque to the compiler) so
    // that the per-channel padding tests are vector arithmetic: as scalar masks, all NP of them were
    // kept live at once and spilled.
    const int Cv = io.opaque(C);
    u16x2 v[H];
#pragma unroll
    for (int c0 = 0; c0 < NP; c0 += 32) {
        uint32_t raw[32];
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            raw[i] = io.load(min(c0 + i, C - 1));
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
        io.barrier();
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
        for (int c = 0; c < C; ++c) s += (double)T::to_f(io.raw(c));
        const double mean = s / (double)C;
        for (int c = 0; c < C; ++c) {
            const double d = (double)T::to_f(io.raw(c)) - mean;
            m2 += d * d;
        }
    }
    sd = (float)sqrt(m2 / (double)(C - 1));  // C == 1: NaN, as the reference
    if (!(exp & 8)) pk_bitonic<NP>(v);
    io.barrier();

    // sorted scan: the median image (position (C-1)/2) and where its run starts; the first longest run
    // of values (the padding's run of 0xFFFF images, after every value, never counts)
    const int mpos = (C - 1) >> 1;
    const int mposv = io.opaque(mpos);  // a VGPR copy, as Cv above: the per-position tests stay vector compares
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
    mi = -1;
    oi = 0;
    int seen = 0;
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

}

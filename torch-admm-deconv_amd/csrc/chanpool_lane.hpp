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

// The lane's LDS column holds one 16-bit element per channel: the value image (position = channel
// while the column is in channel order).  For the introsort trace the mode-valued elements are
// rewritten as channel codes -- images no value takes, so an element carries its channel through the
// partitions and still compares as the mode value: below the image of -inf (the negative NaN bit
// patterns, which ord16 folds onto 0xFFFE) and 0x7FFF (-0, folded onto +0).  bf16: codes 0..126 and
// 0x7FFF for channel 127 (WIDE); f16: codes 0..1022.
template <class T, bool WIDE> struct ModeCode {
    static constexpr uint32_t lim = T::inf == 0x7F80u ? 0x7Fu : 0x3FFu;
    __device__ static uint32_t enc(int c) { return WIDE && (uint32_t)c >= lim ? 0x7FFFu : (uint32_t)c; }
    __device__ static bool is(uint32_t e) { return e < lim || (WIDE && e == 0x7FFFu); }  // one compare unless WIDE
    __device__ static int chan(uint32_t e) { return WIDE && e == 0x7FFFu ? 127 : (int)e; }
};

// std::__adjust_heap / __push_heap / heap sort on the lane's LDS column, compared by value (val:
// element -> value image): the depth-limit fallback, reached only by adversarial orders
template <class V>
__device__ void adjust_heap_col(uint16_t* col, int f, int hole, int len, uint32_t v, const V& val) {
    const int top = hole;
    int sc = hole;
    while (sc < (len - 1) / 2) {
        sc = 2 * (sc + 1);
        if (val(col[(f + sc) * 64]) < val(col[(f + sc - 1) * 64])) --sc;
        col[(f + hole) * 64] = col[(f + sc) * 64];
        hole = sc;
    }
    if ((len & 1) == 0 && sc == (len - 2) / 2) {
        sc = 2 * (sc + 1);
        col[(f + hole) * 64] = col[(f + sc - 1) * 64];
        hole = sc - 1;
    }
    int parent = (hole - 1) / 2;
    while (hole > top && val(col[(f + parent) * 64]) < val(v)) {
        col[(f + hole) * 64] = col[(f + parent) * 64];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    col[(f + hole) * 64] = (uint16_t)v;
}
template <class V> __device__ void heap_sort_col(uint16_t* col, int f, int l, const V& val) {
    const int len = l - f;
    if (len >= 2)
        for (int parent = (len - 2) / 2;; --parent) {
            adjust_heap_col(col, f, parent, len, col[(f + parent) * 64], val);
            if (parent == 0) break;
        }
    for (int last = l; last - f > 1;) {
        --last;
        const uint32_t v = col[last * 64];
        col[last * 64] = col[f * 64];
        adjust_heap_col(col, f, 0, last - f, v, val);
    }
}

// fn(p, element) over the lane's LDS column, positions [f, l) in order, eight reads issued before any
// use (a plain loop waits out one LDS round trip per element)
template <class F> __device__ __forceinline__ void for_channels(const uint16_t* col, int f, int l, F&& fn) {
    int p = f;
    for (; p + 8 <= l; p += 8) {
        uint32_t e[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) e[k] = col[(p + k) * 64];
#pragma unroll
        for (int k = 0; k < 8; ++k) fn(p + k, e[k]);
    }
    for (; p < l; ++p) fn(p, (uint32_t)col[p * 64]);
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

// The mode's channel when the introsort reaches it: follow the rightmost range holding two or more
// mode-valued elements (lmax of them, value image mvl) through libstdc++'s partitions, each carrying
// its channel as a code (ModeCode).  WIDE: a bf16 column of 128 channels (channel 127's code).
template <class T, bool WIDE>
__device__ __forceinline__ int introsort_trace(uint16_t* col, int C, int lmax, uint32_t mvl, int depth_limit) {
    using MC = ModeCode<T, WIDE>;
    int oi = 0;
    for_channels(col, 0, C, [&](int c, uint32_t e) {
        if (e == mvl) col[c * 64] = (uint16_t)MC::enc(c);
    });
    auto val = [mvl](uint32_t e) { return MC::is(e) ? mvl : e; };
    const int lg = 31 - __builtin_clz((unsigned)C);
    int f = 0, l = C, cnt = (int)lmax, depth = depth_limit < 0 ? 2 * lg : depth_limit;
    for (;;) {
        if (cnt == 1 || l - f <= 16 || depth == 0) {
            if (cnt != 1 && l - f > 16) heap_sort_col(col, f, l, val);
            uint32_t last = 0;  // the range's last mode-valued element (the final insertion sort is stable)
            for_channels(col, f, l, [&](int, uint32_t e) { last = MC::is(e) ? e : last; });
            oi = MC::chan(last);
            break;
        }
        --depth;
        // __move_median_to_first(f, f + 1, mid, l - 1)
        const int mid = f + (l - f) / 2;
        const uint32_t kf = col[f * 64], ka = col[(f + 1) * 64], kb = col[mid * 64], kc = col[(l - 1) * 64];
        const uint32_t va = val(ka), vb = val(kb), vc = val(kc);
        int sel;
        uint32_t ks;
        if (va < vb) {
            sel = vb < vc ? mid : (va < vc ? l - 1 : f + 1);
            ks = vb < vc ? kb : (va < vc ? kc : ka);
        } else {
            sel = va < vc ? f + 1 : (vb < vc ? l - 1 : mid);
            ks = va < vc ? ka : (vb < vc ? kc : kb);
        }
        col[f * 64] = (uint16_t)ks;
        col[sel * 64] = (uint16_t)kf;
        // __unguarded_partition(f + 1, l, pivot f) with both scans advancing at once: in a step the
        // left scan (ascending from i, stops at a value >= pivot) and the right scan (descending
        // from j, stops at a value <= pivot) each read their next four positions -- one LDS round
        // trip -- unless already holding their stop; with both stops held, the pair is swapped
        // (i < j) or the partition ends at i.  A round's two scans read positions no swap of that
        // round has touched yet, so running them side by side reads what the sequential algorithm
        // reads.  Reads run at most three positions past a stop (the column is addressable from -3
        // to C + 3) and are never used there: the median-of-three leaves a stop inside [f, l) for
        // either scan.  Branch-free but for the
        // loop exit: a step that swaps nothing writes its two elements to the spare element C.
        const uint32_t pv = val(ks);
        int i = f + 1, j = l - 1;
        bool lf = false, rf = false;
        uint32_t ai = 0, bj = 0;
        for (;;) {
            uint32_t el[4], er[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                el[q] = col[(i + q) * 64];
                er[q] = col[(j - q) * 64];
            }
            int kl = 4, kr = 4;
#pragma unroll
            for (int q = 3; q >= 0; --q) {
                kl = val(el[q]) >= pv ? q : kl;
                kr = val(er[q]) <= pv ? q : kr;
            }
            uint32_t sl = el[0], sr = er[0];
#pragma unroll
            for (int q = 1; q < 4; ++q) {
                sl = kl == q ? el[q] : sl;
                sr = kr == q ? er[q] : sr;
            }
            i += lf ? 0 : kl;
            j -= rf ? 0 : kr;
            ai = lf ? ai : sl;
            bj = rf ? bj : sr;
            lf = lf || kl < 4;
            rf = rf || kr < 4;
            if (lf && rf && !(i < j)) break;
            const bool sw = lf && rf;
            col[(sw ? i : C) * 64] = (uint16_t)bj;
            col[(sw ? j : C) * 64] = (uint16_t)ai;
            i += sw ? 1 : 0;
            j -= sw ? 1 : 0;
            lf = lf && !sw;
            rf = rf && !sw;
        }
        const int cut = i;
        // the left part holds values <= pivot, the right part values >= pivot: mode elements
        // split between the two only when the pivot is the mode value
        int cr = mvl > pv ? cnt : 0;
        if (mvl == pv) for_channels(col, cut, l, [&](int, uint32_t e) { cr += MC::is(e) ? 1 : 0; });
        if (cr > 0) {
            f = cut;
            cnt = cr;
        } else {
            l = cut;
        }
    }
    return oi;
}

// One pixel of the lane kernel: C channel values of one pixel through Io (load(c): raw bits of
// channel c < C, the loads of a chunk issued before any use; raw(c): the same, re-read; opaque(v): v
// in a VGPR, hidden from the compiler's scalar analysis; pack(lo, hi): two 16-bit images in one
// register, where it stands; barrier(): a scheduling barrier), the lane's LDS column col (16-bit
// elements at stride 64, addressable from position -3 to C + 3; C is a spare element) -> the std,
// the median's and the mode's channels.  The
// kernel passes device memory accessors; tests/native/chanpool_lane_host.cpp runs this same function
// on the host against the oracle's restatement.
template <class T, int NP, class Io>
__device__ __forceinline__ void lane_pixel(Io& io, uint16_t* col, int C, int depth_limit, float& sd,
                                           int& mi, int& oi) {
    static_assert(T::bits == 16, "16-bit value images");
    constexpr int H = NP / 2;
    // loads in chunks of 32 channels (the two halves of 16 registers: channels r and r + NP/2), each
    // chunk's loads issued before any use and its images packed as it lands (a scheduling barrier
    // between chunks keeps 32, not NP, unpacked values in flight); channels past C re-read channel
    // C-1 and are replaced by 0 (the sum) and the all-ones image (the sort: after every value, tied
    // only with NaN, which the scans below stop short of by counting positions < C).  As a chunk
    // lands: the value images into the packed registers and, in channel order, into the lane's LDS
    // column.  C goes through a VGPR copy (opaque to the compiler) so
    // that the per-channel padding tests are vector arithmetic: as scalar masks, all NP of them were
    // kept live at once and spilled.
    const int Cv = io.opaque(C);
    u16x2 v[H];
#pragma unroll
    for (int r0 = 0; r0 < H; r0 += 16) {  // a chunk: registers r0 .. r0+15, channels r and r + H of each
        uint32_t raw[32];
#pragma unroll
        for (int i = 0; i < 32; ++i) raw[i] = io.load(min(r0 + (i & 15) + (i >> 4) * H, C - 1));
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            const int c = r0 + (i & 15) + (i >> 4) * H;
            const uint32_t keep = ~(uint32_t)((Cv - 1 - c) >> 31);  // all ones for c < C
            const uint32_t u = raw[i] & keep;
            const uint32_t o = ord16<T::inf>(u) | (~keep & 0xFFFFu);
            col[min(c, Cv) * 64] = (uint16_t)o;  // padding: into the spare element C
            raw[i] = o;
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) v[r0 + i] = io.pack(raw[i], raw[i + 16]);
        io.barrier();
    }
    // the sort right behind the loads: placed after the std passes, the images were packed only
    // there and all NP of them stayed unpacked (one register each) through those loops
    pk_bitonic<NP>(v);
    io.barrier();
    // std: two passes in fp64, channel order (as the wave kernel), over the keys in LDS, 8 reads in
    // flight (in the load loop, the fp64 sum held that chunk's values and doubled the registers).  The
    // image inverts to the value bits but for -0 -> +0 (no effect on the sums) and one NaN for all: a
    // column holding NaN (its first one noted here, for the median rule) re-reads its values from
    // global memory instead, so the NaN that propagates is the one the wave kernel's sum carried.
    auto value = [](uint32_t o) {
        return (double)T::to_f((o & 0x8000u) ? (o ^ 0x8000u) : (~o & 0xFFFFu));
    };
    double s = 0.0;
    int nanc = -1;
    for_channels(col, 0, C, [&](int c, uint32_t e) {
        s += value(e);
        nanc = (nanc < 0 && e == 0xFFFEu) ? c : nanc;
    });
    double m2 = 0.0;
    if (nanc < 0) {
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
    for_channels(col, 0, C, [&](int c, uint32_t e) {
        mi = (e == medv && seen == jm) ? c : mi;
        seen += e == medv ? 1 : 0;
        oi = e == mvl ? c : oi;
    });
    if (nanc >= 0) mi = nanc;

    // oi so far: a unique value, or C <= 16 (only the stable insertion sort)
    if (lmax > 1 && C > 16)
        oi = (ModeCode<T, false>::lim <= 0x7Fu && C > (int)ModeCode<T, false>::lim)
                 ? introsort_trace<T, true>(col, C, (int)lmax, mvl, depth_limit)
                 : introsort_trace<T, false>(col, C, (int)lmax, mvl, depth_limit);
}

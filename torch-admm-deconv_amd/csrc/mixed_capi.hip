// mixed_capi.hip -- launchers of the mixed-radix fused kernels (mixed_kernels.hpp):
// the plan tables dispatched to their template instances.  The solve itself is orchestrated in
// admm_capi.hip (run_forward_mixed).
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "mixed_capi.hpp"
#include "knobs.hpp"
#include "mixed_kernels.hpp"

using namespace admm;

namespace admm_mixed {

namespace {

template <class F> hipError_t with_row(int N, F&& f) {
    switch (N) {
        case 16: return f(std::integral_constant<int, 16>{});
        case 32: return f(std::integral_constant<int, 32>{});
        case 64: return f(std::integral_constant<int, 64>{});
        case 128: return f(std::integral_constant<int, 128>{});
        case 256: return f(std::integral_constant<int, 256>{});
        case 512: return f(std::integral_constant<int, 512>{});
        case 1024: return f(std::integral_constant<int, 1024>{});
        case 240: return f(std::integral_constant<int, 240>{});
        case 320: return f(std::integral_constant<int, 320>{});
        case 360: return f(std::integral_constant<int, 360>{});
        case 480: return f(std::integral_constant<int, 480>{});
        case 540: return f(std::integral_constant<int, 540>{});
        case 640: return f(std::integral_constant<int, 640>{});
        case 960: return f(std::integral_constant<int, 960>{});
        case 1920: return f(std::integral_constant<int, 1920>{});
        case 2048: return f(std::integral_constant<int, 2048>{});
        case 400: return f(std::integral_constant<int, 400>{});
        case 720: return f(std::integral_constant<int, 720>{});
        case 800: return f(std::integral_constant<int, 800>{});
        case 1280: return f(std::integral_constant<int, 1280>{});
        default: return hipErrorInvalidValue;
    }
}

template <class F> hipError_t with_col(int H, F&& f) {
    switch (H) {
        case 16: return f(std::integral_constant<int, 16>{});
        case 32: return f(std::integral_constant<int, 32>{});
        case 64: return f(std::integral_constant<int, 64>{});
        case 128: return f(std::integral_constant<int, 128>{});
        case 256: return f(std::integral_constant<int, 256>{});
        case 512: return f(std::integral_constant<int, 512>{});
        case 1024: return f(std::integral_constant<int, 1024>{});
        case 2048: return f(std::integral_constant<int, 2048>{});
        case 4096: return f(std::integral_constant<int, 4096>{});
        case 240: return f(std::integral_constant<int, 240>{});
        case 360: return f(std::integral_constant<int, 360>{});
        case 480: return f(std::integral_constant<int, 480>{});
        case 540: return f(std::integral_constant<int, 540>{});
        case 720: return f(std::integral_constant<int, 720>{});
        case 960: return f(std::integral_constant<int, 960>{});
        case 1080: return f(std::integral_constant<int, 1080>{});
        case 2160: return f(std::integral_constant<int, 2160>{});
        case 600: return f(std::integral_constant<int, 600>{});
        case 768: return f(std::integral_constant<int, 768>{});
        case 800: return f(std::integral_constant<int, 800>{});
        case 1200: return f(std::integral_constant<int, 1200>{});
        case 1440: return f(std::integral_constant<int, 1440>{});
        case 1536: return f(std::integral_constant<int, 1536>{});
        default: return hipErrorInvalidValue;
    }
}

template <class K> hipError_t lds(K kern, size_t bytes) {
    if (bytes <= 64 * 1024) return hipSuccess;
    return hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)bytes);
}

template <int N, class PL = MRow<N>> unsigned row_blocks(long long items) {
    return (unsigned)((items + MRowG<N, PL>::SG - 1) / MRowG<N, PL>::SG);
}

}  // namespace

bool row_ok(int N) {
    return with_row(N, [](auto) { return hipSuccess; }) == hipSuccess;
}
bool col_ok(int H) {
    return with_col(H, [](auto) { return hipSuccess; }) == hipSuccess;
}
int row_lanes(int N) {
    int l = 0;
    (void)with_row(N, [&](auto n) {
        l = MRowG<decltype(n)::value>::Lg;
        return hipSuccess;
    });
    return l;
}
int pass_a_blocks_per_cu(int N) {
    int nb = 0;
    (void)with_row(N, [&](auto n) {
        constexpr int NN = decltype(n)::value;
        using G = MRowG<NN>;
        if (lds(k_pass_a_m<NN, false, false, false>, G::lds_bytes()) != hipSuccess) return hipSuccess;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_pass_a_m<NN, false, false, false>, G::NT, G::lds_bytes()) !=
            hipSuccess)
            nb = 0;
        return hipSuccess;
    });
    return nb;
}
int col_cols(int H) {
    // the fewest columns a block may take: pass_b launches the plan's C, or 4 or 2 when N = W / 2 is no
    // multiple of it
    int c = 0;
    (void)with_col(H, [&](auto h) {
        c = MColG<decltype(h)::value>::C < 2 ? MColG<decltype(h)::value>::C : 2;
        return hipSuccess;
    });
    return c;
}

hipError_t r2c(int N, const float* img, cf* spec, const cf* twW, long long rows, hipStream_t s) {
    return with_row(N, [&](auto n) {
        constexpr int NN = decltype(n)::value;
        using G = MRowG<NN>;
        if (hipError_t e = lds(k_row_r2c_m<NN>, G::lds_bytes())) return e;
        hipLaunchKernelGGL(k_row_r2c_m<NN>, dim3(row_blocks<NN>(rows)), dim3(G::NT), G::lds_bytes(), s, img, spec, twW, rows);
        return hipGetLastError();
    });
}

hipError_t c2r(int N, const cf* spec, float* img, const cf* twW, long long rows, hipStream_t s) {
    return with_row(N, [&](auto n) {
        constexpr int NN = decltype(n)::value;
        using G = MRowG<NN>;
        if (hipError_t e = lds(k_row_c2r_m<NN>, G::lds_bytes())) return e;
        hipLaunchKernelGGL(k_row_c2r_m<NN>, dim3(row_blocks<NN>(rows)), dim3(G::NT), G::lds_bytes(), s, spec, img, twW, rows);
        return hipGetLastError();
    });
}

hipError_t pass_a(int N, const PassAArgs& a, bool iso, bool first, bool hist, hipStream_t s) {
    return with_row(N, [&](auto n) {
        constexpr int NN = decltype(n)::value;
        // the launch geometry of the kernel's row plan (MPlan: the training plans with HIST)
        auto go = [&](auto kern, auto train) {
            using G = MRowG<NN, MPlan<NN, decltype(train)::value>>;
            const size_t l = G::lds_bytes();
            if (hipError_t e = lds(kern, l)) return e;
            hipLaunchKernelGGL(kern, dim3(row_blocks<NN, MPlan<NN, decltype(train)::value>>(a.nstrips)), dim3(G::NT), l, s,
                               a);
            return hipGetLastError();
        };
        const std::true_type T{};
        const std::false_type F{};
        if (hist) {
            if (iso) return first ? go(k_pass_a_m<NN, true, true, true>, T) : go(k_pass_a_m<NN, true, false, true>, T);
            return first ? go(k_pass_a_m<NN, false, true, true>, T) : go(k_pass_a_m<NN, false, false, true>, T);
        }
        if (iso) return first ? go(k_pass_a_m<NN, true, true, false>, F) : go(k_pass_a_m<NN, true, false, false>, F);
        return first ? go(k_pass_a_m<NN, false, true, false>, F) : go(k_pass_a_m<NN, false, false, false>, F);
    });
}

hipError_t iso_norm(int N, const IsoArgs& a, bool first, bool hist, hipStream_t s) {
    return with_row(N, [&](auto n) {
        constexpr int NN = decltype(n)::value;
        auto go = [&](auto kern, auto train) {
            using G = MRowG<NN, MPlan<NN, decltype(train)::value>>;
            const size_t l = G::lds_bytes();
            if (hipError_t e = lds(kern, l)) return e;
            hipLaunchKernelGGL(kern, dim3(row_blocks<NN, MPlan<NN, decltype(train)::value>>(a.nitems)), dim3(G::NT), l, s,
                               a);
            return hipGetLastError();
        };
        if (first) return go(k_iso_norm_m<NN, true, false>, std::false_type{});
        return hist ? go(k_iso_norm_m<NN, false, true>, std::true_type{})
                    : go(k_iso_norm_m<NN, false, false>, std::false_type{});
    });
}

hipError_t bwd_pass_a(int N, const BwdArgs& a, bool iso, bool lastk, bool firstk, hipStream_t s) {
    return with_row(N, [&](auto n) {
        constexpr int NN = decltype(n)::value;
        using G = MRowG<NN, BPlan<NN>>;  // the reverse passes' plans
        const dim3 grid(row_blocks<NN, BPlan<NN>>(a.nstrips)), blk(G::NT);
        const size_t l = G::lds_bytes();
        auto go = [&](auto kern) {
            if (hipError_t e = lds(kern, l)) return e;
            hipLaunchKernelGGL(kern, grid, blk, l, s, a);
            return hipGetLastError();
        };
        switch ((iso ? 4 : 0) | (lastk ? 2 : 0) | (firstk ? 1 : 0)) {
            case 0: return go(k_bwd_pass_a_m<NN, false, false, false>);
            case 1: return go(k_bwd_pass_a_m<NN, false, false, true>);
            case 2: return go(k_bwd_pass_a_m<NN, false, true, false>);
            case 3: return go(k_bwd_pass_a_m<NN, false, true, true>);
            case 4: return go(k_bwd_pass_a_m<NN, true, false, false>);
            case 5: return go(k_bwd_pass_a_m<NN, true, false, true>);
            case 6: return go(k_bwd_pass_a_m<NN, true, true, false>);
            default: return go(k_bwd_pass_a_m<NN, true, true, true>);
        }
    });
}

hipError_t bwd_iso_q(int N, const BwdIsoArgs& a, bool lastk, hipStream_t s) {
    return with_row(N, [&](auto n) {
        constexpr int NN = decltype(n)::value;
        using G = MRowG<NN, BPlan<NN>>;  // the reverse passes' plans
        const dim3 grid(row_blocks<NN, BPlan<NN>>(a.nitems)), blk(G::NT);
        const size_t l = G::lds_bytes();
        auto go = [&](auto kern) {
            if (hipError_t e = lds(kern, l)) return e;
            hipLaunchKernelGGL(kern, grid, blk, l, s, a);
            return hipGetLastError();
        };
        return lastk ? go(k_bwd_iso_q_m<NN, true>) : go(k_bwd_iso_q_m<NN, false>);
    });
}

int pass_b_cols(int H, int N) {
    int cols = 0;
    (void)with_col(H, [&](auto h) {
        constexpr int C0 = MCol<decltype(h)::value>::C;
        cols = N % C0 == 0 ? C0 : (C0 > 4 && N % 4 == 0) ? 4 : (C0 > 2 && N % 2 == 0) ? 2 : 0;
        return hipSuccess;
    });
    return cols;
}

hipError_t pass_b(int H, cf* spec, const float* fcM, const cf* twH, int N, long long P, hipStream_t s) {
    return with_col(H, [&](auto h) {
        constexpr int HH = decltype(h)::value;
        // tile order (planes per group of the walk; pb_tile): plane-major below H = 1024; above, groups of
        // two planes, or -- for blocks of 8+ columns (64-byte row segments) -- one group of all planes: the
        // column-block pairs walk every plane before the next pair, so each XCD (a contiguous range of the
        // launch) keeps its columns' Wiener factors in its L2 instead of re-reading the table per plane: HD
        // pass B 9.5 -> 8.5 B/px (1.19 -> 1.06x its 8 B/px; profiles/r05_rdreq_hd*.json) at the same time;
        // 4K UHD's 2-column blocks lose 12 % that way (profiles/r05_ab_uhd_passb_order.txt) and keep groups of
        // two.  A/B knobs ADMM_PASSB_M_ORDER (planes per group), ADMM_PASSB_M_FPACK (the column-block-packed
        // factors); read once per process (they change no sizes)
        static const int forced = env_int("ADMM_PASSB_M_ORDER", 0);
        static const int fpack = env_int("ADMM_PASSB_M_FPACK", 1);
        auto go = [&](auto cc) {
            constexpr int CC = decltype(cc)::value;
            using G = MColG<HH, CC>;
            const int order = forced > 0 ? forced
                              : HH < 1024 ? 1
                              : CC >= 8   ? (int)std::min<long long>(P, 1 << 30)
                                          : 2;
            const int colblocks = N / CC;
            if (hipError_t e = lds(k_pass_b_m<HH, CC>, G::lds_bytes())) return e;
            hipLaunchKernelGGL((k_pass_b_m<HH, CC>), dim3((unsigned)(P * colblocks)), dim3(G::NT), G::lds_bytes(), s,
                               spec, fcM, twH, N, colblocks, order, fpack);
            return hipGetLastError();
        };
        // the plan's columns per block, or fewer when N is no multiple of them (e.g. W = 1080 beside the
        // 8-column plans)
        constexpr int C0 = MCol<HH>::C;
        if (N % C0 == 0) return go(std::integral_constant<int, C0>{});
        if constexpr (C0 > 4) {
            if (N % 4 == 0) return go(std::integral_constant<int, 4>{});
        }
        if constexpr (C0 > 2) {
            if (N % 2 == 0) return go(std::integral_constant<int, 2>{});
        }
        return hipErrorInvalidValue;
    });
}

hipError_t pass_b_cm(int H, cf* spec, const cf* mM, const cf* twH, int N, long long P, hipStream_t s) {
    return with_col(H, [&](auto h) {
        constexpr int HH = decltype(h)::value;
        auto go = [&](auto cc) {
            constexpr int CC = decltype(cc)::value;
            using G = MColG<HH, CC>;
            const int colblocks = N / CC;
            if (hipError_t e = lds(k_pass_b_m<HH, CC, true>, G::lds_bytes())) return e;
            hipLaunchKernelGGL((k_pass_b_m<HH, CC, true>), dim3((unsigned)(P * colblocks)), dim3(G::NT), G::lds_bytes(),
                               s, spec, nullptr, twH, N, colblocks, 1, 0, mM);
            return hipGetLastError();
        };
        constexpr int C0 = MCol<HH>::C;
        if (N % C0 == 0) return go(std::integral_constant<int, C0>{});
        if constexpr (C0 > 4) {
            if (N % 4 == 0) return go(std::integral_constant<int, 4>{});
        }
        if constexpr (C0 > 2) {
            if (N % 2 == 0) return go(std::integral_constant<int, 2>{});
        }
        return hipErrorInvalidValue;
    });
}

hipError_t mt_mixed(const cf* mT, cf* mM, int H, int N, hipStream_t s) {
    const long long n = (long long)H * (N + 1);
    hipLaunchKernelGGL(k_mt_mixed, dim3((unsigned)std::min<long long>(4096, (n + 255) / 256)), dim3(256), 0, s, mT, mM,
                       H, N);
    return hipGetLastError();
}

hipError_t fc_mixed(const float* fcT, float* fcM, int H, int N, hipStream_t s) {
    const long long n = (long long)H * (2 * N + 1);
    const int C = pass_b_cols(H, N);
    if (C <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_fc_mixed, dim3((unsigned)std::min<long long>(4096, (n + 255) / 256)), dim3(256), 0, s, fcT, fcM,
                       H, N, C);
    return hipGetLastError();
}

}  // namespace admm_mixed

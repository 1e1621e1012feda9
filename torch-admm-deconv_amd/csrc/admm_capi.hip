// admm_capi.hip -- host side of the MI355X ADMM-TV library: the C ABI declared in
// include/admm_tv.h.  Orchestrates setup kernels and the per-iteration passes on
// the caller's stream; no host synchronisation, no allocation (workspace is the
// caller's), so the whole call is graph-capturable.
//
// Replaces the reference's Python loop  fft_admm_tv  (deconv.py:35-117): ~30 ATen
// launches per iteration there, 2 fused kernels per iteration here (3 for iso).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "gcol_mm.hpp"
#include "knobs.hpp"
#include "mixed_capi.hpp"
#include "odd_capi.hpp"
#include "admm_tv.h"

using namespace admm;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

// ------------------------------------------------------------------ profiling
struct ProfRec {
    int kind, dev;
    hipEvent_t a, b;
};
// process-wide totals (bench.py reads them); every access holds g_prof.mu, so solves on
// several threads / streams may record concurrently
struct Prof {
    std::mutex mu;
    bool on = false;
    std::vector<ProfRec> recs;
    std::vector<std::pair<int, hipEvent_t>> pool;  // (device, event): an event records on its device's streams
    double ms[4] = {0, 0, 0, 0};
    int64_t n[4] = {0, 0, 0, 0};
} g_prof;

hipEvent_t prof_event() {  // caller holds g_prof.mu; an event of the current device
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    for (size_t i = 0; i < g_prof.pool.size(); ++i)
        if (g_prof.pool[i].first == dev) {
            hipEvent_t e = g_prof.pool[i].second;
            g_prof.pool[i] = g_prof.pool.back();
            g_prof.pool.pop_back();
            return e;
        }
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

struct ProfScope {
    int kind, dev = 0;
    hipStream_t s;
    hipEvent_t a = nullptr, b = nullptr;
    ProfScope(int k, hipStream_t st) : kind(k), s(st) {
        std::lock_guard<std::mutex> lk(g_prof.mu);
        if (g_prof.on && hipGetDevice(&dev) == hipSuccess) {
            a = prof_event();
            b = prof_event();
            if (a && b) (void)hipEventRecord(a, s);
        }
    }
    ~ProfScope() {
        if (a && b) {
            (void)hipEventRecord(b, s);
            std::lock_guard<std::mutex> lk(g_prof.mu);
            g_prof.recs.push_back({kind, dev, a, b});
        }
    }
};

// cross-rank reduction hook (iso): carried per call in the descriptor (admm_tv_desc.allreduce)
void allreduce(const admm_tv_desc& d, float* buf, size_t count, hipStream_t s) {
    if (d.allreduce) d.allreduce(buf, count, s, d.allreduce_ctx);
}
// an empty shard of an iso solve over ranks: only its part of the reductions remains
bool participate_only(const admm_tv_desc& d) { return d.iso && d.allreduce && d.B * d.C == 0; }

// ------------------------------------------------------------------ geometry
bool pow2(int64_t v) { return v > 0 && (v & (v - 1)) == 0; }

// fused power-of-two kernels
bool supported_hw(int64_t H, int64_t W) {
    return pow2(H) && pow2(W) && H >= 16 && H <= 4096 && W >= 16 && W <= 2048;
}
// any other size runs on the generic kernels (generic_kernels.hpp): a line of each dimension in
// their LDS image (two line buffers + twiddles and Bluestein tables, the latter read from global
// memory for lines beyond ~6,800 points) up to 10,240 points (5,120 in fp64); longer lines keep
// their two buffers in a global scratch slot per block (GPlan::glb), up to kGenericMax
constexpr int64_t kGenericMax = 65536;
bool gen_fits(int n, bool f64 = false);  // below, with the plans
bool generic_hw(int64_t H, int64_t W) {
    return !supported_hw(H, W) && H >= 1 && W >= 1 && H <= kGenericMax && W <= kGenericMax && gen_fits((int)H) &&
           gen_fits((int)W);
}
// smooth sizes on the fused two-pass iteration with mixed-radix register transforms (mixed_kernels.hpp,
// DESIGN.md §7c): W even with a row plan for W / 2, a column plan for H, not both powers of two (those
// are supported_hw).  Training too (Layout::mixed_train), except with a PSF gradient or grouped modules.
// ADMM_MIXED=0 (A/B knob) keeps them on the generic kernels.
bool mixed_hw(int64_t H, int64_t W) {
    if (supported_hw(H, W) || H < 16 || W < 16 || (W & 1) || H > 4096 || W > 4096) return false;
    if (!admm_mixed::row_ok((int)(W / 2)) || !admm_mixed::col_ok((int)H)) return false;
    return (W / 2) % admm_mixed::col_cols((int)H) == 0 && env_int("ADMM_MIXED", 1) != 0;
}
// odd row lengths with a fused row pass instance (odd_kernels.hpp; BSD's W = 481 = 13 * 37): the
// aniso inference solve runs the two-launch iteration -- the generic column pass, then ONE row pass
// (inverse rows, step, forward rows) -- instead of the generic three.  iso and training keep the generic
// kernels.  ADMM_ODD=0 (A/B knob) keeps every solve on them.
bool odd_hw(int64_t H, int64_t W) {
    return generic_hw(H, W) && !mixed_hw(H, W) && admm_odd::row_ok((int)W) && env_int("ADMM_ODD", 1) != 0;
}
// ... and the transposed orientation (H an odd-path row length, W not: BSD portrait frames, 481 x 321): the
// solve commutes with transposing the image and the PSF (Dx and Dy trade places; the x-update's
// |Dx^|^2 + |Dy^|^2, the shrinkage and the centred H_t are symmetric in them), so the aniso inference solve
// transposes xin and the PSF, runs the odd-length iteration on the W x H problem and transposes the result
// back (two transposes per solve, not per iteration; Layout::tr)
bool odd_t_hw(int64_t H, int64_t W) {
    return generic_hw(H, W) && !mixed_hw(H, W) && !odd_hw(H, W) && odd_hw(W, H);
}
// fp64 solves (ADMM_TV_FLAG_F64) run on the generic kernels' double instantiation at every size
bool is_f64(const admm_tv_desc& d) { return (d.flags & ADMM_TV_FLAG_F64) != 0; }
bool f64_hw(int64_t H, int64_t W) {
    return H >= 1 && W >= 1 && H <= kGenericMax && W <= kGenericMax && gen_fits((int)H, true) && gen_fits((int)W, true);
}

GPlan make_plan(int n, bool f64 = false);  // generic-size transform plan (below)
size_t glb_scratch(int H, int W, long long P, bool f64);  // long lines' scratch bytes (below)
// matrix-core column pass (gcol_mm.hpp): H = S R, odd R in [17, 127] carrying H's largest prime
// factor (>= 17), S in {1, ..., 8} with a kernel instance; ok = false: the LDS column pass
struct MMPlan {
    bool ok;
    int R, S, h, KS, MT, NL, RP;
    size_t lds;
    int nth;  // threads per block (the row inverse; the column pass picks its own)
};
MMPlan mm_plan(int H, int W);
MMPlan mm_plan_row(int W);  // the row inverse (k_grow_inv_mm): W = S R, S in {1..5, 8, 13}

// modules solved together (admm_tv_desc.groups)
int ngroups_of(const admm_tv_desc& d) { return d.groups > 1 ? d.groups : 1; }

constexpr size_t kAlign = 256;
size_t up(size_t v) { return (v + kAlign - 1) / kAlign * kAlign; }

struct Layout {
    size_t spec[2], u[4], b, fcT, mT, twW, twH, twHd, G, part, nsq, sigma, total;
    size_t mM;  // mixed path with a PSF: the multiplier for b = H_t(xin) on the mixed transforms (mt_mixed)
    // generic path: the matrix-core plans, decided once per call (their environment knobs are read
    // here only, so the regions sized below and the kernels launched later always agree)
    MMPlan mm, mmr;
    // mixed-radix fused iteration (mixed_hw; run_forward_mixed): the Wiener factor for its column pass.
    // mixed_train: training forward / backward on it too (not with a PSF gradient, whose column-spectrum
    // history is the generic path's)
    bool mixed, mixed_train;
    size_t fcM;
    // fused odd-length row pass (odd_hw, aniso inference): the second half-spectrum buffer of its ping-pong
    bool odd;
    size_t spec2;
    // transposed odd-length solve (odd_t_hw, aniso inference): xin and the result transposed, the PSF
    // transposed, then the W x H problem's own workspace at tws
    bool tr;
    size_t xT, oT, kT, tws;
    size_t rimg;  // generic path: spec[0] = half spectra [P][H][W/2+1], spec[1] = x image, rimg = r image
    size_t gscr;  // generic path, lines beyond the LDS image: the transform blocks' scratch slots
    int ngroups, ppg;
    bool gen;
    // generic fp32 inference with both matrix-core plans: the half-spectrum row pitch (complex values)
    // padded to a multiple of 16 (128 B), so the column pass's 16-column row segments are whole cache
    // lines (A/B knob ADMM_GEN_PITCH=0: Wh)
    int ldw;
};

admm_tv_desc transposed(const admm_tv_desc& d) {
    admm_tv_desc t = d;
    t.H = d.W;
    t.W = d.H;
    return t;
}

Layout make_layout(const admm_tv_desc& d) {
    Layout L{};
    const bool f64 = is_f64(d);
    const size_t rs = f64 ? sizeof(double) : sizeof(float), csz = 2 * rs;  // real / complex element
    const size_t G = ngroups_of(d);
    const size_t P = (size_t)d.B * d.C * G, H = d.H, W = d.W, N = W / 2;  // all modules' planes
    const size_t img = P * H * W * rs;
    const size_t img_m = (size_t)d.B * d.C * H * W * rs;         // one module's planes
    const int k = d.kh;
    size_t o = 0;
    auto take = [&](size_t bytes) {
        size_t at = o;
        o += up(bytes);
        return at;
    };
    L.gen = f64 || generic_hw(d.H, d.W);
    if (L.gen && !f64) {
        L.mm = mm_plan((int)H, (int)W);
        L.mmr = mm_plan_row((int)W);
    }
    L.mixed = L.gen && !f64 && mixed_hw(d.H, d.W) && (G == 1 || !(d.flags & ADMM_TV_FLAG_PSF_GRAD));
    L.mixed_train = L.mixed && G == 1 && !(k > 0 && (d.flags & ADMM_TV_FLAG_PSF_GRAD));
    L.odd = L.gen && !f64 && G == 1 && !d.iso && odd_hw(d.H, d.W);
    L.ldw = (int)(N + 1);
    if (L.gen && !f64 && L.mm.ok && L.mmr.ok && env_int("ADMM_GEN_PITCH", 1)) L.ldw = (int)((N + 1 + 15) / 16 * 16);
    L.spec[0] = take(L.gen ? P * H * (size_t)L.ldw * csz : img);
    L.spec[1] = take(img);
    // generic path: the r image (unfused step)
    L.rimg = L.gen ? take(img) : 0;
    for (int i = 0; i < 4; ++i) L.u[i] = take(img);
    // b = H_t(xin), shared by the modules; on the fused path also without a PSF (b = xin re-laid
    // out for the inference pass, lane-paired rows)
    L.b = (k > 0 || !L.gen) ? take(img_m) : 0;
    // one Wiener factor per module (its rho); on the fused path followed by their packed copies for
    // the column pass (k_fc_pack)
    // (generic path: a [H][Wh] copy for the matrix-core column pass, k_fc_transpose)
    L.fcT = take(G * (N + 1) * H * rs * ((!L.gen || L.mm.ok) ? 2 : 1));
    L.mT = take((N + 1) * H * csz);
    // twiddles; on the generic path followed by the plan's Bluestein tables (make_plan)
    L.twW = take((W + (L.gen ? make_plan((int)W, f64).ntab : 0)) * csz);
    L.twH = take((H + (L.gen ? make_plan((int)H, f64).ntab : 0)) * csz);
    L.twHd = take(H * sizeof(double2));
    L.G = take((size_t)(k > 0 ? k : 1) * (N + 1) * sizeof(double2));
    L.gscr = L.gen ? take(glb_scratch((int)H, (int)W, (long long)P, f64)) : 0;
    L.fcM = L.mixed ? take(G * (2 * N + 1) * H * sizeof(float)) : 0;  // per module: [H][N + 1] + packed copy, k_fc_mixed
    L.mM = (L.mixed && k > 0) ? take((N + 1) * H * 2 * sizeof(float)) : 0;
    L.spec2 = L.odd ? take(P * H * (size_t)L.ldw * csz) : 0;
    L.sigma = (k > 0 && (d.flags & ADMM_TV_FLAG_PSF_GRAD)) ? take((N + 1) * H * sizeof(double2)) : 0;
    if (d.iso) {
        // plane groups for the iso norm pass: enough (group,row) items to fill the chip
        // planes per group: at most 64 (each group writes and the reduce reads one 2HW partial;
        // C3 iso norm pass: 16 -> 0.49 ms, 32 -> 0.46, 64 -> 0.45; 8 -> 499 it/s, 16 -> 497-507,
        // 64 -> 509),
        // fewer when (group, row) items would not give ~3 waves per SIMD (C5: 48 planes of 512^2
        // -> 4, iso norm -30 %)
        const int lanes = (int)std::min<size_t>(64, N / (N >= 1024 ? 16 : N >= 64 ? 8 : N >= 16 ? 4 : 2));
        const long long want = 3LL * 1024 * 64 / std::max(lanes, 1);
        int ppg = (int)std::max<long long>(1, std::min<long long>(64, (long long)(P * H) / want));
        if (const int e = env_int("ADMM_ISO_PPG", 0); e > 0) ppg = e;  // A/B knob; <= 0: the rule
        if ((size_t)P <= (size_t)ppg) ppg = (int)std::max<long long>(1, P);
        if (G > 1) {  // a plane group must not straddle two modules: a divisor of B*C
            const int pm = (int)(d.B * d.C);
            ppg = std::min(ppg, pm);
            while (pm % ppg) --ppg;
        }
        L.ppg = ppg;
        L.ngroups = (int)((P + ppg - 1) / ppg);
        L.part = take((size_t)L.ngroups * 2 * H * W * rs);
        L.nsq = take(G * 2 * H * W * rs);  // per module
    }
    L.total = o;
    if (!f64 && G == 1 && !d.iso && odd_t_hw(d.H, d.W)) {
        // the transposed inference solve: [xin^T][result^T][PSF^T][the W x H problem's workspace], laid over
        // the regions above (a call uses one or the other: training and the helpers keep this layout)
        size_t t = 0;
        auto takeT = [&](size_t bytes) {
            size_t at = t;
            t += up(bytes);
            return at;
        };
        L.tr = true;
        L.xT = takeT(img);
        L.oT = takeT(img);
        L.kT = takeT((size_t)std::max(1, d.kh * d.kw) * sizeof(float));
        L.tws = takeT(make_layout(transposed(d)).total);
        L.total = std::max(L.total, t);
    }
    return L;
}


template <class T> T* at(void* ws, size_t off) { return reinterpret_cast<T*>(static_cast<char*>(ws) + off); }

#define HIPCHK(expr)                                                                    \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess) return fail(ADMM_TV_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

template <class K> int set_lds(K kern, size_t bytes) {
    if (bytes > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
        if (e != hipSuccess) return fail(ADMM_TV_EHIP, std::string("hipFuncSetAttribute: ") + hipGetErrorString(e));
    }
    return 0;
}

int launch_check(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(ADMM_TV_EHIP, std::string(what) + ": " + hipGetErrorString(e));
    return 0;
}

// lambda / rho gradients of one module from the reverse row pass's per-strip fp64 partials
// ([K][nstrips][2], the module's strips at [soff, soff + spm)) and, iso, the tau^ partials: per-iteration
// sums (K blocks, in place), then the sum over the iterations.  Fixed order: deterministic.
template <class T>
int bwd_scalars(double* part, int K, long long nstrips, long long spm, long long soff, const double* tpart, int ntp,
                int G, int g, const T* lam, const T* rho, T* glam, T* grho, hipStream_t s) {
    if (K < 1) return fail(ADMM_TV_EINVAL, "bwd_scalars: no iterations");
    hipLaunchKernelGGL(k_bwd_iter_sums, dim3((unsigned)K), dim3(256), 0, s, part, nstrips, spm, soff, tpart, ntp, G, g);
    if (int e = launch_check("k_bwd_iter_sums")) return e;
    hipLaunchKernelGGL(k_bwd_scalars<T>, dim3(1), dim3(256), 0, s, (const double*)part, K, nstrips, 1LL, soff,
                       (const double*)nullptr, ntp, G, g, lam, rho, glam, grho);
    return launch_check("k_bwd_scalars");
}

// ------------------------------------------------------------------ row-side ops (templated on N = W/2)
template <int N> struct RowOps {
    using G = RowKernelGeom<N>;
    static unsigned blocks(long long items) { return (unsigned)((items + G::SG - 1) / G::SG); }

    // pl: the lane-paired row layout (admm_kernels.hpp ld_row) for the image side
    static int r2c(const float* img, cf* spec, const cf* twW, long long rows, hipStream_t s, bool pl = false) {
        if (pl)
            hipLaunchKernelGGL((k_row_r2c<N, true>), dim3(blocks(rows)), dim3(G::NT), G::lds_bytes(), s, img, spec, twW, rows);
        else
            hipLaunchKernelGGL((k_row_r2c<N, false>), dim3(blocks(rows)), dim3(G::NT), G::lds_bytes(), s, img, spec, twW, rows);
        return launch_check("k_row_r2c");
    }
    static int c2r(const cf* spec, float* img, const cf* twW, long long rows, hipStream_t s, bool pl = false) {
        if (pl)
            hipLaunchKernelGGL((k_row_c2r<N, true>), dim3(blocks(rows)), dim3(G::NT), G::lds_bytes(), s, spec, img, twW, rows);
        else
            hipLaunchKernelGGL((k_row_c2r<N, false>), dim3(blocks(rows)), dim3(G::NT), G::lds_bytes(), s, spec, img, twW, rows);
        return launch_check("k_row_c2r");
    }
    static int pair(const float* img, float* out, long long rows, hipStream_t s) {
        hipLaunchKernelGGL(k_row_pair<N>, dim3(blocks(rows)), dim3(G::NT), 0, s, img, out, rows);
        return launch_check("k_row_pair");
    }
    template <bool ISO, bool FIRST, bool HIST, bool PL> static void pa(const PassAArgs& a, unsigned nb, hipStream_t s) {
        hipLaunchKernelGGL((k_pass_a<N, ISO, FIRST, HIST, PL>), dim3(nb), dim3(G::NT), G::lds_bytes(), s, a);
    }
    static int pass_a(const PassAArgs& a, bool iso, bool first, bool hist, hipStream_t s, bool pl = false) {
        const unsigned nb = blocks(a.nstrips);
        const int sel = (iso ? 4 : 0) | (first ? 2 : 0) | (hist ? 1 : 0);
        if (pl && !hist) {  // inference: lane-paired images
            switch (sel) {
                case 0: pa<false, false, false, true>(a, nb, s); break;
                case 2: pa<false, true, false, true>(a, nb, s); break;
                case 4: pa<true, false, false, true>(a, nb, s); break;
                default: pa<true, true, false, true>(a, nb, s); break;
            }
            return launch_check("k_pass_a");
        }
        switch (sel) {
            case 0: pa<false, false, false, false>(a, nb, s); break;
            case 1: pa<false, false, true, false>(a, nb, s); break;
            case 2: pa<false, true, false, false>(a, nb, s); break;
            case 3: pa<false, true, true, false>(a, nb, s); break;
            case 4: pa<true, false, false, false>(a, nb, s); break;
            case 5: pa<true, false, true, false>(a, nb, s); break;
            case 6: pa<true, true, false, false>(a, nb, s); break;
            default: pa<true, true, true, false>(a, nb, s); break;
        }
        return launch_check("k_pass_a");
    }
    static int iso_norm(const IsoArgs& a, bool first, bool hist, hipStream_t s, bool pl = false) {
        const unsigned nb = blocks(a.nitems);
        if (first && pl)
            hipLaunchKernelGGL((k_iso_norm<N, true, false, true>), dim3(nb), dim3(G::NT), G::lds_bytes(), s, a);
        else if (first)
            hipLaunchKernelGGL((k_iso_norm<N, true, false, false>), dim3(nb), dim3(G::NT), G::lds_bytes(), s, a);
        else if (hist)
            hipLaunchKernelGGL((k_iso_norm<N, false, true, false>), dim3(nb), dim3(G::NT), G::lds_bytes(), s, a);
        else if (pl)
            hipLaunchKernelGGL((k_iso_norm<N, false, false, true>), dim3(nb), dim3(G::NT), G::lds_bytes(), s, a);
        else
            hipLaunchKernelGGL((k_iso_norm<N, false, false, false>), dim3(nb), dim3(G::NT), G::lds_bytes(), s, a);
        return launch_check("k_iso_norm");
    }
    template <bool ISO, bool LASTK, bool FIRSTK> static void bpa(const BwdArgs& a, unsigned nb, hipStream_t s) {
        using BG = BwdGeom<N>;
        hipLaunchKernelGGL((k_bwd_pass_a<N, ISO, LASTK, FIRSTK>), dim3(nb), dim3(BG::NT), BG::lds_bytes(), s, a);
    }
    static int bwd_pass_a(const BwdArgs& a, bool iso, bool lastk, bool firstk, hipStream_t s) {
        const unsigned nb = (unsigned)((a.nstrips + BwdGeom<N>::SG - 1) / BwdGeom<N>::SG);  // its own strips per block
        const int sel = (iso ? 4 : 0) | (lastk ? 2 : 0) | (firstk ? 1 : 0);
        switch (sel) {
            case 0: bpa<false, false, false>(a, nb, s); break;
            case 1: bpa<false, false, true>(a, nb, s); break;
            case 2: bpa<false, true, false>(a, nb, s); break;
            case 3: bpa<false, true, true>(a, nb, s); break;
            case 4: bpa<true, false, false>(a, nb, s); break;
            case 5: bpa<true, false, true>(a, nb, s); break;
            case 6: bpa<true, true, false>(a, nb, s); break;
            default: bpa<true, true, true>(a, nb, s); break;
        }
        return launch_check("k_bwd_pass_a");
    }
    static int bwd_iso_q(const BwdIsoArgs& a, bool lastk, hipStream_t s) {
        const unsigned nb = blocks(a.nitems);
        if (lastk)
            hipLaunchKernelGGL((k_bwd_iso_q<N, true>), dim3(nb), dim3(G::NT), G::lds_bytes(), s, a);
        else
            hipLaunchKernelGGL((k_bwd_iso_q<N, false>), dim3(nb), dim3(G::NT), G::lds_bytes(), s, a);
        return launch_check("k_bwd_iso_q");
    }
};

template <class F> int with_row(int N, F&& f) {
    switch (N) {
        case 8: return f(RowOps<8>{});
        case 16: return f(RowOps<16>{});
        case 32: return f(RowOps<32>{});
        case 64: return f(RowOps<64>{});
        case 128: return f(RowOps<128>{});
        case 256: return f(RowOps<256>{});
        case 512: return f(RowOps<512>{});
        case 1024: return f(RowOps<1024>{});
        default: return fail(ADMM_TV_EUNSUPPORTED, "unsupported W");
    }
}

// ------------------------------------------------------------------ column-side ops (templated on H, C)
// column-pass tile order (k_pass_b pb_tile): planes per group, 1 = plane-major.  Two planes at
// H >= 1024 (C3 pass B 0.376 -> 0.362 ms, C3 iso 0.381 -> 0.369; 4 and 8 planes slower: DRAM
// locality), plane-major below (C2: neutral).  A/B knob ADMM_PASSB_GROUP.
// values per lane of the column transforms (RowCfg<H>::E)
int col_e(int H) { return H >= 1024 ? 16 : H >= 64 ? 8 : 4; }

int passb_order(int H) { return std::max(1, std::min(64, env_int("ADMM_PASSB_GROUP", H >= 1024 ? 2 : 1))); }

// planes per pass B block (k_pass_b gp): the block keeps its multipliers in registers across them
// and reads the Wiener-factor table once per gp planes.  A divisor of the planes per module (a group
// never straddles two Wiener factors).  Measured at C3 (profiles/r03_ab_passb_gp.txt): gp = 4 takes
// pass B 0.346 -> 0.336 ms but the following pass A +1.5 % (whole iteration +-0), gp = 8 slower;
// default 1.  ADMM_PASSB_GP (A/B knob) overrides it.
int passb_gp(int H, int P, int ppm) {
    (void)H;
    int g = env_int("ADMM_PASSB_GP", 1);
    g = std::max(1, std::min(g, 64));
    while (g > 1 && (ppm % g)) --g;
    (void)P;
    return g;
}

template <int H, int C> int pass_b_hc(const cf* spec, cf* out, const float* fcT, const cf* mT, const cf* twH, int N,
                                      int P, int mode, int ppm, hipStream_t s) {
    using G = ColGeom<H, C>;
    const int colblocks = N / C;
    const int gp = passb_gp(H, P, ppm);
    const dim3 grid((unsigned)((long long)((P + gp - 1) / gp) * colblocks));
    const int order = gp > 1 ? 1 : passb_order(H);
    const int fpack = mode == 0 && env_int("ADMM_PASSB_FPACK", 1) ? 1 : 0;  // A/B knob
    // block remap / plane order (k_pass_b pmode): contiguous XCD ranges (2), plane groups walked
    // forward; the reverse walk (3) takes pass B alone 0.3465 -> 0.3420 ms at C3 but the iteration is
    // faster with the forward one (4 interleaved rounds: C3 706-722 -> 710-728 it/s, C2 5,572 ->
    // 5,624, C3 iso +0.5 %; profiles/r03_sweep_knobs_c3.txt); pair-interleaved remap (4, 5) +9 %
    // (profiles/r03_ab_passb_order.txt)
    const int pmode = env_int("ADMM_PASSB_PMODE", 2);
    if (mode == 0) {
        if (int e = set_lds(k_pass_b<H, C, 0>, G::lds_bytes())) return e;
        hipLaunchKernelGGL((k_pass_b<H, C, 0>), grid, dim3(G::NT), G::lds_bytes(), s, spec, out, fcT, mT, twH, N, colblocks, ppm,
                           order, fpack, gp, P, pmode);
    } else if (mode == 1) {
        if (int e = set_lds(k_pass_b<H, C, 1>, G::lds_bytes())) return e;
        hipLaunchKernelGGL((k_pass_b<H, C, 1>), grid, dim3(G::NT), G::lds_bytes(), s, spec, out, fcT, mT, twH, N, colblocks, ppm,
                           order, fpack, gp, P, pmode);
    } else {
        if (int e = set_lds(k_pass_b<H, C, 2>, G::lds_bytes())) return e;
        hipLaunchKernelGGL((k_pass_b<H, C, 2>), grid, dim3(G::NT), G::lds_bytes(), s, spec, out, fcT, mT, twH, N, colblocks, ppm,
                           order, fpack, gp, P, pmode);
    }
    return launch_check("k_pass_b");
}

template <int H> int pass_b_h(const cf* spec, cf* out, const float* fcT, const cf* mT, const cf* twH, int N, int P,
                              int mode, int ppm, hipStream_t s) {
    constexpr int L = ColGeom<H, 1>::L;
    if constexpr (L <= 64) {
        // column pairs with 16-byte accesses (k_pass_b2): measured faster up to H = 512 (C2: pass B
        // -7.5 %, same bits); at H = 1024 the doubled register set costs occupancy (+30 %)
        if (mode == 0 && N >= 16 && env_int("ADMM_PASSB_PAIR", H <= 512 ? 1 : 0)) {
            using G = ColGeom<H, 8>;
            const int colblocks = N / 16;
            if (int e = set_lds(k_pass_b2<H, 8>, G::lds_bytes())) return e;
            hipLaunchKernelGGL((k_pass_b2<H, 8>), dim3((unsigned)((long long)P * colblocks)), dim3(G::NT), G::lds_bytes(),
                               s, spec, out, fcT, twH, N, colblocks, ppm, passb_order(H), env_int("ADMM_PASSB_FPACK", 1) ? 1 : 0);
            return launch_check("k_pass_b2");
        }
        int C = env_int("ADMM_PASSB_C", 8);
        if (C > N) C = N;
        if (C >= 16) return pass_b_hc<H, 16>(spec, out, fcT, mT, twH, N, P, mode, ppm, s);
        return pass_b_hc<H, 8>(spec, out, fcT, mT, twH, N, P, mode, ppm, s);
    } else if constexpr (L == 128) {
        return pass_b_hc<H, 8>(spec, out, fcT, mT, twH, N, P, mode, ppm, s);
    } else {
        return pass_b_hc<H, 4>(spec, out, fcT, mT, twH, N, P, mode, ppm, s);
    }
}

// column pass; out == spec (in place) or a separate buffer
// ppm: planes per module (module m = plane / ppm uses Wiener factor m); ppm = P for one module
int pass_b_oop(int H, const cf* spec, cf* out, const float* fcT, const cf* mT, const cf* twH, int N, int P, int mode,
               hipStream_t s, int ppm = 0) {
    if (ppm <= 0) ppm = P;
    switch (H) {
        case 16: return pass_b_h<16>(spec, out, fcT, mT, twH, N, P, mode, ppm, s);
        case 32: return pass_b_h<32>(spec, out, fcT, mT, twH, N, P, mode, ppm, s);
        case 64: return pass_b_h<64>(spec, out, fcT, mT, twH, N, P, mode, ppm, s);
        case 128: return pass_b_h<128>(spec, out, fcT, mT, twH, N, P, mode, ppm, s);
        case 256: return pass_b_h<256>(spec, out, fcT, mT, twH, N, P, mode, ppm, s);
        case 512: return pass_b_h<512>(spec, out, fcT, mT, twH, N, P, mode, ppm, s);
        case 1024: return pass_b_h<1024>(spec, out, fcT, mT, twH, N, P, mode, ppm, s);
        case 2048: return pass_b_h<2048>(spec, out, fcT, mT, twH, N, P, mode, ppm, s);
        case 4096: return pass_b_h<4096>(spec, out, fcT, mT, twH, N, P, mode, ppm, s);
        default: return fail(ADMM_TV_EUNSUPPORTED, "unsupported H");
    }
}

int pass_b(int H, cf* spec, const float* fcT, const cf* mT, const cf* twH, int N, int P, int mode, hipStream_t s,
           int ppm = 0) {
    return pass_b_oop(H, spec, spec, fcT, mT, twH, N, P, mode, s, ppm);
}

// cross-spectrum partials sum_{p in group} conj(colFFT U_p) colFFT V_p  -> part[g][N+1][H]
template <int H, int C> int xspec_hc(const cf* U, const cf* V, cf* part, const cf* twH, int N, int P, int ppg,
                                     hipStream_t s) {
    using G = ColGeom<H, C>;
    const int colblocks = N / C;
    const int groups = (P + ppg - 1) / ppg;
    if (int e = set_lds(k_xspec<H, C, true>, G::lds_bytes())) return e;
    if (int e = set_lds(k_xspec<H, C, false>, G::lds_bytes())) return e;
    hipLaunchKernelGGL((k_xspec<H, C, true>), dim3(groups), dim3(G::NT), G::lds_bytes(), s, U, V, part, twH, N,
                       colblocks, P, ppg);
    if (colblocks > 1)
        hipLaunchKernelGGL((k_xspec<H, C, false>), dim3(groups * (colblocks - 1)), dim3(G::NT), G::lds_bytes(), s, U,
                           V, part, twH, N, colblocks, P, ppg);
    return launch_check("k_xspec");
}
template <int H> int xspec_h(const cf* U, const cf* V, cf* part, const cf* twH, int N, int P, int ppg, hipStream_t s) {
    constexpr int L = ColGeom<H, 1>::L;
    if constexpr (L <= 64) return xspec_hc<H, 8>(U, V, part, twH, N, P, ppg, s);
    else if constexpr (L == 128) return xspec_hc<H, 8>(U, V, part, twH, N, P, ppg, s);
    else return xspec_hc<H, 4>(U, V, part, twH, N, P, ppg, s);
}
int xspec(int H, const cf* U, const cf* V, cf* part, const cf* twH, int N, int P, int ppg, hipStream_t s) {
    switch (H) {
        case 16: return xspec_h<16>(U, V, part, twH, N, P, ppg, s);
        case 32: return xspec_h<32>(U, V, part, twH, N, P, ppg, s);
        case 64: return xspec_h<64>(U, V, part, twH, N, P, ppg, s);
        case 128: return xspec_h<128>(U, V, part, twH, N, P, ppg, s);
        case 256: return xspec_h<256>(U, V, part, twH, N, P, ppg, s);
        case 512: return xspec_h<512>(U, V, part, twH, N, P, ppg, s);
        case 1024: return xspec_h<1024>(U, V, part, twH, N, P, ppg, s);
        case 2048: return xspec_h<2048>(U, V, part, twH, N, P, ppg, s);
        case 4096: return xspec_h<4096>(U, V, part, twH, N, P, ppg, s);
        default: return fail(ADMM_TV_EUNSUPPORTED, "unsupported H");
    }
}

// grouped modules train only on the fused power-of-two path (a smooth size solves them one after
// another for inference only; training there takes one call per module)
int grouped_train_check(const admm_tv_desc& d) {
    if (d.groups > 1 && !supported_hw(d.H, d.W))
        return fail(ADMM_TV_EUNSUPPORTED, "grouped training needs power-of-two H, W: one call per module");
    return 0;
}

int validate(const admm_tv_desc* d) {
    if (!d) return fail(ADMM_TV_EINVAL, "null descriptor");
    const bool empty_ok = d->iso && d->allreduce && d->B >= 0 && d->C >= 0;  // see participate_only
    if ((empty_ok ? (d->B < 0 || d->C < 0) : (d->B <= 0 || d->C <= 0)) || d->H <= 0 || d->W <= 0 || d->maxit < 0 ||
        d->kh < 0 || d->kw < 0 || d->groups < 0)
        return fail(ADMM_TV_EINVAL, "invalid sizes or maxit");
    if (d->kh != d->kw) return fail(ADMM_TV_ENONSQUARE, "non-square PSF (the reference's H_t swaps H/W pads)");
    if (is_f64(*d) ? !f64_hw(d->H, d->W) : (!supported_hw(d->H, d->W) && !generic_hw(d->H, d->W)))
        return fail(ADMM_TV_EUNSUPPORTED, "unsupported H, W (admm_tv_supported / admm_tv_supported_f64: up to 65,536)");
    if (is_f64(*d) && d->groups > 1) return fail(ADMM_TV_EUNSUPPORTED, "groups > 1: fp32 only");
    if (d->kh > d->H || d->kw > d->W) return fail(ADMM_TV_EKERNEL, "PSF larger than the image");
    if (d->groups > 1 && ((!supported_hw(d->H, d->W) && !mixed_hw(d->H, d->W)) || (d->flags & ADMM_TV_FLAG_PSF_GRAD)))
        return fail(ADMM_TV_EUNSUPPORTED, "groups > 1 needs power-of-two or smooth H, W and no PSF gradient");
    return 0;
}

// the multiplier tables carry the transforms' normalisation: the packed power-of-two row
// transforms produce 2 rfft, the generic ones rfft
double spectra_scale(int H, int W) {
    return (supported_hw(H, W) ? 0.5 : 1.0) / ((double)H * (double)W);
}

// setup: twiddle tables, PSF spectrum, Wiener factor (if rho given), centred-PSF multiplier
template <class T>
int setup(const admm_tv_desc& d, const Layout& Lo, void* ws, const T* kern, const T* rho, hipStream_t s) {
    using C = cx_t<T>;
    ProfScope ps(3, s);
    const int H = (int)d.H, W = (int)d.W, N = W / 2, k = d.kh;
    const int nt = 256;
    hipLaunchKernelGGL(k_tables<C>, dim3((std::max(H, W) + nt - 1) / nt), dim3(nt), 0, s, at<C>(ws, Lo.twW),
                       at<C>(ws, Lo.twH), at<double2>(ws, Lo.twHd), H, W);
    if (int e = launch_check("k_tables")) return e;
    if (Lo.gen && !std::is_same<T, double>::value) {  // Bluestein tables of the row and column plans
        for (int dim = 0; dim < 2; ++dim) {
            const GPlan pl = make_plan(dim == 0 ? W : H);
            if (pl.ntab == 0) continue;
            hipLaunchKernelGGL(k_blue_tables, dim3((3 * 1024 * 64 + nt - 1) / nt), dim3(nt), 0, s,  // a wave per entry
                               at<cf>(ws, dim == 0 ? Lo.twW : Lo.twH), pl);
            if (int e = launch_check("k_blue_tables")) return e;
        }
    }
    if (k > 0) {
        const int n = k * (N + 1);
        hipLaunchKernelGGL(k_psf_rows<T>, dim3((n + nt - 1) / nt), dim3(nt), 0, s, kern, at<double2>(ws, Lo.G), k, N, W);
        if (int e = launch_check("k_psf_rows")) return e;
    }
    const int n = (N + 1) * H;
    if (rho) {
        for (int g = 0; g < ngroups_of(d); ++g) {  // one Wiener factor per module
            hipLaunchKernelGGL(k_spectra<T>, dim3((n + nt - 1) / nt), dim3(nt), 0, s, at<double2>(ws, Lo.G),
                               at<double2>(ws, Lo.twHd), rho + g, at<T>(ws, Lo.fcT) + (size_t)g * n, at<C>(ws, Lo.mT),
                               k, H, N, W, Lo.sigma ? at<double2>(ws, Lo.sigma) : nullptr,
                               (std::is_same<T, double>::value ? 1.0 / ((double)H * W) : spectra_scale(H, W)));
            if (int e = launch_check("k_spectra")) return e;
            if constexpr (std::is_same<T, float>::value) if (!Lo.gen) {
                float* fc = at<float>(ws, Lo.fcT) + (size_t)g * n;
                hipLaunchKernelGGL(k_fc_pack, dim3((n + nt - 1) / nt), dim3(nt), 0, s, fc,
                                   fc + (size_t)ngroups_of(d) * n, H, N, col_e(H));
                if (int e = launch_check("k_fc_pack")) return e;
            }
            if constexpr (std::is_same<T, float>::value) if (Lo.mixed) {
                hipError_t e = admm_mixed::fc_mixed(at<float>(ws, Lo.fcT) + (size_t)g * n,
                                                    at<float>(ws, Lo.fcM) + (size_t)g * (2 * N + 1) * H, H, N, s);
                if (e != hipSuccess) return fail(ADMM_TV_EHIP, std::string("k_fc_mixed: ") + hipGetErrorString(e));
            }
            if constexpr (std::is_same<T, float>::value) if (Lo.gen && Lo.mm.ok && ngroups_of(d) == 1) {
                float* fc = at<float>(ws, Lo.fcT);  // the generic path has one module (grouped: the mixed path)
                hipLaunchKernelGGL(k_fc_transpose, dim3(std::min(4096, (n + nt - 1) / nt)), dim3(nt), 0, s, fc, fc + n, H,
                                   N + 1);
                if (int e = launch_check("k_fc_transpose")) return e;
            }
        }
        if constexpr (std::is_same<T, float>::value) if (Lo.mixed && k > 0) {
            hipError_t e = admm_mixed::mt_mixed(at<cf>(ws, Lo.mT), at<cf>(ws, Lo.mM), H, N, s);
            if (e != hipSuccess) return fail(ADMM_TV_EHIP, std::string("k_mt_mixed: ") + hipGetErrorString(e));
        }
    }
    return 0;
}

int pow2_floor(int v);

int strip_rows(int H, int N, long long rows, bool aniso_fwd = false) {
    int R = env_int("ADMM_PASSA_R", 0);
    // A/B knob: a strip must tile H exactly (pass A maps strip -> (plane, first row) by H / R),
    // so an override is rounded down to a power of two in [2, H]; <= 0 selects the rule below
    if (R > 0) R = pow2_floor(std::max(2, std::min(R, H)));
    if (R <= 0) {
        // rows per strip (measured on MI355X, tools/sweep.py: R = 8 beats 16 at W = 1024 with
        // the 3-waves/SIMD row pass); halve while there are fewer than ~3 waves per SIMD of
        // strips.  The aniso forward at W = 512 (with the XCD strip remap) takes R = 16 down to
        // ~1.5 waves per SIMD of strips: C2 pass A 0.126 -> 0.120 ms; the iso row pass there
        // keeps the rule (C5 module: R = 4 best).
        const int L = std::min(64, N / (N >= 1024 ? 16 : N >= 64 ? 8 : N >= 16 ? 4 : 2));
        long long want = 3LL * 1024 * 64 / L;
        R = 8;
        if (aniso_fwd && N == 256) {
            R = 16;
            want /= 2;
        }
        while (R > 2 && rows / R < want) R /= 2;
    }
    if (R > H) R = H;
    return R;
}

// The device a call runs on is the device of its stream (the legacy default stream: the current
// device).  Every entry point switches to it for the duration of the call and switches back, so
// an input on cuda:1 solved while the current device is 0 launches, records and waits on device 1.
struct DeviceGuard {
    int prev = -1, dev = -1;
    hipError_t err = hipSuccess;
    explicit DeviceGuard(hipStream_t s) {
        err = hipGetDevice(&prev);
        if (err != hipSuccess) return;
        dev = prev;
        if (s) {
            hipDevice_t d = 0;
            err = hipStreamGetDevice(s, &d);
            if (err != hipSuccess) return;
            dev = (int)d;
        }
        if (dev != prev) err = hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0 && dev != prev) (void)hipSetDevice(prev);
    }
};

// Auxiliary streams of the two-stream solves, one per (device, caller stream): two solves on
// independent caller streams keep independent auxiliary streams (no false dependency between
// them), and every thread that uses the same caller stream shares its auxiliary stream (no
// per-thread leak).  Bounded: beyond kAuxPerDev caller streams per device the entries are reused
// round-robin (a reused entry only adds ordering, never a hazard).  The streams live until the
// process ends (destroying them from a static destructor could race the HIP runtime's teardown).
constexpr int kMaxAux = 3;  // auxiliary streams per caller stream (solves on up to 4 streams)
struct AuxEntry {
    hipStream_t caller = nullptr, aux[kMaxAux] = {};
};
constexpr int kAuxDev = 64, kAuxPerDev = 32;
struct AuxPool {
    std::mutex mu;
    AuxEntry e[kAuxDev][kAuxPerDev];
    int used[kAuxDev] = {}, next[kAuxDev] = {};
} g_aux;

// the k-th auxiliary stream (k < kMaxAux) paired with caller stream s on device dev (the current
// device, see DeviceGuard), created on first use
hipStream_t aux_stream(hipStream_t s, int dev, int k = 0) {
    if (dev < 0 || dev >= kAuxDev || k < 0 || k >= kMaxAux) return nullptr;
    std::lock_guard<std::mutex> lk(g_aux.mu);
    AuxEntry* row = g_aux.e[dev];
    AuxEntry* slot = nullptr;
    for (int i = 0; i < g_aux.used[dev] && !slot; ++i)
        if (row[i].caller == s) slot = &row[i];
    if (!slot) {
        if (g_aux.used[dev] < kAuxPerDev) {
            slot = &row[g_aux.used[dev]++];
        } else {
            slot = &row[g_aux.next[dev]];
            g_aux.next[dev] = (g_aux.next[dev] + 1) % kAuxPerDev;
        }
        slot->caller = s;
    }
    if (!slot->aux[k] && hipStreamCreateWithFlags(&slot->aux[k], hipStreamNonBlocking) != hipSuccess) {
        slot->aux[k] = nullptr;
        return nullptr;
    }
    return slot->aux[k];
}

// fork / join of a solve on several streams: the auxiliary streams start after the work already
// queued on s, and s waits for everything queued on them -- also when a part fails after the fork
// (every join is issued)
struct ForkJoin {
    hipStream_t s;
    std::vector<hipStream_t> aux;
    hipEvent_t fork = nullptr;
    std::vector<hipEvent_t> joins;
    hipError_t err = hipSuccess;
    ForkJoin(hipStream_t a, std::vector<hipStream_t> b) : s(a), aux(std::move(b)), joins(aux.size(), nullptr) {
        if ((err = hipEventCreateWithFlags(&fork, hipEventDisableTiming)) != hipSuccess) return;
        for (auto& j : joins)
            if ((err = hipEventCreateWithFlags(&j, hipEventDisableTiming)) != hipSuccess) return;
        if ((err = hipEventRecord(fork, s)) != hipSuccess) return;
        for (hipStream_t x : aux)
            if ((err = hipStreamWaitEvent(x, fork, 0)) != hipSuccess) return;
    }
    hipError_t finish() {
        hipError_t first = hipSuccess;
        for (size_t i = 0; i < aux.size(); ++i) {
            hipError_t e = hipEventRecord(joins[i], aux[i]);
            if (e == hipSuccess) e = hipStreamWaitEvent(s, joins[i], 0);
            if (first == hipSuccess) first = e;
        }
        return first;
    }
    ~ForkJoin() {
        if (fork) (void)hipEventDestroy(fork);
        for (hipEvent_t j : joins)
            if (j) (void)hipEventDestroy(j);
    }
};

// split of P planes into up to ns parts for the generic row kernels, which transform real rows in
// pairs (rows 2c, 2c + 1 of a launch's range): every part but the last must hold an even number of
// rows, or the pairs of the parts after it would shift and the results would differ in the last
// bits from a one-stream solve.  Returns the parts' first planes (one entry: no split).
std::vector<long long> gen_parts(long long P, int H, int ns) {
    long long c = (P + ns - 1) / std::max(ns, 1);
    if (H & 1) c += c & 1;  // an even plane count per part when H is odd
    std::vector<long long> starts;
    for (long long p = 0; p < P; p += std::max(c, 1LL)) starts.push_back(p);
    return starts;
}


// b = H_t(xin) into `bb` through the FFT passes (scratch: spec)
int psf_transpose_into(const admm_tv_desc& d, const Layout& Lo, void* ws, const float* xin, float* bb, cf* spec,
                       int mode, hipStream_t s, bool pl = false) {
    const long long rows = d.B * d.C * d.H;
    const int H = (int)d.H, N = (int)d.W / 2;
    cf* twW = at<cf>(ws, Lo.twW);
    int e = with_row(N, [&](auto ops) { return decltype(ops)::r2c(xin, spec, twW, rows, s); });
    if (e) return e;
    if ((e = pass_b(H, spec, at<float>(ws, Lo.fcT), at<cf>(ws, Lo.mT), at<cf>(ws, Lo.twH), N, (int)(d.B * d.C), mode, s)))
        return e;
    return with_row(N, [&](auto ops) { return decltype(ops)::c2r(spec, bb, twW, rows, s, pl); });
}


// ------------------------------------------------------------------ generic sizes (generic_kernels.hpp)
GPlan make_plan_radices(int n);

// Bluestein stages (generic_kernels.hpp gstage_blue): a prime radix R >= ADMM_BLUE_MIN (default
// below) with 2R - 1 <= 1024 runs as a chirp-z transform on the register-resident power-of-two FFT;
// larger primes keep the O(R)-per-output stage.  ADMM_BLUE_MIN <= 0 disables it (A/B).
int blue_min() { return env_int("ADMM_BLUE_MIN", 41); }

constexpr size_t kMaxLds = 160 * 1024;
// LDS bytes of a generic transform kernel: twiddles + tables, two line buffers, Bluestein exchange
// (csz: bytes of a complex element, 16 for the fp64 kernels)
size_t glds(int n, int lines, const GPlan& p, size_t csz = sizeof(cf)) {
    if (p.glb) return 0;  // the line buffers live in global scratch
    return csz * ((p.twg ? 0 : (size_t)n + p.ntab) + 2 * (size_t)n * lines + p.xslots);
}

// long-line blocks (GPlan::glb): scratch slots (resident blocks walking their items grid-stride) and
// the bytes of the scratch region a solve needs for its longer dimension
constexpr long long kGlbSlots = 1024;
constexpr size_t kGlbBudget = 512ull << 20;
long long glb_slots(int n, size_t csz) {
    return std::max<long long>(64, std::min<long long>(kGlbSlots, (long long)(kGlbBudget / (2 * (size_t)n * csz))));
}

// fp64 plan: any prime > 5 first (its stage at NS = 1 needs no twiddle pass), then radices 4, 2, 3, 5
// (the radices the double kernels have butterflies for; no Bluestein stages); twiddles from global
// memory when a line's LDS image would not fit
GPlan make_plan_f64(int n) {
    GPlan p{};
    p.n = n;
    int m = n, r = n;
    auto take_all = [&](int q) {
        while (m % q == 0 && m > 1) {
            p.rad[p.nst++] = q;
            m /= q;
        }
    };
    for (int q : {2, 3, 5})
        while (r % q == 0) r /= q;
    for (int f = 7; f * f <= r; f += 2)
        if (r % f == 0) {
            take_all(f);
            while (r % f == 0) r /= f;
        }
    if (r > 1) take_all(r);
    take_all(4);
    take_all(2);
    take_all(3);
    take_all(5);
    p.twg = glds(n, 1, p, sizeof(double2)) > kMaxLds ? 1 : 0;
    p.glb = (p.twg && glds(n, 1, p, sizeof(double2)) > kMaxLds) ? 1 : 0;
    return p;
}

GPlan make_plan(int n, bool f64) {
    if (f64) return make_plan_f64(n);
    GPlan p = make_plan_radices(n);
    const int bmin = blue_min();
    int M = 0;  // one Bluestein size for the plan: M = 2^k >= 2R - 1 for its largest such prime
    for (int s = 0; s < p.nst; ++s) {
        const int R = p.rad[s];
        if (bmin <= 0 || R <= 7 || (R & (R - 1)) == 0 || R < bmin || 2 * R - 1 > 1024) continue;  // primes only
        int m = 32;
        while (m < 2 * R - 1) m *= 2;
        M = std::max(M, m);
    }
    int off = n;
    for (int s = 0; s < p.nst; ++s) {
        const int R = p.rad[s];
        const bool blue = M > 0 && R > 7 && (R & (R - 1)) != 0 && R >= bmin && 2 * R - 1 <= 1024;
        p.bst[s] = blue ? M : 0;
        p.boff[s] = blue ? off : 0;
        if (blue) off += R + 2 * M;
    }
    p.bm = M;
    p.ntab = off - n;
    p.xslots = M > 0 ? (GNT / (M / blue_e(M))) * (M + M / 8) : 0;
    // one line must fit the LDS: else no Bluestein, else twiddles from global memory, else the
    // line buffers too (a global scratch slot per block)
    if (glds(n, 1, p) <= kMaxLds) return p;
    GPlan q = make_plan_radices(n);
    q.twg = glds(n, 1, q) > kMaxLds ? 1 : 0;
    if (q.twg && glds(n, 1, q) > kMaxLds) q.glb = 1;
    return q;
}

bool gen_fits(int n, bool f64) {
    return n >= 1 && n <= kGenericMax && glds(n, 1, make_plan(n, f64), f64 ? sizeof(double2) : sizeof(cf)) <= kMaxLds;
}
// (as many slots as a launch of that dimension uses: min(slots, its items) -- gen_grid)
size_t glb_scratch(int H, int W, long long P, bool f64) {
    const size_t csz = f64 ? sizeof(double2) : sizeof(cf);
    size_t b = 0;
    if (make_plan(W, f64).glb)  // row transforms: two real rows per item
        b = std::max(b, (size_t)std::min(glb_slots(W, csz), (P * H + 1) / 2) * 2 * (size_t)W * csz);
    if (make_plan(H, f64).glb)  // column pass: one column per item
        b = std::max(b, (size_t)std::min(glb_slots(H, csz), P * (W / 2 + 1)) * 2 * (size_t)H * csz);
    return b;
}

// threads per block of the generic transform kernels (A/B knob; 64, 128 or 256)
int gen_threads(const char* knob) {
    const int v = env_int(knob, GNT);
    return v <= 64 ? 64 : v <= 128 ? 128 : v <= 256 || GNT <= 256 ? 256 : GNT;
}

// long lines without Bluestein stages run their transform blocks with 512 threads (a 1,920-point
// row's stages have 480-960 butterflies; 256 threads leave them latency-bound: HD 1080x1920
// 716 -> 850 it/s; BSD-like lines with Bluestein stages are faster at 256).  ADMM_GEN_WIDE_MIN:
// the line length from which it applies (0: never).
constexpr int kGenWide = 512;
bool gen_wide(int n, const GPlan& p) {
    const int mn = env_int("ADMM_GEN_WIDE_MIN", 1024);
    return p.bm == 0 && mn > 0 && n >= mn;
}

// f(integral_constant BM, bool_constant TWG, bool_constant GLB)
template <class F> int with_plan(const GPlan& p, F&& f) {
    if (p.glb) return f(std::integral_constant<int, 0>{}, std::true_type{}, std::true_type{});
    if (p.twg) return f(std::integral_constant<int, 0>{}, std::true_type{}, std::false_type{});
    return with_bm(p.bm, [&](auto bm) { return f(bm, std::false_type{}, std::false_type{}); });
}

// the kernel instantiation for a plan's Bluestein size
template <class F> int with_bm(int bm, F&& f) {
    // f(integral_constant BM, bool_constant TWG): global-memory twiddles only on plans without Bluestein
    switch (bm) {
        case 0: return f(std::integral_constant<int, 0>{});
        case 32: return f(std::integral_constant<int, 32>{});
        case 64: return f(std::integral_constant<int, 64>{});
        case 128: return f(std::integral_constant<int, 128>{});
        case 256: return f(std::integral_constant<int, 256>{});
        case 512: return f(std::integral_constant<int, 512>{});
        case 1024: return f(std::integral_constant<int, 1024>{});
        default: return fail(ADMM_TV_EUNSUPPORTED, "generic plan: Bluestein size");
    }
}

GPlan make_plan_radices(int n) {
    GPlan p{};
    p.n = n;
    int m = n;
    auto take_all = [&](int r) {
        while (m % r == 0 && m > 1) {
            p.rad[p.nst++] = r;
            m /= r;
        }
    };
    if (env_int("ADMM_GPLAN_PRIME_FIRST", 1)) {
        // any other prime first: at NS = 1 its stage needs no twiddle pass (BSD size: column pass
        // 122 -> 112 ms per 250 launches, 1,410 -> 1,491 it/s)
        // (the primes >= 11 of n by trial division of n stripped of 2, 3, 5, 7: O(sqrt n))
        int r = n;
        // (11 and 13 run as compile-time butterflies like 3, 5, 7: after the powers of two)
        for (int q : {2, 3, 5, 7, 11, 13})
            while (r % q == 0) r /= q;
        for (int f = 11; f * f <= r; f += 2)
            if (r % f == 0) {
                take_all(f);
                while (r % f == 0) r /= f;
            }
        if (r > 1) take_all(r);
        // powers of two as radix-16 / 8 stages (one LDS round trip per 16 / 8 instead of two /
        // three radix-4 / 2 ones); ADMM_GPLAN_R16=0 for the radix-4/2 plan (A/B)
        if (env_int("ADMM_GPLAN_R16", 1)) {
            take_all(16);
            take_all(8);
        }
        take_all(4);
        take_all(2);
        take_all(3);
        take_all(5);
        take_all(7);
        take_all(11);
        take_all(13);
        return p;
    }
    take_all(4);
    take_all(2);
    take_all(3);
    take_all(5);
    take_all(7);
    take_all(11);
    take_all(13);
    for (int f = 17; f * f <= m; f += 2) take_all(f);  // any other prime: O(R) per output
    if (m > 1) take_all(m);
    return p;
}

// complex rows (= 2 real rows each) per block of the row transforms / columns per block of
// the column pass
// (powers of two, so the per-item line index is a shift)
int pow2_floor(int v) { int p = 1; while (2 * p <= v) p *= 2; return p; }
// LDS image <= ~32 KB (4+ resident blocks per CU: the prime-radix stages are latency-bound
// chains and need the waves), except where one line alone is bigger
// (A/B knobs ADMM_GROW_LINES / ADMM_GCOL_COLS: rounded down to a power of two in [1, 32])
// With Bluestein stages the column pass takes at least as many columns as make one item per
// sub-group (16x3x509^2: 2 -> 4 columns, 1,125 -> 1,368 it/s; BSD keeps 4).  Either count is
// halved until the block's LDS fits.
int fit_lines(int n, int lines, const GPlan& p, size_t csz = sizeof(cf)) {
    while (lines > 1 && glds(n, lines, p, csz) > kMaxLds) lines /= 2;
    return lines;
}
int grow_lines(int W, const GPlan& p, size_t csz = sizeof(cf)) {
    if (p.glb) return 1;  // one line per scratch slot
    if (csz != sizeof(cf)) return fit_lines(W, pow2_floor(std::max(1, std::min(32, (2048 / W - 1) / 2))), p, csz);
    const int dflt = pow2_floor(std::max(1, std::min(32, (4096 / W - 1) / 2)));
    return fit_lines(W, pow2_floor(std::max(1, std::min(32, env_int("ADMM_GROW_LINES", dflt)))), p);
}
int gcol_cols(int H, const GPlan& p, size_t csz = sizeof(cf)) {
    if (p.glb) return 1;
    if (csz != sizeof(cf)) return fit_lines(H, pow2_floor(std::max(1, std::min(16, (3072 / H - 1) / 2))), p, csz);
    // column blocks: ~48 KB LDS images without Bluestein stages (VGA 480: 2 -> 4 columns +7 %,
    // 500: +4 %, HD 1080: 1 -> 2 columns +6 %; tools/bench_generic_sizes.py), ~32 KB with them
    int dflt = pow2_floor(std::max(1, std::min(16, ((p.bm > 0 ? 4096 : 6144) / H - 1) / 2)));
    if (p.bm > 0) {
        int nb = H;  // butterflies per line of the Bluestein stages (fewest)
        for (int s = 0; s < p.nst; ++s)
            if (p.bst[s] > 0) nb = std::min(nb, H / p.rad[s]);
        const int nsg = GNT / (p.bm / blue_e(p.bm));
        while (dflt * nb < nsg && dflt < 16) dflt *= 2;
    }
    return fit_lines(H, pow2_floor(std::max(1, std::min(32, env_int("ADMM_GCOL_COLS", dflt)))), p);
}

// matrix-core column pass plan (gcol_mm.hpp).  A/B knobs: ADMM_GCOL_MM=0 keeps the LDS column pass,
// ADMM_GCOL_MM_NL the columns per block (8 or 16)
MMPlan mm_plan(int H, int W) {
    MMPlan m{};
    if (!env_int("ADMM_GCOL_MM", 1) || H < 17) return m;
    int r = H, big = 1;  // largest prime factor of H
    for (int f = 2; f * f <= r; ++f)
        while (r % f == 0) {
            big = std::max(big, f);
            r /= f;
        }
    big = std::max(big, r);
    if (big < 17 || big > 127) return m;
    for (int S = 1; S <= 8; ++S) {
        if (S == 7 || H % S) continue;  // instances: S = 1..6, 8
        const int R = H / S;
        if (R > 127 || !(R & 1) || R % big) continue;
        m.R = R;
        m.S = S;
        break;
    }
    if (!m.R) return m;
    m.h = (m.R - 1) / 2;
    m.KS = (m.h + 1 + 3) / 4;
    m.MT = (m.h + 1 + 15) / 16;
    const int G = m.MT == 3 ? 1 : 4 / m.MT;
    int NL = env_int("ADMM_GCOL_MM_NL", 16) >= 16 ? 16 : 8;
    // n-tiles of 16 real columns: ceil(NL S / 8) of them (the last one padded), at most 8 per wave (the
    // accumulator arrays)
    while (NL > 1 && ((NL * m.S + 7) / 8 + G - 1) / G > 8) NL /= 2;
    if (((NL * m.S + 7) / 8 + G - 1) / G > 8) return m;
    m.NL = NL;
    m.RP = std::max(4 * NL * m.S, 32 * ((NL * m.S + 7) / 8));
    while (m.RP % 64 != 32) m.RP += 16;
    m.lds = (size_t)4 * m.KS * m.RP * sizeof(float) + (size_t)H * sizeof(cf);  // image + twiddles
    m.ok = m.lds <= kMaxLds;
    (void)W;
    return m;
}

// row inverse on the matrix cores: lines (row pairs) per block NL, one (line, k1) item per thread,
// at most 8 n-tiles per wave.  A/B knob: ADMM_GROW_MM=0 keeps the LDS row inverse.
MMPlan mm_plan_row(int W) {
    MMPlan m{};
    if (!env_int("ADMM_GROW_MM", 1) || W < 17) return m;
    int r = W, big = 1;
    for (int f = 2; f * f <= r; ++f)
        while (r % f == 0) {
            big = std::max(big, f);
            r /= f;
        }
    big = std::max(big, r);
    if (big < 17 || big > 127) return m;
    for (int S : {1, 2, 3, 4, 5, 8, 13}) {
        if (W % S) continue;
        const int R = W / S;
        if (R > 127 || !(R & 1) || R % big) continue;
        m.R = R;
        m.S = S;
        break;
    }
    if (!m.R) return m;
    m.h = (m.R - 1) / 2;
    m.KS = (m.h + 1 + 3) / 4;
    m.MT = (m.h + 1 + 15) / 16;
    const int G = m.MT == 3 ? 1 : 4 / m.MT;
    // 256-thread blocks; A/B knob ADMM_GROW_MM_NT=512: 2 G waves per row tile, at most 4 n-tiles per wave
    // (BSD two streams 4,281-4,310 -> 4,130 it/s, profiles/r03_grow_inv_mm_nt.txt)
    m.nth = env_int("ADMM_GROW_MM_NT", 256) == 512 ? 512 : 256;
    const int Gt = m.nth == 512 ? 2 * G : G, maxt = m.nth == 512 ? 4 : 8;
    int NL = 16;
    while (NL > 1 && (NL * (m.h + 1) > m.nth || ((NL * m.S + 7) / 8 + Gt - 1) / Gt > maxt)) NL /= 2;
    if (NL * (m.h + 1) > m.nth || ((NL * m.S + 7) / 8 + Gt - 1) / Gt > maxt) return m;  // one (line, k1) item per thread
    m.NL = NL;
    m.RP = std::max(4 * NL * m.S, 32 * ((NL * m.S + 7) / 8));
    while (m.RP % 64 != 32) m.RP += 16;
    const size_t stage = (size_t)2 * NL * (W / 2 + 1) * 2;  // floats
    m.lds = std::max(stage, (size_t)4 * m.KS * m.RP) * sizeof(float) + (size_t)W * sizeof(cf);
    m.ok = m.lds <= kMaxLds;
    return m;
}


// the launchers below are templated on the real type T of the solve: float, or double for fp64
// inputs (ADMM_TV_FLAG_F64: the generic kernels' double instantiation, plans without Bluestein
// stages, 256-thread blocks)
template <class T> constexpr bool kF64 = std::is_same<T, double>::value;
template <class T> constexpr size_t kCsz = sizeof(cx_t<T>);

// f(integral_constant BM, bool_constant TWG) for a plan: the fp64 kernels exist for BM = 0 only
template <class T, class F> int with_plan_t(const GPlan& p, F&& f) {
    if constexpr (kF64<T>) {
        if (p.bm != 0) return fail(ADMM_TV_EUNSUPPORTED, "fp64 plan with a Bluestein stage");
        if (p.glb) return f(std::integral_constant<int, 0>{}, std::true_type{}, std::true_type{});
        if (p.twg) return f(std::integral_constant<int, 0>{}, std::true_type{}, std::false_type{});
        return f(std::integral_constant<int, 0>{}, std::false_type{}, std::false_type{});
    } else {
        return with_plan(p, f);
    }
}
// grid of a transform launch: one block per item, or (long lines) the scratch slots walking them
inline dim3 gen_grid(long long items, const GPlan& p, size_t csz) {
    return dim3((unsigned)(p.glb ? std::min(items, glb_slots(p.n, csz)) : items));
}

#define GLB_CHECK(pl, gscr)                                                                          \
    if ((pl).glb && !(gscr)) return fail(ADMM_TV_EINVAL, "long lines: no scratch region");
template <class T>
int grow_fwd(const T* img, cx_t<T>* spec, const cx_t<T>* tw, int W, long long rows, hipStream_t s,
             cx_t<T>* gscr = nullptr, int ldw = 0) {
    const GPlan pl = make_plan(W, kF64<T>);
    GLB_CHECK(pl, gscr)
    GRowArgsT<T> a{img, spec, nullptr, tw, pl, rows, grow_lines(W, pl, kCsz<T>), gscr, ldw};
    const size_t lds = glds(W, a.lines, a.plan, kCsz<T>);
    return with_plan_t<T>(a.plan, [&](auto bm, auto twg, auto glb) {
        constexpr int BM = decltype(bm)::value;
        constexpr bool TWG = decltype(twg)::value, GLB = decltype(glb)::value;
        const dim3 grid = gen_grid((rows + 2 * a.lines - 1) / (2 * a.lines), pl, kCsz<T>);
        if constexpr (BM == 0 && !kF64<T> && !GLB) {
            if (gen_wide(W, pl)) {
                if (int e = set_lds(k_grow_fwd<BM, TWG, kGenWide>, lds)) return e;
                hipLaunchKernelGGL((k_grow_fwd<BM, TWG, kGenWide>), grid, dim3(kGenWide), lds, s, a);
                return launch_check("k_grow_fwd");
            }
        }
        if (int e = set_lds(k_grow_fwd<BM, TWG, GNT, T, GLB>, lds)) return e;
        hipLaunchKernelGGL((k_grow_fwd<BM, TWG, GNT, T, GLB>), grid,
                           dim3(kF64<T> || GLB ? GNT : gen_threads("ADMM_GROW_NT")), lds, s, a);
        return launch_check("k_grow_fwd");
    });
}
// the step fused into the row transform of r (k_grow_fwd_step; inference iterations)
template <bool ISO, bool FIRST, class T>
int grow_fwd_step_t(const GStepArgsT<T>& g, cx_t<T>* spec, const cx_t<T>* tw, int W, long long rows, hipStream_t s,
                    cx_t<T>* gscr, int ldw) {
    const GPlan pl = make_plan(W, kF64<T>);
    GLB_CHECK(pl, gscr)
    GRowArgsT<T> a{nullptr, spec, nullptr, tw, pl, rows, grow_lines(W, pl, kCsz<T>), gscr, ldw};
    const size_t lds = glds(W, a.lines, a.plan, kCsz<T>);
    return with_plan_t<T>(a.plan, [&](auto bm, auto twg, auto glb) {
        constexpr int BM = decltype(bm)::value;
        constexpr bool TWG = decltype(twg)::value, GLB = decltype(glb)::value;
        const dim3 grid = gen_grid((rows + 2 * a.lines - 1) / (2 * a.lines), pl, kCsz<T>);
        if constexpr (BM == 0 && !kF64<T> && !GLB) {
            if (gen_wide(W, pl)) {
                if (int e = set_lds(k_grow_fwd_step<BM, TWG, ISO, FIRST, kGenWide>, lds)) return e;
                hipLaunchKernelGGL((k_grow_fwd_step<BM, TWG, ISO, FIRST, kGenWide>), grid, dim3(kGenWide), lds, s, a, g);
                return launch_check("k_grow_fwd_step");
            }
        }
        if (int e = set_lds(k_grow_fwd_step<BM, TWG, ISO, FIRST, GNT, T, GLB>, lds)) return e;
        hipLaunchKernelGGL((k_grow_fwd_step<BM, TWG, ISO, FIRST, GNT, T, GLB>), grid,
                           dim3(kF64<T> || GLB ? GNT : gen_threads("ADMM_GROW_NT")), lds, s, a, g);
        return launch_check("k_grow_fwd_step");
    });
}
template <class T>
int grow_fwd_step(const GStepArgsT<T>& g, cx_t<T>* spec, const cx_t<T>* tw, int W, long long rows, bool iso,
                  bool first, hipStream_t s, cx_t<T>* gscr = nullptr, int ldw = 0) {
    if (iso) return first ? grow_fwd_step_t<true, true>(g, spec, tw, W, rows, s, gscr, ldw)
                          : grow_fwd_step_t<true, false>(g, spec, tw, W, rows, s, gscr, ldw);
    return first ? grow_fwd_step_t<false, true>(g, spec, tw, W, rows, s, gscr, ldw)
                 : grow_fwd_step_t<false, false>(g, spec, tw, W, rows, s, gscr, ldw);
}
template <int S> int grow_inv_mm_launch(const GRowInvMMArgs& a, size_t lds, int nth, hipStream_t s) {
    const dim3 grid((unsigned)((a.rows + 2 * a.NL - 1) / (2 * a.NL)));
    if (nth == 512) {
        if (int e = set_lds(k_grow_inv_mm<S, 512>, lds)) return e;
        hipLaunchKernelGGL((k_grow_inv_mm<S, 512>), grid, dim3(512), lds, s, a);
        return launch_check("k_grow_inv_mm");
    }
    if (int e = set_lds(k_grow_inv_mm<S>, lds)) return e;
    hipLaunchKernelGGL(k_grow_inv_mm<S>, grid, dim3(256), lds, s, a);
    return launch_check("k_grow_inv_mm");
}
// mmr: the layout's row-inverse plan (Layout::mmr)
template <class T>
int grow_inv(const cx_t<T>* spec, T* img, const cx_t<T>* tw, int W, long long rows, hipStream_t s,
             cx_t<T>* gscr, const MMPlan& mmr, int ldw = 0) {
    if constexpr (!kF64<T>) {
        const MMPlan m = mmr;
        if (m.ok && rows > 0) {
            const int Wh = W / 2 + 1;
            GRowInvMMArgs a{spec, img, tw, rows, W, m.R, m.h, m.KS, m.MT, m.NL, m.RP, Wh, 2 * m.NL * Wh * 2,
                            ldw ? ldw : Wh};
            switch (m.S) {
                case 1: return grow_inv_mm_launch<1>(a, m.lds, m.nth, s);
                case 2: return grow_inv_mm_launch<2>(a, m.lds, m.nth, s);
                case 3: return grow_inv_mm_launch<3>(a, m.lds, m.nth, s);
                case 4: return grow_inv_mm_launch<4>(a, m.lds, m.nth, s);
                case 5: return grow_inv_mm_launch<5>(a, m.lds, m.nth, s);
                case 8: return grow_inv_mm_launch<8>(a, m.lds, m.nth, s);
                default: return grow_inv_mm_launch<13>(a, m.lds, m.nth, s);
            }
        }
    }
    const GPlan pl = make_plan(W, kF64<T>);
    GLB_CHECK(pl, gscr)
    GRowArgsT<T> a{nullptr, const_cast<cx_t<T>*>(spec), img, tw, pl, rows, grow_lines(W, pl, kCsz<T>), gscr, ldw};
    const size_t lds = glds(W, a.lines, a.plan, kCsz<T>);
    return with_plan_t<T>(a.plan, [&](auto bm, auto twg, auto glb) {
        constexpr int BM = decltype(bm)::value;
        constexpr bool TWG = decltype(twg)::value, GLB = decltype(glb)::value;
        const dim3 grid = gen_grid((rows + 2 * a.lines - 1) / (2 * a.lines), pl, kCsz<T>);
        if constexpr (BM == 0 && !kF64<T> && !GLB) {
            if (gen_wide(W, pl)) {
                if (int e = set_lds(k_grow_inv<BM, TWG, kGenWide>, lds)) return e;
                hipLaunchKernelGGL((k_grow_inv<BM, TWG, kGenWide>), grid, dim3(kGenWide), lds, s, a);
                return launch_check("k_grow_inv");
            }
        }
        if (int e = set_lds(k_grow_inv<BM, TWG, GNT, T, GLB>, lds)) return e;
        hipLaunchKernelGGL((k_grow_inv<BM, TWG, GNT, T, GLB>), grid,
                           dim3(kF64<T> || GLB ? GNT : gen_threads("ADMM_GROW_NT")), lds, s, a);
        return launch_check("k_grow_inv");
    });
}

template <int MODE, int BM, bool TWG, bool GLB, class T>
int gcol_launch(const GColArgsT<T>& a, size_t lds, dim3 grid, hipStream_t s) {
    if constexpr (BM == 0 && !kF64<T> && !GLB) {
        if (gen_wide(a.plan.n, a.plan)) {
            if (int e = set_lds(k_gcol<MODE, BM, TWG, kGenWide>, lds)) return e;
            hipLaunchKernelGGL((k_gcol<MODE, BM, TWG, kGenWide>), grid, dim3(kGenWide), lds, s, a);
            return launch_check("k_gcol");
        }
    }
    if (int e = set_lds(k_gcol<MODE, BM, TWG, GNT, T, GLB>, lds)) return e;
    hipLaunchKernelGGL((k_gcol<MODE, BM, TWG, GNT, T, GLB>), grid,
                       dim3(kF64<T> || GLB ? GNT : gen_threads("ADMM_GCOL_NT")), lds, s, a);
    return launch_check("k_gcol");
}
template <int S> int gcol_mm_launch(const GColMMArgs& a, size_t lds, hipStream_t s) {
    const dim3 grid((unsigned)(a.P * a.colblocks));
    // 512-thread blocks for S <= 4 (NL = 16: at most 8 n-tiles, 2+ waves per row tile -> at most 4 per
    // wave; BSD 4,191-4,230 -> 4,343-4,354 it/s, profiles/r03_gcol_mm_nt.txt); A/B knob ADMM_GCOL_MM_NT
    if constexpr (S <= 4) {
        if (a.NL == 16 && env_int("ADMM_GCOL_MM_NT", 512) == 512) {
            if (int e = set_lds(k_gcol_mm<S, 512>, lds)) return e;
            hipLaunchKernelGGL((k_gcol_mm<S, 512>), grid, dim3(512), lds, s, a);
            return launch_check("k_gcol_mm");
        }
    }
    if (int e = set_lds(k_gcol_mm<S>, lds)) return e;
    hipLaunchKernelGGL(k_gcol_mm<S>, grid, dim3(256), lds, s, a);
    return launch_check("k_gcol_mm");
}
// phase skips of the matrix-core column pass for timing experiments (results invalid): only in a
// library built with -DADMM_MM_DBG_BUILD=1 (tools/build_variant.sh), never from the environment of a
// product build
#ifndef ADMM_MM_DBG_BUILD
#define ADMM_MM_DBG_BUILD 0
#endif
inline int mm_dbg() { return ADMM_MM_DBG_BUILD ? env_int("ADMM_MM_DBG", 0) : 0; }

// mm: the layout's column-pass plan (Layout::mm; its factor copy was sized and written for it)
template <class T>
int gcol(cx_t<T>* spec, cx_t<T>* dump, const T* fcT, const cx_t<T>* mT, const cx_t<T>* tw, int H, int W, long long P,
         int mode, hipStream_t s, cx_t<T>* gscr, const MMPlan& mm, int ldw = 0) {
    if constexpr (!kF64<T>) {
        const MMPlan m = mm;
        if (mode == 0 && m.ok) {  // the factor's [H][Wh] copy follows fcT (setup, k_fc_transpose)
            const int Wh = W / 2 + 1;
            GColMMArgs a{spec, dump, fcT + (size_t)Wh * H, tw, H, m.R, m.h, m.KS, m.MT, m.NL, __builtin_ctz(m.NL), m.RP,
                         Wh, (Wh + m.NL - 1) / m.NL, P, mm_dbg(), ldw ? ldw : Wh};
            switch (m.S) {
                case 1: return gcol_mm_launch<1>(a, m.lds, s);
                case 2: return gcol_mm_launch<2>(a, m.lds, s);
                case 3: return gcol_mm_launch<3>(a, m.lds, s);
                case 4: return gcol_mm_launch<4>(a, m.lds, s);
                case 5: return gcol_mm_launch<5>(a, m.lds, s);
                case 6: return gcol_mm_launch<6>(a, m.lds, s);
                default: return gcol_mm_launch<8>(a, m.lds, s);
            }
        }
    }
    const GPlan pl = make_plan(H, kF64<T>);
    GLB_CHECK(pl, gscr)
    const int Wh = W / 2 + 1, cols = gcol_cols(H, pl, kCsz<T>);
    if (ldw && ldw != Wh) return fail(ADMM_TV_EINVAL, "padded spectrum pitch without the matrix-core column pass");
    const int colblocks = (Wh + cols - 1) / cols;
    GColArgsT<T> a{spec, dump, fcT, mT, tw, pl, Wh, cols, colblocks, P, gscr};
    const size_t lds = glds(H, cols, a.plan, kCsz<T>);
    const dim3 grid = gen_grid(P * colblocks, pl, kCsz<T>);
    return with_plan_t<T>(a.plan, [&](auto bm, auto twg, auto glb) {
        constexpr int BM = decltype(bm)::value;
        constexpr bool TWG = decltype(twg)::value, GLB = decltype(glb)::value;
        switch (mode) {
            case 0: return gcol_launch<0, BM, TWG, GLB>(a, lds, grid, s);
            case 1: return gcol_launch<1, BM, TWG, GLB>(a, lds, grid, s);
            case 2: return gcol_launch<2, BM, TWG, GLB>(a, lds, grid, s);
            default: return gcol_launch<3, BM, TWG, GLB>(a, lds, grid, s);
        }
    });
}
// img_out = real part of the 2-D transform chain  rowFFT -> column pass (mode) -> rowIFFT  of img_in
template <class T>
int gapply(const T* img_in, T* img_out, cx_t<T>* spec, const Layout& Lo, void* ws, const admm_tv_desc& d, int mode,
           hipStream_t s) {
    using C = cx_t<T>;
    const long long P = d.B * d.C, rows = P * d.H;
    const int H = (int)d.H, W = (int)d.W;
    C* twW = at<C>(ws, Lo.twW);
    C* gs = at<C>(ws, Lo.gscr);
    if (int e = grow_fwd(img_in, spec, twW, W, rows, s, gs)) return e;
    if (int e = gcol<T>(spec, nullptr, at<T>(ws, Lo.fcT), at<C>(ws, Lo.mT), at<C>(ws, Lo.twH), H, W, P, mode, s, gs,
                        Lo.mm))
        return e;
    return grow_inv<T>(spec, img_out, twW, W, rows, s, gs, Lo.mmr);
}

template <class T> int gstep(const GStepArgsT<T>& a, bool iso, bool first, bool hist, hipStream_t s) {
    // one block row per image row (P H <= 2^31 - 1 rows), column chunks of 256 pixels
    const long long rows = a.npx / a.W;
    if (rows <= 0) return 0;
    if (rows > 0x7fffffffLL) return fail(ADMM_TV_EUNSUPPORTED, "too many image rows for the generic step kernel");
    const dim3 grid((unsigned)rows, (unsigned)((a.W + 255) / 256)), blk(256);
    const int sel = (iso ? 4 : 0) | (first ? 2 : 0) | (hist ? 1 : 0);
    switch (sel) {
        case 0: hipLaunchKernelGGL((k_gstep<false, false, false, T>), grid, blk, 0, s, a); break;
        case 1: hipLaunchKernelGGL((k_gstep<false, false, true, T>), grid, blk, 0, s, a); break;
        case 2: hipLaunchKernelGGL((k_gstep<false, true, false, T>), grid, blk, 0, s, a); break;
        case 3: hipLaunchKernelGGL((k_gstep<false, true, true, T>), grid, blk, 0, s, a); break;
        case 4: hipLaunchKernelGGL((k_gstep<true, false, false, T>), grid, blk, 0, s, a); break;
        case 5: hipLaunchKernelGGL((k_gstep<true, false, true, T>), grid, blk, 0, s, a); break;
        case 6: hipLaunchKernelGGL((k_gstep<true, true, false, T>), grid, blk, 0, s, a); break;
        default: hipLaunchKernelGGL((k_gstep<true, true, true, T>), grid, blk, 0, s, a); break;
    }
    return launch_check("k_gstep");
}

template <class T> int gbwd(const GBwdArgsT<T>& a, bool iso, bool lastk, bool firstk, hipStream_t s) {
    const dim3 grid((unsigned)((a.npx + 255) / 256)), blk(256);
    const int sel = (iso ? 4 : 0) | (lastk ? 2 : 0) | (firstk ? 1 : 0);
    switch (sel) {
        case 0: hipLaunchKernelGGL((k_gbwd<false, false, false, T>), grid, blk, 0, s, a); break;
        case 1: hipLaunchKernelGGL((k_gbwd<false, false, true, T>), grid, blk, 0, s, a); break;
        case 2: hipLaunchKernelGGL((k_gbwd<false, true, false, T>), grid, blk, 0, s, a); break;
        case 3: hipLaunchKernelGGL((k_gbwd<false, true, true, T>), grid, blk, 0, s, a); break;
        case 4: hipLaunchKernelGGL((k_gbwd<true, false, false, T>), grid, blk, 0, s, a); break;
        case 5: hipLaunchKernelGGL((k_gbwd<true, false, true, T>), grid, blk, 0, s, a); break;
        case 6: hipLaunchKernelGGL((k_gbwd<true, true, false, T>), grid, blk, 0, s, a); break;
        default: hipLaunchKernelGGL((k_gbwd<true, true, true, T>), grid, blk, 0, s, a); break;
    }
    return launch_check("k_gbwd");
}

// history (training) storage: a_k for k = 1..K (x and y images), iso norms N_k
struct Hist {
    size_t a_slot;     // bytes of one image
    size_t t_slot;     // bytes of one kept spectrum (fast path: row spectra; generic: 2-D half spectra)
    size_t n_slot;     // bytes of one norm pair [2][H][W]
    size_t n_off;      // offset of the norm history
    size_t t_off;      // offset of the r_k spectra (PSF gradient only)
    bool keep_t;
    size_t total;
};
Hist make_hist(const admm_tv_desc& d) {
    Hist h{};
    const size_t rs = is_f64(d) ? sizeof(double) : sizeof(float);
    const size_t G = ngroups_of(d);
    const size_t img = G * d.B * d.C * d.H * d.W * rs;
    h.a_slot = up(img);
    h.n_slot = d.iso ? up(G * 2 * (size_t)d.H * d.W * rs) : 0;
    h.n_off = (size_t)d.maxit * 2 * h.a_slot;
    h.t_off = h.n_off + (size_t)d.maxit * h.n_slot;
    h.keep_t = d.kh > 0 && (d.flags & ADMM_TV_FLAG_PSF_GRAD);
    h.t_slot = (is_f64(d) || generic_hw(d.H, d.W)) ? up((size_t)d.B * d.C * d.H * (d.W / 2 + 1) * 2 * rs) : h.a_slot;
    h.total = h.t_off + (h.keep_t ? (size_t)d.maxit * h.t_slot : 0);
    return h;
}


// generic-size forward (same contract as run_forward; generic_kernels.hpp)
template <class T>
int run_forward_gen(const admm_tv_desc& d, const Layout& Lo, const T* xin, const T* lam, const T* rho, T* out, void* ws,
                    void* hist, hipStream_t s) {
    using C = cx_t<T>;
    const long long P = d.B * d.C;
    const int H = (int)d.H, W = (int)d.W;
    C* twW = at<C>(ws, Lo.twW);
    C* twH = at<C>(ws, Lo.twH);
    T* fcT = at<T>(ws, Lo.fcT);
    C* mT = at<C>(ws, Lo.mT);
    C* spec = at<C>(ws, Lo.spec[0]);
    C* gs = at<C>(ws, Lo.gscr);  // long lines: the transform blocks' scratch slots
    T* ximg = at<T>(ws, Lo.spec[1]);
    T* rimg = at<T>(ws, Lo.rimg);
    T* u[4] = {at<T>(ws, Lo.u[0]), at<T>(ws, Lo.u[1]), at<T>(ws, Lo.u[2]), at<T>(ws, Lo.u[3])};
    const bool train = hist != nullptr;
    const Hist Hs = make_hist(d);
    auto ha = [&](int k, int comp) -> T* {
        return reinterpret_cast<T*>(static_cast<char*>(hist) + (size_t)(2 * (k - 1) + comp) * Hs.a_slot);
    };
    auto hn = [&](int k) -> T* {
        return reinterpret_cast<T*>(static_cast<char*>(hist) + Hs.n_off + (size_t)(k - 1) * Hs.n_slot);
    };
    const bool keep_t = train && Hs.keep_t;  // PSF gradient: keep every r_k's 2-D spectrum
    auto ht = [&](int k) -> C* {
        return reinterpret_cast<C*>(static_cast<char*>(hist) + Hs.t_off + (size_t)(k - 1) * Hs.t_slot);
    };
    const T* bimg = xin;
    if (d.kh > 0) {  // b = H_t(xin) once
        ProfScope ps(3, s);
        T* bb = at<T>(ws, Lo.b);
        if (int e = gapply(xin, bb, spec, Lo, ws, d, 1, s)) return e;
        bimg = bb;
    }
    // the iteration loop over planes [p0, p0 + np) on stream st (every plane, or -- aniso inference,
    // whose planes are independent -- one half per stream, ADMM_GEN_STREAMS)
    auto solve_planes = [&](long long p0, long long np, hipStream_t st) -> int {
    // the inference iteration's spectrum pitch (Layout::ldw); training keeps Wh (its history layout)
    const int ld = train ? W / 2 + 1 : Lo.ldw;
    const size_t so = (size_t)p0 * H * ld, io = (size_t)p0 * H * W;  // cf / float offsets
    C* cspec = spec + so;
    T* cx = ximg + io;
    T* crimg = rimg + io;
    T* cout = out + io;
    const T* cb = bimg + io;
    const long long crows = np * H;
    {
        ProfScope ps(3, st);
        if (int e = grow_fwd(cb, cspec, twW, W, crows, st, gs, ld)) return e;  // r_1 = b
    }
    if constexpr (!kF64<T>) {
        if (Lo.odd && !train) {
            // the two-launch iteration (odd_kernels.hpp): the column pass in place on spec[cur], then pass A
            // (inverse rows, step, forward rows) from spec[cur] into spec[1 - cur]; u ping-pong as below
            C* sp[2] = {cspec, at<C>(ws, Lo.spec2) + so};
            const int rs = admm_odd::strip_rows(W);
            const int ns = (H + rs - 1) / rs;
            int cur = 0, ui = 0;
            for (int it = 1; it <= d.maxit; ++it) {
                {
                    ProfScope ps(1, st);
                    if (int e = gcol<T>(sp[cur], nullptr, fcT, mT, twH, H, W, np, 0, st, gs, Lo.mm, ld)) return e;
                }
                if (it == d.maxit) {
                    ProfScope ps(3, st);
                    return grow_inv<T>(sp[cur], cout, twW, W, crows, st, gs, Lo.mmr, ld);
                }
                ProfScope ps(0, st);
                OddPassAArgs oa{sp[cur], sp[1 - cur], cb, u[2 * ui] + io, u[2 * ui + 1] + io, u[2 * (1 - ui)] + io,
                                u[2 * (1 - ui) + 1] + io, lam, rho, H, ld, ns, np * ns};
                const hipError_t he = admm_odd::pass_a(W, oa, it == 1, st);
                if (he != hipSuccess) return fail(ADMM_TV_EHIP, std::string("k_pass_a_odd: ") + hipGetErrorString(he));
                cur = 1 - cur;
                ui = 1 - ui;
            }
            return 0;
        }
    }
    int uin = 0;
    for (int it = 1; it <= d.maxit; ++it) {
        const bool last = it == d.maxit;
        {
            ProfScope ps(1, st);
            if (int e = gcol<T>(cspec, keep_t ? ht(it) : nullptr, fcT, mT, twH, H, W, np, 0, st, gs, Lo.mm, ld)) return e;
            if (int e = grow_inv<T>(cspec, last ? cout : cx, twW, W, crows, st, gs, Lo.mmr, ld)) return e;
        }
        if (last && !train) break;
        const T* xk = last ? cout : cx;
        const bool first = it == 1;
        const T *uxi, *uyi, *nprev = nullptr;
        T *uxo, *uyo;
        if (train) {
            uxi = first ? nullptr : ha(it - 1, 0);
            uyi = first ? nullptr : ha(it - 1, 1);
            uxo = ha(it, 0);
            uyo = ha(it, 1);
            if (d.iso && !first) nprev = hn(it - 1);
        } else {
            uxi = u[2 * uin] + io;
            uyi = u[2 * uin + 1] + io;
            uxo = u[2 * (1 - uin)] + io;
            uyo = u[2 * (1 - uin) + 1] + io;
        }
        const T* nsq = nullptr;
        if (d.iso) {
            ProfScope ps(2, st);
            T* nout = train ? hn(it) : at<T>(ws, Lo.nsq);
            const long long hw = (long long)H * W;
            const dim3 grid((unsigned)((hw + 255) / 256)), blk(256);
            if (first)
                hipLaunchKernelGGL((k_giso_norm<true, false, T>), grid, blk, 0, st, xk, uxi, uyi, nprev, lam, rho, nout, H, W, np);
            else if (train)
                hipLaunchKernelGGL((k_giso_norm<false, true, T>), grid, blk, 0, st, xk, uxi, uyi, nprev, lam, rho, nout, H, W, np);
            else
                hipLaunchKernelGGL((k_giso_norm<false, false, T>), grid, blk, 0, st, xk, uxi, uyi, nprev, lam, rho, nout, H, W, np);
            if (int e = launch_check("k_giso_norm")) return e;
            allreduce(d, reinterpret_cast<float*>(nout), 2ull * H * W, st);
            nsq = nout;
        }
        {
            ProfScope ps(0, st);
            GStepArgsT<T> ga{xk, cb, uxi, uyi, uxo, uyo, last ? nullptr : crimg, nsq, nprev, lam, rho, H, W, np * H * W};
            // inference: the step runs inside the row transform of r (ADMM_GSTEP_FUSE=0: separate)
            if (!train && !last && env_int("ADMM_GSTEP_FUSE", 1)) {
                if (int e = grow_fwd_step(ga, cspec, twW, W, crows, d.iso != 0, first, st, gs, ld)) return e;
            } else {
                if (int e = gstep(ga, d.iso != 0, first, train, st)) return e;
                if (!last)
                    if (int e = grow_fwd(crimg, cspec, twW, W, crows, st, gs, ld)) return e;
            }
        }
        uin = 1 - uin;
    }
    return 0;
    };
    // plane parts on several streams (the caller's and auxiliary ones, aux_stream): one part's
    // compute-bound column pass overlaps another part's row / step passes (ADMM_GEN_STREAMS parts,
    // default 2: BSD 2,790 -> 3,150 it/s, every generic size measured gains).
    // Not under stream capture: a captured solve stays on the caller's stream.
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    HIPCHK(hipStreamIsCapturing(s, &cap));
    const int ns = std::max(1, std::min(kMaxAux + 1, env_setting("ADMM_GEN_STREAMS", 2)));
    const std::vector<long long> parts = gen_parts(P, H, ns);
    // (long lines: the parts would share the transform blocks' scratch slots -- one stream)
    const bool glb = make_plan(H, kF64<T>).glb || make_plan(W, kF64<T>).glb;
    if (!d.iso && !train && parts.size() > 1 && !glb && cap == hipStreamCaptureStatusNone) {
        int dev = 0;
        HIPCHK(hipGetDevice(&dev));
        std::vector<hipStream_t> aux;
        for (size_t i = 1; i < parts.size(); ++i) {
            hipStream_t x = aux_stream(s, dev, (int)i - 1);
            if (!x) return fail(ADMM_TV_EHIP, "auxiliary stream");
            aux.push_back(x);
        }
        ForkJoin fj(s, aux);
        if (fj.err != hipSuccess) return fail(ADMM_TV_EHIP, std::string("fork: ") + hipGetErrorString(fj.err));
        int e = 0;
        for (size_t i = 0; i < parts.size() && !e; ++i) {
            const long long p1 = i + 1 < parts.size() ? parts[i + 1] : P;
            e = solve_planes(parts[i], p1 - parts[i], i == 0 ? s : aux[i - 1]);
        }
        const hipError_t je = fj.finish();
        if (e) return e;
        if (je != hipSuccess) return fail(ADMM_TV_EHIP, std::string("join: ") + hipGetErrorString(je));
        return 0;
    }
    return solve_planes(0, P, s);
}

// rows per strip of the mixed row pass: the R dividing H that minimises (rounds of blocks over the chip)
// x (R + 1) -- a strip of R rows inverts R + 1 row spectra (one halo row), and the blocks run in rounds
// of (CUs x resident blocks per CU), so a short last round costs a whole one.  HD (1080 rows, 2 blocks of
// 2 strips per CU): R = 15 -> 1,981 it/s against 1,910-1,927 with R = 8, and the model orders R = 8, 10,
// 12, 15, 20, 24 as measured (profiles/r04_ab_hd_r.txt).  A/B knob ADMM_MIXED_R.
// The block slots (CUs x resident pass A blocks) are queried once per (device, N) and cached.
long long mixed_slots(int N) {
    static std::mutex mu;
    static std::vector<std::pair<std::pair<int, int>, long long>> cache;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 512;
    std::lock_guard<std::mutex> lk(mu);
    for (const auto& c : cache)
        if (c.first.first == dev && c.first.second == N) return c.second;
    long long slots = 0;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess)
        slots = (long long)cus * std::max(1, admm_mixed::pass_a_blocks_per_cu(N));
    if (slots <= 0) return 512;  // not cached: a failed query is retried
    cache.push_back({{dev, N}, slots});
    return slots;
}
// slots <= 0: this device's (mixed_slots); the training backward's layout passes a fixed count (its
// workspace size must not depend on the device)
int strip_rows_mixed(int H, long long rows, int N, long long slots = 0) {
    if (const int e = env_int("ADMM_MIXED_R", 0); e > 0 && H % e == 0) return e;
    const int sg = 256 / std::max(1, admm_mixed::row_lanes(N));  // strips per block
    if (slots <= 0) slots = mixed_slots(N);
    int best = 1;
    double best_t = 1e300;
    for (int R = 1; R <= 32 && R <= H; ++R) {
        if (H % R) continue;
        const long long strips = rows / R;
        const long long blocks = (strips + sg - 1) / sg;
        const double t = (double)((blocks + slots - 1) / slots) * (R + 1);
        if (t < best_t - 1e-9 || (t < best_t + 1e-9 && R > best)) {
            best_t = t;
            best = R;
        }
    }
    return best;
}

// The inference solve of a smooth size (mixed_hw) on the fused two-pass iteration (mixed_kernels.hpp):
// the same sequence as run_forward's fused loop -- b = H_t(xin) once (here through the generic
// transforms, mode 1: once per solve), r_1 = rowFFT(b), then per iteration pass B (column FFT, Wiener
// factor, column IFFT), [iso: the norm pass, its reduce and the cross-rank hook], pass A -- inside
// the generic layout's regions (spec[0] / spec[1] hold the packed row spectra ping-pong, u[0..3] the
// u images; the generic b region or xin is b, in pixel order).
// hist: the training forward (Layout::mixed_train) -- a_k and N_k into the history as run_forward's
// fused loop writes them (make_hist), and the last iteration's pass A also runs.
int run_forward_mixed(const admm_tv_desc& d, const Layout& Lo, const float* xin, const float* lam, const float* rho,
                      float* out, void* ws, void* hist, hipStream_t s) {
    const long long P = d.B * d.C;
    const bool train = hist != nullptr;
    const Hist Hs = make_hist(d);
    auto ha = [&](int k, int comp) -> float* {  // a_k image (k >= 1), comp 0 = x, 1 = y
        return reinterpret_cast<float*>(static_cast<char*>(hist) + (size_t)(2 * (k - 1) + comp) * Hs.a_slot);
    };
    auto hn = [&](int k) -> float* {  // N_k (k >= 1)
        return reinterpret_cast<float*>(static_cast<char*>(hist) + Hs.n_off + (size_t)(k - 1) * Hs.n_slot);
    };
    const int H = (int)d.H, W = (int)d.W, N = W / 2;
    cf* twW = at<cf>(ws, Lo.twW);
    cf* twH = at<cf>(ws, Lo.twH);
    cf* spec[2] = {at<cf>(ws, Lo.spec[0]), at<cf>(ws, Lo.spec[1])};
    float* u[4] = {at<float>(ws, Lo.u[0]), at<float>(ws, Lo.u[1]), at<float>(ws, Lo.u[2]), at<float>(ws, Lo.u[3])};
    auto hchk = [&](hipError_t e, const char* what) {
        return e == hipSuccess ? 0 : fail(ADMM_TV_EHIP, std::string(what) + ": " + hipGetErrorString(e));
    };
    const long long rows = P * H;
    const float* bimg = xin;
    {
        ProfScope ps(3, s);
        if (d.kh > 0) {  // b = H_t(xin) once, into the generic b region
            float* bb = at<float>(ws, Lo.b);
            // on the mixed transforms: row r2c, the column pass with the PSF multiplier, row c2r (HD: three
            // fast launches in place of the generic transforms' ~1 ms); A/B knob ADMM_MIXED_BGEN=1: the
            // generic transforms (half spectra as scratch)
            if (env_int("ADMM_MIXED_BGEN", 0)) {
                if (int e = gapply<float>(xin, bb, spec[0], Lo, ws, d, 1, s)) return e;
            } else {
                if (int e = hchk(admm_mixed::r2c(N, xin, spec[0], twW, rows, s), "k_row_r2c_m")) return e;
                if (int e = hchk(admm_mixed::pass_b_cm(H, spec[0], at<cf>(ws, Lo.mM), twH, N, P, s), "k_pass_b_m<cm>"))
                    return e;
                if (int e = hchk(admm_mixed::c2r(N, spec[0], bb, twW, rows, s), "k_row_c2r_m")) return e;
            }
            bimg = bb;
        }
        if (int e = hchk(admm_mixed::r2c(N, bimg, spec[0], twW, rows, s), "k_row_r2c_m")) return e;  // r_1 = b
    }
    const int R = strip_rows_mixed(H, rows, N);
    // grouped modules (desc.groups, inference only): one module after another through the iteration,
    // each with its own Wiener factor, lambda, rho and (iso) norm, sharing b and the tables
    const int G = ngroups_of(d);
    const int gpm = Lo.ngroups / G;  // iso plane groups per module (a group never straddles two)
    for (int g = 0; g < G; ++g) {
    const float* fcM = at<float>(ws, Lo.fcM) + (size_t)g * (2 * N + 1) * H;
    const float* lamg = lam + g;
    const float* rhog = rho + g;
    float* outg = out + (size_t)g * P * H * W;
    if (g > 0) {  // r_1 = b again: the previous module's iterations overwrote it
        ProfScope ps(3, s);
        if (int e = hchk(admm_mixed::r2c(N, bimg, spec[0], twW, rows, s), "k_row_r2c_m")) return e;
    }
    int cur = 0, uin = 0;
    for (int it = 1; it <= d.maxit; ++it) {
        {
            ProfScope ps(1, s);
            if (int e = hchk(admm_mixed::pass_b(H, spec[cur], fcM, twH, N, P, s), "k_pass_b_m")) return e;
        }
        if (it == d.maxit) {
            ProfScope ps(3, s);
            if (int e = hchk(admm_mixed::c2r(N, spec[cur], outg, twW, rows, s), "k_row_c2r_m")) return e;
            if (!train) break;
        }
        const bool first = it == 1;
        const float *uxi, *uyi, *nprev = nullptr;
        float *uxo, *uyo;
        if (train) {  // a_{k-1} in, a_k out (u is rebuilt from a in the kernels)
            uxi = first ? nullptr : ha(it - 1, 0);
            uyi = first ? nullptr : ha(it - 1, 1);
            uxo = ha(it, 0);
            uyo = ha(it, 1);
            if (d.iso && !first) nprev = hn(it - 1);
        } else {
            uxi = u[2 * uin];
            uyi = u[2 * uin + 1];
            uxo = u[2 * (1 - uin)];
            uyo = u[2 * (1 - uin) + 1];
        }
        const float* nsq = nullptr;
        if (d.iso) {
            ProfScope ps(2, s);
            float* nout = train ? hn(it) : at<float>(ws, Lo.nsq);
            IsoArgs ia{spec[cur], uxi, uyi, nprev, lamg, rhog, at<float>(ws, Lo.part), twW, (int)P, H, Lo.ppg,
                       (long long)gpm * H, P};
            if (int e = hchk(admm_mixed::iso_norm(N, ia, first, train, s), "k_iso_norm_m")) return e;
            const long long n4 = 2LL * H * W / 4;
            hipLaunchKernelGGL(k_iso_reduce, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, at<float4>(ws, Lo.part),
                               reinterpret_cast<float4*>(nout), gpm, n4);
            if (int e = launch_check("k_iso_reduce")) return e;
            allreduce(d, nout, 2ull * H * W, s);  // sharded batch: sums over every rank's planes
            nsq = nout;
        }
        {
            ProfScope ps(0, s);
            PassAArgs pa{spec[cur], spec[1 - cur], bimg, uxi, uyi, uxo, uyo, nsq, nprev, lamg, rhog, twW, H, R,
                         rows / R, P, 0};
            if (int e = hchk(admm_mixed::pass_a(N, pa, d.iso != 0, first, train, s), "k_pass_a_m")) return e;
        }
        cur = 1 - cur;
        uin = 1 - uin;
    }
    }
    return 0;
}

// The forward solver.  hist == nullptr: inference (u ping-pong).  Otherwise training mode:
// a_k -> hist slot k-1 (x image at 2(k-1), y image at 2(k-1)+1), N_k -> norm slot k-1, and
// the last iteration's pass A also runs (a_K is needed by the backward).
int run_forward(const admm_tv_desc& d, const float* xin, const float* kern, const float* lam, const float* rho,
                float* out, void* ws, size_t ws_bytes, void* hist, hipStream_t s) {
    const Layout Lo = make_layout(d);
    if (!ws || ws_bytes < Lo.total || (reinterpret_cast<uintptr_t>(ws) % kAlign) != 0)
        return fail(ADMM_TV_EWORKSPACE, "workspace too small or not 256-byte aligned");
    if (Lo.tr && !hist && d.maxit > 0) {  // the transposed odd-length solve (odd_t_hw)
        const long long P = d.B * d.C;
        const int H = (int)d.H, W = (int)d.W;
        float* xT = at<float>(ws, Lo.xT);
        float* oT = at<float>(ws, Lo.oT);
        float* kT = d.kh > 0 ? at<float>(ws, Lo.kT) : nullptr;
        {
            ProfScope ps(3, s);
            hipError_t e = admm_odd::transpose(xin, xT, H, W, P, s);
            if (e == hipSuccess && kT) e = admm_odd::transpose(kern, kT, d.kh, d.kw, 1, s);
            if (e != hipSuccess) return fail(ADMM_TV_EHIP, std::string("k_transpose: ") + hipGetErrorString(e));
        }
        const admm_tv_desc dT = transposed(d);
        if (int e = run_forward(dT, xT, kT, lam, rho, oT, at<char>(ws, Lo.tws), ws_bytes - Lo.tws, nullptr, s)) return e;
        ProfScope ps(3, s);
        const hipError_t e = admm_odd::transpose(oT, out, W, H, P, s);
        return e == hipSuccess ? 0 : fail(ADMM_TV_EHIP, std::string("k_transpose: ") + hipGetErrorString(e));
    }
    const int G = ngroups_of(d);
    const long long Pm = d.B * d.C, P = G * Pm;  // planes of one module, of all modules
    const int H = (int)d.H, W = (int)d.W, N = W / 2;
    const size_t img_bytes = (size_t)P * H * W * sizeof(float);
    if (d.maxit == 0) {
        if (img_bytes) HIPCHK(hipMemsetAsync(out, 0, img_bytes, s));  // the reference returns x = zeros (deconv.py:61,117)
        return 0;
    }
    if (participate_only(d)) {  // the same reductions as run_forward's iso loop, contributing zeros
        // (grouped modules at a smooth size: one module's iterations after another, 2HW per reduction)
        const bool by_module = Lo.gen && G > 1;
        const size_t n = (Lo.gen ? 1 : (size_t)G) * 2 * H * W;
        for (int g = 0; g < (by_module ? G : 1); ++g)
            for (int it = 1; it <= d.maxit; ++it) {
                if (it == d.maxit && !hist) break;
                HIPCHK(hipMemsetAsync(at<float>(ws, Lo.nsq), 0, n * sizeof(float), s));
                allreduce(d, at<float>(ws, Lo.nsq), n, s);
            }
        return 0;
    }
    if (int e = setup(d, Lo, ws, kern, rho, s)) return e;
    if (Lo.mixed && (!hist || Lo.mixed_train)) return run_forward_mixed(d, Lo, xin, lam, rho, out, ws, hist, s);
    if (Lo.gen) return run_forward_gen(d, Lo, xin, lam, rho, out, ws, hist, s);
    cf* twW = at<cf>(ws, Lo.twW);
    cf* twH = at<cf>(ws, Lo.twH);
    float* fcT = at<float>(ws, Lo.fcT);
    cf* mT = at<cf>(ws, Lo.mT);
    cf* spec[2] = {at<cf>(ws, Lo.spec[0]), at<cf>(ws, Lo.spec[1])};
    float* u[4] = {at<float>(ws, Lo.u[0]), at<float>(ws, Lo.u[1]), at<float>(ws, Lo.u[2]), at<float>(ws, Lo.u[3])};
    const bool train = hist != nullptr;
    const Hist Hs = make_hist(d);
    auto ha = [&](int k, int comp) -> float* {  // a_k image (k >= 1), comp 0 = x, 1 = y
        return reinterpret_cast<float*>(static_cast<char*>(hist) + (size_t)(2 * (k - 1) + comp) * Hs.a_slot);
    };
    auto hn = [&](int k) -> float* {  // N_k (k >= 1)
        return reinterpret_cast<float*>(static_cast<char*>(hist) + Hs.n_off + (size_t)(k - 1) * Hs.n_slot);
    };
    const bool keep_t = train && Hs.keep_t;
    auto ht = [&](int k) -> cf* {  // r_k row spectra (k >= 1), kept for the PSF gradient
        return reinterpret_cast<cf*>(static_cast<char*>(hist) + Hs.t_off + (size_t)(k - 1) * Hs.t_slot);
    };

    // The inference path keeps its internal images (u, b, iso norm maps) in the lane-paired row
    // layout (16-byte accesses, admm_kernels.hpp ld_row); the training history stays in pixel order.
    // ADMM_PL=0 for the pixel-order layout (A/B).
    // Default on for iso (C3 iso 507-514 -> 533-544 it/s) and rows up to 512 (C2 +1 %), off for aniso
    // rows of 1,024+ where the pixel-order streams measured faster (C3 pass A 1.0355 -> 1.0295 ms, 4
    // interleaved rounds, profiles/r03_sweep_knobs_c3.txt).
    const bool pl = !train && env_int("ADMM_PL", (d.iso || W < 1024) ? 1 : 0) != 0;

    // b = H_t(xin) once (the reference recomputes it every iteration, deconv.py:104)
    const float* bimg = xin;
    if (d.kh > 0) {
        ProfScope ps(3, s);
        float* bb = at<float>(ws, Lo.b);
        if (int e = psf_transpose_into(d, Lo, ws, xin, bb, spec[0], 1, s, pl)) return e;
        bimg = bb;
    } else if (pl) {  // b = xin, re-laid out
        ProfScope ps(3, s);
        float* bb = at<float>(ws, Lo.b);
        if (int e = with_row(N, [&](auto ops) { return decltype(ops)::pair(xin, bb, Pm * H, s); })) return e;
        bimg = bb;
    }
    for (int g = 0; g < G; ++g) {  // r_1 = b for every module
        ProfScope ps(3, s);
        cf* t0 = (keep_t ? ht(1) : spec[0]) + (size_t)g * Pm * H * N;
        int e = with_row(N, [&](auto ops) { return decltype(ops)::r2c(bimg, t0, twW, Pm * H, s, pl); });
        if (e) return e;
    }
    // Planes [p0, p0 + np) through all iterations (ppm: planes per module of that range).
    auto solve_planes = [&](long long p0, long long np, long long ppm, hipStream_t st) -> int {
    const size_t so = (size_t)p0 * H * N, io = (size_t)p0 * H * W;  // cf / float offsets
    cf* cspec[2] = {spec[0] + so, spec[1] + so};
    const long long crows = np * H;
    const float* cb = bimg + io;
    float* cout = out + io;
    const int R = strip_rows(H, N, crows, !d.iso && !hist);

    int cur = 0, uin = 0;  // spec[cur] holds the current r spectra; u[2*uin], u[2*uin+1] = u_x, u_y in
    for (int it = 1; it <= d.maxit; ++it) {
        {
            ProfScope ps(1, st);
            // PSF-gradient training keeps r_k's spectrum: the column pass then runs out of place
            const cf* tin = keep_t ? ht(it) : cspec[cur];
            if (int e = pass_b_oop(H, tin, cspec[cur], fcT, mT, twH, N, (int)np, 0, st, (int)ppm)) return e;
        }
        if (it == d.maxit) {
            ProfScope ps(3, st);
            int e = with_row(N, [&](auto ops) { return decltype(ops)::c2r(cspec[cur], cout, twW, crows, st); });
            if (e) return e;
            if (!train) break;
        }
        const bool first = (it == 1);
        const float *uxi, *uyi, *nprev = nullptr;
        float *uxo, *uyo;
        if (train) {
            uxi = first ? nullptr : ha(it - 1, 0);
            uyi = first ? nullptr : ha(it - 1, 1);
            uxo = ha(it, 0);
            uyo = ha(it, 1);
            if (d.iso && !first) nprev = hn(it - 1);
        } else {
            uxi = u[2 * uin] + io;
            uyi = u[2 * uin + 1] + io;
            uxo = u[2 * (1 - uin)] + io;
            uyo = u[2 * (1 - uin) + 1] + io;
        }
        const float* nsq = nullptr;
        if (d.iso) {
            ProfScope ps(2, st);
            float* nout = train ? hn(it) : at<float>(ws, Lo.nsq);
            IsoArgs ia{cspec[cur], uxi, uyi, nprev, lam, rho, at<float>(ws, Lo.part), twW, (int)P, H, Lo.ppg,
                       (long long)Lo.ngroups * H, Pm};
            int e = with_row(N, [&](auto ops) { return decltype(ops)::iso_norm(ia, first, train, st, pl); });
            if (e) return e;
            const long long n4 = 2LL * H * W / 4;
            const int gpm = Lo.ngroups / G;  // plane groups per module
            for (int g = 0; g < G; ++g) {     // each module's norm over its own planes
                hipLaunchKernelGGL(k_iso_reduce, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st,
                                   at<float4>(ws, Lo.part) + (size_t)g * gpm * n4,  // n4 float4 = 2HW floats
                                   reinterpret_cast<float4*>(nout) + (size_t)g * n4, gpm, n4);
                if ((e = launch_check("k_iso_reduce"))) return e;
            }
            // sharded batch: the per-pixel sums must cover every rank's planes
            allreduce(d, nout, (size_t)G * 2 * H * W, st);
            nsq = nout;
        }
        {
            ProfScope ps(0, st);
            cf* tout = (keep_t && it < d.maxit) ? ht(it + 1) : cspec[1 - cur];
            PassAArgs pa{cspec[cur], tout, cb, uxi, uyi, uxo, uyo, nsq, nprev, lam, rho, twW, H, R, crows / R, ppm,
                         env_int("ADMM_PASSA_REV", 0)};
            int e = with_row(N, [&](auto ops) { return decltype(ops)::pass_a(pa, d.iso != 0, first, train, st, pl); });
            if (e) return e;
        }
        cur = 1 - cur;
        uin = 1 - uin;
    }
    return 0;
    };
    // (measured and removed: plane chunks kept resident in the Infinity Cache through all iterations, and
    // two plane halves on two streams -- DESIGN.md §9; both no faster at C3)
    return solve_planes(0, P, Pm, s);
}

// backward workspace = forward layout + a^ ping-pong (4 images) + b^ + per-iteration partials
struct BwdLayout {
    Layout f;
    size_t abar[4], bbar, part, tpart, q, xpart, aacc, zacc, total;
    long long nstrips;
    int R, ntp, xgroups, xppg;
};
BwdLayout make_bwd_layout(const admm_tv_desc& d) {
    BwdLayout B{};
    B.f = make_layout(d);
    const size_t rs = is_f64(d) ? sizeof(double) : sizeof(float);
    const size_t G = ngroups_of(d);
    const size_t img = G * d.B * d.C * d.H * d.W * rs;  // all modules' planes
    size_t o = B.f.total;
    auto take = [&](size_t bytes) {
        size_t at_ = o;
        o += up(bytes);
        return at_;
    };
    for (int i = 0; i < 4; ++i) B.abar[i] = take(img);
    B.bbar = take(img);  // per module; summed into gxin at the end
    const long long rows = (long long)G * d.B * d.C * d.H;
    if (B.f.mixed_train) {  // mixed-radix reverse row pass: strips of R rows (a device-independent rule)
        B.R = strip_rows_mixed((int)d.H, rows, (int)d.W / 2, 512);
        B.nstrips = rows / B.R;
    } else if (B.f.gen) {  // generic backward: one partial pair per 256-pixel block
        B.R = 0;
        B.nstrips = (rows * d.W + 255) / 256;
    } else {
        B.R = strip_rows((int)d.H, (int)d.W / 2, rows);
        B.nstrips = rows / B.R;
    }
    // the lambda / rho gradient partials are fp64 in every solve (admm_backward.hpp)
    B.part = take((size_t)std::max(d.maxit, 1) * B.nstrips * 2 * sizeof(double));
    // tau^ partials per iteration and module: one per block of the fused paths' Q reduce (k_iso_reduce_tau,
    // 1,024 values per block); the generic path's k_iso_tau_partial runs that many blocks too
    B.ntp = (int)std::max<long long>(1, ((long long)d.H * d.W / 2 + 255) / 256);
    B.tpart = take((size_t)std::max(d.maxit, 1) * G * B.ntp * sizeof(double));  // [K][G][ntp]
    B.q = take(G * 2 * (size_t)d.H * d.W * rs);
    if (d.kh > 0 && (d.flags & ADMM_TV_FLAG_PSF_GRAD)) {
        const size_t nf = ((size_t)d.W / 2 + 1) * d.H;
        B.xppg = 8;
        B.xgroups = (int)((d.B * d.C + B.xppg - 1) / B.xppg);
        // fast path: per-plane-group cross-spectrum partials; generic: one 2-D spectrum set
        B.xpart = take((B.f.gen ? (size_t)d.B * d.C : (size_t)B.xgroups) * nf * 2 * rs);
        B.aacc = take(nf * sizeof(double2));
        B.zacc = take(nf * sizeof(double2));
    }
    B.total = o;
    return B;
}


// generic-size backward (same contract as admm_tv_backward, PSF gradient excluded)
template <class T>
int run_backward_gen(const admm_tv_desc& d, const BwdLayout& BL, const T* xin, const T* lam, const T* rho,
                     const T* gout, const void* hist, T* gxin, T* glam, T* grho, T* gkern, void* ws, hipStream_t s) {
    using C = cx_t<T>;
    const Layout& Lo = BL.f;
    const long long P = d.B * d.C;
    const int H = (int)d.H, W = (int)d.W, K = d.maxit;
    const long long npx = P * H * W;
    const long long HW = (long long)H * W;
    const Hist Hs = make_hist(d);
    char* hb = static_cast<char*>(const_cast<void*>(hist));
    auto ha = [&](int k, int comp) -> const T* {
        return reinterpret_cast<const T*>(hb + (size_t)(2 * (k - 1) + comp) * Hs.a_slot);
    };
    auto hn = [&](int k) -> const T* { return reinterpret_cast<const T*>(hb + Hs.n_off + (size_t)(k - 1) * Hs.n_slot); };
    auto ht = [&](int k) -> const C* { return reinterpret_cast<const C*>(hb + Hs.t_off + (size_t)(k - 1) * Hs.t_slot); };
    const bool psf_grad = gkern != nullptr;
    const int Wh = W / 2 + 1;
    const long long nf = (long long)Wh * H;
    C* xspec = psf_grad ? at<C>(ws, BL.xpart) : nullptr;  // 2-D spectra of x^_k (then of b^)
    if (psf_grad) {
        HIPCHK(hipMemsetAsync(at<double2>(ws, BL.aacc), 0, nf * sizeof(double2), s));
        HIPCHK(hipMemsetAsync(at<double2>(ws, BL.zacc), 0, nf * sizeof(double2), s));
    }
    C* twW = at<C>(ws, Lo.twW);
    C* twH = at<C>(ws, Lo.twH);
    C* gs = at<C>(ws, Lo.gscr);  // long lines: the transform blocks' scratch slots
    T* fcT = at<T>(ws, Lo.fcT);
    const long long rows = P * H;
    const dim3 fgrid((unsigned)((nf + 255) / 256)), fblk(256);
    C* spec = at<C>(ws, Lo.spec[0]);
    T* rb = at<T>(ws, Lo.spec[1]);   // r^_k
    T* xbuf[2] = {at<T>(ws, Lo.rimg), at<T>(ws, Lo.u[0])};  // x^ ping-pong
    T* ab[4] = {at<T>(ws, BL.abar[0]), at<T>(ws, BL.abar[1]), at<T>(ws, BL.abar[2]),
                    at<T>(ws, BL.abar[3])};
    T* bbar = (d.kh == 0 && gxin) ? gxin : at<T>(ws, BL.bbar);
    double* part = at<double>(ws, BL.part);
    double* tpart = at<double>(ws, BL.tpart);
    T* q = at<T>(ws, BL.q);
    if (d.iso) HIPCHK(hipMemsetAsync(tpart, 0, (size_t)K * BL.ntp * sizeof(double), s));
    const T* xbk = gout;
    int ain = 0, xo = 0;
    for (int k = K; k >= 1; --k) {
        const bool lastk = (k == K), firstk = (k == 1);
        {
            ProfScope ps(1, s);
            // r^_k = M x^_k; with the PSF gradient the column pass also dumps X^_k's spectrum and
            // A += fc^2 Re(sum_p conj(X^_k) R_k)
            if (int e = grow_fwd(xbk, spec, twW, W, rows, s, gs)) return e;
            if (int e = gcol<T>(spec, xspec, fcT, at<C>(ws, Lo.mT), twH, H, W, P, 0, s, gs, Lo.mm)) return e;
            if (int e = grow_inv<T>(spec, rb, twW, W, rows, s, gs, Lo.mmr)) return e;
            if (psf_grad) {
                hipLaunchKernelGGL(k_gxspec_acc<T>, fgrid, fblk, 0, s, xspec, ht(k), P, H, Wh, fcT, at<double2>(ws, BL.aacc));
                if (int e = launch_check("k_gxspec_acc")) return e;
            }
        }
        if (d.iso && !firstk) {
            ProfScope ps(2, s);
            const dim3 grid((unsigned)((HW + 255) / 256)), blk(256);
            if (lastk)
                hipLaunchKernelGGL((k_giso_q<true, T>), grid, blk, 0, s, rb, ab[2 * ain], ab[2 * ain + 1], ha(k - 1, 0),
                                   ha(k - 1, 1), rho, q, H, W, P);
            else
                hipLaunchKernelGGL((k_giso_q<false, T>), grid, blk, 0, s, rb, ab[2 * ain], ab[2 * ain + 1], ha(k - 1, 0),
                                   ha(k - 1, 1), rho, q, H, W, P);
            if (int e = launch_check("k_giso_q")) return e;
            hipLaunchKernelGGL(k_iso_tau_partial<T>, dim3(BL.ntp), dim3(256), 0, s, q, hn(k - 1), lam, rho,
                               tpart + (size_t)(K - k) * BL.ntp, 2LL * HW);
            if (int e = launch_check("k_iso_tau_partial")) return e;
            allreduce(d, reinterpret_cast<float*>(q), 2ull * H * W, s);
        }
        {
            ProfScope ps(0, s);
            GBwdArgsT<T> ba{rb, xbuf[xo], bbar,
                        ab[2 * ain], ab[2 * ain + 1], ab[2 * (1 - ain)], ab[2 * (1 - ain) + 1],
                        ha(k, 0), ha(k, 1),
                        firstk ? nullptr : ha(k - 1, 0), firstk ? nullptr : ha(k - 1, 1),
                        (d.iso && !firstk) ? hn(k - 1) : nullptr, q, lam, rho,
                        part + (size_t)(K - k) * BL.nstrips * 2, H, W, npx};
            if (int e = gbwd(ba, d.iso != 0, lastk, firstk, s)) return e;
        }
        xbk = xbuf[xo];
        xo = 1 - xo;
        ain = 1 - ain;
    }
    if (glam && grho) {
        if (int e = bwd_scalars<T>(part, K, BL.nstrips, BL.nstrips, 0LL, d.iso ? tpart : nullptr, BL.ntp, 1, 0, lam, rho,
                                   glam, grho, s))
            return e;
    } else if (glam || grho) {
        return fail(ADMM_TV_EINVAL, "glam and grho must be given together");
    }
    if (psf_grad) {  // Z = sum_p conj(Bbar_p) Xin_p, then the k x k taps
        if (int e = grow_fwd(bbar, spec, twW, W, rows, s, gs)) return e;
        if (int e = gcol<T>(spec, xspec, nullptr, nullptr, twH, H, W, P, 3, s, gs, Lo.mm)) return e;
        if (int e = grow_fwd(xin, spec, twW, W, rows, s, gs)) return e;
        if (int e = gcol<T>(spec, spec, nullptr, nullptr, twH, H, W, P, 3, s, gs, Lo.mm)) return e;
        hipLaunchKernelGGL(k_gxspec_acc<T>, fgrid, fblk, 0, s, xspec, spec, P, H, Wh, nullptr, at<double2>(ws, BL.zacc));
        if (int e = launch_check("k_gxspec_acc")) return e;
        hipLaunchKernelGGL(k_psf_grad<T>, dim3(d.kh * d.kw), dim3(256), 0, s, at<double2>(ws, BL.aacc),
                           at<double2>(ws, BL.zacc), at<double2>(ws, Lo.sigma), d.kh, H, W, gkern, 1.0);
        if (int e = launch_check("k_psf_grad")) return e;
    }
    if (gxin && d.kh > 0)  // x^_in = H_t^T b^
        if (int e = gapply<T>(bbar, gxin, spec, Lo, ws, d, 2, s)) return e;
    return 0;
}

// ------------------------------------------------------------------ fp64 solves (ADMM_TV_FLAG_F64)
// The forward of an fp64 solve: run_forward's contract on the generic kernels' double instantiation.
// training backward at a smooth size (Layout::mixed_train; one module, no PSF gradient): the fused
// path's reverse sequence (admm_tv_backward) on the mixed transforms -- r^_k = M x^_k by the inference
// column pass, [iso: Q_{k-1} and its tau^ partial], the reverse row pass; then the scalars, and
// x^_in = H_t^T b^ through the generic transforms when there is a PSF.
int run_backward_mixed(const admm_tv_desc& d, const BwdLayout& BL, const float* lam, const float* rho,
                       const float* gout, const void* hist, float* gxin, float* glam, float* grho, void* ws,
                       hipStream_t s) {
    const Layout& Lo = BL.f;
    const long long P = d.B * d.C;
    const int H = (int)d.H, W = (int)d.W, N = W / 2, K = d.maxit;
    const Hist Hs = make_hist(d);
    const char* hb = static_cast<const char*>(hist);
    auto ha = [&](int k, int comp) -> const float* {
        return reinterpret_cast<const float*>(hb + (size_t)(2 * (k - 1) + comp) * Hs.a_slot);
    };
    auto hn = [&](int k) -> const float* { return reinterpret_cast<const float*>(hb + Hs.n_off + (size_t)(k - 1) * Hs.n_slot); };
    auto hchk = [&](hipError_t e, const char* what) {
        return e == hipSuccess ? 0 : fail(ADMM_TV_EHIP, std::string(what) + ": " + hipGetErrorString(e));
    };
    cf* twW = at<cf>(ws, Lo.twW);
    cf* twH = at<cf>(ws, Lo.twH);
    const float* fcM = at<float>(ws, Lo.fcM);
    cf* spec[2] = {at<cf>(ws, Lo.spec[0]), at<cf>(ws, Lo.spec[1])};
    float* ab[4] = {at<float>(ws, BL.abar[0]), at<float>(ws, BL.abar[1]), at<float>(ws, BL.abar[2]),
                    at<float>(ws, BL.abar[3])};
    float* bbar = (d.kh == 0 && gxin) ? gxin : at<float>(ws, BL.bbar);  // no PSF: x^_in = b^
    double* part = at<double>(ws, BL.part);
    double* tpart = at<double>(ws, BL.tpart);
    float* q = at<float>(ws, BL.q);
    const long long rows = P * H;
    if (d.iso) HIPCHK(hipMemsetAsync(tpart, 0, (size_t)K * BL.ntp * sizeof(double), s));
    if (int e = hchk(admm_mixed::r2c(N, gout, spec[0], twW, rows, s), "k_row_r2c_m")) return e;
    int cur = 0, ain = 0;
    for (int k = K; k >= 1; --k) {
        {
            ProfScope ps(1, s);
            if (int e = hchk(admm_mixed::pass_b(H, spec[cur], fcM, twH, N, P, s), "k_pass_b_m")) return e;
        }
        const bool lastk = (k == K), firstk = (k == 1);
        if (d.iso && !firstk) {
            ProfScope ps(2, s);
            BwdIsoArgs qa{spec[cur], ab[2 * ain], ab[2 * ain + 1], ha(k - 1, 0), ha(k - 1, 1), rho,
                          at<float>(ws, Lo.part), twW, (int)P, H, Lo.ppg, (long long)Lo.ngroups * H, P};
            if (int e = hchk(admm_mixed::bwd_iso_q(N, qa, lastk, s), "k_bwd_iso_q_m")) return e;
            const long long n4 = 2LL * H * W / 4;
            // Q and the tau^ partials from this rank's Q (N is already global), then Q over every rank's planes
            hipLaunchKernelGGL(k_iso_reduce_tau, dim3((unsigned)BL.ntp), dim3(256), 0, s, at<float4>(ws, Lo.part),
                               reinterpret_cast<float4*>(q), Lo.ngroups, n4, reinterpret_cast<const float4*>(hn(k - 1)),
                               lam, rho, tpart + (size_t)(K - k) * BL.ntp);
            if (int e = launch_check("k_iso_reduce_tau")) return e;
            allreduce(d, q, 2ull * H * W, s);
        }
        {
            ProfScope ps(0, s);
            BwdArgs ba{spec[cur], spec[1 - cur], bbar,
                       ab[2 * ain], ab[2 * ain + 1], ab[2 * (1 - ain)], ab[2 * (1 - ain) + 1],
                       ha(k, 0), ha(k, 1),
                       firstk ? nullptr : ha(k - 1, 0), firstk ? nullptr : ha(k - 1, 1),
                       (d.iso && !firstk) ? hn(k - 1) : nullptr, q, lam, rho,
                       part + (size_t)(K - k) * BL.nstrips * 2, twW, H, BL.R, BL.nstrips, P};
            if (int e = hchk(admm_mixed::bwd_pass_a(N, ba, d.iso != 0, lastk, firstk, s), "k_bwd_pass_a_m")) return e;
        }
        cur = 1 - cur;
        ain = 1 - ain;
    }
    if (glam && grho) {
        if (int e = bwd_scalars<float>(part, K, BL.nstrips, BL.nstrips, 0LL, d.iso ? tpart : nullptr, BL.ntp, 1, 0, lam,
                                       rho, glam, grho, s))
            return e;
    } else if (glam || grho) {
        return fail(ADMM_TV_EINVAL, "glam and grho must be given together");
    }
    if (gxin && d.kh > 0)  // x^_in = H_t^T b^ (the conjugate multiplier, generic transforms)
        if (int e = gapply<float>(bbar, gxin, spec[0], Lo, ws, d, 2, s)) return e;
    return 0;
}

int run_forward_f64(const admm_tv_desc& d, const double* xin, const double* kern, const double* lam,
                    const double* rho, double* out, void* ws, size_t ws_bytes, void* hist, hipStream_t s) {
    const Layout Lo = make_layout(d);
    if (!ws || ws_bytes < Lo.total || (reinterpret_cast<uintptr_t>(ws) % kAlign) != 0)
        return fail(ADMM_TV_EWORKSPACE, "workspace too small or not 256-byte aligned");
    const int H = (int)d.H, W = (int)d.W;
    const size_t img_bytes = (size_t)d.B * d.C * H * W * sizeof(double);
    if (d.maxit == 0) {
        if (img_bytes) HIPCHK(hipMemsetAsync(out, 0, img_bytes, s));  // the reference returns x = zeros
        return 0;
    }
    if (participate_only(d)) {  // the same reductions as the iso loop, contributing zeros
        for (int it = 1; it <= d.maxit; ++it) {
            if (it == d.maxit && !hist) break;
            HIPCHK(hipMemsetAsync(at<double>(ws, Lo.nsq), 0, 2ull * H * W * sizeof(double), s));
            allreduce(d, at<float>(ws, Lo.nsq), 2ull * H * W, s);
        }
        return 0;
    }
    if (int e = setup<double>(d, Lo, ws, kern, rho, s)) return e;
    return run_forward_gen<double>(d, Lo, xin, lam, rho, out, ws, hist, s);
}

int run_backward_f64(const admm_tv_desc& d, const double* xin, const double* kern, const double* lam,
                     const double* rho, const double* gout, const void* hist, size_t hist_bytes, double* gxin,
                     double* glam, double* grho, double* gkern, void* ws, size_t ws_bytes, hipStream_t s) {
    const BwdLayout BL = make_bwd_layout(d);
    if (!ws || ws_bytes < BL.total || (reinterpret_cast<uintptr_t>(ws) % kAlign) != 0)
        return fail(ADMM_TV_EWORKSPACE, "workspace too small or not 256-byte aligned");
    const int H = (int)d.H, W = (int)d.W, K = d.maxit;
    const size_t img_bytes = (size_t)d.B * d.C * H * W * sizeof(double);
    if (gkern && (d.kh == 0 || !(d.flags & ADMM_TV_FLAG_PSF_GRAD) || (!xin && !participate_only(d))))
        return fail(ADMM_TV_EINVAL, "gkern needs a PSF, ADMM_TV_FLAG_PSF_GRAD (forward and backward) and xin");
    if ((glam == nullptr) != (grho == nullptr)) return fail(ADMM_TV_EINVAL, "glam and grho must be given together");
    if (K == 0 || participate_only(d)) {
        if (participate_only(d) && K > 0)
            for (int k = K; k >= 2; --k) {
                HIPCHK(hipMemsetAsync(at<double>(ws, BL.q), 0, 2ull * H * W * sizeof(double), s));
                allreduce(d, at<float>(ws, BL.q), 2ull * H * W, s);
            }
        if (gxin && img_bytes) HIPCHK(hipMemsetAsync(gxin, 0, img_bytes, s));
        if (glam) HIPCHK(hipMemsetAsync(glam, 0, sizeof(double), s));
        if (grho) HIPCHK(hipMemsetAsync(grho, 0, sizeof(double), s));
        if (gkern) HIPCHK(hipMemsetAsync(gkern, 0, sizeof(double) * d.kh * d.kw, s));
        return 0;
    }
    if (!hist || hist_bytes < make_hist(d).total) return fail(ADMM_TV_EWORKSPACE, "history buffer too small");
    if (int e = setup<double>(d, BL.f, ws, kern, rho, s)) return e;
    return run_backward_gen<double>(d, BL, xin, lam, rho, gout, hist, gxin, glam, grho, gkern, ws, s);
}

}  // namespace

// ============================================================================ C ABI
extern "C" {

int admm_tv_abi_version(void) { return ADMM_TV_ABI_VERSION; }

int admm_tv_supported(int64_t H, int64_t W) {
    return supported_hw(H, W) ? 1 : mixed_hw(H, W) ? 3 : (odd_hw(H, W) || odd_t_hw(H, W)) ? 4 : generic_hw(H, W) ? 2 : 0;
}

int admm_tv_supported_f64(int64_t H, int64_t W) { return f64_hw(H, W) ? 1 : 0; }

int admm_tv_path(const admm_tv_desc* d, int train) {
    if (int e = validate(d)) return e;
    if (train) {
        if (int e = grouped_train_check(*d)) return e;
    }
    if (is_f64(*d)) return ADMM_TV_PATH_GENERIC;  // the generic kernels' double instantiation
    const Layout Lo = make_layout(*d);
    if (Lo.tr) return train ? ADMM_TV_PATH_GENERIC : ADMM_TV_PATH_ODD;
    if (!Lo.gen) return ADMM_TV_PATH_FUSED;
    if (Lo.mixed && (!train || Lo.mixed_train)) return ADMM_TV_PATH_MIXED;
    if (Lo.odd && !train) return ADMM_TV_PATH_ODD;
    return ADMM_TV_PATH_GENERIC;
}

const char* admm_tv_last_error(void) { return g_err.c_str(); }

int admm_tv_workspace_size(const admm_tv_desc* d, size_t* bytes) {
    if (int e = validate(d)) return e;
    if (!bytes) return fail(ADMM_TV_EINVAL, "null bytes");
    *bytes = make_layout(*d).total;
    return 0;
}

int admm_tv_forward(const admm_tv_desc* dp, const float* xin, const float* kern, const float* lam, const float* rho,
                    float* out, void* ws, size_t ws_bytes, void* stream) {
    if (int e = validate(dp)) return e;
    if (is_f64(*dp)) return fail(ADMM_TV_EINVAL, "ADMM_TV_FLAG_F64: use admm_tv_forward_f64");
    if (((!xin || !out) && !participate_only(*dp)) || !lam || !rho || (dp->kh > 0 && !kern))
        return fail(ADMM_TV_EINVAL, "null pointer argument");
    DeviceGuard dg(reinterpret_cast<hipStream_t>(stream));
    if (dg.err != hipSuccess) return fail(ADMM_TV_EHIP, std::string("device of the stream: ") + hipGetErrorString(dg.err));
    return run_forward(*dp, xin, kern, lam, rho, out, ws, ws_bytes, nullptr, reinterpret_cast<hipStream_t>(stream));
}

int admm_tv_history_size(const admm_tv_desc* d, size_t* bytes) {
    if (int e = validate(d)) return e;
    if (int e = grouped_train_check(*d)) return e;
    if (!bytes) return fail(ADMM_TV_EINVAL, "null bytes");
    *bytes = make_hist(*d).total;
    return 0;
}

int admm_tv_forward_train(const admm_tv_desc* dp, const float* xin, const float* kern, const float* lam,
                          const float* rho, float* out, void* hist, size_t hist_bytes, void* ws, size_t ws_bytes,
                          void* stream) {
    if (int e = validate(dp)) return e;
    if (int e = grouped_train_check(*dp)) return e;
    if (is_f64(*dp)) return fail(ADMM_TV_EINVAL, "ADMM_TV_FLAG_F64: use admm_tv_forward_train_f64");
    if (((!xin || !out) && !participate_only(*dp)) || !lam || !rho || (dp->kh > 0 && !kern))
        return fail(ADMM_TV_EINVAL, "null pointer argument");
    if (dp->maxit > 0 && (!hist || hist_bytes < make_hist(*dp).total))
        return fail(ADMM_TV_EWORKSPACE, "history buffer too small");
    DeviceGuard dg(reinterpret_cast<hipStream_t>(stream));
    if (dg.err != hipSuccess) return fail(ADMM_TV_EHIP, std::string("device of the stream: ") + hipGetErrorString(dg.err));
    return run_forward(*dp, xin, kern, lam, rho, out, ws, ws_bytes, dp->maxit > 0 ? hist : nullptr,
                       reinterpret_cast<hipStream_t>(stream));
}

int admm_tv_backward_workspace_size(const admm_tv_desc* d, size_t* bytes) {
    if (int e = validate(d)) return e;
    if (int e = grouped_train_check(*d)) return e;
    if (!bytes) return fail(ADMM_TV_EINVAL, "null bytes");
    *bytes = make_bwd_layout(*d).total;
    return 0;
}

int admm_tv_backward(const admm_tv_desc* dp, const float* xin, const float* kern, const float* lam,
                     const float* rho, const float* gout, const void* hist, size_t hist_bytes, float* gxin,
                     float* glam, float* grho, float* gkern, void* ws, size_t ws_bytes, void* stream) {
    if (int e = validate(dp)) return e;
    if (int e = grouped_train_check(*dp)) return e;
    if (is_f64(*dp)) return fail(ADMM_TV_EINVAL, "ADMM_TV_FLAG_F64: use admm_tv_backward_f64");
    const admm_tv_desc d = *dp;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    DeviceGuard dg(reinterpret_cast<hipStream_t>(stream));
    if (dg.err != hipSuccess) return fail(ADMM_TV_EHIP, std::string("device of the stream: ") + hipGetErrorString(dg.err));
    if ((!gout && !participate_only(d)) || !lam || !rho || (d.kh > 0 && !kern))
        return fail(ADMM_TV_EINVAL, "null pointer argument");
    const BwdLayout BL = make_bwd_layout(d);
    const Layout& Lo = BL.f;
    if (!ws || ws_bytes < BL.total || (reinterpret_cast<uintptr_t>(ws) % kAlign) != 0)
        return fail(ADMM_TV_EWORKSPACE, "workspace too small or not 256-byte aligned");
    const int G = ngroups_of(d);
    const long long Pm = d.B * d.C, P = G * Pm;  // planes of one module, of all modules
    const int H = (int)d.H, W = (int)d.W, N = W / 2, K = d.maxit;
    const size_t img_bytes = (size_t)Pm * H * W * sizeof(float);  // gxin: one module's planes
    const bool psf_grad = gkern != nullptr;
    if (psf_grad && (d.kh == 0 || !(d.flags & ADMM_TV_FLAG_PSF_GRAD) || (!xin && !participate_only(d))))
        return fail(ADMM_TV_EINVAL, "gkern needs a PSF, ADMM_TV_FLAG_PSF_GRAD (forward and backward) and xin");
    if (K == 0) {  // output is identically zero
        if (gxin) HIPCHK(hipMemsetAsync(gxin, 0, img_bytes, s));
        if (glam) HIPCHK(hipMemsetAsync(glam, 0, sizeof(float) * G, s));
        if (grho) HIPCHK(hipMemsetAsync(grho, 0, sizeof(float) * G, s));
        if (gkern) HIPCHK(hipMemsetAsync(gkern, 0, sizeof(float) * d.kh * d.kw, s));
        return 0;
    }
    if (participate_only(d)) {  // the same reductions as the iso backward below, contributing zeros
        const size_t n = (size_t)G * 2 * H * W;
        for (int k = K; k >= 2; --k) {
            HIPCHK(hipMemsetAsync(at<float>(ws, BL.q), 0, n * sizeof(float), s));
            allreduce(d, at<float>(ws, BL.q), Lo.gen ? 2ull * H * W : n, s);
        }
        if (glam) HIPCHK(hipMemsetAsync(glam, 0, sizeof(float) * G, s));
        if (grho) HIPCHK(hipMemsetAsync(grho, 0, sizeof(float) * G, s));
        if (gkern) HIPCHK(hipMemsetAsync(gkern, 0, sizeof(float) * d.kh * d.kw, s));
        return 0;
    }
    if (!hist || hist_bytes < make_hist(d).total) return fail(ADMM_TV_EWORKSPACE, "history buffer too small");
    if (int e = setup(d, Lo, ws, kern, rho, s)) return e;
    if (Lo.mixed_train) return run_backward_mixed(d, BL, lam, rho, gout, hist, gxin, glam, grho, ws, s);
    if (Lo.gen) return run_backward_gen(d, BL, xin, lam, rho, gout, hist, gxin, glam, grho, gkern, ws, s);
    const Hist Hs = make_hist(d);
    char* hb = static_cast<char*>(const_cast<void*>(hist));
    auto ha = [&](int k, int comp) -> const float* {
        return reinterpret_cast<const float*>(hb + (size_t)(2 * (k - 1) + comp) * Hs.a_slot);
    };
    auto hn = [&](int k) -> const float* { return reinterpret_cast<const float*>(hb + Hs.n_off + (size_t)(k - 1) * Hs.n_slot); };
    auto ht = [&](int k) -> const cf* { return reinterpret_cast<const cf*>(hb + Hs.t_off + (size_t)(k - 1) * Hs.t_slot); };
    const long long nf = (long long)(N + 1) * H;
    if (psf_grad) {
        HIPCHK(hipMemsetAsync(at<double2>(ws, BL.aacc), 0, nf * sizeof(double2), s));
        HIPCHK(hipMemsetAsync(at<double2>(ws, BL.zacc), 0, nf * sizeof(double2), s));
    }
    cf* twW = at<cf>(ws, Lo.twW);
    cf* twH = at<cf>(ws, Lo.twH);
    float* fcT = at<float>(ws, Lo.fcT);
    cf* mT = at<cf>(ws, Lo.mT);
    cf* spec[2] = {at<cf>(ws, Lo.spec[0]), at<cf>(ws, Lo.spec[1])};
    float* ab[4] = {at<float>(ws, BL.abar[0]), at<float>(ws, BL.abar[1]), at<float>(ws, BL.abar[2]),
                    at<float>(ws, BL.abar[3])};
    // b^ accumulates straight into gxin when there is no PSF and one module (x^_in = b^)
    float* bbar = (d.kh == 0 && gxin && G == 1) ? gxin : at<float>(ws, BL.bbar);
    double* part = at<double>(ws, BL.part);
    double* tpart = at<double>(ws, BL.tpart);
    float* q = at<float>(ws, BL.q);
    const long long rows = P * H;
    if (d.iso) HIPCHK(hipMemsetAsync(tpart, 0, (size_t)K * G * BL.ntp * sizeof(double), s));
    int e = with_row(N, [&](auto ops) { return decltype(ops)::r2c(gout, spec[0], twW, rows, s); });
    if (e) return e;
    int cur = 0, ain = 0;
    for (int k = K; k >= 1; --k) {
        if (psf_grad) {  // A += fc^2 Re(sum_p conj(X^_k) R_k), before the column pass rewrites X^_k
            if ((e = xspec(H, spec[cur], ht(k), at<cf>(ws, BL.xpart), twH, N, (int)P, BL.xppg, s))) return e;
            hipLaunchKernelGGL(k_xspec_reduce, dim3((unsigned)((nf + 255) / 256)), dim3(256), 0, s,
                               at<cf>(ws, BL.xpart), BL.xgroups, nf, fcT, at<double2>(ws, BL.aacc));
            if ((e = launch_check("k_xspec_reduce"))) return e;
        }
        {
            ProfScope ps(1, s);
            if ((e = pass_b(H, spec[cur], fcT, mT, twH, N, (int)P, 0, s, (int)Pm))) return e;
        }
        const bool lastk = (k == K), firstk = (k == 1);
        if (d.iso && !firstk) {
            ProfScope ps(2, s);
            BwdIsoArgs qa{spec[cur], ab[2 * ain], ab[2 * ain + 1], ha(k - 1, 0), ha(k - 1, 1), rho,
                          at<float>(ws, Lo.part), twW, (int)P, H, Lo.ppg, (long long)Lo.ngroups * H, Pm};
            if ((e = with_row(N, [&](auto ops) { return decltype(ops)::bwd_iso_q(qa, lastk, s); }))) return e;
            const long long n4 = 2LL * H * W / 4;
            const int gpm = Lo.ngroups / G;
            for (int g = 0; g < G; ++g) {  // per module: Q over its planes, then its tau^ partial
                float* qg = q + (size_t)g * 2 * H * W;
                // Q and the tau^ partials from this rank's Q (the norm N is already global): summing the
                // ranks' lambda/rho gradients then counts every plane once
                hipLaunchKernelGGL(k_iso_reduce_tau, dim3((unsigned)BL.ntp), dim3(256), 0, s,
                                   at<float4>(ws, Lo.part) + (size_t)g * gpm * n4, reinterpret_cast<float4*>(qg), gpm, n4,
                                   reinterpret_cast<const float4*>(hn(k - 1) + (size_t)g * 2 * H * W), lam + g, rho + g,
                                   tpart + ((size_t)(K - k) * G + g) * BL.ntp);
                if ((e = launch_check("k_iso_reduce_tau"))) return e;
            }
            allreduce(d, q, (size_t)G * 2 * H * W, s);
        }
        {
            ProfScope ps(0, s);
            BwdArgs ba{spec[cur], spec[1 - cur], bbar,
                       ab[2 * ain], ab[2 * ain + 1], ab[2 * (1 - ain)], ab[2 * (1 - ain) + 1],
                       ha(k, 0), ha(k, 1),
                       firstk ? nullptr : ha(k - 1, 0), firstk ? nullptr : ha(k - 1, 1),
                       (d.iso && !firstk) ? hn(k - 1) : nullptr, q, lam, rho,
                       part + (size_t)(K - k) * BL.nstrips * 2, twW, H, BL.R, BL.nstrips, Pm};
            if ((e = with_row(N, [&](auto ops) { return decltype(ops)::bwd_pass_a(ba, d.iso != 0, lastk, firstk, s); })))
                return e;
        }
        cur = 1 - cur;
        ain = 1 - ain;
    }
    if (glam && grho) {
        const long long spm = BL.nstrips / G;  // strips of one module (module-major planes)
        for (int g = 0; g < G; ++g) {
            if ((e = bwd_scalars<float>(part, K, BL.nstrips, spm, (long long)g * spm, d.iso ? tpart : nullptr, BL.ntp, G, g,
                                        lam + g, rho + g, glam + g, grho + g, s)))
                return e;
        }
    } else if (glam || grho) {
        return fail(ADMM_TV_EINVAL, "glam and grho must be given together");
    }
    if (psf_grad) {  // Z = sum_p conj(Bbar_p) Xin_p, then the k x k taps
        if ((e = with_row(N, [&](auto ops) { return decltype(ops)::r2c(bbar, spec[0], twW, rows, s); }))) return e;
        if ((e = with_row(N, [&](auto ops) { return decltype(ops)::r2c(xin, spec[1], twW, rows, s); }))) return e;
        if ((e = xspec(H, spec[0], spec[1], at<cf>(ws, BL.xpart), twH, N, (int)P, BL.xppg, s))) return e;
        hipLaunchKernelGGL(k_xspec_reduce, dim3((unsigned)((nf + 255) / 256)), dim3(256), 0, s, at<cf>(ws, BL.xpart),
                           BL.xgroups, nf, nullptr, at<double2>(ws, BL.zacc));
        if ((e = launch_check("k_xspec_reduce"))) return e;
        hipLaunchKernelGGL(k_psf_grad<float>, dim3(d.kh * d.kw), dim3(256), 0, s, at<double2>(ws, BL.aacc),
                           at<double2>(ws, BL.zacc), at<double2>(ws, Lo.sigma), d.kh, H, W, gkern, 0.25);
        if ((e = launch_check("k_psf_grad"))) return e;
    }
    if (gxin && G > 1) {  // the modules share xin: x^_in collects every module's b^
        const long long n4 = Pm * H * W / 4;
        float* sum = d.kh > 0 ? bbar : gxin;  // with a PSF, sum in place (module 0's slot) first
        hipLaunchKernelGGL(k_sum_modules, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s,
                           reinterpret_cast<const float4*>(bbar), reinterpret_cast<float4*>(sum), G, n4);
        if ((e = launch_check("k_sum_modules"))) return e;
    }
    if (gxin && d.kh > 0) {
        // x^_in = H_t^T b^ : the conjugate multiplier (pass B mode 2)
        if ((e = psf_transpose_into(d, Lo, ws, bbar, gxin, spec[0], 2, s))) return e;
    }
    return 0;
}

int admm_tv_psf_transpose(const admm_tv_desc* dp, const float* xin, const float* kern, float* out, void* ws,
                          size_t ws_bytes, void* stream) {
    if (int e = validate(dp)) return e;
    if (is_f64(*dp)) return fail(ADMM_TV_EINVAL, "ADMM_TV_FLAG_F64: fp32 entry point");
    const admm_tv_desc d = *dp;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    DeviceGuard dg(reinterpret_cast<hipStream_t>(stream));
    if (dg.err != hipSuccess) return fail(ADMM_TV_EHIP, std::string("device of the stream: ") + hipGetErrorString(dg.err));
    const Layout Lo = make_layout(d);
    if (!ws || ws_bytes < Lo.total) return fail(ADMM_TV_EWORKSPACE, "workspace too small");
    const long long P = d.B * d.C;
    const int H = (int)d.H, W = (int)d.W, N = W / 2;
    if (d.kh == 0) {
        HIPCHK(hipMemcpyAsync(out, xin, (size_t)P * H * W * sizeof(float), hipMemcpyDeviceToDevice, s));
        return 0;
    }
    if (int e = setup<float>(d, Lo, ws, kern, nullptr, s)) return e;
    const int n = (N + 1) * H;
    // k_spectra needs a rho pointer: point it at a zeroed float inside the workspace (fcT region)
    HIPCHK(hipMemsetAsync(at<float>(ws, Lo.fcT), 0, sizeof(float), s));
    hipLaunchKernelGGL(k_spectra<float>, dim3((n + 255) / 256), dim3(256), 0, s, at<double2>(ws, Lo.G),
                       at<double2>(ws, Lo.twHd), at<float>(ws, Lo.fcT), at<float>(ws, Lo.spec[1]),
                       at<cf>(ws, Lo.mT), d.kh, H, N, W, nullptr, spectra_scale(H, W));
    if (int e = launch_check("k_spectra")) return e;
    if (Lo.gen) return gapply(xin, out, at<cf>(ws, Lo.spec[0]), Lo, ws, d, 1, s);
    return psf_transpose_into(d, Lo, ws, xin, out, at<cf>(ws, Lo.spec[0]), 1, s);
}

int admm_tv_forward_f64(const admm_tv_desc* dp, const double* xin, const double* kern, const double* lam,
                        const double* rho, double* out, void* ws, size_t ws_bytes, void* stream) {
    if (int e = validate(dp)) return e;
    if (!is_f64(*dp)) return fail(ADMM_TV_EINVAL, "admm_tv_forward_f64 needs ADMM_TV_FLAG_F64");
    if (((!xin || !out) && !participate_only(*dp)) || !lam || !rho || (dp->kh > 0 && !kern))
        return fail(ADMM_TV_EINVAL, "null pointer argument");
    DeviceGuard dg(reinterpret_cast<hipStream_t>(stream));
    if (dg.err != hipSuccess) return fail(ADMM_TV_EHIP, std::string("device of the stream: ") + hipGetErrorString(dg.err));
    return run_forward_f64(*dp, xin, kern, lam, rho, out, ws, ws_bytes, nullptr, reinterpret_cast<hipStream_t>(stream));
}

int admm_tv_forward_train_f64(const admm_tv_desc* dp, const double* xin, const double* kern, const double* lam,
                              const double* rho, double* out, void* hist, size_t hist_bytes, void* ws, size_t ws_bytes,
                              void* stream) {
    if (int e = validate(dp)) return e;
    if (!is_f64(*dp)) return fail(ADMM_TV_EINVAL, "admm_tv_forward_train_f64 needs ADMM_TV_FLAG_F64");
    if (((!xin || !out) && !participate_only(*dp)) || !lam || !rho || (dp->kh > 0 && !kern))
        return fail(ADMM_TV_EINVAL, "null pointer argument");
    if (dp->maxit > 0 && (!hist || hist_bytes < make_hist(*dp).total))
        return fail(ADMM_TV_EWORKSPACE, "history buffer too small");
    DeviceGuard dg(reinterpret_cast<hipStream_t>(stream));
    if (dg.err != hipSuccess) return fail(ADMM_TV_EHIP, std::string("device of the stream: ") + hipGetErrorString(dg.err));
    return run_forward_f64(*dp, xin, kern, lam, rho, out, ws, ws_bytes, dp->maxit > 0 ? hist : nullptr,
                           reinterpret_cast<hipStream_t>(stream));
}

int admm_tv_backward_f64(const admm_tv_desc* dp, const double* xin, const double* kern, const double* lam,
                         const double* rho, const double* gout, const void* hist, size_t hist_bytes, double* gxin,
                         double* glam, double* grho, double* gkern, void* ws, size_t ws_bytes, void* stream) {
    if (int e = validate(dp)) return e;
    if (!is_f64(*dp)) return fail(ADMM_TV_EINVAL, "admm_tv_backward_f64 needs ADMM_TV_FLAG_F64");
    if ((!gout && !participate_only(*dp)) || !lam || !rho || (dp->kh > 0 && !kern))
        return fail(ADMM_TV_EINVAL, "null pointer argument");
    DeviceGuard dg(reinterpret_cast<hipStream_t>(stream));
    if (dg.err != hipSuccess) return fail(ADMM_TV_EHIP, std::string("device of the stream: ") + hipGetErrorString(dg.err));
    return run_backward_f64(*dp, xin, kern, lam, rho, gout, hist, hist_bytes, gxin, glam, grho, gkern, ws, ws_bytes,
                            reinterpret_cast<hipStream_t>(stream));
}

int admm_tv_profile_enable(int enable) {
    std::lock_guard<std::mutex> lk(g_prof.mu);
    g_prof.on = enable != 0;
    return 0;
}

int admm_tv_profile_reset(void) {
    std::lock_guard<std::mutex> lk(g_prof.mu);
    for (auto& r : g_prof.recs) {
        (void)hipEventSynchronize(r.b);
        g_prof.pool.push_back({r.dev, r.a});
        g_prof.pool.push_back({r.dev, r.b});
    }
    g_prof.recs.clear();
    for (int i = 0; i < 4; ++i) {
        g_prof.ms[i] = 0;
        g_prof.n[i] = 0;
    }
    return 0;
}

int admm_tv_profile_read(double* ms4, int64_t* count4) {
    std::lock_guard<std::mutex> lk(g_prof.mu);
    for (auto& r : g_prof.recs) {
        if (hipEventSynchronize(r.b) != hipSuccess) return fail(ADMM_TV_EHIP, "hipEventSynchronize");
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
            g_prof.ms[r.kind] += ms;
            g_prof.n[r.kind] += 1;
        }
        g_prof.pool.push_back({r.dev, r.a});
        g_prof.pool.push_back({r.dev, r.b});
    }
    g_prof.recs.clear();
    for (int i = 0; i < 4; ++i) {
        if (ms4) ms4[i] = g_prof.ms[i];
        if (count4) count4[i] = g_prof.n[i];
    }
    return 0;
}

}  // extern "C"

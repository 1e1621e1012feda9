// fft_core.hpp -- register/LDS FFT building blocks for the ADMM-TV passes (gfx950).
//
// Layout convention used everywhere ("natural layout"): a transform of length N
// is owned by a group of L lanes ("sub-group"), each lane holding E = N / L
// complex values in registers; lane t, register j holds element  t + L*j.
// Coalesced global loads/stores of consecutive elements therefore map 1:1 onto
// registers, and a Stockham autosort FFT whose first and last stages read and
// write exactly that layout needs LDS only between stages.
//
// Stockham radix-R stage at span NS (Govindaraju et al. formulation): virtual
// thread vt in [0, N/R) takes inputs vt + k*N/R, multiplies input k by
// W_{NS*R}^{(vt mod NS) k}, runs an R-point DFT and writes output k to
// (vt/NS)*NS*R + (vt mod NS) + k*NS.  A lane runs Q = E/R virtual threads
// vt = t + L*q, so its inputs sit in registers q + Q*k (natural layout) and, at
// the last stage (NS*R = N), its outputs land in the same registers.
//
// Twiddles come from an accurate table tw[i] = exp(-2*pi*i*i_/TWN) (computed in
// fp64 on the device, stored fp32): W_{NS*R}^m = tw[m * TWN/(NS*R)].
#pragma once
#include <hip/hip_runtime.h>
#include <type_traits>

namespace admm {

typedef float2 cf;

__device__ __forceinline__ cf mkc(float r, float i) { cf z; z.x = r; z.y = i; return z; }
__device__ __forceinline__ cf cadd(cf a, cf b) { return mkc(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ cf csub(cf a, cf b) { return mkc(a.x - b.x, a.y - b.y); }
// Complex products with explicit fused multiply-adds.  The library is compiled with
// -ffp-contract=off, so every rounding is spelled out here and identical in every
// inlined copy (a row transformed as a halo row rounds exactly like the same row
// transformed as an interior row: results do not depend on strip boundaries).
__device__ __forceinline__ cf cmul(cf a, cf b) {
    return mkc(fmaf(a.x, b.x, -(a.y * b.y)), fmaf(a.x, b.y, a.y * b.x));
}
// a * conj(b)
__device__ __forceinline__ cf cmulc(cf a, cf b) {
    return mkc(fmaf(a.x, b.x, a.y * b.y), fmaf(a.y, b.x, -(a.x * b.y)));
}
__device__ __forceinline__ cf cconj(cf a) { return mkc(a.x, -a.y); }
__device__ __forceinline__ cf cscale(cf a, float s) { return mkc(a.x * s, a.y * s); }
// multiply by DIR*i  (DIR = -1: -i, forward;  DIR = +1: +i, inverse)
template <int DIR> __device__ __forceinline__ cf mul_i(cf a) {
    return DIR < 0 ? mkc(a.y, -a.x) : mkc(-a.y, a.x);
}

// fp64 complex values (the generic kernels' double instantiation: fp64 inputs are solved in fp64,
// as the reference computes in xin.dtype).  Same operation order as the fp32 helpers above.
typedef double2 cd;
__device__ __forceinline__ cd mkcd(double r, double i) { cd z; z.x = r; z.y = i; return z; }
__device__ __forceinline__ cd cadd(cd a, cd b) { return mkcd(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ cd csub(cd a, cd b) { return mkcd(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ cd cmul(cd a, cd b) { return mkcd(fma(a.x, b.x, -(a.y * b.y)), fma(a.x, b.y, a.y * b.x)); }
__device__ __forceinline__ cd cmulc(cd a, cd b) { return mkcd(fma(a.x, b.x, a.y * b.y), fma(a.y, b.x, -(a.x * b.y))); }
__device__ __forceinline__ cd cconj(cd a) { return mkcd(a.x, -a.y); }
__device__ __forceinline__ cd cscale(cd a, double s) { return mkcd(a.x * s, a.y * s); }
template <int DIR> __device__ __forceinline__ cd mul_i(cd a) { return DIR < 0 ? mkcd(a.y, -a.x) : mkcd(-a.y, a.x); }

// real type -> complex type, and a constructor usable from code templated on the real type
template <class T> struct CxOf;
template <> struct CxOf<float> { using type = cf; };
template <> struct CxOf<double> { using type = cd; };
template <class T> using cx_t = typename CxOf<T>::type;
template <class T> __device__ __forceinline__ cx_t<T> mkx(T r, T i) {
    if constexpr (std::is_same<T, float>::value) return mkc(r, i);
    else return mkcd(r, i);
}
// the real type of a complex type (cf -> float, cd -> double)
template <class C> struct ReOf;
template <> struct ReOf<cf> { using type = float; };
template <> struct ReOf<cd> { using type = double; };
template <class C> using re_t = typename ReOf<C>::type;
__device__ __forceinline__ float fmat(float a, float b, float c) { return fmaf(a, b, c); }
__device__ __forceinline__ double fmat(double a, double b, double c) { return fma(a, b, c); }

// cos(2*pi*m/64) for m in [0,16] with exact 0 at m = 16
__device__ __forceinline__ constexpr double cos64q(int m) {
    constexpr double Q[17] = {1.0, 0.99518472667219693, 0.98078528040323043, 0.95694033573220882,
                              0.92387953251128674, 0.88192126434835505, 0.83146961230254524,
                              0.77301045336273699, 0.70710678118654757, 0.63439328416364549,
                              0.55557023301960229, 0.47139673682599781, 0.38268343236508984,
                              0.29028467725446233, 0.19509032201612833, 0.09801714032956077, 0.0};
    return Q[m];
}
__device__ __forceinline__ constexpr double cos64(int m) {
    m &= 63;
    return m <= 16 ? cos64q(m) : m <= 32 ? -cos64q(32 - m) : m <= 48 ? -cos64q(m - 32) : cos64q(64 - m);
}
__device__ __forceinline__ constexpr double sin64(int m) { return cos64(16 - m); }

// exp(DIR * 2*pi*i * k / R) as a compile-time constant (R | 64)
template <int R, int DIR, int K> struct ConstTw {
    static constexpr int m = (K * (64 / R)) & 63;
    static constexpr float re = (float)cos64(m);
    static constexpr float im = (float)(DIR * sin64(m));
};

template <int R, int DIR, int K> __device__ __forceinline__ cf tw_mul(cf a) {
    constexpr int m = (K * (64 / R)) & 63;
    if constexpr (m == 0) {
        return a;
    } else if constexpr (m == 16) {
        return mul_i<DIR>(a);
    } else if constexpr (m == 32) {
        return mkc(-a.x, -a.y);
    } else if constexpr (m == 48) {
        return mul_i<-DIR>(a);
    } else if constexpr (m == 8 || m == 24 || m == 40 || m == 56) {
        // (+-1 +- i)/sqrt2 : 2 mul + 2 add
        constexpr float h = 0.70710678118654752f;
        constexpr float cr = ConstTw<R, DIR, K>::re, ci = ConstTw<R, DIR, K>::im;
        constexpr float sr = cr > 0 ? 1.f : -1.f, si = ci > 0 ? 1.f : -1.f;
        // (sr + i si) h * (x + i y) = h (sr x - si y) + i h (sr y + si x)
        return mkc(h * (sr * a.x - si * a.y), h * (sr * a.y + si * a.x));  // sr, si = +-1: exact
    } else {
        return cmul(a, mkc(ConstTw<R, DIR, K>::re, ConstTw<R, DIR, K>::im));
    }
}

// ---------------------------------------------------------------------------
// buffer-resource memory access (T8): 32-bit per-lane offset + wave-uniform SGPR
// offset, so strided per-lane streams need one VGPR instead of one 64-bit address
// per element.  Descriptors must be built from wave-uniform values.
// ---------------------------------------------------------------------------
typedef __amdgpu_buffer_rsrc_t rsrc_t;
__device__ __forceinline__ rsrc_t make_rsrc(const void* base, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
// AUX: cache policy bits (2 = nt, streaming)
template <int AUX = 0> __device__ __forceinline__ cf bload_cf(rsrc_t r, int voff, int soff) {
    return __builtin_bit_cast(cf, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, AUX));
}
template <int AUX = 0> __device__ __forceinline__ void bstore_cf(rsrc_t r, int voff, int soff, cf v) {
    typedef decltype(__builtin_amdgcn_raw_buffer_load_b64(r, 0, 0, 0)) V2;
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(V2, v), r, voff, soff, AUX);
}

// Streaming-data cache policy of pass A (-DADMM_NT=mask overrides for A/B runs): bit 0 stores nt,
// bit 1 spectrum loads nt, bit 5 spectrum loads nt only for W >= 1024, bit 4 u / b loads nt; bit 2
// pass B stores nt, bit 3 pass B loads nt.  Default 0x31, measured (tools/ab_variants.sh,
// DESIGN.md §4): C3 666 -> 706 it/s, C2 4702 -> 5213 it/s; nt in pass B is slower (its paired
// column blocks share lines through L2).
#ifndef ADMM_NT
#define ADMM_NT 0x31
#endif
typedef float v2f_t __attribute__((ext_vector_type(2)));
template <bool NT> __device__ __forceinline__ cf ld_pol(const cf* p) {
    if constexpr (NT) return __builtin_bit_cast(cf, __builtin_nontemporal_load(reinterpret_cast<const v2f_t*>(p)));
    else return *p;
}
template <int BIT = 2> __device__ __forceinline__ cf lda(const cf* p) { return ld_pol<(ADMM_NT & BIT) != 0>(p); }
template <bool NT> __device__ __forceinline__ void st_pol(cf* p, cf v) {
    if constexpr (NT) __builtin_nontemporal_store(__builtin_bit_cast(v2f_t, v), reinterpret_cast<v2f_t*>(p));
    else *p = v;
}
// the training backward's reverse row pass (-DADMM_NT_BWD=0 for A/B runs)
#ifndef ADMM_NT_BWD
#define ADMM_NT_BWD 1
#endif
__device__ __forceinline__ void sta(cf* p, cf v) {
    if constexpr ((ADMM_NT & 1) != 0) __builtin_nontemporal_store(__builtin_bit_cast(v2f_t, v), reinterpret_cast<v2f_t*>(p));
    else *p = v;
}
__device__ __forceinline__ float bload_f(rsrc_t r, int voff, int soff) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}

// ---------------------------------------------------------------------------
// in-register DFT of size R (power of two), natural-order in and out.
// v[s*STRIDE] for s in [0,R) are the operands (STRIDE lets a lane run several
// interleaved butterflies over one register array).
// ---------------------------------------------------------------------------
template <int R, int DIR> struct DFT;

template <int DIR> struct DFT<1, DIR> {
    template <int STRIDE, int OFF, int E> __device__ __forceinline__ static void run(cf (&)[E]) {}
};

template <int DIR> struct DFT<2, DIR> {
    template <int STRIDE, int OFF, int E> __device__ __forceinline__ static void run(cf (&v)[E]) {
        cf a = v[OFF], b = v[OFF + STRIDE];
        v[OFF] = cadd(a, b);
        v[OFF + STRIDE] = csub(a, b);
    }
};

template <int DIR> struct DFT<4, DIR> {
    template <int STRIDE, int OFF, int E> __device__ __forceinline__ static void run(cf (&v)[E]) {
        cf a0 = v[OFF], a1 = v[OFF + STRIDE], a2 = v[OFF + 2 * STRIDE], a3 = v[OFF + 3 * STRIDE];
        cf t0 = cadd(a0, a2), t1 = csub(a0, a2), t2 = cadd(a1, a3), t3 = mul_i<DIR>(csub(a1, a3));
        v[OFF] = cadd(t0, t2);
        v[OFF + 2 * STRIDE] = csub(t0, t2);
        v[OFF + STRIDE] = cadd(t1, t3);
        v[OFF + 3 * STRIDE] = csub(t1, t3);
    }
};

// radix-2 decimation in time on top of DFT<R/2>
template <int R, int DIR> struct DFT {
    template <int K, int STRIDE, int OFF, int E>
    __device__ __forceinline__ static void combine(cf (&v)[E], cf (&e)[R / 2], cf (&o)[R / 2]) {
        if constexpr (K < R / 2) {
            cf t = tw_mul<R, DIR, K>(o[K]);
            v[OFF + K * STRIDE] = cadd(e[K], t);
            v[OFF + (K + R / 2) * STRIDE] = csub(e[K], t);
            combine<K + 1, STRIDE, OFF>(v, e, o);
        }
    }
    template <int STRIDE, int OFF, int E> __device__ __forceinline__ static void run(cf (&v)[E]) {
        cf e[R / 2], o[R / 2];
#pragma unroll
        for (int i = 0; i < R / 2; ++i) {
            e[i] = v[OFF + (2 * i) * STRIDE];
            o[i] = v[OFF + (2 * i + 1) * STRIDE];
        }
        DFT<R / 2, DIR>::template run<1, 0>(e);
        DFT<R / 2, DIR>::template run<1, 0>(o);
        combine<0, STRIDE, OFF>(v, e, o);
    }
};

// ---------------------------------------------------------------------------
// Radix schedules: product of radices = N, each radix divides E.
// ---------------------------------------------------------------------------
template <int... Rs> struct Sched {};

template <int N> struct RowCfg;  // transform length N -> E (values per lane), schedule
template <> struct RowCfg<8> { static constexpr int E = 2; using S = Sched<2, 2, 2>; };
template <> struct RowCfg<16> { static constexpr int E = 4; using S = Sched<4, 4>; };
template <> struct RowCfg<32> { static constexpr int E = 4; using S = Sched<4, 4, 2>; };
template <> struct RowCfg<64> { static constexpr int E = 8; using S = Sched<8, 8>; };
template <> struct RowCfg<128> { static constexpr int E = 8; using S = Sched<8, 8, 2>; };
template <> struct RowCfg<256> { static constexpr int E = 8; using S = Sched<8, 8, 4>; };
template <> struct RowCfg<512> { static constexpr int E = 8; using S = Sched<8, 8, 8>; };
template <> struct RowCfg<1024> { static constexpr int E = 16; using S = Sched<16, 16, 4>; };
template <> struct RowCfg<2048> { static constexpr int E = 16; using S = Sched<16, 16, 8>; };
template <> struct RowCfg<4096> { static constexpr int E = 16; using S = Sched<16, 16, 16>; };

// ---------------------------------------------------------------------------
// LDS exchange buffers.  Index -> LDS slot mapping (padding / interleaving).
//   RowBuf: one transform per sub-group, contiguous, padded by 1 slot per 8.
//   ColBuf: C transforms interleaved element-major ([element][C]), column c.
// SYNC: 0 = the sub-group lives in one wave (wave-level ordering suffices),
//       1 = the sub-group spans waves (block barrier).
// ---------------------------------------------------------------------------
struct RowBuf {
    cf* base;
    __device__ __forceinline__ cf& at(int i) const { return base[i + (i >> 3)]; }
    static constexpr int slots(int n) { return n + n / 8; }
};
template <int C> struct ColBuf {
    cf* base;  // already offset by the column index c
    __device__ __forceinline__ cf& at(int i) const { return base[i * C]; }
};

// SYNC 1: a block barrier (__syncthreads: also waits for the wave's outstanding global loads);
// SYNC 2: a block barrier for LDS traffic only, so global loads issued before it stay in flight across it
// (the mixed pass B prefetches the next plane's columns through its inverse transform's exchanges)
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
template <int SYNC> __device__ __forceinline__ void xsync() {
    if constexpr (SYNC == 2) {
        lds_barrier();
    } else if constexpr (SYNC) {
        __syncthreads();
    } else {
        // all lanes of a sub-group are in one wave: LDS ops of a wave execute
        // in order; stop the compiler from moving LDS accesses across.
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

template <int I, int NI, class F> __device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I < NI) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, NI>(f);
    }
}

// One Stockham stage.  The twiddle table holds tw[i] = exp(-2 pi i i_ / (N*TWMUL))
// for i_ in [0, N*TWMUL); W_{NS*R}^{m} = tw[m * (N/(NS*R)) * TWMUL].
template <int N, int L, int E, int R, int NS, int DIR, bool FIRST, bool LAST, int SYNC, int TWMUL, class Buf>
__device__ __forceinline__ void stage(cf (&v)[E], const Buf& buf, const cf* __restrict__ tw, int t) {
    constexpr int Q = E / R;
    if constexpr (!FIRST) {
#pragma unroll
        for (int j = 0; j < E; ++j) v[j] = buf.at(t + L * j);
    }
    static_for<0, Q>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        if constexpr (NS > 1) {
            const int m = (t + L * q) & (NS - 1);
#pragma unroll
            for (int k = 1; k < R; ++k) {
                cf w = tw[(m * k) * (N / (NS * R)) * TWMUL];
                v[q + Q * k] = DIR < 0 ? cmul(v[q + Q * k], w) : cmulc(v[q + Q * k], w);
            }
        }
        DFT<R, DIR>::template run<Q, q>(v);
    });
    if constexpr (!LAST) {
        xsync<SYNC>();  // everyone has read before anyone overwrites
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int vt = t + L * q;
            const int base = (vt / NS) * NS * R + (vt & (NS - 1));
#pragma unroll
            for (int k = 0; k < R; ++k) buf.at(base + k * NS) = v[q + Q * k];
        }
        xsync<SYNC>();
    }
}

template <int N, int L, int E, int NS, int DIR, bool FIRST, int SYNC, int TWMUL, class Buf, int R, int... Rest>
__device__ __forceinline__ void run_sched(cf (&v)[E], const Buf& buf, const cf* __restrict__ tw, int t) {
    constexpr bool LAST = sizeof...(Rest) == 0;
    stage<N, L, E, R, NS, DIR, FIRST, LAST, SYNC, TWMUL>(v, buf, tw, t);
    if constexpr (!LAST) run_sched<N, L, E, NS * R, DIR, false, SYNC, TWMUL, Buf, Rest...>(v, buf, tw, t);
}

template <int N, int L, int DIR, int SYNC, int TWMUL, class Buf, int... Rs>
__device__ __forceinline__ void fft_dispatch(cf (&v)[RowCfg<N>::E], const Buf& buf, const cf* __restrict__ tw, int t,
                                             Sched<Rs...>) {
    run_sched<N, L, RowCfg<N>::E, 1, DIR, true, SYNC, TWMUL, Buf, Rs...>(v, buf, tw, t);
}

// the same with E values per lane and an explicit schedule (each radix divides E)
template <int N, int L, int E, int DIR, int SYNC, int TWMUL, class Buf, int... Rs>
__device__ __forceinline__ void fft_e(cf (&v)[E], const Buf& buf, const cf* __restrict__ tw, int t, Sched<Rs...>) {
    run_sched<N, L, E, 1, DIR, true, SYNC, TWMUL, Buf, Rs...>(v, buf, tw, t);
}

// Full N-point complex FFT (DIR -1 forward / +1 inverse, unnormalised) in natural layout.
template <int N, int L, int DIR, int SYNC, int TWMUL, class Buf>
__device__ __forceinline__ void fft(cf (&v)[RowCfg<N>::E], const Buf& buf, const cf* __restrict__ tw, int t) {
    fft_dispatch<N, L, DIR, SYNC, TWMUL>(v, buf, tw, t, typename RowCfg<N>::S{});
}

}  // namespace admm

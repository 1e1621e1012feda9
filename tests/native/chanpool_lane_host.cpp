// Host build of the one-pixel-per-lane ChannelPool forward (torch-admm-deconv_amd/csrc/chanpool_lane.hpp):
// the kernel's per-pixel function lane_pixel, compiled for the CPU with plain memory accessors, so that
// tests/test_chanpool_lane_host.py can check its logic (sort network, scans, the introsort trace) against
// torch's CPU median / mode and the oracle on many pixels without a GPU.  Test infrastructure only.
//   chanpool_lane_host <bf16|f16> C npix depth_limit in.u16 out.bin
//   in.u16: npix x C values, channel-major ([C][npix]); out.bin: per pixel float std, int32 median
//   channel, int32 mode channel (three arrays of npix).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <vector>

#define __device__
#define __host__
#define __forceinline__ inline
using std::max;
using std::min;
static inline float __uint_as_float(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }
static inline uint32_t __float_as_uint(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
typedef _Float16 __half;
static inline __half __ushort_as_half(unsigned short u) { __half h; std::memcpy(&h, &u, 2); return h; }
static inline unsigned short __half_as_ushort(__half h) { unsigned short u; std::memcpy(&u, &h, 2); return u; }
static inline float __half2float(__half h) { return (float)h; }
static inline __half __float2half_rn(float f) { return (__half)f; }

#include "../../torch-admm-deconv_amd/csrc/chanpool_lane.hpp"

struct HostIo {
    const uint16_t* px;
    long long stride;
    uint32_t load(int c) const { return px[(size_t)c * stride]; }
    uint32_t raw(int c) const { return px[(size_t)c * stride]; }
    int opaque(int v) const { return v; }
    u16x2 pack(uint32_t lo, uint32_t hi) const { return u16x2{(unsigned short)lo, (unsigned short)hi}; }
    void barrier() const {}
};

template <class T, int NP>
static void run(const std::vector<uint16_t>& x, int C, long long npix, int depth, float* sd, int32_t* mi, int32_t* oi) {
    std::vector<uint16_t> col((size_t)(C + 7) * 64);
    for (long long p = 0; p < npix; ++p) {
        HostIo io{x.data() + p, npix};
        int m, o;
        lane_pixel<T, NP>(io, col.data() + 3 * 64, C, depth, sd[p], m, o);
        mi[p] = m;
        oi[p] = o;
    }
}

int main(int argc, char** argv) {
    if (argc != 7) {
        std::fprintf(stderr, "usage: %s <bf16|f16> C npix depth_limit in.u16 out.bin\n", argv[0]);
        return 2;
    }
    const bool bf = std::strcmp(argv[1], "bf16") == 0;
    const int C = std::atoi(argv[2]), depth = std::atoi(argv[4]);
    const long long npix = std::atoll(argv[3]);
    if (C < 1 || C > 128 || npix < 1) return 2;
    std::vector<uint16_t> x((size_t)C * npix);
    FILE* f = std::fopen(argv[5], "rb");
    if (!f || std::fread(x.data(), 2, x.size(), f) != x.size()) return 3;
    std::fclose(f);
    std::vector<float> sd(npix);
    std::vector<int32_t> mi(npix), oi(npix);
    if (bf) {
        if (C <= 64) run<BF16T, 64>(x, C, npix, depth, sd.data(), mi.data(), oi.data());
        else run<BF16T, 128>(x, C, npix, depth, sd.data(), mi.data(), oi.data());
    } else {
        if (C <= 64) run<F16T, 64>(x, C, npix, depth, sd.data(), mi.data(), oi.data());
        else run<F16T, 128>(x, C, npix, depth, sd.data(), mi.data(), oi.data());
    }
    FILE* g = std::fopen(argv[6], "wb");
    if (!g) return 3;
    std::fwrite(sd.data(), 4, npix, g);
    std::fwrite(mi.data(), 4, npix, g);
    std::fwrite(oi.data(), 4, npix, g);
    std::fclose(g);
    return 0;
}

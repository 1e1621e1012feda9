// odd_capi.hip -- launchers of the fused odd-length row pass (odd_kernels.hpp).
#include "odd_capi.hpp"

#include <algorithm>

#include "odd_kernels.hpp"

namespace admm_odd {

using namespace admm;

namespace {

constexpr int kThreads = ADMM_ODD_NT;  // independent waves per block x 64 (a launch granule, no barrier)

template <int W1, int W2, int NLD> struct Inst {
    static constexpr int W = W1 * W2;
    static constexpr int RS = 2 * NLD;
    static hipError_t launch(const OddPassAArgs& a, bool first, hipStream_t s) {
        const size_t lds = (size_t)(kThreads / 64) * odd_wave_lds<W, NLD>();
        const unsigned blocks = (unsigned)((a.nstrips + kThreads / 64 - 1) / (kThreads / 64));
        auto kern = first ? k_pass_a_odd<W1, W2, NLD, true> : k_pass_a_odd<W1, W2, NLD, false>;
        if (lds > 64 * 1024) {
            const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(kThreads), lds, s, a);
        return hipGetLastError();
    }
};

// instances: BSD's 481 = 13 * 37 (3 row pairs + the halo line per wave: 17.3 KB of LDS; A/B builds:
// -DADMM_ODD_NLD row pairs per wave)
#ifndef ADMM_ODD_NLD
#define ADMM_ODD_NLD 3
#endif
using I481 = Inst<13, 37, ADMM_ODD_NLD>;

// out[p][j][i] = in[p][i][j]: 32 x 32 tiles through LDS (odd word pitch: no bank conflicts), both sides
// coalesced; planes on grid.z (strided beyond 65,535)
__global__ void __launch_bounds__(256) k_transpose(const float* __restrict__ in, float* __restrict__ out, int H, int W,
                                                   long long P) {
    __shared__ float t[32][33];
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8 threads
    const int j0 = blockIdx.x * 32, i0 = blockIdx.y * 32;
    for (long long p = blockIdx.z; p < P; p += gridDim.z) {
        const float* src = in + (size_t)p * H * W;
        float* dst = out + (size_t)p * H * W;
        for (int r = ty; r < 32; r += 8) {
            const int i = i0 + r, j = j0 + tx;
            if (i < H && j < W) t[r][tx] = src[(size_t)i * W + j];
        }
        __syncthreads();
        for (int r = ty; r < 32; r += 8) {
            const int j = j0 + r, i = i0 + tx;
            if (i < H && j < W) dst[(size_t)j * H + i] = t[tx][r];
        }
        __syncthreads();
    }
}

}  // namespace

hipError_t transpose(const float* in, float* out, int H, int W, long long P, hipStream_t s) {
    if (P <= 0) return hipSuccess;
    const dim3 grid((unsigned)((W + 31) / 32), (unsigned)((H + 31) / 32), (unsigned)std::min<long long>(P, 65535));
    hipLaunchKernelGGL(k_transpose, grid, dim3(256), 0, s, in, out, H, W, P);
    return hipGetLastError();
}

bool row_ok(int W) { return W == I481::W; }

int strip_rows(int W) { return W == I481::W ? I481::RS : 0; }

hipError_t pass_a(int W, const OddPassAArgs& a, bool first, hipStream_t s) {
    if (W == I481::W) return I481::launch(a, first, s);
    return hipErrorInvalidValue;
}

}  // namespace admm_odd

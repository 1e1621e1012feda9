// odd_capi.hip -- launchers of the fused odd-length row pass (odd_kernels.hpp).
#include "odd_capi.hpp"

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

}  // namespace

bool row_ok(int W) { return W == I481::W; }

int strip_rows(int W) { return W == I481::W ? I481::RS : 0; }

hipError_t pass_a(int W, const OddPassAArgs& a, bool first, hipStream_t s) {
    if (W == I481::W) return I481::launch(a, first, s);
    return hipErrorInvalidValue;
}

}  // namespace admm_odd

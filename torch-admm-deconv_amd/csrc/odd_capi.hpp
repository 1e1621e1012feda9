// odd_capi.hpp -- launchers of the fused odd-length row pass (odd_kernels.hpp), compiled in their own
// translation unit (odd_capi.hip) and called by the generic solve's orchestration in admm_capi.hip.
#pragma once
#include <hip/hip_runtime.h>

#include "admm_kernels.hpp"

namespace admm {
// arguments of the fused odd-length row pass (odd_kernels.hpp k_pass_a_odd)
struct OddPassAArgs {
    const cf* sin;    // x half spectra (output of the column pass)   [P][H][ld]
    cf* sout;         // r half spectra for the next column pass       [P][H][ld]
    const float* b;   // H_t(xin)                                      [P][H][W]
    const float* uxi; // u_{k-1}
    const float* uyi;
    float* uxo;       // u_k
    float* uyo;
    const float* lam;
    const float* rho;
    int H, ld;        // rows per plane, spectrum row pitch (complex values, >= W/2 + 1)
    int ns;           // strips per plane
    long long nstrips;  // P ns
};
}

namespace admm_odd {

// a fused row pass instance exists for the row length W (odd, W = W1 W2 with both factors in registers)
bool row_ok(int W);
// rows per strip (one wave each) of the instance for W
int strip_rows(int W);
// pass A of one iteration over a.nstrips strips; first: u_{k-1} = 0 (not read)
hipError_t pass_a(int W, const admm::OddPassAArgs& a, bool first, hipStream_t s);
// out[p][j][i] = in[p][i][j] for P planes of H x W floats (the transposed odd-length solve, odd_t_hw)
hipError_t transpose(const float* in, float* out, int H, int W, long long P, hipStream_t s);

}  // namespace admm_odd

// odd_capi.hpp -- launchers of the fused odd-length row pass (odd_kernels.hpp), compiled in their own
// translation unit (odd_capi.hip) and called by the generic solve's orchestration in admm_capi.hip.
#pragma once
#include <hip/hip_runtime.h>

#include "admm_kernels.hpp"

namespace admm {
struct OddPassAArgs;
}

namespace admm_odd {

// a fused row pass instance exists for the row length W (odd, W = W1 W2 with both factors in registers)
bool row_ok(int W);
// rows per strip (one wave each) of the instance for W
int strip_rows(int W);
// pass A of one iteration over a.nstrips strips; first: u_{k-1} = 0 (not read)
hipError_t pass_a(int W, const admm::OddPassAArgs& a, bool first, hipStream_t s);

}  // namespace admm_odd

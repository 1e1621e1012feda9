// mixed_capi.hpp -- launchers of the mixed-radix fused kernels (mixed_kernels.hpp), compiled in their
// own translation unit (mixed_capi.hip) and called by the solver's orchestration in admm_capi.hip.
// Every launcher returns hipSuccess or the launch error.
#pragma once
#include <hip/hip_runtime.h>

#include "admm_backward.hpp"
#include "admm_kernels.hpp"

namespace admm_mixed {

using admm::cf;

// plans exist for the row length N = W/2 / the column length H
bool row_ok(int N);
bool col_ok(int H);
int col_cols(int H);  // the fewest columns per column-pass block (N must be a multiple)
int pass_b_cols(int H, int N);  // the columns per block pass_b launches (0: N fits no plan)
int row_lanes(int N);  // lanes of a row group (up to 256: several waves)
int pass_a_blocks_per_cu(int N);  // resident 256-thread blocks of the row pass per CU (occupancy query)

hipError_t r2c(int N, const float* img, cf* spec, const cf* twW, long long rows, hipStream_t s);
hipError_t c2r(int N, const cf* spec, float* img, const cf* twW, long long rows, hipStream_t s);
// hist: the training forward (a_k into the history; admm_kernels.hpp k_pass_a HIST)
hipError_t pass_a(int N, const admm::PassAArgs& a, bool iso, bool first, bool hist, hipStream_t s);
hipError_t iso_norm(int N, const admm::IsoArgs& a, bool first, bool hist, hipStream_t s);
// the training backward's reverse row pass and iso Q pass (admm_backward.hpp, mixed transforms)
hipError_t bwd_pass_a(int N, const admm::BwdArgs& a, bool iso, bool lastk, bool firstk, hipStream_t s);
hipError_t bwd_iso_q(int N, const admm::BwdIsoArgs& a, bool lastk, hipStream_t s);
hipError_t pass_b(int H, cf* spec, const float* fcM, const cf* twH, int N, long long P, hipStream_t s);
// fcM: [H][N + 1] then the column-block-packed copy [N / C][H][C] (C = pass_b_cols): H (2N + 1) floats
hipError_t fc_mixed(const float* fcT, float* fcM, int H, int N, hipStream_t s);
// b = H_t(xin) on the mixed transforms: the column pass with the complex PSF multiplier mM ([H][N + 1],
// mt_mixed of the generic path's mT [N + 1][H], halved for the packed row transforms)
hipError_t pass_b_cm(int H, cf* spec, const cf* mM, const cf* twH, int N, long long P, hipStream_t s);
hipError_t mt_mixed(const cf* mT, cf* mM, int H, int N, hipStream_t s);

}  // namespace admm_mixed

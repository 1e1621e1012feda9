/* admm_chanstat.h -- C ABI of the per-pixel channel statistics used by the config-5 caller.
 *
 * Replaces the reference's ChannelPool (/root/reference/src/admmtor/elayers/attentions.py:36-47),
 * the spatial gate of CBAM inside DivergentAttention:
 *
 *     torch.cat((torch.std(x, 1), torch.median(x, 1).values, torch.mode(x, 1).values), dim=1)
 *
 * which PyTorch runs as three separate sort/select reductions over the channel dim
 * (46 % of the config-5 training step on MI355X, profiles/r01_c5_kernel_stats.csv).  Here it is
 * one kernel: each lane owns a pixel, sorts its C channel values in LDS as
 * (order-preserving value bits, channel index) keys, and writes all three statistics plus the
 * two selected channel indices (for the backward scatter).
 *
 * Semantics (the reference's CPU rules; PyTorch's GPU mode leaves ties unspecified):
 *   std    : unbiased (C - 1), evaluated in fp64 (two-pass) and rounded to the input dtype;
 *   median : lower median, the element at position (C-1)/2 of a STABLE ascending sort
 *            (value and index as torch.median on the CPU);
 *   mode   : the smallest of the most frequent values (== ties: -0.0 == +0.0); its index is the
 *            one torch.mode on the CPU returns: the channel of the last element of that value's
 *            run after libstdc++ std::sort of the (value, channel) pairs compared by value
 *            (introsort; not stable for C > 16, so the kernel runs the same algorithm);
 *   NaN    : unpinned (the reference's `<` comparator is not a strict weak order with NaN);
 *            here every NaN sorts above +inf. */

/* (the backward of the three statistics, admm_chanstat_pool_backward below)
 *   gx[c] = g_std (x_c - mean) / ((C-1) std) + [c == median idx] g_median + [c == mode idx] g_mode
 * the reference's std_backward / value_selecting_reduction_backward, evaluated in fp32 with the
 * forward's (rounded) std and rounded once to the dtype; where the std is 0 its term is 0 (as the
 * reference's masked_fill_).
 *
 * Conventions as admm_tv.h: DEVICE pointers, C-contiguous, `stream` a hipStream_t as void*,
 * asynchronous, 0 on success or a negative ADMM_TV_E* code (admm_tv.h).
 */
#ifndef ADMM_CHANSTAT_H
#define ADMM_CHANSTAT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    ADMM_CHANSTAT_F32 = 0,
    ADMM_CHANSTAT_BF16 = 1,
    ADMM_CHANSTAT_F16 = 2
};

/* largest channel count the kernel takes for a dtype (256 for 16-bit types, 128 for fp32) */
int admm_chanstat_max_channels(int dtype);

/* x   : [B][C][HW] elements of `dtype`
 * out : [B][3][HW] of `dtype`: std, median, mode (ChannelPool's output layout)
 * idx : [B][2][HW] int16 channel indices of the median and the mode, or NULL */
int admm_chanstat_pool(int dtype, const void* x, int64_t B, int64_t C, int64_t HW, void* out, int16_t* idx,
                       void* stream);

/* test hook: admm_chanstat_pool with the introsort depth budget forced to `depth_limit` (0..16;
 * -1 = std::sort's own 2*floor(log2 C)), so the heapsort fallback can be checked against the
 * oracle on ordinary inputs */
int admm_chanstat_pool_depth(int dtype, const void* x, int64_t B, int64_t C, int64_t HW, void* out, int16_t* idx,
                             int depth_limit, void* stream);

/* x, out, idx : as admm_chanstat_pool returned them (idx required)
 * gout        : [B][3][HW] gradient of `out`
 * gx          : [B][C][HW] gradient of x (written, not accumulated) */
int admm_chanstat_pool_backward(int dtype, const void* x, const void* out, const int16_t* idx, const void* gout,
                                int64_t B, int64_t C, int64_t HW, void* gx, void* stream);

/* ---- whole-plane median and mode (ChannelWiseAttention's amedian / amodes, reference
 * elayers/cwa.py: x.view(B, C, -1).median(-1) / .mode(-1)).
 * x          : [P][N] elements of `dtype` (ADMM_CHANSTAT_BF16 or _F16; ADMM_CHANSTAT_F32 for
 *              the median only: mode_idx must then be NULL, else ADMM_TV_EUNSUPPORTED)
 * median_idx : [P] int64, flat index of torch.median's (CPU) element, or NULL; a plane holding
 *              NaN gives its first NaN, as torch.median does
 * mode_idx   : [P] int64, flat index of torch.mode's (CPU) element, or NULL
 * ws         : device workspace of admm_planestat_workspace_size(P, N) bytes (24 N B per plane)
 * depth_limit: -1 (std::sort's 2*floor(log2 N)); >= 0 forces the introsort depth budget (tests)
 * Values are x at those indices; semantics as ChannelPool's median / mode above. */
int admm_planestat_workspace_size(int64_t P, int64_t N, size_t* bytes);
int admm_planestat_median_mode(int dtype, const void* x, int64_t P, int64_t N, int64_t* median_idx,
                               int64_t* mode_idx, void* ws, size_t ws_bytes, int depth_limit, void* stream);

/* The same selection for any of the three dtypes (fp32 included) from per-plane statistics the
 * caller computed (e.g. from a segmented sort): stats[P][4] int32 = {mode code, mode count,
 * median code, rank of the median within its run of equal values}, codes being the
 * order-preserving unsigned images of the value bits (-0 folded onto +0, NaN the all-ones code;
 * 32-bit codes stored as their int32 bit patterns). */
int admm_planestat_select(int dtype, const void* x, int64_t P, int64_t N, const int32_t* stats, int64_t* median_idx,
                          int64_t* mode_idx, void* ws, size_t ws_bytes, int depth_limit, void* stream);

#ifdef __cplusplus
}
#endif
#endif

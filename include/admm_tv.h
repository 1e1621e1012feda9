/* admm_tv.h -- C ABI of the MI355X (gfx950) ADMM-TV deconvolution library.
 *
 * This is the drop-in boundary for the hot path of georgegrosu1/torch-admm-deconv
 * ("admmtor").  The reference is pure Python/PyTorch, so its "FFI" for this path
 * is the Python call  admmtor.eops.deconv.fft_admm_tv(xin, lmbd, rho, kern, iso,
 * maxit)  (/root/reference/src/admmtor/eops/deconv.py:35-40) and the module
 * ADMMDeconv.forward (/root/reference/src/admmtor/elayers/admmdeconv.py:63-64).
 * The Python mirror in torch-admm-deconv_amd/admmtor binds the entry points below
 * through ctypes (see INTEGRATION.md for the binding a maintainer would add).
 *
 * Conventions
 *  - All pointers are DEVICE pointers (hipMalloc / PyTorch caching allocator),
 *    fp32, C-contiguous NCHW.  lambda / rho are device scalars, read on the GPU
 *    (no host synchronisation, graph-capturable).
 *  - `stream` is a hipStream_t passed as void* (0 = legacy default stream).
 *    Every call is asynchronous with respect to the host, like an ATen op.
 *  - The caller owns input, output and workspace.  The workspace must be at
 *    least admm_tv_workspace_size() bytes and 256-byte aligned.
 *  - Return value: 0 on success, a negative ADMM_TV_E* code otherwise.  Error
 *    classes mirror the reference's exceptions: the Python
 *    wrapper validates shapes first (ValueError / IndexError / RuntimeError as
 *    the reference raises them) and maps any native error to RuntimeError.
 */
#ifndef ADMM_TV_H
#define ADMM_TV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ADMM_TV_ABI_VERSION 7

enum {
    ADMM_TV_OK = 0,
    ADMM_TV_EINVAL = -1,        /* null pointer / negative sizes / maxit < 0       */
    ADMM_TV_EUNSUPPORTED = -2,  /* H, W not supported (admm_tv_supported == 0)               */
    ADMM_TV_ENONSQUARE = -3,    /* kh != kw  (reference: RuntimeError, deconv.py:90-96) */
    ADMM_TV_EWORKSPACE = -4,    /* workspace too small / misaligned                 */
    ADMM_TV_EHIP = -5,          /* a HIP runtime call or kernel launch failed       */
    ADMM_TV_EKERNEL = -6        /* PSF larger than the image                        */
};

/* Cross-rank reduction for iso (block) shrinkage over a batch sharded across GPUs
 * (SURVEY.md §8 e2).  The per-pixel norm couples every (b,c) plane, so each iteration the
 * library calls allreduce(buf, count, stream, allreduce_ctx) on its per-pixel sums
 * (count = groups*2*H*W floats, device memory inside the caller's workspace or history
 * buffer) and expects an in-place SUM all-reduce ordered on `stream` (e.g. RCCL).  The
 * backward calls it the same way on the cross-plane products Q.  The callback runs on the
 * calling thread, inside the admm_tv_forward* / admm_tv_backward call that was given it. */
typedef void (*admm_tv_allreduce_fn)(float* buf, size_t count, void* stream, void* ctx);

/* Problem descriptor.  Replaces the shapes/flags of fft_admm_tv's arguments
 * (deconv.py:35-42): xin (B,C,H,W), kern (1,1,kh,kw) or empty (kh = kw = 0),
 * iso (False = soft/anisotropic shrink, True = block shrink with the per-pixel
 * norm over batch AND channel, deconv.py:19-24), maxit (>= 0).
 * Sizes: see admm_tv_supported.
 *
 * groups (0 or 1: one solve): G > 1 solves G modules that share the input xin and the
 * PSF but have their own lambda[g], rho[g] (device arrays of G floats) in one pass
 * sequence -- the two ADMMDeconv modules of DivergentAttention's first level
 * (blocks.py:187-196).  out / gout / history then hold G*B*C planes (module-major),
 * glam / grho G values, gxin the sum over modules.  Each module's iso norm runs over its
 * own (B,C).  No PSF gradient.  Power-of-two sizes: every launch covers all modules' planes
 * (inference and training); smooth sizes (admm_tv_supported == 3): the modules are solved one
 * after another inside the call, sharing b = H_t(xin) and the tables -- inference only
 * (training entry points return ADMM_TV_EUNSUPPORTED there: one call per module).
 *
 * allreduce / allreduce_ctx: the per-call cross-rank hook above (NULL: single process;
 * ignored for iso = 0).  Everything a call needs is in its arguments: the library keeps no
 * per-solve global state, so calls on different threads / streams are independent.
 * With a hook, B*C may be 0 (a rank whose shard is empty): the call then only takes part
 * in the reductions (zeros), so the other ranks' collectives complete. */
typedef struct admm_tv_desc {
    int64_t B, C, H, W;
    int32_t kh, kw;
    int32_t iso;
    int32_t maxit;
    int32_t flags;   /* ADMM_TV_FLAG_*; 0 for plain use */
    int32_t groups;  /* modules solved together (0 or 1: one) */
    admm_tv_allreduce_fn allreduce;  /* iso over a sharded batch; NULL otherwise */
    void* allreduce_ctx;
} admm_tv_desc;

/* flags: the training forward also keeps the spectra of every r_k so that
 * admm_tv_backward can form the PSF gradient (history grows by 4 B/pixel/iteration). */
#define ADMM_TV_FLAG_PSF_GRAD 1
/* flags: fp64 solve.  The reference computes in xin.dtype (deconv.py:49,61-67,104-106), so fp64
 * callers get fp64 arithmetic: every array of the *_f64 entry points below is double (input, PSF,
 * lambda, rho, output, gradients; the all-reduce hook's buffer holds `count` doubles), and the
 * size queries (admm_tv_workspace_size, admm_tv_history_size, admm_tv_backward_workspace_size)
 * return the fp64 sizes.  fp64 solves run on the generic (any-size) kernels' double instantiation at
 * every H, W that admm_tv_supported_f64 accepts; groups must be 0 or 1. */
#define ADMM_TV_FLAG_F64 2

/* ABI version (ADMM_TV_ABI_VERSION). */
int admm_tv_abi_version(void);

/* Provenance: the first 16 hex digits of the SHA-256 of the sources the library was built
 * from (the .hip / .hpp files of csrc, the .h files of include, csrc/Makefile). */
const char* admm_tv_build_hash(void);

/* 1: (H, W) runs on the fused power-of-two kernels (H in [16,4096], W in [16,2048]);
 * 3: a smooth size (2^a 3^b 5^c with a transform plan: W/2 in {240, 320, 360, 400, 480, 540, 640, 720,
 *    800, 960, 1280, 1920} or a power of two up to 2048, H in {240, 360, 480, 540, 600, 720, 768, 800,
 *    960, 1080, 1200, 1440, 1536, 2160} or a power of two up to 4096, W/2 even, e.g. 1080x1920,
 *    720x1280, 480x640, 2160x3840, 600x800): admm_tv_forward runs the same fused two-pass iteration
 *    with mixed-radix register transforms (ABI v6), and so do the training forward / backward of
 *    one module without a PSF gradient (with one, or with grouped modules, they run on the generic
 *    kernels, as for 2);
 * 4: an odd row length with a fused row pass instance (W = 481 = 13 * 37, the BSD image width, any H up
 *    to 65,536): admm_tv_forward's aniso solve runs the two-launch iteration -- the generic column pass
 *    and ONE row pass (inverse rows, step, forward rows; prime-factor transforms in LDS, ABI v7) -- iso
 *    and the training entry points run on the generic kernels, as for 2;
 * 2: any other size up to 65,536 points per side, run on the generic kernels (mixed-radix
 *    transforms, per-pixel step; the reference accepts any size, deconv.py:103-106): lines up to
 *    10,240 points transform in the kernels' LDS image, longer ones in a global scratch slot per
 *    block (part of the workspace);
 * 0: unsupported. */
int admm_tv_supported(int64_t H, int64_t W);

/* The kernel path a solve of `desc` takes (train = 0: admm_tv_forward; 1: admm_tv_forward_train and
 * admm_tv_backward): one of the ADMM_TV_PATH_* codes, or a negative ADMM_TV_E* code for an invalid
 * descriptor.  Host-only (no device call); tests and benchmarks name the path they measured with it. */
#define ADMM_TV_PATH_FUSED 1    /* power-of-two two-pass iteration (admm_kernels.hpp) */
#define ADMM_TV_PATH_GENERIC 2  /* generic kernels: column pass, row inverse, step + row forward */
#define ADMM_TV_PATH_MIXED 3    /* smooth-size two-pass iteration (mixed_kernels.hpp) */
#define ADMM_TV_PATH_ODD 4      /* odd-length two-launch iteration (odd_kernels.hpp) */
int admm_tv_path(const admm_tv_desc* desc, int train);

/* 1 when an fp64 solve (ADMM_TV_FLAG_F64) of (H, W) is supported (up to 65,536 points per side;
 * lines beyond 5,120 points transform in global scratch), 0 otherwise. */
int admm_tv_supported_f64(int64_t H, int64_t W);

/* Workspace bytes needed by admm_tv_forward for `desc`. */
int admm_tv_workspace_size(const admm_tv_desc* desc, size_t* bytes);

/* The whole solver: replaces fft_admm_tv(xin, lmbd, rho, kern, iso, maxit)
 * (deconv.py:35-117).  Computes b = H_t(xin) once, freq_c from the PSF spectrum
 * and rho, then `maxit` ADMM iterations (two fused passes each, three for iso),
 * and writes the final x to `out` (B,C,H,W).  maxit == 0 writes zeros.
 * kern may be NULL iff kh == kw == 0 (pure TV denoising, sigma = 1).            */
int admm_tv_forward(const admm_tv_desc* desc, const float* xin, const float* kern,
                    const float* lambda_dev, const float* rho_dev, float* out,
                    void* workspace, size_t workspace_bytes, void* stream);

/* fp64 variants (desc->flags must hold ADMM_TV_FLAG_F64; the plain entry points refuse it): the
 * same contracts as admm_tv_forward / admm_tv_forward_train / admm_tv_backward with double arrays. */
int admm_tv_forward_f64(const admm_tv_desc* desc, const double* xin, const double* kern,
                        const double* lambda_dev, const double* rho_dev, double* out,
                        void* workspace, size_t workspace_bytes, void* stream);
int admm_tv_forward_train_f64(const admm_tv_desc* desc, const double* xin, const double* kern,
                              const double* lambda_dev, const double* rho_dev, double* out,
                              void* hist, size_t hist_bytes,
                              void* workspace, size_t workspace_bytes, void* stream);
int admm_tv_backward_f64(const admm_tv_desc* desc, const double* xin, const double* kern,
                         const double* lambda_dev, const double* rho_dev, const double* gout,
                         const void* hist, size_t hist_bytes,
                         double* gxin, double* glam, double* grho, double* gkern,
                         void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------- autograd
 * Replaces the reference's implicit autograd through the unrolled loop
 * (deconv.py:103-115 differentiated by PyTorch).
 *
 * Training forward: same result as admm_tv_forward, and additionally stores, for
 * every iteration k, a_k = D x_k + u_{k-1} (x and y images) and, for iso, the
 * per-pixel norms N_k in `hist` (admm_tv_history_size bytes; kept by the caller
 * until the backward).                                                          */
int admm_tv_history_size(const admm_tv_desc* desc, size_t* bytes);
int admm_tv_forward_train(const admm_tv_desc* desc, const float* xin, const float* kern,
                          const float* lambda_dev, const float* rho_dev, float* out,
                          void* hist, size_t hist_bytes,
                          void* workspace, size_t workspace_bytes, void* stream);

/* Backward: given gout = dL/dx_K and the training history, writes dL/dxin
 * (gxin, may be NULL), dL/dlambda and dL/drho (glam, grho: device scalars, both or
 * neither) and, when desc->flags has ADMM_TV_FLAG_PSF_GRAD (also at the forward),
 * dL/dkern (gkern, kh*kw floats; xin must then be given).                         */
int admm_tv_backward_workspace_size(const admm_tv_desc* desc, size_t* bytes);
int admm_tv_backward(const admm_tv_desc* desc, const float* xin, const float* kern,
                     const float* lambda_dev, const float* rho_dev, const float* gout,
                     const void* hist, size_t hist_bytes,
                     float* gxin, float* glam, float* grho, float* gkern,
                     void* workspace, size_t workspace_bytes, void* stream);

/* b = H_t(xin): the reference's circular PSF "adjoint" (a centred circular
 * CONVOLUTION, deconv.py:86-101), via the same FFT passes.  Exposed for tests. */
int admm_tv_psf_transpose(const admm_tv_desc* desc, const float* xin, const float* kern,
                          float* out, void* workspace, size_t workspace_bytes, void* stream);

/* Per-kernel timing of the iteration passes (HIP events on the launch stream),
 * used by bench.py for the roofline line (process-wide, behind a lock: calls from several
 * threads add to the same totals).  enable != 0 starts recording;
 * read() synchronises on the recorded events and returns totals since the last
 * reset: ms[k], count[k] for k = 0 pass A (row pass), 1 pass B (column pass),
 * 2 iso norm pass, 3 setup.                                                    */
int admm_tv_profile_enable(int enable);
int admm_tv_profile_reset(void);
int admm_tv_profile_read(double* ms4, int64_t* count4);

/* Human-readable text for the last error on this thread. */
const char* admm_tv_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* ADMM_TV_H */

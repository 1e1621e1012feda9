"""torch.library registration of the HIP solver: the dispatcher ops ``admm_hip::*``.

The reference's solver is ~30 plain ATen ops per iteration (``deconv.py:103-115``), so
``torch.compile`` / FX / ``torch.export`` see through it.  Here the solver is one native call, so
it is registered as custom operators with fake (meta) kernels: tracing keeps it as one node of the
graph, with no graph break, and the autograd formula is registered on the op itself.

  admm_hip::fft_admm_tv_fwd(x, lam, rho, kern, iso, maxit) -> out
      inference solve (admm_tv_forward); out has G*B planes for G = lam.numel() modules
  admm_hip::fft_admm_tv_fwd_train(x, lam, rho, kern, iso, maxit, psf_grad) -> (out, hist)
      the training forward (admm_tv_forward_train): hist is the uint8 history the backward reads
  admm_hip::fft_admm_tv_bwd(gout, x, lam, rho, kern, hist, iso, maxit, psf_grad,
                            need_x, need_s, need_k) -> (gx, glam, grho, gkern)
      admm_tv_backward; gradients that are not needed come back as empty tensors

All tensor arguments share one dtype -- fp32, or fp64 for an fp64 solve (ADMM_TV_FLAG_F64: the
reference computes in xin.dtype, so fp64 inputs get fp64 arithmetic) -- and are contiguous, on one
ROCm device (the public wrapper in ``admmtor.eops.deconv`` stages host / half inputs).  The backward op
has an autograd formula of its own (``admmtor._unrolled.double_backward``), so a gradient taken with
``create_graph=True`` can be differentiated again, as through the reference's unrolled ATen graph;
first-order values stay the native kernels'.  The cross-rank all-reduce hook of the
sharded iso solve (``admmtor.sharded``) is a Python callable and cannot be an op argument: that
path keeps the ``autograd.Function`` in ``admmtor._backward`` (first order only).
"""
from __future__ import annotations

from typing import Tuple

import torch
from torch import Tensor

from . import _native

__all__ = ["fft_admm_tv_fwd", "fft_admm_tv_fwd_train", "fft_admm_tv_bwd"]


def _k(kern: Tensor) -> int:
    return int(kern.shape[-1]) if kern.numel() > 0 else 0


def _f64(x: Tensor) -> bool:
    return x.dtype == torch.float64


def _desc(x: Tensor, lam: Tensor, kern: Tensor, iso: bool, maxit: int, flags: int = 0):
    B, C, H, W = x.shape
    return _native.desc(B, C, H, W, _k(kern), iso, maxit, flags, lam.numel(), f64=_f64(x))


def _check_supported(H: int, W: int, f64: bool) -> None:
    if not _native.supported(H, W, f64):
        raise NotImplementedError(f"admmtor (MI355X build): H={H}, W={W} unsupported (admm_tv_supported"
                                  f"{'_f64' if f64 else ''}: any size whose lines fit the generic kernels' LDS, "
                                  "up to 65,536)")


def _flags(kern: Tensor, psf_grad: bool) -> int:
    return _native.ADMM_TV_FLAG_PSF_GRAD if (psf_grad and kern.numel() > 0) else 0


def _stream(dev) -> int:
    return torch.cuda.current_stream(dev).cuda_stream


def _check_device(*ts: Tensor) -> None:
    for t in ts:
        if t.numel() > 0 and not t.is_cuda:
            raise RuntimeError("admm_hip ops take ROCm device tensors only (no CPU kernel)")


# ---------------------------------------------------------------- inference
@torch.library.custom_op("admm_hip::fft_admm_tv_fwd", mutates_args=())
def fft_admm_tv_fwd(x: Tensor, lam: Tensor, rho: Tensor, kern: Tensor, iso: bool, maxit: int) -> Tensor:
    """admm_tv_forward (include/admm_tv.h) -- replaces fft_admm_tv's loop (deconv.py:35-117)."""
    _check_device(x, lam, rho, kern)
    B, C, H, W = x.shape
    _check_supported(H, W, _f64(x))
    d = _desc(x, lam, kern, iso, maxit)
    x, lam, rho, kern = x.contiguous(), lam.contiguous(), rho.contiguous(), kern.contiguous()
    ws = torch.empty(_native.workspace_size(d), dtype=torch.uint8, device=x.device)
    out = torch.empty((lam.numel() * B, C, H, W), dtype=x.dtype, device=x.device)
    _native.check(_native.entry("admm_tv_forward", _f64(x))(
        d, x.data_ptr(), kern.data_ptr() if _k(kern) > 0 else None, lam.data_ptr(), rho.data_ptr(),
        out.data_ptr(), ws.data_ptr(), ws.numel(), _stream(x.device)))
    return out


@fft_admm_tv_fwd.register_fake
def _(x, lam, rho, kern, iso, maxit):
    B, C, H, W = x.shape
    return x.new_empty((lam.shape[0] * B, C, H, W), dtype=x.dtype)


# ---------------------------------------------------------------- training forward + backward
def _is_concrete(*vals) -> bool:
    return all(isinstance(v, int) for v in vals)


@torch.library.custom_op("admm_hip::fft_admm_tv_fwd_train", mutates_args=())
def fft_admm_tv_fwd_train(x: Tensor, lam: Tensor, rho: Tensor, kern: Tensor, iso: bool, maxit: int,
                          psf_grad: bool) -> Tuple[Tensor, Tensor]:
    """admm_tv_forward_train: the solve plus the history its backward reads (a_k per iteration,
    iso norms, and with psf_grad the r_k spectra)."""
    _check_device(x, lam, rho, kern)
    B, C, H, W = x.shape
    _check_supported(H, W, _f64(x))
    d = _desc(x, lam, kern, iso, maxit, _flags(kern, psf_grad))
    x, lam, rho, kern = x.contiguous(), lam.contiguous(), rho.contiguous(), kern.contiguous()
    ws = torch.empty(_native.workspace_size(d), dtype=torch.uint8, device=x.device)
    hist = torch.empty(max(_native.history_size(d), 1), dtype=torch.uint8, device=x.device)
    out = torch.empty((lam.numel() * B, C, H, W), dtype=x.dtype, device=x.device)
    _native.check(_native.entry("admm_tv_forward_train", _f64(x))(
        d, x.data_ptr(), kern.data_ptr() if _k(kern) > 0 else None, lam.data_ptr(), rho.data_ptr(),
        out.data_ptr(), hist.data_ptr(), hist.numel(), ws.data_ptr(), ws.numel(), _stream(x.device)))
    return out, hist


@fft_admm_tv_fwd_train.register_fake
def _(x, lam, rho, kern, iso, maxit, psf_grad):
    B, C, H, W = x.shape
    G = lam.shape[0]
    out = x.new_empty((G * B, C, H, W), dtype=x.dtype)
    k = kern.shape[-1] if kern.numel() > 0 else 0
    if _is_concrete(B, C, H, W, G, k):
        n = max(_native.history_size(_native.desc(B, C, H, W, k, iso, maxit, _flags(kern, psf_grad), G,
                                                  f64=_f64(x))), 1)
    else:  # symbolic shapes: the history size is a closed form of the native planner, opaque here
        n = torch.library.get_ctx().new_dynamic_size()
    return out, x.new_empty((n,), dtype=torch.uint8)


@torch.library.custom_op("admm_hip::fft_admm_tv_bwd", mutates_args=())
def fft_admm_tv_bwd(gout: Tensor, x: Tensor, lam: Tensor, rho: Tensor, kern: Tensor, hist: Tensor, iso: bool,
                    maxit: int, psf_grad: bool, need_x: bool, need_s: bool,
                    need_k: bool) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """admm_tv_backward: (dL/dx, dL/dlam, dL/drho, dL/dkern) from dL/dout and the history."""
    _check_device(gout, x, lam, rho, kern, hist)
    f64 = lam.dtype == torch.float64
    G = lam.numel()
    GB, C, H, W = gout.shape
    B = GB // G
    k = _k(kern)
    flags = _flags(kern, psf_grad)
    if need_k and not flags:
        raise RuntimeError("admmtor: PSF gradient requested but the forward did not keep the spectra")
    if flags and tuple(x.shape) != (B, C, H, W):
        raise RuntimeError("admm_hip::fft_admm_tv_bwd: the PSF gradient needs the forward's input x")
    d = _native.desc(B, C, H, W, k, iso, maxit, flags, G, f64=f64)
    dev = gout.device
    dt = lam.dtype
    g = gout.contiguous().to(dt)
    e = torch.empty(0, dtype=dt, device=dev)
    gx = torch.empty((B, C, H, W), dtype=dt, device=dev) if need_x else e
    gl = torch.empty(G, dtype=dt, device=dev) if need_s else e.clone()
    gr = torch.empty(G, dtype=dt, device=dev) if need_s else e.clone()
    gk = torch.empty((1, 1, k, k), dtype=dt, device=dev) if (need_k and k > 0) else e.clone()
    ws = torch.empty(_native.backward_workspace_size(d), dtype=torch.uint8, device=dev)
    xc = x.contiguous() if flags else None
    _native.check(_native.entry("admm_tv_backward", f64)(
        d, xc.data_ptr() if flags else None, kern.contiguous().data_ptr() if k > 0 else None,
        lam.contiguous().data_ptr(), rho.contiguous().data_ptr(), g.data_ptr(), hist.data_ptr(), hist.numel(),
        gx.data_ptr() if need_x else None, gl.data_ptr() if need_s else None,
        gr.data_ptr() if need_s else None, gk.data_ptr() if gk.numel() else None,
        ws.data_ptr(), ws.numel(), _stream(dev)))
    return gx, gl, gr, gk


@fft_admm_tv_bwd.register_fake
def _(gout, x, lam, rho, kern, hist, iso, maxit, psf_grad, need_x, need_s, need_k):
    G = lam.shape[0]
    GB, C, H, W = gout.shape
    B = GB // G
    k = kern.shape[-1] if kern.numel() > 0 else 0
    def mk(shape):
        return gout.new_empty(shape, dtype=lam.dtype)
    gx = mk((B, C, H, W)) if need_x else mk((0,))
    gl = mk((G,)) if need_s else mk((0,))
    gr = mk((G,)) if need_s else mk((0,))
    gk = mk((1, 1, k, k)) if (need_k and kern.numel() > 0) else mk((0,))
    return gx, gl, gr, gk


def _setup_context(ctx, inputs, output):
    x, lam, rho, kern, iso, maxit, psf_grad = inputs
    _, hist = output
    ctx.iso, ctx.maxit, ctx.psf_grad = iso, maxit, psf_grad
    # hist (uint8) never has a gradient: without this autograd would hand _backward a materialised
    # zero tensor of the whole history (10 GB at the C5 shape, 1.5 ms of fills per backward)
    ctx.set_materialize_grads(False)
    # x: read by the native backward only for the PSF gradient (b = H_t(x) path), and by a double
    # backward (admmtor._unrolled rebuilds the iteration from it).  An x that requires grad is saved
    # as itself (the double backward must reach it; autograd's usual version check applies, as for
    # any op that saves its input).  The reference's graph saves no reference to xin (its circular pad
    # copies), so a caller may modify xin in place after the forward and still call backward: with a
    # PSF gradient a private copy is kept (one image next to the 2 K images of history); otherwise x
    # is only referenced with its version, the first-order backward does not read it, and a double
    # backward after such a modification raises instead of differentiating the wrong input.
    # An inference tensor (made under torch.inference_mode) tracks no version counter, so it cannot be
    # referenced with one: it gets the private copy too.
    ctx.xref = None
    if x.requires_grad:
        xs = x
    elif psf_grad or x.is_inference():
        xs = x.detach().clone()
    else:
        xs = x.new_empty(0)
        ctx.xref = (x.detach(), x._version)
    ctx.save_for_backward(xs, lam, rho, kern, hist)


def _backward(ctx, gout, ghist):
    if gout is None:  # grads are not materialised (above): no gradient reached the solve's output
        return (None,) * 7
    x, lam, rho, kern, hist = ctx.saved_tensors
    if ctx.xref is not None and ctx.xref[0]._version == ctx.xref[1]:
        x = ctx.xref[0]  # unmodified since the forward (else x stays empty: no double backward)
    need_x = ctx.needs_input_grad[0]
    need_s = ctx.needs_input_grad[1] or ctx.needs_input_grad[2]
    need_k = ctx.needs_input_grad[3] and kern.numel() > 0
    gx, gl, gr, gk = torch.ops.admm_hip.fft_admm_tv_bwd(
        gout, x, lam, rho, kern, hist, ctx.iso, ctx.maxit, ctx.psf_grad, need_x, need_s, need_k)
    return (gx if need_x else None,
            gl if ctx.needs_input_grad[1] else None,
            gr if ctx.needs_input_grad[2] else None,
            gk if need_k else None, None, None, None)


torch.library.register_autograd("admm_hip::fft_admm_tv_fwd_train", _backward, setup_context=_setup_context)


# ---------------------------------------------------------------- double backward
def _bwd_setup_context(ctx, inputs, output):
    gout, x, lam, rho, kern, hist, iso, maxit, psf_grad, need_x, need_s, need_k = inputs
    ctx.iso, ctx.maxit = iso, maxit
    ctx.produced = (need_x, need_s, need_s, need_k)
    ctx.save_for_backward(gout, x, lam, rho, kern)


def _bwd_backward(ctx, ggx, ggl, ggr, ggk):
    """Derivative of admm_tv_backward's result (admmtor._unrolled: the first-order gradient rebuilt
    on a differentiable restatement of the same iteration, deconv.py:103-115)."""
    from ._unrolled import double_backward
    gout, x, lam, rho, kern = ctx.saved_tensors
    wanted = tuple(ctx.needs_input_grad[:5])
    grads = double_backward(gout, x, lam, rho, kern, ctx.iso, ctx.maxit, ctx.produced,
                            (ggx, ggl, ggr, ggk), wanted)
    return grads + (None,) * 7


torch.library.register_autograd("admm_hip::fft_admm_tv_bwd", _bwd_backward, setup_context=_bwd_setup_context)

"""Autograd of fft_admm_tv through the HIP solver (unrolled-iteration adjoint).

The reference gets its gradients from PyTorch autograd replaying ~30 ATen ops per
iteration (about 10-16 saved tensors of the image size per
iteration).  Here the forward runs the same fused HIP passes in "training mode",
keeping only a_k = D x_k + u_{k-1} (two images per iteration) plus, for iso, the
per-pixel norms; the backward (admm_tv_backward, csrc/admm_backward.hpp) replays
the iteration in reverse with the same two-pass structure: r^_k = M x^_k in the
column pass, then one fused row pass for the stencils and shrink Jacobians.

Gradients: xin (through H_t and every iteration), lambda and rho (scalars; rho also
through the Wiener factor, using dM/drho = -M D^T D M) and the PSF (through b = H_t(xin)
and through |sigma|^2 in the Wiener factor: a per-frequency cross-spectrum accumulated over
planes and iterations, csrc/admm_backward.hpp).  The PSF path keeps each iteration's r_k
spectrum (4 B/pixel/iteration more history) and is only enabled when the PSF requires grad.

The normal path goes through the dispatcher ops of ``admmtor._ops`` (autograd registered on
``admm_hip::fft_admm_tv_fwd_train``).  This ``autograd.Function`` carries only the sharded iso
solve, whose per-call all-reduce hook (a Python callable) cannot be an op argument.
"""
from __future__ import annotations

import torch
from torch.autograd.function import once_differentiable

from . import _native


def _scalar_input(v, device, dtype=torch.float32):
    """-> ((1,) device tensor of the solve's dtype, differentiable?)"""
    if isinstance(v, torch.Tensor):
        if v.numel() != 1:
            raise NotImplementedError("lmbd / rho must be scalars or 1-element tensors")
        return v.reshape(1).to(device=device, dtype=dtype), v.requires_grad
    return torch.full((1,), float(v), dtype=dtype, device=device), False


class AdmmTvFunction(torch.autograd.Function):
    """out = fft_admm_tv(xin, lam, rho, kern, iso, maxit) with a native backward."""

    @staticmethod
    def forward(ctx, x32, lam, rho, k32, iso: bool, maxit: int, hook=None, psf_grad: bool = False):
        f64 = x32.dtype == torch.float64  # an fp64 solve (ADMM_TV_FLAG_F64)
        B, C, H, W = x32.shape
        G = lam.numel()  # > 1: modules sharing x32 (fft_admm_tv_grouped); output (G B, C, H, W)
        k = int(k32.shape[-1]) if k32.numel() > 0 else 0
        flags = _native.ADMM_TV_FLAG_PSF_GRAD if (psf_grad and k > 0) else 0
        hook = hook if iso else None
        bound = hook.bind(f64=f64) if hook is not None else None
        d = _native.desc(B, C, H, W, k, iso, maxit, flags, G, bound, f64=f64)
        x32 = x32.contiguous()
        k32c = k32.contiguous()
        lam_c, rho_c = lam.contiguous(), rho.contiguous()
        ws = torch.empty(_native.workspace_size(d), dtype=torch.uint8, device=x32.device)
        hist = torch.empty(max(_native.history_size(d), 1), dtype=torch.uint8, device=x32.device)
        out = torch.empty((G * B, C, H, W), dtype=x32.dtype, device=x32.device)
        stream = torch.cuda.current_stream(x32.device).cuda_stream
        if bound is not None:
            bound.add(ws, hist)
        _native.check(_native.entry("admm_tv_forward_train", f64)(
            d, x32.data_ptr(), k32c.data_ptr() if k > 0 else None, lam_c.data_ptr(), rho_c.data_ptr(),
            out.data_ptr(), hist.data_ptr(), hist.numel(), ws.data_ptr(), ws.numel(), stream))
        if bound is not None:
            bound.check()
        del ws, bound
        ctx.hook = hook
        ctx.save_for_backward(k32c, lam_c, rho_c, x32 if flags else None)
        ctx.hist = hist
        ctx.desc = (B, C, H, W, k, iso, maxit, flags, G, f64)
        return out

    @staticmethod
    @once_differentiable
    def backward(ctx, gout):
        if ctx.hist is None:
            raise RuntimeError("admmtor: fft_admm_tv's native backward was already run for this graph and its "
                               "history released; backward through it twice (retain_graph=True) is not supported")
        k32, lam, rho, x32 = ctx.saved_tensors
        B, C, H, W, k, iso, maxit, flags, G, f64 = ctx.desc
        bound = ctx.hook.bind(f64=f64) if ctx.hook is not None else None
        d = _native.desc(B, C, H, W, k, iso, maxit, flags, G, bound, f64=f64)
        need_k = ctx.needs_input_grad[3] and k > 0
        if need_k and not flags:
            raise RuntimeError("admmtor: PSF gradient requested but the forward did not keep the spectra")
        dev = gout.device
        dt = torch.float64 if f64 else torch.float32
        g = gout.contiguous().to(dt)
        need_x = ctx.needs_input_grad[0]
        need_s = ctx.needs_input_grad[1] or ctx.needs_input_grad[2]
        gx = torch.empty((B, C, H, W), dtype=dt, device=dev) if need_x else None
        gl = torch.empty(G, dtype=dt, device=dev) if need_s else None
        gr = torch.empty(G, dtype=dt, device=dev) if need_s else None
        gk = torch.empty((1, 1, k, k), dtype=dt, device=dev) if need_k else None
        ws = torch.empty(_native.backward_workspace_size(d), dtype=torch.uint8, device=dev)
        stream = torch.cuda.current_stream(dev).cuda_stream
        if bound is not None:
            bound.add(ws, ctx.hist)
        _native.check(_native.entry("admm_tv_backward", f64)(
            d, x32.data_ptr() if x32 is not None else None, k32.data_ptr() if k > 0 else None,
            lam.data_ptr(), rho.data_ptr(), g.data_ptr(), ctx.hist.data_ptr(), ctx.hist.numel(),
            gx.data_ptr() if gx is not None else None,
            gl.data_ptr() if gl is not None else None,
            gr.data_ptr() if gr is not None else None,
            gk.data_ptr() if gk is not None else None,
            ws.data_ptr(), ws.numel(), stream))
        if bound is not None:
            bound.check()
        ctx.hist = None  # release the history as soon as the gradient is formed
        return (gx,
                gl if ctx.needs_input_grad[1] else None,
                gr if ctx.needs_input_grad[2] else None,
                gk, None, None, None, None)


def fft_admm_tv_autograd(xin, lmbd, rho, kern, iso, maxit, hook=None):
    dev = xin.device
    dt = torch.float64 if xin.dtype == torch.float64 else torch.float32  # fp64 inputs: an fp64 solve
    x32 = xin.to(dt)  # differentiable cast (autocast / half inputs)
    k32 = kern.to(device=dev, dtype=dt) if kern.numel() > 0 else torch.empty(0, dtype=dt, device=dev)
    lam_t, _ = _scalar_input(lmbd, dev, dt)
    rho_t, _ = _scalar_input(rho, dev, dt)
    psf_grad = isinstance(kern, torch.Tensor) and kern.requires_grad and kern.numel() > 0
    out = AdmmTvFunction.apply(x32, lam_t, rho_t, k32, bool(iso), int(maxit), hook, psf_grad)
    return out

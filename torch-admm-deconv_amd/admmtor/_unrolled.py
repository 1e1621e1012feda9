"""Higher-order autograd for the HIP solver: the autograd formula of ``admm_hip::fft_admm_tv_bwd``.

The reference's solver is ~30 ATen ops per iteration (``deconv.py:103-115``), so PyTorch can
differentiate its gradient again: ``torch.autograd.grad(..., create_graph=True)`` followed by a
second backward (gradient penalties, Hessian-vector products, meta-learning through the solver).
Here the first-order gradient is one native call (``admm_tv_backward``).  Its own derivative --
needed only when a caller actually differentiates a gradient -- comes from this module:

* the solve is re-expressed as a differentiable graph of device tensor ops in the solve's dtype on
  the solve's ROCm device (``unrolled_solve``: the Fourier form of ``deconv.py:35-117`` that the
  kernels implement, DESIGN §3: ``b = H_t(xin)`` once, ``r = b + rho D^T (z - u)``,
  ``x = F^-1 freq_c F r``, shrink, dual update);
* the first-order gradient is rebuilt on it with ``create_graph=True`` and differentiated against
  the incoming second-order seeds (``double_backward``).

So the values every first-order caller sees stay the native kernels' (``fft_admm_tv_bwd`` still
runs for them, with ``create_graph`` or not); the second-order terms -- which involve d/d rho of
the Wiener factor, d/d PSF of ``|sigma|^2`` and ``H_t``, and the forward-mode (tangent) solve that
d/d gout is -- are those of the reference's own autograd through the same iteration.  Any order
works: the result is built from ordinary differentiable ops when grad mode is on.  This is not a
fallback of the solver: it runs only inside the backward of a backward, never for a forward or a
first-order gradient, and it needs the same ROCm device tensors the native call had.
"""
from __future__ import annotations

import math
from typing import Optional, Sequence, Tuple

import torch
from torch import Tensor

__all__ = ["unrolled_solve", "double_backward"]


def _laplacian_symbol(H: int, W: int, dtype, device) -> Tensor:
    """|Dx^|^2 + |Dy^|^2 on the (H, W//2+1) half plane (deconv.py:51-57), built in fp64."""
    ky = torch.arange(H, dtype=torch.float64, device=device).reshape(H, 1)
    kx = torch.arange(W // 2 + 1, dtype=torch.float64, device=device).reshape(1, -1)
    lap = (2.0 - 2.0 * torch.cos((2.0 * math.pi / W) * kx)) + (2.0 - 2.0 * torch.cos((2.0 * math.pi / H) * ky))
    return lap.to(dtype)


def _psf_spectra(kern: Tensor, H: int, W: int, dtype) -> Tuple[Tensor, Tensor]:
    """(|sigma|^2, spectrum of H_t): sigma = rfft2(kern, s=(H, W)) (deconv.py:49); H_t is the
    circular convolution with the PSF anchored at ceil((k-1)/2) (deconv.py:89-101), i.e. sigma
    times the phase of that anchor.  Both differentiable in kern."""
    k = kern.shape[-1]
    sig = torch.fft.rfftn(kern.reshape(kern.shape[-2:]).to(dtype), s=(H, W))
    s2 = sig.real * sig.real + sig.imag * sig.imag
    a = k // 2
    ky = torch.arange(H, dtype=torch.float64, device=kern.device).reshape(H, 1)
    kx = torch.arange(W // 2 + 1, dtype=torch.float64, device=kern.device).reshape(1, -1)
    phase = torch.polar(torch.ones_like(ky * kx), (2.0 * math.pi * a) * (ky / H + kx / W)).to(sig.dtype)
    return s2, sig * phase


def _soft(a: Tensor, tau: Tensor) -> Tensor:
    return torch.sign(a) * torch.clamp_min(torch.abs(a) - tau, 0.0)


def _block_pair(ax: Tensor, ay: Tensor, tau: Tensor) -> Tuple[Tensor, Tensor]:
    """Block shrink with the per-pixel norm over (B, C) of each difference image (deconv.py:19-24)."""
    out = []
    for a in (ax, ay):
        nrm = torch.sqrt(torch.sum(a * a, dim=(0, 1)) + 1e-15)
        out.append(torch.clamp_min(1.0 - tau / (nrm + 1e-15), 0.0) * a)
    return out[0], out[1]


def _solve_module(xin: Tensor, lam: Tensor, rho: Tensor, s2: Optional[Tensor], bspec: Optional[Tensor],
                  lap: Tensor, iso: bool, maxit: int) -> Tensor:
    B, C, H, W = xin.shape
    tau = lam / rho
    if bspec is None:
        b = xin
    else:
        b = torch.fft.irfftn(torch.fft.rfftn(xin, dim=(2, 3)) * bspec, s=(H, W), dim=(2, 3))
    fc = 1.0 / ((s2 if s2 is not None else 1.0) + rho * lap)
    x = torch.zeros_like(xin)
    ux = torch.zeros_like(xin)
    uy = torch.zeros_like(xin)
    wx = torch.zeros_like(xin)  # z - u
    wy = torch.zeros_like(xin)
    for _ in range(maxit):
        # D^T w = w - shift(w, -1) along each axis; D x = x - shift(x, +1)
        v = (wx - torch.roll(wx, -1, dims=3)) + (wy - torch.roll(wy, -1, dims=2))
        r = b + rho * v
        x = torch.fft.irfftn(fc * torch.fft.rfftn(r, dim=(2, 3)), s=(H, W), dim=(2, 3))
        ax = (x - torch.roll(x, 1, dims=3)) + ux
        ay = (x - torch.roll(x, 1, dims=2)) + uy
        if iso:
            zx, zy = _block_pair(ax, ay, tau)
        else:
            zx, zy = _soft(ax, tau), _soft(ay, tau)
        ux = ax - zx
        uy = ay - zy
        wx = zx - ux
        wy = zy - uy
    return x


def unrolled_solve(xin: Tensor, lam: Tensor, rho: Tensor, kern: Tensor, iso: bool, maxit: int) -> Tensor:
    """The solve as differentiable device tensor ops: xin (B, C, H, W), lam / rho (G,) for G modules
    sharing xin (module-major output, as ``admm_hip::fft_admm_tv_fwd``), kern (1, 1, k, k) or empty."""
    B, C, H, W = xin.shape
    dt = xin.dtype
    lap = _laplacian_symbol(H, W, dt, xin.device)
    s2 = bspec = None
    if kern.numel() > 0:
        s2, bspec = _psf_spectra(kern, H, W, dt)
    lam = lam.reshape(-1).to(dt)
    rho = rho.reshape(-1).to(dt)
    outs = [_solve_module(xin, lam[g], rho[g], s2, bspec, lap, iso, int(maxit)) for g in range(lam.numel())]
    return outs[0] if len(outs) == 1 else torch.cat(outs, 0)


def double_backward(gout: Tensor, x: Tensor, lam: Tensor, rho: Tensor, kern: Tensor, iso: bool, maxit: int,
                    produced: Sequence[bool], seeds: Sequence[Optional[Tensor]],
                    wanted: Sequence[bool]) -> Tuple[Optional[Tensor], ...]:
    """Gradients of ``sum_i <seeds[i], g_i>`` with respect to (gout, x, lam, rho, kern), where
    ``g = (dL/dx, dL/dlam, dL/drho, dL/dkern)`` is what ``admm_hip::fft_admm_tv_bwd`` returned for
    ``gout``.  ``produced[i]``: the first-order op computed g_i; ``wanted``: which of the five
    inputs need a gradient.  Built with ``create_graph`` when grad mode is on (third order and up)."""
    outer = torch.is_grad_enabled()
    none = (None,) * 5
    if x.numel() == 0:
        raise RuntimeError("admmtor: double backward needs the forward's input x (not kept by this call)")
    with torch.enable_grad():
        def live(t: Tensor) -> Tensor:
            return t if t.requires_grad else t.detach().requires_grad_(True)
        has_k = kern.numel() > 0
        go, xi, li, ri = live(gout), live(x), live(lam), live(rho)
        ki = live(kern) if has_k else kern
        prims = (xi, li, ri, ki)
        pick = [i for i in range(4) if produced[i] and seeds[i] is not None and seeds[i].numel() > 0
                and (i < 3 or has_k)]
        if not pick:
            return none
        y = unrolled_solve(xi, li, ri, ki, iso, maxit)
        g1 = torch.autograd.grad(y, [prims[i] for i in pick], go.to(y.dtype), create_graph=True,
                                 allow_unused=True)
        outs, seeds_used = [], []
        for g, i in zip(g1, pick):
            if g is not None and g.requires_grad:
                outs.append(g)
                seeds_used.append(seeds[i].to(g.dtype))
        targets = [(j, t) for j, t in enumerate((go, xi, li, ri, ki)) if wanted[j] and (j != 4 or has_k)]
        if not outs or not targets:
            return none
        # retain_graph: the traversal reaches nodes of the caller's graph through gout (e.g. the
        # derivative of the loss that produced it), which its own backward still has to run
        res = torch.autograd.grad(outs, [t for _, t in targets], seeds_used, create_graph=outer, retain_graph=True,
                                  allow_unused=True)
    full = [None] * 5
    for (j, t), r in zip(targets, res):
        full[j] = r if r is not None else torch.zeros_like(t)
    return tuple(full)

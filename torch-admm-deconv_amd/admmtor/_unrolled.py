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

__all__ = ["unrolled_solve", "tangent_solve", "double_backward"]


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


# ---------------------------------------------------------------------------------------------
# Forward-mode (tangent) solve with checkpointed segments: the memory-bounded second order
# ---------------------------------------------------------------------------------------------
def _soft_dual(a: Tensor, da: Tensor, tau: Tensor, dtau: Tensor) -> Tuple[Tensor, Tensor]:
    """soft threshold and its tangent, with torch's derivative conventions for the same expression
    (clamp_min passes the gradient at equality, sign has none, abs has sign(a) -- so 0 at a = 0, where
    tau <= 0 still passes the clamp)."""
    sg = torch.sign(a)
    m = torch.abs(a) - tau
    z = sg * torch.clamp_min(m, 0.0)
    dz = torch.where(m >= 0, sg * sg * da - sg * dtau, torch.zeros_like(da))
    return z, dz


def _block_dual(a: Tensor, da: Tensor, tau: Tensor, dtau: Tensor) -> Tuple[Tensor, Tensor]:
    """block shrink over (B, C) (deconv.py:19-24) and its tangent."""
    n = torch.sqrt(torch.sum(a * a, dim=(0, 1)) + 1e-15)
    dn = torch.sum(a * da, dim=(0, 1)) / n
    ne = n + 1e-15
    q = 1.0 - tau / ne
    f = torch.clamp_min(q, 0.0)
    df = torch.where(q >= 0, -dtau / ne + tau * dn / (ne * ne), torch.zeros_like(dn))
    return f * a, f * da + df * a


def _dual_iterations(n: int, consts, iso: bool, state):
    """n iterations of the solve and of its tangent (the directional derivative of every operation,
    written out: D and D^T, the Wiener solve with d fc, the shrink Jacobians).  state = (u_x, u_y, w_x,
    w_y) and their tangents; returns (x, x_dot, new state)."""
    b, db, fc, dfc, rho, drho, tau, dtau = consts
    ux, uy, wx, wy, dux, duy, dwx, dwy = state
    H, W = b.shape[-2:]
    x = dx = None
    for _ in range(n):
        v = (wx - torch.roll(wx, -1, dims=3)) + (wy - torch.roll(wy, -1, dims=2))
        dv = (dwx - torch.roll(dwx, -1, dims=3)) + (dwy - torch.roll(dwy, -1, dims=2))
        r = b + rho * v
        dr = db + drho * v + rho * dv
        R = torch.fft.rfftn(r, dim=(2, 3))
        dR = torch.fft.rfftn(dr, dim=(2, 3))
        x = torch.fft.irfftn(fc * R, s=(H, W), dim=(2, 3))
        dx = torch.fft.irfftn(dfc * R + fc * dR, s=(H, W), dim=(2, 3))
        ax = (x - torch.roll(x, 1, dims=3)) + ux
        ay = (x - torch.roll(x, 1, dims=2)) + uy
        dax = (dx - torch.roll(dx, 1, dims=3)) + dux
        day = (dx - torch.roll(dx, 1, dims=2)) + duy
        shrink = _block_dual if iso else _soft_dual
        zx, dzx = shrink(ax, dax, tau, dtau)
        zy, dzy = shrink(ay, day, tau, dtau)
        ux, uy, dux, duy = ax - zx, ay - zy, dax - dzx, day - dzy
        wx, wy, dwx, dwy = zx - ux, zy - uy, dzx - dux, dzy - duy
    return x, dx, (ux, uy, wx, wy, dux, duy, dwx, dwy)


def tangent_solve(xin: Tensor, lam: Tensor, rho: Tensor, kern: Tensor, iso: bool, maxit: int,
                  tangents: Sequence[Optional[Tensor]], segment: int = 0) -> Tuple[Tensor, Tensor]:
    """(y, y_dot): the solve (as unrolled_solve) and its directional derivative along
    tangents = (x_dot, lam_dot, rho_dot, kern_dot) (None: zero).  segment > 0 runs the iterations in
    checkpointed segments of that many iterations (torch.utils.checkpoint, non-reentrant): a reverse pass
    through y_dot then keeps only the segment-boundary states plus one segment's activations, instead
    of the whole unrolled graph."""
    from torch.utils.checkpoint import checkpoint
    B, C, H, W = xin.shape
    dt = xin.dtype
    tx, tl, tr, tk = tangents
    lap = _laplacian_symbol(H, W, dt, xin.device)
    lam = lam.reshape(-1).to(dt)
    rho = rho.reshape(-1).to(dt)
    G = lam.numel()
    zl = torch.zeros(G, dtype=dt, device=xin.device)
    tl = zl if tl is None else tl.reshape(-1).to(dt)
    tr = zl if tr is None else tr.reshape(-1).to(dt)
    s2 = ds2 = None
    b, db = xin, (tx.to(dt) if tx is not None else torch.zeros_like(xin))
    if kern.numel() > 0:
        k = kern.shape[-1]
        sig = torch.fft.rfftn(kern.reshape(k, k).to(dt), s=(H, W))
        s2 = sig.real * sig.real + sig.imag * sig.imag
        a = k // 2
        ky = torch.arange(H, dtype=torch.float64, device=xin.device).reshape(H, 1)
        kx = torch.arange(W // 2 + 1, dtype=torch.float64, device=xin.device).reshape(1, -1)
        phase = torch.polar(torch.ones_like(ky * kx), (2.0 * math.pi * a) * (ky / H + kx / W)).to(sig.dtype)
        X = torch.fft.rfftn(xin, dim=(2, 3))
        dX = torch.fft.rfftn(db, dim=(2, 3))
        b = torch.fft.irfftn(X * (sig * phase), s=(H, W), dim=(2, 3))
        dB = dX * (sig * phase)
        if tk is not None:
            dsig = torch.fft.rfftn(tk.reshape(k, k).to(dt), s=(H, W))
            ds2 = 2.0 * (sig.real * dsig.real + sig.imag * dsig.imag)
            dB = dB + X * (dsig * phase)
        db = torch.fft.irfftn(dB, s=(H, W), dim=(2, 3))
    ys, dys = [], []
    for g in range(G):
        r, dr = rho[g], tr[g]
        tau = lam[g] / r
        dtau = tl[g] / r - lam[g] * dr / (r * r)
        den = (s2 if s2 is not None else 1.0) + r * lap
        fc = 1.0 / den
        dfc = -(fc * fc) * ((ds2 if ds2 is not None else 0.0) + dr * lap)
        consts = (b, db, fc, dfc, r, dr, tau, dtau)
        z = torch.zeros_like(xin)
        state = (z,) * 8
        x = dx = z
        left = int(maxit)
        while left > 0:
            n = min(segment, left) if segment > 0 else left
            if segment > 0:
                out = checkpoint(lambda c, *st, n=n: (lambda x_, dx_, st_: (x_, dx_) + tuple(st_))(
                                     *_dual_iterations(n, c, iso, st)), consts, *state, use_reentrant=False)
                x, dx, state = out[0], out[1], tuple(out[2:])
            else:
                x, dx, state = _dual_iterations(n, consts, iso, state)
            left -= n
        ys.append(x)
        dys.append(dx)
    if G == 1:
        return ys[0], dys[0]
    return torch.cat(ys, 0), torch.cat(dys, 0)


def _double_backward_tangent(gout, x, lam, rho, kern, iso, maxit, pick, seeds, wanted, segment):
    """Second order without the unrolled graph of the first-order gradient: with g = J^T gout
    (J = dy/d theta), sum_i <s_i, g_i> = <gout, J s> = <gout, y_dot>, y_dot the tangent solve along the
    seeds s.  So the gradient for gout is y_dot itself, and the gradient for theta = (x, lam, rho, kern)
    is the reverse pass through <gout, y_dot(theta)> -- a first-order gradient of a checkpointed
    function: memory bounded by the segment states plus one segment's activations."""
    has_k = kern.numel() > 0
    leaf = [t.detach().requires_grad_(True) for t in (x, lam, rho)]
    kl = kern.detach().requires_grad_(True) if has_k else kern
    tangents = [None, None, None, None]
    for i in pick:
        tangents[i] = seeds[i].detach()
    with torch.enable_grad():
        _, ydot = tangent_solve(leaf[0], leaf[1], leaf[2], kl, iso, maxit, tangents, segment)
        prims = (leaf[0], leaf[1], leaf[2], kl)
        targets = [(j, prims[j - 1]) for j in range(1, 5) if wanted[j] and (j != 4 or has_k)]
        res = []
        if targets:
            obj = torch.sum(gout.detach().to(ydot.dtype) * ydot)
            res = torch.autograd.grad(obj, [t for _, t in targets], allow_unused=True)
    full = [None] * 5
    if wanted[0]:
        full[0] = ydot.detach().to(gout.dtype)
    for (j, t), r in zip(targets, res):
        full[j] = r if r is not None else torch.zeros_like(t)
    return tuple(full)


# iterations per checkpointed segment of the tangent solve (second order without create_graph): about
# sqrt(maxit); ADMM_SO_SEGMENT overrides (0: no checkpointing), ADMM_SO_UNROLLED=1 selects the unrolled
# create_graph formulation below (A/B)
def _segment(maxit: int) -> int:
    import os
    v = os.environ.get("ADMM_SO_SEGMENT")
    if v is not None:
        return max(0, int(v))
    return max(1, int(round(math.sqrt(max(int(maxit), 1)))))


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
        raise RuntimeError("admmtor: double backward needs the forward's input x, which was modified in place "
                           "after the forward (or not kept by this call)")
    import os
    if not outer and os.environ.get("ADMM_SO_UNROLLED", "0") == "0":
        # the usual second order (no graph of the result needed): the tangent formulation, checkpointed
        has_k = kern.numel() > 0
        pick = [i for i in range(4) if produced[i] and seeds[i] is not None and seeds[i].numel() > 0
                and (i < 3 or has_k)]
        if not pick:
            return none
        return _double_backward_tangent(gout, x, lam, rho, kern, iso, maxit, pick, seeds, wanted, _segment(maxit))
    # third order and up (grad mode on): the first-order gradient rebuilt with create_graph on the
    # unrolled graph, so the result is itself differentiable
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

"""CPU oracle for the ADMM-TV deconvolution hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product package (``admmtor``) may
import, call or execute this file.  Only ``tests/``, ``__graft_entry__.smoke()``
and the ``cpu_baseline`` leg of ``bench.py`` use it, and only as the checker /
the timed CPU baseline, never as the thing measured or shipped.

It restates, in two independent ways, the algorithm of the reference solver
``fft_admm_tv`` (``/root/reference/src/admmtor/eops/deconv.py:35-117``):

* :func:`solve_spatial` follows the reference's operator sequence: every linear
  operator is a circular pad followed by a depthwise ``conv2d`` and the PSF
  adjoint ``H_t(xin)`` is re-evaluated inside the loop, exactly as the reference
  does (deconv.py:98-104).  It is the ``cpu_baseline`` ("port") timed by
  ``bench.py``: same op mix, same cost profile as the reference on the same cores.
* :func:`solve_fourier` is the Fourier-domain restatement the HIP path
  implements (``b = H_t(xin)`` once, differences by ``roll``, the Wiener factor
  applied to the 2-D real spectrum).  It runs in any float dtype; in fp64 it
  agrees with the reference's fp64 output to ~1e-14.

Parity pinning: both restatements are checked against golden vectors produced
by importing the reference itself in the build container
(``tests/golden/make_golden.py`` -> ``tests/golden/*.npz``; test
``tests/test_oracle_golden.py``).

Semantics restated (all circular, per (b,c) plane; line numbers in deconv.py):

* ``Dx a = a[i,j] - a[i,j-1]``, ``Dy a = a[i,j] - a[i-1,j]``          (:51-52, 74-78)
* ``Dx_t a = a[i,j] - a[i,j+1]``, ``Dy_t a = a[i,j] - a[i+1,j]``      (:80-84)
* ``H_t`` = circular *convolution* with the PSF anchored at
  ``c = ceil((k-1)/2)`` (pads ``(floor, ceil)`` on each side, flipped kernel,
  cross-correlation) -- not the adjoint for non-centrosymmetric PSFs  (:86-101)
* ``freq_c = 1 / (|sigma|^2 + rho (|Dx^|^2 + |Dy^|^2))``, ``sigma = rfft2(kern, s=(H,W))`` (:46-57)
* soft shrink ``sign(a) max(|a|-tau, 0)``; block shrink
  ``max(1 - tau/(sqrt(sum_{b,c} a^2 + 1e-15) + 1e-15), 0) a`` (norm over dims 0,1)  (:15-24)
* ``tau = lmbd / rho``; ``x = z = u = 0`` initially; returns the last ``x``  (:44, 61-67, 103-117)
"""
from __future__ import annotations

import math
from typing import Callable

import torch
import torch.nn.functional as F

__all__ = [
    "kink_margins",
    "psf_conv_pads",
    "apply_psf_transpose",
    "shrink_soft",
    "shrink_block",
    "wiener_factor",
    "solve_spatial",
    "solve_fourier",
    "solve_fourier_jvp",
    "rel_l2",
]


# --------------------------------------------------------------------------
# small helpers
# --------------------------------------------------------------------------
def rel_l2(a: torch.Tensor, b: torch.Tensor) -> float:
    """||a-b|| / ||b|| in fp64."""
    a = torch.as_tensor(a).double()
    b = torch.as_tensor(b).double()
    den = torch.linalg.vector_norm(b).item()
    num = torch.linalg.vector_norm(a - b).item()
    return num / den if den > 0 else num


def psf_conv_pads(k: int) -> tuple[int, int]:
    """(before, after) circular padding of H_t for a k-tap axis (deconv.py:90-96).

    The reference pads ``floor((k-1)/2)`` before and ``ceil((k-1)/2)`` after and
    cross-correlates with the flipped PSF, i.e. convolves with the PSF anchored
    at ``ceil((k-1)/2)``.
    """
    return (k - 1) // 2, k // 2  # floor((k-1)/2), ceil((k-1)/2)


def _dw(stencil, C: int, like: torch.Tensor) -> torch.Tensor:
    w = torch.tensor(stencil, dtype=like.dtype, device=like.device).reshape(1, 1, 2, 2)
    return w.expand(C, 1, 2, 2).contiguous()


def _circ_dwconv(a: torch.Tensor, w: torch.Tensor, pad: tuple[int, int, int, int]) -> torch.Tensor:
    return F.conv2d(F.pad(a, pad, mode="circular"), w, groups=a.shape[1])


def apply_psf_transpose(x: torch.Tensor, kern: torch.Tensor) -> torch.Tensor:
    """H_t(x) as the reference evaluates it: circular pad + depthwise conv with the flipped PSF."""
    if kern.numel() == 0:
        return x
    kh, kw = kern.shape[-2:]
    if kh != kw:
        raise RuntimeError("non-square PSF: the reference's H_t pads are swapped and fail (deconv.py:90-96)")
    C = x.shape[1]
    lo, hi = psf_conv_pads(kh)
    w = kern.flip((2, 3)).expand(C, 1, kh, kw).contiguous()
    return F.conv2d(F.pad(x, (lo, hi, lo, hi), mode="circular"), w, groups=C)


def shrink_soft(a: torch.Tensor, tau) -> torch.Tensor:
    """sign(a) * max(|a| - tau, 0)  (deconv.py:15-16)."""
    return torch.sign(a) * torch.clamp_min(torch.abs(a) - tau, 0.0)


def shrink_block(a: torch.Tensor, tau) -> torch.Tensor:
    """max(1 - tau / (||a||_(B,C) + 1e-15), 0) * a with the norm over dims (0,1) (deconv.py:19-24)."""
    nrm = torch.sqrt(torch.sum(a * a, dim=(0, 1)) + 1e-15)
    return torch.clamp_min(1.0 - tau / (nrm + 1e-15), 0.0) * a


def wiener_factor(H: int, W: int, kern: torch.Tensor, rho, dtype=torch.float64) -> torch.Tensor:
    """freq_c on the (H, W//2+1) half-plane (deconv.py:46-57), computed in ``dtype``."""
    ky = torch.arange(H, dtype=torch.float64).reshape(H, 1)
    kx = torch.arange(W // 2 + 1, dtype=torch.float64).reshape(1, -1)
    lap = (2.0 - 2.0 * torch.cos(2 * math.pi * kx / W)) + (2.0 - 2.0 * torch.cos(2 * math.pi * ky / H))
    if kern.numel() == 0:
        s2 = torch.ones((H, W // 2 + 1), dtype=torch.float64)
    else:
        sig = torch.fft.rfftn(kern.detach().double().reshape(kern.shape[-2:]), s=(H, W))
        s2 = sig.real ** 2 + sig.imag ** 2
    rho_d = torch.as_tensor(rho, dtype=torch.float64).reshape(())
    return (1.0 / (s2 + rho_d * lap)).to(dtype)


# --------------------------------------------------------------------------
# restatement 1: the reference's operator sequence (timed CPU baseline)
# --------------------------------------------------------------------------
def solve_spatial(xin: torch.Tensor, lmbd, rho, kern: torch.Tensor, iso: bool = False,
                  maxit: int = 100, iters_cb: Callable[[int, torch.Tensor], None] | None = None) -> torch.Tensor:
    """ADMM-TV with the reference's op mix: pad+depthwise-conv operators, FFT x-update.

    Differentiable w.r.t. xin, lmbd, rho and kern through ordinary autograd.
    """
    if xin.dim() != 4:
        raise ValueError("expected a 4-D (B,C,H,W) input")
    B, C, H, W = xin.shape
    dt = xin.dtype
    lmbd = torch.as_tensor(lmbd, dtype=dt)
    rho = torch.as_tensor(rho, dtype=dt)
    tau = lmbd / rho

    # Wiener factor in the working dtype, built like deconv.py:46-57
    if kern.numel() == 0:
        s2 = torch.ones((), dtype=dt)
    else:
        sig = torch.fft.rfftn(kern, s=(H, W), dim=(2, 3))
        s2 = sig.real ** 2 + sig.imag ** 2
    kx = torch.arange(W // 2 + 1, dtype=dt)
    ky = torch.arange(H, dtype=dt).reshape(H, 1)
    lap = (2 - 2 * torch.cos(2 * math.pi * kx / W)) + (2 - 2 * torch.cos(2 * math.pi * ky / H))
    fc = 1.0 / (s2 + rho * lap)

    wdx = _dw([[0, 0], [-1, 1]], C, xin)
    wdy = _dw([[0, -1], [0, 1]], C, xin)
    wdxt = _dw([[1, -1], [0, 0]], C, xin)
    wdyt = _dw([[1, 0], [-1, 0]], C, xin)
    back = (1, 0, 1, 0)
    fwd = (0, 1, 0, 1)
    shrink = shrink_block if iso else shrink_soft

    x = torch.zeros_like(xin)
    zx = torch.zeros_like(xin)
    zy = torch.zeros_like(xin)
    ux = torch.zeros_like(xin)
    uy = torch.zeros_like(xin)
    for it in range(int(maxit)):
        rhs = apply_psf_transpose(xin, kern) + rho * (
            _circ_dwconv(zx - ux, wdxt, fwd) + _circ_dwconv(zy - uy, wdyt, fwd))
        x = torch.fft.irfftn(fc * torch.fft.rfftn(rhs, dim=(2, 3)), s=(H, W), dim=(2, 3))
        gx = _circ_dwconv(x, wdx, back)
        gy = _circ_dwconv(x, wdy, back)
        zx = shrink(gx + ux, tau)
        zy = shrink(gy + uy, tau)
        ux = ux + gx - zx
        uy = uy + gy - zy
        if iters_cb is not None:
            iters_cb(it, x)
    return x


# --------------------------------------------------------------------------
# restatement 2: Fourier-domain form (what the HIP path computes)
# --------------------------------------------------------------------------
def _psf_centered_spectrum(kern: torch.Tensor, H: int, W: int) -> torch.Tensor:
    """Spectrum of the circular convolution that H_t applies (PSF anchored at ceil((k-1)/2))."""
    k = kern.shape[-1]
    c = k // 2
    sig = torch.fft.rfftn(kern.reshape(kern.shape[-2:]), s=(H, W))
    ky = torch.arange(H, dtype=torch.float64).reshape(H, 1)
    kx = torch.arange(W // 2 + 1, dtype=torch.float64).reshape(1, -1)
    ph = torch.exp(2j * math.pi * c * (ky / H + kx / W)).to(sig.dtype)
    return sig * ph


def solve_fourier(xin: torch.Tensor, lmbd, rho, kern: torch.Tensor, iso: bool = False,
                  maxit: int = 100, return_state: bool = False, norm_allreduce=None):
    """Fourier-domain restatement (b once, roll differences) in xin's dtype.

    norm_allreduce (iso only; test hook for a batch sharded over ranks): called every iteration
    with the local per-pixel sums over (B, C) of a_x^2 and a_y^2 as one (2, H, W) tensor, which it
    must replace in place by the sums over all ranks -- the contract of admm_tv_desc.allreduce."""
    B, C, H, W = xin.shape
    dt = xin.dtype
    lmbd = torch.as_tensor(lmbd, dtype=dt)
    rho = torch.as_tensor(rho, dtype=dt)
    tau = lmbd / rho
    if kern.numel() == 0:
        b = xin
    else:
        if kern.shape[-1] != kern.shape[-2]:
            raise RuntimeError("non-square PSF")
        b = torch.fft.irfftn(torch.fft.rfftn(xin, dim=(2, 3)) * _psf_centered_spectrum(kern.to(dt), H, W),
                             s=(H, W), dim=(2, 3))
    fc = wiener_factor(H, W, kern, rho, dtype=torch.float64).to(dt)

    def Dx(a):
        return a - torch.roll(a, 1, dims=3)

    def Dy(a):
        return a - torch.roll(a, 1, dims=2)

    def DxT(a):
        return a - torch.roll(a, -1, dims=3)

    def DyT(a):
        return a - torch.roll(a, -1, dims=2)

    shrink = shrink_block if iso else shrink_soft
    if iso and norm_allreduce is not None:
        def shrink_pair(ax, ay, tau):
            sums = torch.stack([torch.sum(ax * ax, dim=(0, 1)), torch.sum(ay * ay, dim=(0, 1))])
            norm_allreduce(sums)
            fx = torch.clamp_min(1.0 - tau / (torch.sqrt(sums[0] + 1e-15) + 1e-15), 0.0)
            fy = torch.clamp_min(1.0 - tau / (torch.sqrt(sums[1] + 1e-15) + 1e-15), 0.0)
            return fx * ax, fy * ay
    else:
        def shrink_pair(ax, ay, tau):
            return shrink(ax, tau), shrink(ay, tau)
    x = torch.zeros_like(xin)
    ux = torch.zeros_like(xin)
    uy = torch.zeros_like(xin)
    wx = torch.zeros_like(xin)  # z - u
    wy = torch.zeros_like(xin)
    for _ in range(int(maxit)):
        r = b + rho * (DxT(wx) + DyT(wy))
        x = torch.fft.irfftn(fc * torch.fft.rfftn(r, dim=(2, 3)), s=(H, W), dim=(2, 3))
        ax = Dx(x) + ux
        ay = Dy(x) + uy
        zx, zy = shrink_pair(ax, ay, tau)
        ux = ax - zx
        uy = ay - zy
        wx = zx - ux
        wy = zy - uy
    if return_state:
        return x, dict(b=b, fc=fc, ux=ux, uy=uy)
    return x


def solve_fourier_jvp(xin: torch.Tensor, lmbd, rho, kern: torch.Tensor, iso: bool, maxit: int,
                      tx: torch.Tensor, tl: torch.Tensor, tr: torch.Tensor, progress: Callable | None = None):
    """(y, y_dot): solve_fourier and its directional derivatives along K tangents at once, written out
    (forward mode, O(state) memory: no graph is kept, so the full config-5 shape fits where the fp64
    unrolled graph would need ~100 GB).  tx (K, B, C, H, W) are tangents of xin, tl / tr (K,) of lmbd /
    rho; y_dot is (K, B, C, H, W).  The PSF is held constant.  Torch's derivative conventions for the
    same expressions (clamp_min passes the derivative at equality, sign and abs have none at 0), so it
    equals torch.func.jvp of solve_fourier (tests/test_oracle_golden.py checks that at small size).

    Per iteration (deconv.py:103-115, Fourier form):
      r = b + rho v,  v = Dx^T w_x + Dy^T w_y       r' = b' + rho' v + rho v'
      x = F^-1 fc F r,  fc = 1/(s2 + rho lap)        x' = F^-1 (fc F r' + fc' F r),  fc' = -fc^2 rho' lap
      a = D x + u,  z = S(a; tau),  tau = lmbd/rho   a' = D x' + u',  z' = S'(a; tau) (a', tau')
      u = a - z,  w = z - u

    progress(it) is called after every iteration (long CPU runs report that they are alive)."""
    B, C, H, W = xin.shape
    dt = xin.dtype
    K = tx.shape[0]
    lm = float(lmbd)
    rh = float(rho)
    tau = lm / rh
    tl = tl.to(dt).reshape(K, 1, 1, 1, 1)
    tr = tr.to(dt).reshape(K, 1, 1, 1, 1)
    dtau = tl / rh - lm * tr / (rh * rh)
    if kern.numel() == 0:
        b, db = xin, tx.to(dt)
    else:
        spec = _psf_centered_spectrum(kern.to(dt), H, W)
        b = torch.fft.irfftn(torch.fft.rfftn(xin, dim=(2, 3)) * spec, s=(H, W), dim=(2, 3))
        db = torch.fft.irfftn(torch.fft.rfftn(tx.to(dt), dim=(-2, -1)) * spec, s=(H, W), dim=(-2, -1))
    fc = wiener_factor(H, W, kern, rh, dtype=torch.float64).to(dt)
    ky = torch.arange(H, dtype=torch.float64).reshape(H, 1)
    kx = torch.arange(W // 2 + 1, dtype=torch.float64).reshape(1, -1)
    lap = ((2.0 - 2.0 * torch.cos(2 * math.pi * kx / W)) + (2.0 - 2.0 * torch.cos(2 * math.pi * ky / H))).to(dt)
    dfc = -(fc * fc * lap) * tr  # (K, 1, 1, H, W/2+1)

    def dxt(a):
        return a - torch.roll(a, -1, dims=-1)

    def dyt(a):
        return a - torch.roll(a, -1, dims=-2)

    def dx_(a):
        return a - torch.roll(a, 1, dims=-1)

    def dy_(a):
        return a - torch.roll(a, 1, dims=-2)

    def shrink(a, da):
        if iso:
            n = torch.sqrt(torch.sum(a * a, dim=(0, 1)) + 1e-15)
            dn = torch.sum(a * da, dim=(1, 2)) / n           # (K, H, W)
            ne = n + 1e-15
            q = 1.0 - tau / ne
            f = torch.clamp_min(q, 0.0)
            df = torch.where(q >= 0, -dtau.reshape(K, 1, 1) / ne + tau * dn / (ne * ne), torch.zeros_like(dn))
            return f * a, f * da + df.unsqueeze(1).unsqueeze(1) * a
        sg = torch.sign(a)
        m = torch.abs(a) - tau
        z = sg * torch.clamp_min(m, 0.0)
        dz = torch.where(m >= 0, sg * sg * da - sg * dtau, torch.zeros_like(da))
        return z, dz

    # primal and tangents stacked along a leading axis (index 0 = primal): one FFT call per direction
    bs = torch.cat([b.unsqueeze(0), db])
    ux = uy = wx = wy = torch.zeros((K + 1,) + tuple(xin.shape), dtype=dt)
    xs = ux
    for step in range(int(maxit)):
        v = dxt(wx) + dyt(wy)                            # v_0 and its tangents
        r = bs + rh * v
        r[1:] += tr * v[0]
        Rs = torch.fft.rfftn(r, dim=(-2, -1))
        Xs = fc * Rs
        Xs[1:] += dfc * Rs[0]
        xs = torch.fft.irfftn(Xs, s=(H, W), dim=(-2, -1))
        ax, ay = dx_(xs) + ux, dy_(xs) + uy
        zx0, dzx = shrink(ax[0], ax[1:])
        zy0, dzy = shrink(ay[0], ay[1:])
        zx = torch.cat([zx0.unsqueeze(0), dzx])
        zy = torch.cat([zy0.unsqueeze(0), dzy])
        ux, uy = ax - zx, ay - zy
        wx, wy = zx - ux, zy - uy
        if progress is not None:
            progress(step + 1)
    return xs[0], xs[1:]


def kink_margins(xin: torch.Tensor, lmbd, rho, kern: torch.Tensor, maxit: int) -> torch.Tensor:
    """Per-plane min over iterations 1..maxit-1 and pixels of ||a| - tau| / tau (soft shrink).

    The soft threshold is not differentiable at |a| = tau: where the fp64 trajectory passes closer
    to the kink than fp32 can resolve (~1e-6 relative), an fp32 solver may take the other branch
    and its gradient legitimately differs.  Tests use this to scope their strict gates.
    """
    x = xin.double()
    B, C, H, W = x.shape
    tau = float(lmbd) / float(rho)
    _, st = solve_fourier(x, lmbd, rho, kern.double() if kern.numel() else kern.double(), False, 0, return_state=True)
    b, fc = st["b"], st["fc"]
    ux = torch.zeros_like(x)
    uy = torch.zeros_like(x)
    wx = torch.zeros_like(x)
    wy = torch.zeros_like(x)
    out = torch.full((B, C), float("inf"), dtype=torch.float64)
    for it in range(int(maxit) - 1):
        r = b + float(rho) * ((wx - torch.roll(wx, -1, 3)) + (wy - torch.roll(wy, -1, 2)))
        xx = torch.fft.irfftn(fc * torch.fft.rfftn(r, dim=(2, 3)), s=(H, W), dim=(2, 3))
        ax = xx - torch.roll(xx, 1, 3) + ux
        ay = xx - torch.roll(xx, 1, 2) + uy
        d = torch.minimum((ax.abs() - tau).abs().amin(dim=(2, 3)), (ay.abs() - tau).abs().amin(dim=(2, 3))) / tau
        out = torch.minimum(out, d)
        zx = shrink_soft(ax, tau)
        zy = shrink_soft(ay, tau)
        ux, uy = ax - zx, ay - zy
        wx, wy = zx - ux, zy - uy
    return out

"""Synthetic inputs for the ADMM-TV benchmarks and parity fixtures.

There is no dataset in this environment, so every benchmark image is generated:
piecewise-constant random rectangles and disks in [0, 1], blurred by circular
convolution with a centred PSF, plus AWGN (sigma = 0.01).  PSFs follow the
BASELINE.json configs: Gaussians (C1 9x9 sigma 1.5, C3/C4 21x21 sigma 3) and a
one-sided 30-degree linear motion blur (C2 15x15, non-centrosymmetric, so the
reference's ``H_t`` convolution-vs-correlation quirk is exercised).

Everything here is plain torch and runs on CPU or on the GPU (the bench
generates its batch directly in HBM).
"""
from __future__ import annotations

import math

import torch

__all__ = ["gaussian_psf", "motion_psf", "make_psf", "clean_images", "blurred_batch", "CONFIG_SEED"]

CONFIG_SEED = 20251205  # seed base; config i uses CONFIG_SEED + i


def gaussian_psf(k: int, sigma: float, dtype=torch.float32) -> torch.Tensor:
    r = torch.arange(k, dtype=torch.float64) - (k - 1) / 2.0
    g = torch.exp(-(r[:, None] ** 2 + r[None, :] ** 2) / (2.0 * sigma * sigma))
    g = g / g.sum()
    return g.to(dtype).reshape(1, 1, k, k)


def motion_psf(k: int, angle_deg: float = 30.0, dtype=torch.float32) -> torch.Tensor:
    """One-sided linear motion blur starting at the centre tap (non-centrosymmetric)."""
    c = (k - 1) / 2.0
    img = torch.zeros((k, k), dtype=torch.float64)
    th = math.radians(angle_deg)
    n = 8 * k
    for s in range(n):  # supersampled line from the centre outwards
        t = (k / 2.0) * s / (n - 1)
        yy = c - t * math.sin(th)
        xx = c + t * math.cos(th)
        iy, ix = int(round(yy)), int(round(xx))
        if 0 <= iy < k and 0 <= ix < k:
            img[iy, ix] += 1.0
    img = img / img.sum()
    return img.to(dtype).reshape(1, 1, k, k)


def make_psf(kind: str, k: int, dtype=torch.float32) -> torch.Tensor:
    if k == 0 or kind == "none":
        return torch.empty(0, dtype=dtype)
    if kind.startswith("gauss"):
        sigma = float(kind.split(":")[1]) if ":" in kind else max(k / 6.0, 0.5)
        return gaussian_psf(k, sigma, dtype)
    if kind == "motion":
        return motion_psf(k, 30.0, dtype)
    if kind == "random":
        g = torch.Generator().manual_seed(1234 + k)
        w = torch.rand((k, k), generator=g, dtype=torch.float64)
        return (w / w.sum()).to(dtype).reshape(1, 1, k, k)
    raise ValueError(f"unknown psf kind {kind!r}")


def clean_images(B: int, C: int, H: int, W: int, seed: int, device="cpu",
                 n_shapes: int = 10, dtype=torch.float32) -> torch.Tensor:
    """Piecewise-constant images: random rectangles and disks, values in [0, 1]."""
    g = torch.Generator(device="cpu").manual_seed(int(seed))
    img = torch.rand((B, C, 1, 1), generator=g).to(device=device, dtype=dtype).expand(B, C, H, W).clone()
    yy = torch.arange(H, device=device, dtype=torch.float32).reshape(1, 1, H, 1)
    xx = torch.arange(W, device=device, dtype=torch.float32).reshape(1, 1, 1, W)
    for s in range(n_shapes):
        cy = (torch.rand((B, 1, 1, 1), generator=g) * H).to(device)
        cx = (torch.rand((B, 1, 1, 1), generator=g) * W).to(device)
        ry = (torch.rand((B, 1, 1, 1), generator=g) * 0.25 * H + 0.05 * H).to(device)
        rx = (torch.rand((B, 1, 1, 1), generator=g) * 0.25 * W + 0.05 * W).to(device)
        val = torch.rand((B, C, 1, 1), generator=g).to(device=device, dtype=dtype)
        if s % 2 == 0:
            m = ((yy - cy).abs() <= ry) & ((xx - cx).abs() <= rx)
        else:
            m = ((yy - cy) / ry) ** 2 + ((xx - cx) / rx) ** 2 <= 1.0
        img = torch.where(m, val, img)
    return img.contiguous()


def blurred_batch(B: int, C: int, H: int, W: int, psf: torch.Tensor, seed: int, device="cpu",
                  noise: float = 0.01, dtype=torch.float32) -> torch.Tensor:
    """clean images (*) centred PSF (circular) + AWGN; returns a contiguous NCHW float tensor."""
    x = clean_images(B, C, H, W, seed, device=device, dtype=torch.float32)
    if psf.numel() > 0:
        k = psf.shape[-1]
        c = k // 2
        ker = torch.zeros((H, W), dtype=torch.float32, device=device)
        ker[:k, :k] = psf.reshape(k, k).to(device=device, dtype=torch.float32)
        ker = torch.roll(ker, shifts=(-c, -c), dims=(0, 1))
        x = torch.fft.irfftn(torch.fft.rfftn(x, dim=(2, 3)) * torch.fft.rfftn(ker), s=(H, W), dim=(2, 3))
    if noise > 0:
        g = torch.Generator(device="cpu").manual_seed(int(seed) + 7)
        if str(device).startswith("cpu"):
            x = x + noise * torch.randn(x.shape, generator=g, dtype=torch.float32)
        else:
            gd = torch.Generator(device=device).manual_seed(int(seed) + 7)
            x = x + noise * torch.randn(x.shape, generator=gd, dtype=torch.float32, device=device)
    return x.to(dtype).contiguous()

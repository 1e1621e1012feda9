"""admmtor.elayers.admmdeconv -- the ADMMDeconv layer over the MI355X solver.

Mirror of ``/root/reference/src/admmtor/elayers/admmdeconv.py:6-64``: identical
constructor keywords, parameter / buffer names, shapes, registration order and
initialisation (so reference checkpoints load and seeded inits match), and the
same ``forward = activation(fft_admm_tv(x, lmbda, rho, w, iso, max_iters) + b)``.
"""
from __future__ import annotations

from typing import Callable, Tuple

import torch

from admmtor.eops.deconv import fft_admm_tv, identity

__all__ = ["ADMMDeconv"]


class ADMMDeconv(torch.nn.Module):
    """Unrolled ADMM-TV deconvolution layer.

    kern_size  ``(kh, kw)`` -> learnable PSF ``w`` (1,1,kh,kw), xavier-uniform init;
               ``()`` / falsy -> no PSF (empty buffer ``w``, pure TV denoising)
    max_iters  ADMM iterations per forward
    lmbda, rho falsy (None or 0) -> learnable ``Parameter(1,)`` ~ U(0, 1);
               otherwise a fixed fp32 buffer
    iso        block (True, default) or soft (False) shrinkage
    bias       learnable scalar bias ``b`` ~ U(0, 1), else buffer 0
    activation applied to the biased output
    """

    def __init__(self,
                 kern_size: Tuple[int, int],
                 max_iters: int,
                 lmbda: float = None,
                 rho: float = None,
                 iso: bool = True,
                 bias: bool = False,
                 activation: Callable = identity):
        super().__init__()
        # registration order w, lmbda, rho, b as in the reference (admmdeconv.py:17-23)
        self._make_psf(kern_size)
        self.max_iters = max_iters
        self._make_scalar("lmbda", lmbda)
        self._make_scalar("rho", rho)
        self.iso = iso
        self._make_bias(bias)
        self.activation = activation

    def _make_psf(self, kern_size):
        if kern_size:
            self.w = torch.nn.Parameter(torch.empty((1, 1, *kern_size)), requires_grad=True)
            torch.nn.init.xavier_uniform_(self.w)
        else:
            self.register_buffer("w", torch.tensor([], dtype=torch.float32))

    def _make_scalar(self, name: str, value):
        if not value:  # None or 0.0 -> learnable, as in admmdeconv.py:27-29, 36-38
            p = torch.nn.Parameter(torch.empty(1), requires_grad=True)
            torch.nn.init.uniform_(p, a=0.0, b=1.0)
            setattr(self, name, p)
        else:
            self.register_buffer(name, torch.tensor([value], dtype=torch.float32))

    def _make_bias(self, bias: bool):
        if bias:
            self.b = torch.nn.Parameter(torch.empty(1), requires_grad=True)
            torch.nn.init.uniform_(self.b, a=0.0, b=1.0)
        else:
            self.register_buffer("b", torch.tensor([0], dtype=torch.float32))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.activation(fft_admm_tv(x, self.lmbda, self.rho, self.w, self.iso, self.max_iters) + self.b)

    def extra_repr(self) -> str:
        k = tuple(self.w.shape[-2:]) if self.w.numel() else ()
        return f"kern_size={k}, max_iters={self.max_iters}, iso={self.iso}"

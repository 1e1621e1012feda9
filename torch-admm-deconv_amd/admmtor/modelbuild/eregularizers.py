"""Parameter clamps applied to ADMMDeconv modules between optimizer steps.

Mirror of ``/root/reference/src/admmtor/modelbuild/eregularizers.py:5-33`` (same class names,
constructor arguments and behaviour, used as ``model.apply(clipper)``):

* ``ADMMWeightClipper(keep_range)`` clamps ``module.w`` (the learnable PSF) into ``keep_range``;
* ``ADMMClipper(max_val)`` clamps ``module.lmbda`` and ``module.rho`` into ``(1e-9, max_val)``.
  Like the reference, a module exposing ``bias`` gets ``bias = clamp(rho)`` (the reference's
  line 27; ``ADMMDeconv`` names its bias ``b``, so it is unaffected).

``WeightClipper`` of ``scripts/train.py:27-38`` (clamp lmbda / rho into [1e-12, 5]) is provided
too, so the training script's regulariser works on this build's modules.
"""
from __future__ import annotations

import torch
import torch.nn as nn

__all__ = ["ADMMWeightClipper", "ADMMClipper", "WeightClipper"]


class ADMMWeightClipper:
    def __init__(self, keep_range: tuple[float, float]):
        self.keep_range = keep_range

    def __call__(self, module: nn.Module):
        if hasattr(module, "w"):
            module.w.data = torch.clamp(module.w.data, *self.keep_range)


class ADMMClipper:
    def __init__(self, max_val: float):
        self.keep_range = (1e-9, max_val)

    def __call__(self, module: nn.Module):
        if hasattr(module, "lmbda"):
            module.lmbda.data = torch.clamp(module.lmbda.data, *self.keep_range)
        if hasattr(module, "rho"):
            module.rho.data = torch.clamp(module.rho.data, *self.keep_range)
        if hasattr(module, "bias"):  # reference quirk (eregularizers.py:26-27), kept as is
            module.bias.data = torch.clamp(module.rho.data, *self.keep_range)


class WeightClipper:
    """scripts/train.py:27-38: clamp lmbda and rho into [1e-12, 5]."""

    def __call__(self, module: nn.Module):
        for name in ("lmbda", "rho"):
            if hasattr(module, name):
                p = getattr(module, name)
                p.data = p.data.clamp(1e-12, 5)

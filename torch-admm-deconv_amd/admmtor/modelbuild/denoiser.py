"""DivergentRestorer -- the model scripts/train.py trains (config 5).

Mirrors /root/reference/src/admmtor/modelbuild/denoiser.py:7-63 (module names
blocks.{i}, scas.{i}; same construction order, so the same seed gives the same
weights).  Level 0 holds the ADMM-TV modules: with train.py's configuration
(`DivergentRestorer([2, 8, 32], 3, 3, 86, 86, 8, output_activation=Sigmoid(),
admms=[DECONV1, DECONV2])`, train.py:70-73) that is two iso solvers with 100
iterations each, run by the HIP kernels with their own backward.

Data flow (denoiser.py:53-62):
  out = sca_0(block_0(x))
  out = sca_i(block_i([out, x]))            for the middle levels
  out = block_L(  [sca_L(out), x])           for the last level
"""
import torch
import torch.nn as nn

from admmtor.elayers.cwa import ChannelWiseAttention
from admmtor.modelbuild.blocks import DivergentAttention


class DivergentRestorer(nn.Module):
    def __init__(self, level_branches: list, in_channels: int, final_channels: int, filters: int,
                 gate_channels: int, attention_reduction: int, intermediate_activation: nn.Module = None,
                 output_activation: nn.Module = None, admms: list = None):
        super().__init__()
        self._level_branches = level_branches
        last = len(level_branches) - 1
        self.blocks = nn.ModuleList()
        self.scas = nn.ModuleList()
        for level, branches in enumerate(level_branches):
            self.scas.append(ChannelWiseAttention(filters))
            first = level == 0
            self.blocks.append(DivergentAttention(
                branches=branches,
                in_channels=in_channels if first else filters + in_channels,
                out_channels=final_channels if (level == last and not first) else filters,
                conv_filters=filters, gate_channels=gate_channels, attention_reduction=attention_reduction,
                out_activation=output_activation if (level == last and not first) else intermediate_activation,
                admms=admms if first else None))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        n = len(self.blocks)
        out = self.scas[0](self.blocks[0](x))
        for level in range(1, n):
            if level < n - 1:
                out = self.scas[level](self.blocks[level](torch.cat([out, x], dim=1)))
            else:
                out = self.blocks[level](torch.cat([self.scas[level](out), x], dim=1))
        return out

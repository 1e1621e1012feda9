"""CBAM attention used by the config-5 caller.

Mirrors the module tree and parameter names of
/root/reference/src/admmtor/elayers/attentions.py so reference checkpoints load:

  CBAM.channel_gate : ChannelGate  (mlp.1 / mlp.3 Linear layers)         attentions.py:63-96, 98-111
  CBAM.spatial_gate : SpatialGate  (spatial.conv, spatial.norm)          attentions.py:50-60
  BasicConv         : conv -> InstanceNorm2d(affine) -> GELU|Identity    attentions.py:13-33

These are plain PyTorch (GEMM/conv-shaped work goes to MIOpen/hipBLASLt); only
the ADMM solver on this path is a hand-written kernel.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F


def logsumexp_2d(x: torch.Tensor) -> torch.Tensor:
    """(B, C, H, W) -> (B, C, 1): log-sum-exp over the spatial extent (attentions.py:6-10)."""
    flat = x.reshape(x.shape[0], x.shape[1], -1)
    peak = flat.amax(dim=2, keepdim=True)
    return peak + (flat - peak).exp().sum(dim=2, keepdim=True).log()


class BasicConv(nn.Module):
    """conv -> instance norm (affine) -> GELU (attentions.py:13-33)."""

    def __init__(self, in_planes, out_planes, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                 use_activation=True, norm=True, bias=True):
        super().__init__()
        self.out_channels = out_planes
        self.conv = nn.Conv2d(in_planes, out_planes, kernel_size=kernel_size, stride=stride, padding=padding,
                              dilation=dilation, groups=groups, bias=bias)
        self.norm = nn.InstanceNorm2d(out_planes, eps=1e-5, momentum=0.01, affine=True) if norm else nn.Identity()
        self.activation = nn.GELU() if use_activation else nn.Identity()

    def forward(self, x):
        return self.activation(self.norm(self.conv(x)))


class ChannelPool(nn.Module):
    """Per-pixel statistics across channels: unbiased std, lower median, mode (attentions.py:36-47)."""

    @staticmethod
    def forward(x: torch.Tensor) -> torch.Tensor:
        stats = (x.std(dim=1, keepdim=True),
                 x.median(dim=1, keepdim=True).values,
                 x.mode(dim=1, keepdim=True).values)
        return torch.cat(stats, dim=1)


class SpatialGate(nn.Module):
    """x * sigmoid(BasicConv(3 -> 1, k x k)(ChannelPool(x))) (attentions.py:50-60)."""

    def __init__(self, kernel_size: int = 7, use_activation: bool = False):
        super().__init__()
        self.compress = ChannelPool()
        self.spatial = BasicConv(3, 1, kernel_size, stride=1, padding=(kernel_size - 1) // 2,
                                 use_activation=use_activation)

    def forward(self, x):
        return x * torch.sigmoid(self.spatial(self.compress(x)))


def _global_pool(x: torch.Tensor, kind: str) -> torch.Tensor:
    """(B, C, H, W) -> (B, C) global pooling of the kinds ChannelGate accepts (attentions.py:77-89)."""
    if kind == "avg":
        return x.mean(dim=(2, 3))
    if kind == "max":
        return x.amax(dim=(2, 3))
    if kind == "lp":          # lp_pool2d with p = 2 over the whole plane: sqrt(sum x^2)
        return x.square().sum(dim=(2, 3)).sqrt()
    if kind == "lse":
        return logsumexp_2d(x).squeeze(2)
    raise ValueError(f"unknown pool type {kind!r}")


class ChannelGate(nn.Module):
    """x * sigmoid(sum_pool MLP(pool(x))) with a shared 2-layer MLP (attentions.py:63-96)."""

    def __init__(self, gate_channels, reduction_ratio=16, pool_types=("avg", "max")):
        super().__init__()
        self.gate_channels = gate_channels
        hidden = gate_channels // reduction_ratio
        self.mlp = nn.Sequential(nn.Flatten(), nn.Linear(gate_channels, hidden), nn.GELU(),
                                 nn.Linear(hidden, gate_channels))
        self.pool_types = pool_types

    def forward(self, x):
        logits = None
        for kind in self.pool_types:
            term = self.mlp(_global_pool(x, kind))
            logits = term if logits is None else logits + term
        return x * torch.sigmoid(logits)[:, :, None, None]


class CBAM(nn.Module):
    """Channel gate, then (optionally) spatial gate (attentions.py:98-111)."""

    def __init__(self, gate_channels, reduction_ratio=16, pool_types=("avg", "max"), use_spatial=False):
        super().__init__()
        self.channel_gate = ChannelGate(gate_channels, reduction_ratio, pool_types)
        self.spatial_gate = SpatialGate() if use_spatial else None

    def forward(self, x):
        y = self.channel_gate(x)
        return self.spatial_gate(y) if self.spatial_gate is not None else y

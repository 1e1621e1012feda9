"""CBAM attention used by the config-5 caller.

Mirrors the module tree and parameter names of
/root/reference/src/admmtor/elayers/attentions.py so reference checkpoints load:

  CBAM.channel_gate : ChannelGate  (mlp.1 / mlp.3 Linear layers)         attentions.py:63-96, 98-111
  CBAM.spatial_gate : SpatialGate  (spatial.conv, spatial.norm)          attentions.py:50-60
  BasicConv         : conv -> InstanceNorm2d(affine) -> GELU|Identity    attentions.py:13-33

These are plain PyTorch (GEMM/conv-shaped work goes to MIOpen/hipBLASLt), except the spatial
gate's per-pixel channel statistics (ChannelPool), which are one HIP kernel on the GPU
(include/admm_chanstat.h) -- PyTorch's sort-based mode/median were 46 % of the config-5 step.
"""
import os

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


_CHANSTAT_DTYPES = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}


def _chanstat_native(x: torch.Tensor, depth_limit=None):
    """(B, C, H, W) device tensor -> (out (B, 3, H, W), idx (B, 2, H, W) int16) via the HIP kernel of
    include/admm_chanstat.h; idx holds the channels the median and the mode were taken from."""
    from .. import _native
    lib = _native.load()
    B, C, H, W = x.shape
    out = torch.empty((B, 3, H, W), dtype=x.dtype, device=x.device)
    idx = torch.empty((B, 2, H, W), dtype=torch.int16, device=x.device)
    stream = torch.cuda.current_stream(x.device).cuda_stream
    dt = _CHANSTAT_DTYPES[x.dtype]
    if depth_limit is None:
        code = lib.admm_chanstat_pool(dt, x.data_ptr(), B, C, H * W, out.data_ptr(), idx.data_ptr(), stream)
    else:
        code = lib.admm_chanstat_pool_depth(dt, x.data_ptr(), B, C, H * W, out.data_ptr(), idx.data_ptr(),
                                            int(depth_limit), stream)
    _native.check(code)
    return out, idx


class _ChannelPoolFn(torch.autograd.Function):
    """ChannelPool's forward and backward as two HIP kernels (include/admm_chanstat.h)."""

    @staticmethod
    def forward(ctx, x):
        out, idx = _chanstat_native(x)
        ctx.save_for_backward(x, out, idx)
        return out

    @staticmethod
    def backward(ctx, gout):
        from .. import _native
        x, out, idx = ctx.saved_tensors
        gout = gout.to(x.dtype).contiguous()
        gx = torch.empty_like(x)
        B, C, H, W = x.shape
        stream = torch.cuda.current_stream(x.device).cuda_stream
        _native.check(_native.load().admm_chanstat_pool_backward(
            _CHANSTAT_DTYPES[x.dtype], x.data_ptr(), out.data_ptr(), idx.data_ptr(), gout.data_ptr(), B, C, H * W,
            gx.data_ptr(), stream))
        return gx


def channel_pool_reference_ops(x: torch.Tensor) -> torch.Tensor:
    """The reference's op sequence (attentions.py:44-47): std, lower median, mode over dim 1."""
    stats = (x.std(dim=1, keepdim=True),
             x.median(dim=1, keepdim=True).values,
             x.mode(dim=1, keepdim=True).values)
    return torch.cat(stats, dim=1)


def native_channel_pool_applies(x: torch.Tensor) -> bool:
    """GPU tensors of fp32/bf16/fp16 with at most 128 (fp32) / 256 channels take the HIP kernel."""
    if not x.is_cuda or x.dim() != 4 or x.dtype not in _CHANSTAT_DTYPES or os.environ.get("ADMMTOR_CHANPOOL") == "torch":
        return False
    return x.shape[1] <= (128 if x.dtype == torch.float32 else 256)


class ChannelPool(nn.Module):
    """Per-pixel statistics across channels: unbiased std, lower median, mode (attentions.py:36-47).

    On the GPU one HIP kernel computes all three with the reference's CPU tie rules (median: stable
    rank (C-1)/2; mode: the smallest most frequent value, at the index libstdc++ std::sort leaves it
    -- PyTorch's GPU mode leaves that unspecified) and a second one the backward.  CPU tensors (and
    fp64 or very wide inputs, or ADMMTOR_CHANPOOL=torch for A/B runs) take the reference's op sequence.
    """

    @staticmethod
    def forward(x: torch.Tensor) -> torch.Tensor:
        if native_channel_pool_applies(x):
            return _ChannelPoolFn.apply(x.contiguous())
        return channel_pool_reference_ops(x)


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

"""Channel-wise attention used between DivergentRestorer levels.

Mirrors /root/reference/src/admmtor/elayers/cwa.py (parameter names conv1, conv2,
compress_weight.{i}):

  weights = sum_m  w_m * stat_m(x)          per (b, c), stats over the whole plane    cwa.py:73-77
  out     = x * sigmoid(conv2(conv1(x)) * weights)                                    cwa.py:79-84
"""
import torch
import torch.nn as nn


def _planes(x: torch.Tensor) -> torch.Tensor:
    return x.reshape(x.shape[0], x.shape[1], -1)


def amedian(x):
    return _planes(x).median(dim=-1).values


def amodes(x):
    return _planes(x).mode(dim=-1).values


def amean(x):
    return _planes(x).mean(dim=-1)


def astd(x):
    return _planes(x).std(dim=-1)


def amax(x):
    return _planes(x).amax(dim=-1)


def amin(x):
    return _planes(x).amin(dim=-1)


class ChannelCompression:
    """Names of the per-plane statistics (cwa.py:30-36).  As in the reference, a member
    is the statistic function itself."""
    STD = staticmethod(astd)
    MEAN = staticmethod(amean)
    MAX = staticmethod(amax)
    MEDIAN = staticmethod(amedian)
    MODE = staticmethod(amodes)
    MIN = staticmethod(amin)


class ChannelWiseAttention(nn.Module):
    """cwa.py:40-90."""

    def __init__(self, in_channels: int,
                 channel_compress_methods=(ChannelCompression.STD, ChannelCompression.MEDIAN,
                                           ChannelCompression.MODE, ChannelCompression.MAX,
                                           ChannelCompression.MEAN),
                 probas_ch_factor: int = 2, compress_judges_mult: int = 10, reduce_probas_space: bool = False,
                 reduce_mean: bool = False, probas_only: bool = False):
        super().__init__()
        self.in_channels = in_channels
        self.probas_ch_factor = probas_ch_factor
        self.reduce_probas_space = reduce_probas_space
        self.reduce_mean = reduce_mean
        self.probas_only = probas_only
        self.compress_judges_mult = compress_judges_mult
        self.probas_space_size = (in_channels // probas_ch_factor if reduce_probas_space
                                  else in_channels * probas_ch_factor)
        self.conv1 = nn.Conv2d(in_channels, self.probas_space_size, kernel_size=1, bias=True)
        self.conv2 = nn.Conv2d(self.probas_space_size, in_channels, kernel_size=1, bias=True)
        self.compress_methods = tuple(channel_compress_methods)
        self.compress_weight = nn.ParameterList(
            [nn.Parameter(torch.ones(1)) for _ in self.compress_methods])
        self.prob_func = nn.Sigmoid()

    def _get_compressed_vals(self, x: torch.Tensor) -> torch.Tensor:
        acc = None
        for stat, weight in zip(self.compress_methods, self.compress_weight):
            term = stat(x) * weight
            acc = term if acc is None else acc + term
        return acc.reshape(x.shape[0], x.shape[1], 1, 1)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        gate = self.prob_func(self.conv2(self.conv1(x)) * self._get_compressed_vals(x))
        out = gate if self.probas_only else x * gate
        return out.mean(dim=(2, 3)) if self.reduce_mean else out

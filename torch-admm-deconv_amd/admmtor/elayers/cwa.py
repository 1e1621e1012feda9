"""Channel-wise attention used between DivergentRestorer levels.

Mirrors /root/reference/src/admmtor/elayers/cwa.py (parameter names conv1, conv2,
compress_weight.{i}):

  weights = sum_m  w_m * stat_m(x)          per (b, c), stats over the whole plane    cwa.py:73-77
  out     = x * sigmoid(conv2(conv1(x)) * weights)                                    cwa.py:79-84

The per-plane median and mode run as HIP kernels on the GPU (include/admm_chanstat.h,
csrc/plane_stats.hip) with the reference's CPU tie rules; PyTorch's GPU median/mode over 512^2
planes are per-slice thrust sorts (thousands of launches per step).  16-bit inputs get their
value statistics from an LDS histogram, fp32 from one segmented sort; CPU tensors and fp64 take
the reference's op sequence.
"""
import os

import torch
import torch.nn as nn

_PLANE_DTYPES = {torch.bfloat16: 1, torch.float16: 2, torch.float32: 0}


def _planes(x: torch.Tensor) -> torch.Tensor:
    return x.reshape(x.shape[0], x.shape[1], -1)


def _ord32(v: torch.Tensor) -> torch.Tensor:
    """Order-preserving unsigned image of fp32 bits (-0 -> +0, NaN -> all ones), as int64."""
    b = v.contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    mag = b & 0x7FFFFFFF
    b = torch.where(mag == 0, torch.zeros_like(b), b)
    o = torch.where((b & 0x80000000) != 0, (~b) & 0xFFFFFFFF, b | 0x80000000)
    return torch.where(mag > 0x7F800000, torch.full_like(o, 0xFFFFFFFF), o)


def _plane_mode_stats_f32(flat: torch.Tensor) -> torch.Tensor:
    """(P, N) fp32 -> (P, 4) int32 {mode code, mode count, 0, 0} from the runs of one segmented
    sort (the 16-bit types get these from the kernels' LDS histogram, the fp32 median from a
    radix select in the library)."""
    P, N = flat.shape
    st = torch.zeros((P, 4), dtype=torch.int64, device=flat.device)
    sv = torch.sort(flat, dim=1).values
    start = torch.ones((P, N), dtype=torch.bool, device=flat.device)
    start[:, 1:] = sv[:, 1:] != sv[:, :-1]
    pos = torch.arange(N, device=flat.device, dtype=torch.int32).expand(P, N)
    # next run start after each position (N past the last), by a reversed running minimum
    nxt = torch.full((P, N), N, device=flat.device, dtype=torch.int32)
    nxt[:, :-1] = torch.where(start[:, 1:], pos[:, 1:], nxt[:, 1:])
    nxt = torch.flip(torch.cummin(torch.flip(nxt, [1]), dim=1).values, [1])
    length = torch.where(start, nxt - pos, torch.zeros_like(pos))
    mcount = length.max(dim=1).values
    first = torch.argmax((length == mcount[:, None]).to(torch.int8), dim=1)  # first longest run
    st[:, 0] = _ord32(sv.gather(1, first[:, None]).squeeze(1))
    st[:, 1] = mcount.to(torch.int64)
    st = torch.where(st >= 2 ** 31, st - 2 ** 32, st)  # 32-bit codes as int32 bit patterns
    return st.to(torch.int32).contiguous()


def plane_select_native(x: torch.Tensor, which: str, depth_limit=None) -> torch.Tensor:
    """(B, C, H, W) ROCm bf16/fp16/fp32 tensor -> (B*C,) int64 flat indices of torch.median's
    ("median") or torch.mode's ("mode") element of each plane, by the HIP kernels."""
    from .. import _native
    import ctypes
    lib = _native.load()
    xs = _planes(x).contiguous()
    P, N = xs.shape[0] * xs.shape[1], xs.shape[2]
    idx = torch.empty(P, dtype=torch.int64, device=x.device)
    stream = torch.cuda.current_stream(x.device).cuda_stream
    # planes per call: workspace (24 N bytes per plane) up to 8 GiB, calls balanced (each call
    # should cover the chip: one workgroup per plane)
    most = max(1, (8 << 30) // max(1, 24 * N))
    ncall = -(-P // most)
    chunk = -(-P // ncall)
    nb = ctypes.c_size_t(0)
    _native.check(lib.admm_planestat_workspace_size(chunk, N, ctypes.byref(nb)))
    ws = torch.empty(nb.value, dtype=torch.uint8, device=x.device)
    flat = xs.reshape(P, N)
    for p0 in range(0, P, chunk):
        n = min(chunk, P - p0)
        out = idx[p0:p0 + n].data_ptr()
        dl = -1 if depth_limit is None else int(depth_limit)
        if x.dtype == torch.float32 and which == "mode":
            st = _plane_mode_stats_f32(flat[p0:p0 + n])
            _native.check(lib.admm_planestat_select(
                0, flat[p0].data_ptr(), n, N, st.data_ptr(), None, out, ws.data_ptr(), ws.numel(), dl, stream))
        else:
            _native.check(lib.admm_planestat_median_mode(
                _PLANE_DTYPES[x.dtype], flat[p0].data_ptr(), n, N, out if which == "median" else None,
                out if which == "mode" else None, ws.data_ptr(), ws.numel(), dl, stream))
    return idx


class _PlaneSelect(torch.autograd.Function):
    """value of each plane at the selected flat index; the gradient goes to that element
    (the reference's value_selecting_reduction_backward)."""

    @staticmethod
    def forward(ctx, x, which):
        idx = plane_select_native(x, which)
        B, C = x.shape[0], x.shape[1]
        flat = _planes(x).reshape(B * C, -1)
        ctx.save_for_backward(idx)
        ctx.shape = x.shape
        return flat.gather(1, idx[:, None]).reshape(B, C)

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        B, C = ctx.shape[0], ctx.shape[1]
        gx = torch.zeros((B * C, ctx.shape[2] * ctx.shape[3]), dtype=g.dtype,
                         device=g.device)
        gx.scatter_(1, idx[:, None], g.reshape(B * C, 1))
        return gx.reshape(ctx.shape), None


def _native_plane_applies(x: torch.Tensor) -> bool:
    return (x.is_cuda and x.dim() == 4 and x.dtype in _PLANE_DTYPES and x.shape[2] * x.shape[3] > 0
            and os.environ.get("ADMMTOR_PLANESTAT") != "torch")


def amedian(x):
    if _native_plane_applies(x):
        return _PlaneSelect.apply(x, "median")
    return _planes(x).median(dim=-1).values


def amodes(x):
    if _native_plane_applies(x):
        return _PlaneSelect.apply(x, "mode")
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

"""admmtor.eops.deconv -- MI355X build of the ADMM-TV proximal operator.

Drop-in for ``/root/reference/src/admmtor/eops/deconv.py``:

* :func:`fft_admm_tv` keeps the reference signature and argument meaning
  (deconv.py:35-40) and its error behaviour (deconv.py:42, 90-96),
  but runs the whole solver as hand-written HIP kernels for gfx950 through the
  C ABI of ``include/admm_tv.h`` (two fused HBM passes per iteration).  There is
  no CPU fallback: host tensors are staged to the current GPU (``_stage``) and the
  result is returned on that device; without a GPU or the HIP library the call
  raises.
* the small public helpers of the reference module (``torch_abs2``,
  ``hard_thresh``, ``soft_thresh``, ``block_thresh``, ``pixelnorm``,
  ``identity``, ``conv_circular``; deconv.py:7-32) keep their names and
  semantics; they are plain tensor expressions used by callers (``identity`` is
  imported by ``ADMMDeconv``), not part of the solver's hot path.
"""
from __future__ import annotations

from typing import Tuple

import torch
import torch.nn.functional as F

from .. import _native
from .. import _ops  # noqa: F401  (registers the admm_hip::* dispatcher ops)

__all__ = [
    "torch_abs2",
    "hard_thresh",
    "soft_thresh",
    "block_thresh",
    "pixelnorm",
    "identity",
    "conv_circular",
    "fft_admm_tv",
]


# ---------------------------------------------------------------- public helpers (deconv.py:7-32)
def torch_abs2(x: torch.Tensor) -> torch.Tensor:
    """|x|^2 (deconv.py:7-8)."""
    return torch.abs(x) ** 2


def hard_thresh(x: torch.Tensor, tau: float) -> torch.Tensor:
    """x where |x| > tau, else 0 (deconv.py:11-12)."""
    return x * (torch.abs(x) > tau)


def soft_thresh(x: torch.Tensor, tau: float) -> torch.Tensor:
    """sign(x) * max(|x| - tau, 0) (deconv.py:15-16)."""
    zero = torch.zeros(1, dtype=x.dtype, device=x.device)
    return torch.sign(x) * torch.maximum(torch.abs(x) - tau, zero)


def pixelnorm(x: torch.Tensor) -> torch.Tensor:
    """sqrt(sum over dims (0,1) of x^2 + 1e-15) (deconv.py:23-24)."""
    return torch.sqrt(torch.sum(x * x, (0, 1)) + 1e-15)


def block_thresh(x: torch.Tensor, tau: torch.Tensor) -> torch.Tensor:
    """max(1 - tau / (pixelnorm(x) + 1e-15), 0) * x (deconv.py:19-20)."""
    zero = torch.zeros(1, dtype=x.dtype, device=x.device)
    return torch.maximum(1 - tau / (pixelnorm(x) + 1e-15), zero) * x


def identity(x: torch.Tensor) -> torch.Tensor:
    return x


def conv_circular(x: torch.Tensor, w: torch.Tensor, pads: Tuple, groups: int) -> torch.Tensor:
    """circular pad + conv2d (deconv.py:31-32)."""
    return F.conv2d(F.pad(x, pads, mode="circular"), w, groups=groups)


# ---------------------------------------------------------------- boundary checks
def _check_inputs(xin: torch.Tensor, kern: torch.Tensor):
    if not isinstance(xin, torch.Tensor):
        raise TypeError("xin must be a torch.Tensor")
    if xin.dim() != 4:
        # the reference fails unpacking xin.shape into (B, C, H, W) (deconv.py:42)
        raise ValueError(f"fft_admm_tv expects a 4-D (B, C, H, W) input, got shape {tuple(xin.shape)}")
    if not isinstance(kern, torch.Tensor):
        raise TypeError("kern must be a torch.Tensor (use an empty tensor for no PSF)")
    autocast = xin.is_cuda and torch.is_autocast_enabled("cuda")
    if xin.dtype in (torch.float16, torch.bfloat16) and not autocast:
        # the reference's torch.fft rejects half types outside autocast
        raise RuntimeError(f"Unsupported dtype {xin.dtype}")
    if kern.numel() > 0:
        if kern.dim() < 3:
            raise IndexError("Dimension out of range: kern must be (1, 1, kh, kw)")
        if kern.dim() != 4 or kern.shape[0] != 1 or kern.shape[1] != 1:
            raise RuntimeError(f"kern must have shape (1, 1, kh, kw), got {tuple(kern.shape)}")
        if kern.shape[2] != kern.shape[3]:
            raise RuntimeError("non-square PSF: the reference's circular pads are swapped between H and W "
                               f"(deconv.py:90-96) and fail for shape {tuple(kern.shape)}")
        if not autocast and kern.dtype != xin.dtype:
            raise RuntimeError(f"expected kern dtype {xin.dtype}, got {kern.dtype}")


def _as_device_scalar(v, device, dtype=torch.float32) -> torch.Tensor:
    if isinstance(v, torch.Tensor):
        if v.numel() != 1:
            raise NotImplementedError("lmbd / rho must be scalars or 1-element tensors")
        return v.detach().reshape(1).to(device=device, dtype=dtype)
    return torch.full((1,), float(v), dtype=dtype, device=device)


def _scalar_input(v, device, dtype=torch.float32) -> torch.Tensor:
    """lmbd / rho -> (1,) device tensor of the solve's dtype; differentiable when v is a tensor that
    requires grad."""
    if isinstance(v, torch.Tensor):
        if v.numel() != 1:
            raise NotImplementedError("lmbd / rho must be scalars or 1-element tensors")
        return v.reshape(1).to(device=device, dtype=dtype)
    return torch.full((1,), float(v), dtype=dtype, device=device)


def _rocm_device() -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("admmtor (MI355X build): fft_admm_tv runs its HIP kernels on a ROCm device and none "
                           "is visible. There is no CPU path.")
    return torch.device("cuda", torch.cuda.current_device())


def _stage(xin, lmbd, rho, kern):
    """Host inputs -> the current ROCm device (the reference accepts CPU tensors, e.g.
    test_torch_admm.ipynb:249,302).  The copies are differentiable ``.to()`` calls, so gradients
    flow back to host tensors / parameters.  Device inputs pass through unchanged."""
    if xin.device.type in ("cuda", "meta"):  # meta: shape inference through the ops' fake kernels
        return xin, lmbd, rho, kern
    dev = _rocm_device()
    mv = (lambda v: v.to(dev) if isinstance(v, torch.Tensor) else v)
    return xin.to(dev), mv(lmbd), mv(rho), kern.to(dev)


def _solve(x32: torch.Tensor, k32: torch.Tensor, lam: torch.Tensor, rho: torch.Tensor, iso: bool, maxit: int,
           hook=None):
    """Run the HIP solver: x32 (B,C,H,W) fp32 (or fp64: an fp64 solve) contiguous on the device -> new
    tensor.  Without a hook this is the dispatcher op admm_hip::fft_admm_tv_fwd (admmtor._ops).
    `hook`: an _native.AllReduceHook for iso over a batch sharded across ranks; its callback is
    bound to this call's workspace only (no process-global state)."""
    if hook is None or not iso:
        return torch.ops.admm_hip.fft_admm_tv_fwd(x32, lam, rho, k32, bool(iso), int(maxit))
    f64 = x32.dtype == torch.float64
    B, C, H, W = x32.shape
    G = lam.numel()  # modules solved together (fft_admm_tv_grouped); 1 for fft_admm_tv
    k = int(k32.shape[-1]) if k32.numel() > 0 else 0
    bound = hook.bind(f64=f64)
    d = _native.desc(B, C, H, W, k, iso, maxit, 0, G, bound, f64=f64)
    if not _native.supported(H, W, f64):
        raise NotImplementedError(f"admmtor (MI355X build): H={H}, W={W} unsupported (admm_tv_supported: any "
                                  "size up to 65,536 per side)")
    ws = torch.empty(_native.workspace_size(d), dtype=torch.uint8, device=x32.device)
    bound.add(ws)
    out = torch.empty((G * B, C, H, W), dtype=x32.dtype, device=x32.device)
    stream = torch.cuda.current_stream(x32.device).cuda_stream
    _native.check(_native.entry("admm_tv_forward", f64)(
        d, x32.data_ptr(), k32.data_ptr() if k > 0 else None, lam.data_ptr(), rho.data_ptr(),
        out.data_ptr(), ws.data_ptr(), ws.numel(), stream))
    bound.check()
    return out


def fft_admm_tv(xin: torch.Tensor,
                lmbd: torch.Tensor,
                rho: torch.Tensor,
                kern: torch.Tensor,
                iso: bool = False,
                maxit: int = 100) -> torch.Tensor:
    """ADMM total-variation deconvolution, ``min_x 1/2 ||k * x - y||^2 + lmbd ||D x||_1``.

    Same contract as the reference (deconv.py:35-117): circular boundaries,
    forward differences, ``H_t`` = centred circular convolution with ``kern``,
    soft (``iso=False``) or batch/channel-coupled block (``iso=True``)
    shrinkage, ``tau = lmbd / rho``, ``maxit`` iterations from zero, returns the
    last x with xin's shape, on xin's device.  The solve always runs as HIP kernels on a ROCm
    device: host tensors are staged to the current device and the result copied back
    (autograd flows through both copies).  Arithmetic follows xin's dtype, as the reference's
    (deconv.py:49,61-67,104-106): fp32 inputs compute in fp32, fp64 inputs in fp64 (the generic
    kernels' double instantiation, ADMM_TV_FLAG_F64), bf16/fp16 under ``torch.autocast`` compute in
    fp32 and return fp32, as the reference does.
    """
    return _fft_admm_tv_impl(xin, lmbd, rho, kern, iso, maxit)


# A line whose length has a prime factor R beyond Bluestein's reach (2R - 1 > 1024, or any R on lines
# longer than 10,240 points) runs that factor as an any-prime stage: every output a sum of R terms, O(R)
# per output.  In fp32 those sums lose accuracy as R grows (13,001: 7.1e-6 vs the fp64 oracle, the 1e-5
# gate close); fp32 solves with a prime factor above this bound -- the largest prime measured in fp32 --
# therefore compute in fp64 (the generic kernels' double instantiation) and return fp32: same kernels,
# same cost order (O(n R) per line), fp64 accuracy.  tests/test_gpu_generic.py runs 13,001 in fp32 and
# 13,003 / 16,381 / 65,521 (the largest prime line accepted) through fp64.
F32_MAX_PRIME = 13001


def _largest_prime(n: int) -> int:
    big, f = 1, 2
    while f * f <= n:
        while n % f == 0:
            big, n = f, n // f
        f += 1
    return max(big, n)


def _fft_admm_tv_impl(xin, lmbd, rho, kern, iso=False, maxit=100, hook=None) -> torch.Tensor:
    """fft_admm_tv with an optional cross-rank all-reduce hook (admmtor.sharded)."""
    if not isinstance(kern, torch.Tensor):
        kern = torch.as_tensor(kern)
    _check_inputs(xin, kern)
    home, out_dtype = xin.device, (torch.float64 if xin.dtype == torch.float64 else torch.float32)
    cdt = out_dtype  # the solve's arithmetic: fp64 for fp64 inputs, else fp32
    if cdt == torch.float32 and max(_largest_prime(int(xin.shape[2])), _largest_prime(int(xin.shape[3]))) > F32_MAX_PRIME:
        cdt = torch.float64  # see F32_MAX_PRIME
    maxit = max(0, int(maxit))  # the reference loops over torch.arange(0, maxit): negative -> no iteration
    # empty batch: the reference's ops return an empty result of the same shape.  An empty shard of
    # an iso solve over ranks still runs: it must take part in every iteration's all-reduce.
    shard_member = hook is not None and iso and xin.shape[2] > 0 and xin.shape[3] > 0
    if xin.numel() == 0 and not shard_member:
        return torch.zeros(xin.shape, dtype=out_dtype, device=home)
    xin, lmbd, rho, kern = _stage(xin, lmbd, rho, kern)
    dev = xin.device
    needs_grad = torch.is_grad_enabled() and (
        xin.requires_grad or (isinstance(lmbd, torch.Tensor) and lmbd.requires_grad)
        or (isinstance(rho, torch.Tensor) and rho.requires_grad) or kern.requires_grad)
    if needs_grad:
        if hook is not None and iso:
            from .._backward import fft_admm_tv_autograd
            out = fft_admm_tv_autograd(xin, lmbd, rho, kern, bool(iso), maxit, hook=hook)
        else:
            xc = xin.to(cdt).contiguous()  # differentiable cast (autocast half inputs)
            kc = kern.to(device=dev, dtype=cdt).contiguous() if kern.numel() > 0 else \
                torch.empty(0, dtype=cdt, device=dev)
            psf_grad = kern.requires_grad and kern.numel() > 0
            out, _ = torch.ops.admm_hip.fft_admm_tv_fwd_train(
                xc, _scalar_input(lmbd, dev, cdt), _scalar_input(rho, dev, cdt), kc, bool(iso), maxit, psf_grad)
    else:
        xc = xin.detach().to(cdt).contiguous()
        kc = kern.detach().to(device=dev, dtype=cdt).contiguous() if kern.numel() > 0 else \
            torch.empty(0, dtype=cdt, device=dev)
        out = _solve(xc, kc, _as_device_scalar(lmbd, dev, cdt), _as_device_scalar(rho, dev, cdt), bool(iso), maxit,
                     hook=hook)
    return out.to(device=home, dtype=out_dtype)


def fft_admm_tv_grouped(xin: torch.Tensor, lmbds, rhos, kern: torch.Tensor, iso: bool = False,
                        maxit: int = 100) -> list:
    """G ADMM-TV solves of the SAME input with per-module lambda / rho, in one pass sequence.

    ``[fft_admm_tv(xin, l, r, kern, iso, maxit) for l, r in zip(lmbds, rhos)]`` as one native
    call (desc.groups = G): every launch covers all modules' planes, each module keeps its own
    Wiener factor (its rho) and, for iso, its own per-pixel norm over its (B, C).  This is how
    DivergentAttention's ADMM modules that share x run (blocks.py:187-196).
    Autograd reaches xin (summed over modules) and every lambda / rho.  Power-of-two H, W run
    on the fused kernels (inference and training); smooth sizes (``admm_tv_supported == 3``)
    solve the modules one after another inside one native call on the mixed-radix kernels,
    sharing b = H_t(xin) and the tables (inference), and train as one call per module.  The PSF
    must not require grad; returns G tensors.
    """
    if not isinstance(kern, torch.Tensor):
        kern = torch.as_tensor(kern)
    _check_inputs(xin, kern)
    if not xin.is_cuda:
        raise RuntimeError("admmtor (MI355X build): fft_admm_tv runs on ROCm device tensors only; "
                           "move xin (and kern) to the GPU. There is no CPU path.")
    G = len(lmbds)
    if G != len(rhos) or G < 1:
        raise ValueError("lmbds and rhos must have the same, non-zero length")
    B, C, H, W = xin.shape
    sup = _native.load().admm_tv_supported(H, W)
    if sup not in (1, 3) or (kern.requires_grad and kern.numel() > 0):
        raise NotImplementedError("grouped solve: power-of-two or smooth H, W and a fixed PSF only")
    maxit = max(0, int(maxit))
    dev = xin.device
    needs_grad = torch.is_grad_enabled() and (
        xin.requires_grad or any(isinstance(v, torch.Tensor) and v.requires_grad for v in (*lmbds, *rhos)))
    if needs_grad and sup == 3:
        # grouped training is power-of-two only (include/admm_tv.h): one training call per module
        return [fft_admm_tv(xin, l, r, kern, iso, maxit) for l, r in zip(lmbds, rhos)]
    if needs_grad:
        # lambda and rho stacked into (G,) tensors differentiably, so each module's parameters get theirs
        x32 = xin.to(torch.float32).contiguous()
        k32 = kern.detach().to(device=dev, dtype=torch.float32).contiguous() if kern.numel() > 0 else \
            torch.empty(0, dtype=torch.float32, device=dev)
        lam_t = torch.cat([_scalar_input(v, dev) for v in lmbds])
        rho_t = torch.cat([_scalar_input(v, dev) for v in rhos])
        out, _ = torch.ops.admm_hip.fft_admm_tv_fwd_train(x32, lam_t, rho_t, k32, bool(iso), maxit, False)
    else:
        x32 = xin.detach().to(torch.float32).contiguous()
        k32 = kern.detach().to(device=dev, dtype=torch.float32).contiguous() if kern.numel() > 0 else \
            torch.empty(0, dtype=torch.float32, device=dev)
        lam = torch.cat([_as_device_scalar(v, dev) for v in lmbds])
        rh = torch.cat([_as_device_scalar(v, dev) for v in rhos])
        out = _solve(x32, k32, lam, rh, bool(iso), maxit)
    return list(out.split(B, dim=0))

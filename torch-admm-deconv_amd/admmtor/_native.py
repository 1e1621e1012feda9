"""ctypes binding of the MI355X C ABI (include/admm_tv.h -> admmtor/_lib/libadmm_tv.so).

The shared library is the product: there is no CPU or PyTorch fallback.  If the
library is missing or fails to load, every entry point raises loudly.
"""
from __future__ import annotations

import contextlib
import ctypes
import glob
import hashlib
import os
import threading

# The release library.  The package reads no environment variable to pick another one: tuning tools
# and A/B test runs call use_library() explicitly before the first native call (tools/sweep.py,
# tests/conftest.py), so a user's job always loads this file.
RELEASE_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libadmm_tv.so")
_LIB_PATH = RELEASE_LIB_PATH
# the same sources built with -DADMM_AB_BUILD=1 (csrc/knobs.hpp): its A/B knobs follow the environment.
# Never used by the package itself; tests that compare alternative kernels select it with ab_library().
AB_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libadmm_tv_ab.so")

ADMM_TV_OK = 0
ADMM_TV_EINVAL = -1
ADMM_TV_EUNSUPPORTED = -2
ADMM_TV_ENONSQUARE = -3
ADMM_TV_EWORKSPACE = -4
ADMM_TV_EHIP = -5
ADMM_TV_EKERNEL = -6

# every symbol include/admm_tv.h declares (checked by tests/test_capi_symbols.py)
EXPORTED = (
    "admm_tv_abi_version",
    "admm_tv_build_hash",
    "admm_tv_supported",
    "admm_tv_supported_f64",
    "admm_tv_path",
    "admm_tv_workspace_size",
    "admm_tv_forward",
    "admm_tv_forward_f64",
    "admm_tv_forward_train_f64",
    "admm_tv_backward_f64",
    "admm_tv_psf_transpose",
    "admm_tv_history_size",
    "admm_tv_forward_train",
    "admm_tv_backward_workspace_size",
    "admm_tv_backward",
    "admm_tv_profile_enable",
    "admm_tv_profile_reset",
    "admm_tv_profile_read",
    "admm_tv_last_error",
)
# every symbol include/admm_chanstat.h declares
EXPORTED_CHANSTAT = (
    "admm_chanstat_max_channels",
    "admm_chanstat_pool",
    "admm_chanstat_pool_depth",
    "admm_chanstat_pool_backward",
    "admm_planestat_workspace_size",
    "admm_planestat_median_mode",
    "admm_planestat_select",
)
CHANSTAT_F32, CHANSTAT_BF16, CHANSTAT_F16 = 0, 1, 2


# admm_tv_allreduce_fn: (float* buf, size_t count, void* stream, void* ctx)
ALLREDUCE_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p)


class AdmmTvDesc(ctypes.Structure):
    _fields_ = [
        ("B", ctypes.c_int64),
        ("C", ctypes.c_int64),
        ("H", ctypes.c_int64),
        ("W", ctypes.c_int64),
        ("kh", ctypes.c_int32),
        ("kw", ctypes.c_int32),
        ("iso", ctypes.c_int32),
        ("maxit", ctypes.c_int32),
        ("flags", ctypes.c_int32),
        ("groups", ctypes.c_int32),
        ("allreduce", ALLREDUCE_FN),      # per-call cross-rank hook (iso over a sharded batch)
        ("allreduce_ctx", ctypes.c_void_p),
    ]


ADMM_TV_FLAG_PSF_GRAD = 1
ADMM_TV_FLAG_F64 = 2  # fp64 solve: the *_f64 entry points, double arrays
ABI_VERSION = 7
# admm_tv_path codes (include/admm_tv.h)
PATHS = {1: "fused", 2: "generic", 3: "fused mixed-radix", 4: "fused odd-length"}


class NativeError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"admm_tv native error {code}: {msg}")
        self.code = code


_lib = None
_lock = threading.Lock()

_CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc")


def source_hash():
    """The hash csrc/Makefile embeds (admm_tv_build_hash): SHA-256 of the library's sources in
    byte-wise sorted path order, then the Makefile; None when the sources are not in the tree."""
    if not os.path.isfile(os.path.join(_CSRC, "Makefile")):
        return None
    rel = sorted(glob.glob("*.hip", root_dir=_CSRC) + glob.glob("*.hpp", root_dir=_CSRC)
                 + glob.glob("../../include/*.h", root_dir=_CSRC), key=lambda p: p.encode())
    h = hashlib.sha256()
    for r in rel + ["Makefile"]:
        with open(os.path.join(_CSRC, r), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def lib_path() -> str:
    return _LIB_PATH


def use_library(path: str) -> None:
    """Tuning and A/B tooling only (tools/sweep.py, tests/conftest.py): load `path` (a variant of the
    library built from the same sources, e.g. tools/_variants/*.so or the A/B build) instead of the
    release library.  Must run before the first native call of the process."""
    global _LIB_PATH
    with _lock:
        if _lib is not None and os.path.abspath(path) != os.path.abspath(_LIB_PATH):
            raise RuntimeError("admmtor: use_library() after the native library was loaded")
        _LIB_PATH = path


def load() -> ctypes.CDLL:
    """Load (once) and return the native library; raises ImportError if absent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        _lib = _open(_LIB_PATH)
        return _lib


_ab_lib = None


@contextlib.contextmanager
def ab_library():
    """Tests and tuning only: inside the block every native call of this process goes to the A/B
    build (AB_LIB_PATH), whose ADMM_* knobs follow the environment, e.g. a solve on the generic kernels
    at a smooth size (ADMM_MIXED=0) to compare two kernel paths.  Not thread-safe (swaps the module's
    library handle)."""
    global _lib, _ab_lib
    prev = load()
    with _lock:
        if _ab_lib is None:
            _ab_lib = _open(AB_LIB_PATH)
        _lib = _ab_lib
    try:
        yield _ab_lib
    finally:
        _lib = prev


def _open(path: str) -> ctypes.CDLL:
    if not os.path.exists(path):
        raise ImportError(
            f"admmtor: the HIP library {path} is missing. Build it with "
            "`python __graft_entry__.py build` (or `make -C torch-admm-deconv_amd/csrc`). "
            "There is no CPU fallback.")
    L = ctypes.CDLL(path)
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    dp = ctypes.POINTER(AdmmTvDesc)
    L.admm_tv_abi_version.restype = ctypes.c_int
    L.admm_tv_abi_version.argtypes = []
    L.admm_tv_build_hash.restype = ctypes.c_char_p
    L.admm_tv_build_hash.argtypes = []
    L.admm_tv_supported.restype = ctypes.c_int
    L.admm_tv_supported.argtypes = [ctypes.c_int64, ctypes.c_int64]
    L.admm_tv_supported_f64.restype = ctypes.c_int
    L.admm_tv_supported_f64.argtypes = [ctypes.c_int64, ctypes.c_int64]
    L.admm_tv_path.restype = ctypes.c_int
    L.admm_tv_path.argtypes = [dp, ctypes.c_int]
    L.admm_tv_workspace_size.restype = ctypes.c_int
    L.admm_tv_workspace_size.argtypes = [dp, ctypes.POINTER(sz)]
    for f in ("admm_tv_forward", "admm_tv_forward_f64"):
        getattr(L, f).restype = ctypes.c_int
        getattr(L, f).argtypes = [dp, vp, vp, vp, vp, vp, vp, sz, vp]
    L.admm_tv_history_size.restype = ctypes.c_int
    L.admm_tv_history_size.argtypes = [dp, ctypes.POINTER(sz)]
    for f in ("admm_tv_forward_train", "admm_tv_forward_train_f64"):
        getattr(L, f).restype = ctypes.c_int
        getattr(L, f).argtypes = [dp, vp, vp, vp, vp, vp, vp, sz, vp, sz, vp]
    L.admm_tv_backward_workspace_size.restype = ctypes.c_int
    L.admm_tv_backward_workspace_size.argtypes = [dp, ctypes.POINTER(sz)]
    for f in ("admm_tv_backward", "admm_tv_backward_f64"):
        getattr(L, f).restype = ctypes.c_int
        getattr(L, f).argtypes = [dp, vp, vp, vp, vp, vp, vp, sz, vp, vp, vp, vp, vp, sz, vp]
    L.admm_tv_psf_transpose.restype = ctypes.c_int
    L.admm_tv_psf_transpose.argtypes = [dp, vp, vp, vp, vp, sz, vp]
    L.admm_tv_profile_enable.restype = ctypes.c_int
    L.admm_tv_profile_enable.argtypes = [ctypes.c_int]
    L.admm_tv_profile_reset.restype = ctypes.c_int
    L.admm_tv_profile_reset.argtypes = []
    L.admm_tv_profile_read.restype = ctypes.c_int
    L.admm_tv_profile_read.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)]
    L.admm_tv_last_error.restype = ctypes.c_char_p
    L.admm_tv_last_error.argtypes = []
    i64 = ctypes.c_int64
    L.admm_chanstat_max_channels.restype = ctypes.c_int
    L.admm_chanstat_max_channels.argtypes = [ctypes.c_int]
    L.admm_chanstat_pool.restype = ctypes.c_int
    L.admm_chanstat_pool.argtypes = [ctypes.c_int, vp, i64, i64, i64, vp, vp, vp]
    L.admm_chanstat_pool_depth.restype = ctypes.c_int
    L.admm_chanstat_pool_depth.argtypes = [ctypes.c_int, vp, i64, i64, i64, vp, vp, ctypes.c_int, vp]
    L.admm_chanstat_pool_backward.restype = ctypes.c_int
    L.admm_chanstat_pool_backward.argtypes = [ctypes.c_int, vp, vp, vp, vp, i64, i64, i64, vp, vp]
    L.admm_planestat_workspace_size.restype = ctypes.c_int
    L.admm_planestat_workspace_size.argtypes = [i64, i64, ctypes.POINTER(sz)]
    L.admm_planestat_median_mode.restype = ctypes.c_int
    L.admm_planestat_median_mode.argtypes = [ctypes.c_int, vp, i64, i64, vp, vp, vp, sz, ctypes.c_int, vp]
    L.admm_planestat_select.restype = ctypes.c_int
    L.admm_planestat_select.argtypes = [ctypes.c_int, vp, i64, i64, vp, vp, vp, vp, sz, ctypes.c_int, vp]
    if L.admm_tv_abi_version() != ABI_VERSION:
        raise ImportError("admmtor: native library ABI version mismatch")
    want, have = source_hash(), L.admm_tv_build_hash().decode()
    if want is not None and want != have:
        raise ImportError(f"admmtor: {path} was built from other sources (build hash {have}, tree "
                          f"{want}); rebuild it: `python __graft_entry__.py build`")
    return L


def check(code: int) -> None:
    if code != ADMM_TV_OK:
        msg = load().admm_tv_last_error().decode(errors="replace")
        raise NativeError(code, msg)


def desc(B, C, H, W, k, iso, maxit, flags=0, groups=1, allreduce=None, f64=False) -> AdmmTvDesc:
    """allreduce: a BoundAllReduce (AllReduceHook.bind) for iso over a sharded batch, or None.
    f64: an fp64 solve (ADMM_TV_FLAG_F64; the *_f64 entry points)."""
    flags = int(flags) | (ADMM_TV_FLAG_F64 if f64 else 0)
    return AdmmTvDesc(int(B), int(C), int(H), int(W), int(k), int(k), int(bool(iso)), int(maxit), flags,
                      int(groups), allreduce.cfn if allreduce is not None else ALLREDUCE_FN(), None)


def entry(name: str, f64: bool):
    """The C entry point `name` of the solve's precision (admm_tv_forward / admm_tv_forward_f64 ...)."""
    return getattr(load(), name + ("_f64" if f64 else ""))


def workspace_size(d: AdmmTvDesc) -> int:
    n = ctypes.c_size_t(0)
    check(load().admm_tv_workspace_size(ctypes.byref(d), ctypes.byref(n)))
    return int(n.value)


def history_size(d: AdmmTvDesc) -> int:
    n = ctypes.c_size_t(0)
    check(load().admm_tv_history_size(ctypes.byref(d), ctypes.byref(n)))
    return int(n.value)


def backward_workspace_size(d: AdmmTvDesc) -> int:
    n = ctypes.c_size_t(0)
    check(load().admm_tv_backward_workspace_size(ctypes.byref(d), ctypes.byref(n)))
    return int(n.value)


def path(d: AdmmTvDesc, train: bool = False) -> str:
    """The kernel path a solve of descriptor `d` takes (admm_tv_path): "fused", "generic",
    "fused mixed-radix" or "fused odd-length"."""
    code = load().admm_tv_path(ctypes.byref(d), 1 if train else 0)
    if code < 0:
        check(code)
    return PATHS[code]


def supported(H: int, W: int, f64: bool = False) -> bool:
    if f64:
        return bool(load().admm_tv_supported_f64(int(H), int(W)))
    return bool(load().admm_tv_supported(int(H), int(W)))


# --------------------------------------------------------------------------- cross-rank hook
class BoundAllReduce:
    """The all-reduce callback of ONE native call (admm_tv_desc.allreduce).  The library hands it
    raw device pointers inside the buffers this call allocated (workspace, history); they are
    mapped back to views of exactly those tensors.  Nothing is shared between calls, so solves on
    several threads / streams each carry their own.  A Python exception inside the callback
    cannot cross the C frame: it is kept and re-raised by check() after the call returns."""

    def __init__(self, dist, group, tensors=(), f64=False):
        self._dist, self._group = dist, group
        self._f64 = f64  # an fp64 solve hands `count` doubles
        self._bufs = []
        self.add(*tensors)
        self.error = None
        self.cfn = ALLREDUCE_FN(self._call)  # referenced by self for the duration of the call

    def add(self, *tensors):
        """Buffers of this call the library may hand to the callback (workspace, history)."""
        self._bufs.extend(t for t in tensors if t is not None)

    def _view_of(self, ptr: int, count: int):
        import torch
        dt = torch.float64 if self._f64 else torch.float32
        nbytes = (8 if self._f64 else 4) * count
        for t in self._bufs:
            base = t.data_ptr()
            if base <= ptr and ptr + nbytes <= base + t.numel() * t.element_size():
                off = ptr - base
                return t.view(torch.uint8)[off:off + nbytes].view(dt)
        raise RuntimeError("admmtor: all-reduce buffer not inside this call's workspace")

    def _call(self, ptr, count, stream, ctx):
        if self.error is not None:
            return
        try:
            import torch
            buf = self._view_of(int(ptr), int(count))
            # The collective must be ordered on the stream the library queued the sums on (its
            # `stream` argument), whatever torch's current stream is: RCCL / gloo order a
            # collective against torch's current stream, so make that stream current for the call.
            if buf.is_cuda:
                st = torch.cuda.ExternalStream(int(stream), device=buf.device) if stream \
                    else torch.cuda.default_stream(buf.device)
                with torch.cuda.device(buf.device), torch.cuda.stream(st):
                    self._dist.all_reduce(buf, op=self._dist.ReduceOp.SUM, group=self._group)
            else:
                self._dist.all_reduce(buf, op=self._dist.ReduceOp.SUM, group=self._group)
        except BaseException as e:  # noqa: BLE001 -- re-raised by check()
            self.error = e

    def check(self):
        if self.error is not None:
            raise RuntimeError("admmtor: cross-rank all-reduce failed inside the solve") from self.error


class AllReduceHook:
    """SUM all-reduce over a torch.distributed group for iso over a sharded batch.  bind() makes
    the per-call callback; the hook itself holds no per-solve state."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self._dist = dist
        self._group = group

    def bind(self, *tensors, f64: bool = False) -> BoundAllReduce:
        return BoundAllReduce(self._dist, self._group, tensors, f64=f64)


def profile_enable(on: bool) -> None:
    check(load().admm_tv_profile_enable(1 if on else 0))


def profile_reset() -> None:
    check(load().admm_tv_profile_reset())


def profile_read():
    """-> (ms[4], count[4]) for pass A, pass B, iso norm, setup."""
    ms = (ctypes.c_double * 4)()
    n = (ctypes.c_int64 * 4)()
    check(load().admm_tv_profile_read(ms, n))
    return list(ms), list(n)

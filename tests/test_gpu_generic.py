"""Generic sizes: every H, W in [1, 65,536] that the fused power-of-two kernels
do not take runs on the generic HIP kernels (mixed-radix LDS transforms + per-pixel step; lines
beyond 10,240 points keep their two buffers in a global scratch slot per block).

Parity as for the fast path: rel-L2 <= 1e-5 against the reference's fp64 output (golden 15x17
case) or the fp64 oracle pinned to it; gradients as in test_gpu_grad.py (1e-4 without PSF,
1e-3 with one, kink-aware where the oracle reports a plane near the shrink kink).
"""
import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu

TOL_REF64 = 1e-5


def rel(a, b):
    a = torch.as_tensor(a).double().cpu().reshape(-1)
    b = torch.as_tensor(b).double().cpu().reshape(-1)
    return (torch.linalg.vector_norm(a - b) / torch.linalg.vector_norm(b)).item()


def solve(x, psf, lam, rho, iso, it, dev):
    from admmtor.eops.deconv import fft_admm_tv
    x = torch.as_tensor(x).float().to(dev)
    k = torch.as_tensor(psf).float().to(dev) if psf is not None else torch.empty(0, device=dev)
    out = fft_admm_tv(x, lam, rho, k, iso, it)
    torch.cuda.synchronize()
    return out.cpu()


def oracle(x, psf, lam, rho, iso, it):
    from oracle.admm_oracle import solve_fourier
    k = torch.as_tensor(psf).double() if psf is not None else torch.empty(0, dtype=torch.float64)
    return solve_fourier(torch.as_tensor(x).double(), lam, rho, k, iso, it)


def test_generic_path_is_taken():
    from admmtor import _native
    assert _native.load().admm_tv_supported(15, 17) == 2 and _native.load().admm_tv_supported(64, 64) == 1


def test_g7_odd_size_vs_reference(cuda_dev):
    e = load_golden("g7_edges")
    out = solve(e["odd_x"], e["odd_psf"], 0.01, 0.02, False, 20, cuda_dev)
    err = rel(out, e["odd_out"])
    print("15x17 even-PSF vs reference fp64:", err)
    assert err <= TOL_REF64


@pytest.mark.parametrize("shape,psf,iso,it", [
    ((1, 2, 15, 17), None, True, 30),
    ((2, 3, 24, 40), ("gauss:1.0", 5), False, 25),
    ((1, 1, 100, 75), ("motion", 9), True, 20),
    ((1, 3, 481, 321), ("gauss:1.5", 9), False, 30),      # a BSD-sized image
    ((2, 1, 8, 64), None, False, 15),                      # power of two below the fast path's 16
    ((1, 1, 1, 32), None, False, 10),                      # one row
    ((1, 1, 7, 1), None, True, 10),                        # one column
    ((1, 2, 97, 101), ("gauss:2", 7), False, 20),          # prime sizes (generic radix stages)
    ((1, 1, 360, 1000), ("motion", 15), False, 10),        # 2^3 3^2 5 x 2^3 5^3
    ((1, 1, 64, 4096), ("gauss:2", 11), False, 5),         # W beyond the fast path
    ((1, 1, 143, 121), ("gauss:1.5", 7), True, 15),        # 11*13 x 11^2: the radix-11 / 13 butterflies
    ((1, 2, 66, 130), ("motion", 7), False, 12),           # 2*3*11 x 2*5*13: radix 11 / 13 after other stages
    ((1, 1, 509, 37), ("motion", 9), False, 10),           # prime 509: Bluestein at M = 1024
    ((1, 2, 509, 509), ("gauss:1.5", 9), False, 10),        # 509 x 509 (VERDICT r5 item 1's parity shapes)
    ((1, 1, 1080, 1921), ("gauss:1.5", 9), False, 6),      # 1921 = 17 * 113 rows beside HD columns
    ((1, 2, 26, 1021), None, False, 8),                    # prime 1021 > 512: the direct prime stage
    ((1, 1, 214, 321), ("gauss:2", 7), True, 12),          # 2*107 x 3*107
    ((1, 1, 12, 6000), ("gauss:1.5", 9), False, 6),        # lines beyond 4096 (one line per block)
    ((1, 1, 5120, 9), ("motion", 5), True, 5),             # a 5120-point column pass
    ((1, 1, 10, 8192), ("gauss:1.5", 9), False, 4),        # 8192-point rows: twiddles from global memory
    ((1, 1, 7680, 6), None, True, 4),                      # 7680-point columns (an 8K frame width)
    ((1, 1, 9, 12000), ("gauss:1.5", 9), False, 6),        # lines beyond 10,240: global line buffers
    ((1, 1, 1, 12000), None, True, 6),                     # the panorama row of VERDICT r2 #7
    ((1, 3, 2160, 3840), ("gauss:2", 11), False, 4),       # a 4K UHD frame (2^4 3^3 5 x 2^8 3 5)
    ((2, 1, 12000, 3), None, True, 4),                     # 12,000-point columns in global scratch
    ((1, 1, 5, 13001), ("motion", 5), False, 3),           # a prime line beyond 10,240 (any-prime stage)
    ((1, 1, 5, 13003), ("motion", 5), False, 3),           # the next prime: past F32_MAX_PRIME, solved in fp64
    ((1, 1, 16381, 2), None, False, 2),                    # the largest prime under 2^14, fp64
    ((1, 1, 8, 65521), ("motion", 5), False, 2),           # the largest prime line: fp32 input solved in fp64
    ((1, 1, 65521, 2), None, True, 2),                     #   (eops.deconv.F32_MAX_PRIME), O(n^2) per line
])
def test_generic_shapes_vs_oracle(cuda_dev, shape, psf, iso, it):
    from admmtor.synth import blurred_batch, make_psf
    k = make_psf(*psf) if psf else None
    x = blurred_batch(*shape, k if k is not None else torch.empty(0), seed=sum(shape))
    got = solve(x, k, 0.01, 0.02, iso, it, cuda_dev)
    ref = oracle(x, k, 0.01, 0.02, iso, it)
    err = rel(got, ref)
    print(shape, psf, "iso" if iso else "aniso", "rel vs fp64 oracle:", err)
    assert err <= TOL_REF64


@pytest.mark.parametrize("shape", [(2, 3, 321, 481), (1, 2, 143, 509), (1, 1, 37, 74)])
def test_bluestein_matches_direct_prime_stages(cuda_dev, shape, monkeypatch):
    """Chirp-z (Bluestein) stages vs the O(R)-per-output prime stages (ADMM_BLUE_MIN=0): both are
    fp32 evaluations of the same transform; Bluestein must meet the fp64-oracle gate and be no less
    accurate than the direct stages (within 2x + 1e-6; the direct O(R) stage itself drifts to ~1e-5
    for R = 509)."""
    from admmtor.synth import blurred_batch, make_psf
    k = make_psf("gauss:1.5", 9)
    x = blurred_batch(*shape, k, seed=7)
    ref = oracle(x, k, 0.01, 0.02, False, 15)
    from admmtor import _native
    e_blue0 = rel(solve(x, k, 0.01, 0.02, False, 15, cuda_dev), ref)  # the release library's plan
    with _native.ab_library():  # the Bluestein threshold is an A/B knob
        monkeypatch.setenv("ADMM_BLUE_MIN", "0")
        e_direct = rel(solve(x, k, 0.01, 0.02, False, 15, cuda_dev), ref)
        monkeypatch.setenv("ADMM_BLUE_MIN", "11")
        e_blue = rel(solve(x, k, 0.01, 0.02, False, 15, cuda_dev), ref)
    assert e_blue0 <= TOL_REF64
    print(shape, f"vs fp64 oracle: bluestein {e_blue:.3e}, direct {e_direct:.3e}")
    assert e_blue <= TOL_REF64
    assert e_blue <= 2 * e_direct + 1e-6


@pytest.mark.parametrize("shape,iso", [((2, 3, 321, 481), False), ((1, 3, 100, 75), True), ((2, 1, 7, 9), False)])
def test_fused_step_is_bit_identical(cuda_dev, shape, iso, monkeypatch):
    """The inference path runs the per-pixel step inside the row transform of r
    (k_grow_fwd_step); the separate kernels (ADMM_GSTEP_FUSE=0) give the same bits."""
    from admmtor.synth import blurred_batch, make_psf
    k = make_psf("gauss:1.5", 5)
    x = blurred_batch(*shape, k, seed=3)
    from admmtor import _native
    monkeypatch.setenv("ADMM_GSTEP_FUSE", "0")
    with _native.ab_library():  # the separate kernels: an A/B knob
        a = solve(x, k, 0.01, 0.02, iso, 12, cuda_dev)
    b = solve(x, k, 0.01, 0.02, iso, 12, cuda_dev)  # the release library: fused
    assert torch.equal(a, b)


def test_generic_psf_transpose(cuda_dev):
    import ctypes
    from admmtor import _native
    from admmtor.synth import make_psf
    from oracle.admm_oracle import apply_psf_transpose
    x = torch.rand(2, 3, 45, 30, generator=torch.Generator().manual_seed(3))
    k = make_psf("motion", 7)
    xd, kd = x.to(cuda_dev), k.to(cuda_dev)
    d = _native.desc(2, 3, 45, 30, 7, False, 1)
    ws = torch.empty(_native.workspace_size(d), dtype=torch.uint8, device=cuda_dev)
    got = torch.empty_like(xd)
    _native.check(_native.load().admm_tv_psf_transpose(
        ctypes.byref(d), xd.data_ptr(), kd.data_ptr(), got.data_ptr(), ws.data_ptr(), ws.numel(),
        torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    ref = apply_psf_transpose(x.double(), k.double())
    assert rel(got.cpu(), ref) <= 1e-6


@pytest.mark.parametrize("shape,iso,it,psf", [((2, 2, 15, 17), False, 6, None), ((2, 2, 15, 17), True, 6, None),
                                              ((1, 3, 24, 36), False, 4, ("gauss:1.0", 5)),
                                              ((2, 1, 20, 12), True, 5, ("motion", 5))])
def test_generic_grads_vs_oracle(cuda_dev, shape, iso, it, psf):
    from admmtor.synth import blurred_batch, make_psf
    from test_gpu_grad import hip_grads, oracle_grads
    from oracle.admm_oracle import kink_margins
    k = make_psf(*psf) if psf else None
    x = blurred_batch(*shape, k if k is not None else torch.empty(0), seed=7)
    cot = torch.randn(x.shape, generator=torch.Generator().manual_seed(2))
    o1, gx1, gl1, gr1 = hip_grads(x, k, 0.03, 0.07, iso, it, cot, cuda_dev)
    o2, gx2, gl2, gr2 = oracle_grads(x, k, 0.03, 0.07, iso, it, cot)
    margins = kink_margins(x.double(), 0.03, 0.07, k.double() if k is not None else torch.empty(0, dtype=torch.float64),
                           it) if not iso else None
    e = (rel(o1, o2), rel(gx1, gx2), rel(gl1, gl2), rel(gr1, gr2))
    print(shape, "iso" if iso else "aniso", it, psf, "out/gx/glam/grho rel:", e)
    tol = 1e-3 if psf else 1e-4
    assert e[0] <= TOL_REF64
    near_kink = margins is not None and float(margins.min()) < 1e-5
    if not near_kink:
        assert e[1] <= tol and e[2] <= tol and e[3] <= tol


@pytest.mark.parametrize("iso,it,psf,shape", [(False, 6, ("gauss:1.0", 5), (2, 2, 15, 17)),
                                              (True, 5, ("motion", 5), (1, 3, 24, 36)),
                                              (False, 8, ("random", 4), (1, 2, 30, 45))])
def test_generic_psf_gradient_vs_oracle(cuda_dev, iso, it, psf, shape):
    """dL/dPSF on the generic path vs the fp64 oracle's autograd (gate as in test_gpu_grad:
    max(1e-3, the reference op sequence's own fp32 error))."""
    from admmtor.synth import blurred_batch, make_psf
    from oracle.admm_oracle import solve_spatial
    from test_gpu_grad import hip_grads_psf
    k = make_psf(*psf)
    x = blurred_batch(*shape, k, seed=5)
    cot = torch.randn(x.shape, generator=torch.Generator().manual_seed(4))
    _, gx1, gl1, gr1, gk1 = hip_grads_psf(x, k, 0.02, 0.05, iso, it, cot, cuda_dev)
    ref = {}
    for dt in (torch.float64, torch.float32):
        xd = x.to(dt).requires_grad_(True)
        kd = k.to(dt).requires_grad_(True)
        ld = torch.tensor([0.02], dtype=dt, requires_grad=True)
        rd = torch.tensor([0.05], dtype=dt, requires_grad=True)
        o = solve_spatial(xd, ld, rd, kd, iso, it)
        ref[dt] = torch.autograd.grad(o, (xd, ld, rd, kd), cot.to(dt), allow_unused=True)
    g64, g32 = ref[torch.float64], ref[torch.float32]
    ours = (rel(gx1, g64[0]), rel(gl1, g64[1]), rel(gr1, g64[2]), rel(gk1, g64[3]))
    floor = (rel(g32[0], g64[0]), rel(g32[1], g64[1]), rel(g32[2], g64[2]), rel(g32[3], g64[3]))
    print("generic psf grad", shape, iso, it, psf, "ours (x, lam, rho, psf)", ours, "fp32 floor", floor)
    for e, f in zip(ours, floor):
        assert e <= max(1e-3, 2 * f)


def test_long_lines_fp64_and_two_stream_fallback(cuda_dev):
    """fp64 lines beyond 5,120 points (global line buffers in the double kernels) vs the fp64 oracle
    at the fp64 gate, and an aniso batch with long lines (its solve stays on one stream: the halves
    would share the scratch slots) equal to its one-stream result bit for bit."""
    import os
    from admmtor.eops.deconv import fft_admm_tv
    from admmtor.synth import blurred_batch, make_psf
    k = make_psf("gauss:1.5", 7)
    x = blurred_batch(1, 2, 8, 6000, k, seed=4).double()
    out = fft_admm_tv(x.to(cuda_dev), 0.01, 0.02, k.double().to(cuda_dev), True, 5)
    assert out.dtype == torch.float64
    e = rel(out, oracle(x, k, 0.01, 0.02, True, 5))
    print("fp64 8x6000 iso:", e)
    assert e <= 1e-12
    x = blurred_batch(3, 1, 8, 11000, k, seed=5)
    a = solve(x, k, 0.01, 0.02, False, 4, cuda_dev)
    os.environ["ADMM_GEN_STREAMS"] = "1"
    try:
        b = solve(x, k, 0.01, 0.02, False, 4, cuda_dev)
    finally:
        del os.environ["ADMM_GEN_STREAMS"]
    assert torch.equal(a, b)
    assert rel(a, oracle(x, k, 0.01, 0.02, False, 4)) <= TOL_REF64

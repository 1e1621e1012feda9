"""The fused two-pass iteration at smooth sizes (mixed-radix register transforms, mixed_kernels.hpp;
admm_tv_supported == 3): HD, 720p, VGA and other 2^a 3^b 5^c frames, and power-of-two widths / heights
paired with a smooth other side.  The reference runs every H, W through the same op sequence
(deconv.py:42,104-106); here each case is checked against the fp64 oracle (north-star gate 1e-5) and
against the generic kernels' solve of the same input (ADMM_MIXED=0: the same algorithm with other
roundings, so the two agree to fp32 noise)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

TOL_REF64 = 1e-5


def rel(a, b):
    a, b = a.double().reshape(-1), b.double().reshape(-1)
    return ((a - b).norm() / b.norm()).item()


def solve(x, k, iso, it, dev, lam=0.01, rho=0.02):
    from admmtor.eops.deconv import fft_admm_tv
    kk = k.to(dev) if k is not None else torch.empty(0, device=dev)
    out = fft_admm_tv(x.to(dev), lam, rho, kk, iso, it)
    torch.cuda.synchronize()
    return out.cpu()


def oracle(x, k, iso, it, lam=0.01, rho=0.02):
    from oracle.admm_oracle import solve_fourier
    kk = k.double() if k is not None else torch.empty(0, dtype=torch.float64)
    return solve_fourier(x.double(), lam, rho, kk, iso, it)


def test_supported_codes():
    from admmtor import _native
    lib = _native.load()
    assert [lib.admm_tv_supported(*hw) for hw in ((1080, 1920), (720, 1280), (480, 640), (2160, 1024), (1024, 960),
                                                  (540, 1080), (360, 720), (240, 480), (2160, 3840), (4096, 4096),
                                                  (600, 800), (768, 1024), (1200, 1600), (1536, 2048), (1080, 1440),
                                                  (1440, 2560), (800, 800))] == [3] * 17
    assert [lib.admm_tv_supported(*hw) for hw in ((1024, 1024), (4096, 2048))] == [1] * 2
    assert [lib.admm_tv_supported(*hw) for hw in ((1080, 1921), (1080, 7680), (1000, 1920), (509, 509))] == [2] * 4


CASES = [
    # (B, C, H, W), psf, iso, iterations
    ((1, 3, 1080, 1920), ("gauss:1.5", 9), False, 20),   # HD frame: rows 960 = 8*15*8 (2-wave groups), cols 9*15*8
    ((2, 3, 720, 1280), ("motion", 15), False, 15),      # 720p: rows 640 = 5*16*8 (2-wave groups), cols 9*16*5
    ((2, 2, 480, 640), ("gauss:1.5", 7), True, 20),      # VGA, iso: rows 320 = 16*4*5, cols 15*16*2
    ((3, 1, 240, 480), None, True, 12),                  # 32-lane row groups (30 pixel lanes), no PSF
    ((1, 2, 360, 720), ("motion", 9), False, 10),        # 45 active pixel lanes of 64
    ((1, 1, 540, 1080), ("gauss:2", 9), True, 10),       # 9 pixel pairs per lane, 12-point spectrum edge
    ((1, 1, 2160, 1024), ("gauss:2", 11), False, 6),     # power-of-two rows, 2160-point columns (9*16*15)
    ((2, 1, 1024, 960), ("gauss:1.5", 9), False, 8),     # power-of-two columns, 480-point rows
    ((1, 2, 960, 512), None, True, 8),                   # 960-point columns (15*16*4)
    ((1, 1, 1080, 1920), ("random", 5), True, 3),        # iso, non-centrosymmetric PSF, 3 iterations
    ((2, 1, 720, 1280), None, False, 1),                 # one iteration
    ((1, 1, 2160, 3840), ("gauss:2", 11), False, 5),     # 4K UHD: 4-wave row groups (1920 = 8*15*16), 2160 columns
    ((1, 1, 4096, 4096), ("gauss:1.5", 9), True, 4),     # 4096-wide power-of-two rows: 4-wave groups (8*4*8*8)
    ((1, 2, 1080, 2048), None, False, 6),                # 2048-wide rows as 2-wave groups beside 1080 columns
    ((2, 2, 600, 800), ("motion", 9), False, 10),        # SVGA: rows 400 = 10*5*8, cols 6*10*10
    ((1, 2, 768, 1024), ("gauss:1.5", 9), True, 8),      # XGA: power-of-two rows, 768-point columns (6*2*8*8)
    ((1, 1, 1200, 1600), ("gauss:2", 11), False, 6),     # UXGA: 4-wave row groups, 5 pixel pairs per lane
    ((1, 1, 1536, 2048), None, False, 4),                # QXGA: 1536-point columns, 4 per block
    ((1, 1, 1080, 1440), ("random", 5), True, 5),        # rows 720 = 12*10*6 over 120 of 128 lanes
    ((1, 1, 1440, 2560), ("gauss:1.5", 9), False, 4),    # QHD: rows 1280 = 8*4*8*5, cols 12*8*15
    ((1, 1, 800, 800), ("motion", 7), True, 6),          # 800-point columns beside 400-point rows
]


@pytest.mark.parametrize("shape,psf,iso,it", CASES)
def test_mixed_vs_oracle_and_generic(cuda_dev, monkeypatch, shape, psf, iso, it):
    from admmtor import _native
    from admmtor.synth import blurred_batch, make_psf
    assert _native.load().admm_tv_supported(shape[2], shape[3]) == 3
    k = make_psf(*psf) if psf else None
    x = blurred_batch(*shape, k if k is not None else torch.empty(0), seed=sum(shape) + it)
    got = solve(x, k, iso, it, cuda_dev)
    ref = oracle(x, k, iso, it)
    monkeypatch.setenv("ADMM_MIXED", "0")  # the same solve on the generic kernels (an A/B knob)
    with _native.ab_library():
        gen = solve(x, k, iso, it, cuda_dev)
    e_ref, e_gen, e_gen_ref = rel(got, ref), rel(got, gen), rel(gen, ref)
    print(shape, psf, "iso" if iso else "aniso", it, f"mixed vs fp64 oracle {e_ref:.2e}, vs generic {e_gen:.2e} "
          f"(generic vs oracle {e_gen_ref:.2e})")
    assert e_ref <= TOL_REF64
    assert e_gen <= 2 * max(e_gen_ref, 1e-7) + e_ref


def test_mixed_planes_independent(cuda_dev):
    """aniso planes are independent: a plane solved inside a batch equals the plane solved alone, bit
    for bit (no cross-plane state in the strips / column blocks)."""
    from admmtor.synth import blurred_batch, make_psf
    k = make_psf("gauss:1.5", 9)
    x = blurred_batch(3, 2, 720, 1280, k, seed=5)
    full = solve(x, k, False, 10, cuda_dev)
    one = solve(x[1:2, 1:2].contiguous(), k, False, 10, cuda_dev)
    assert torch.equal(full[1:2, 1:2], one)


TRAIN_CASES = [
    # (B, C, H, W), psf (fixed), iso, iterations
    ((1, 2, 240, 480), None, True, 8),                 # 240-point rows over a 32-lane group
    ((1, 1, 360, 720), ("gauss:1.5", 5), False, 10),   # 360-point rows, a fixed PSF (x^_in = H_t^T b^)
    ((2, 1, 360, 800), None, True, 6),                 # 400-point rows, two planes coupled by the iso norm
    ((1, 1, 240, 1920), ("motion", 5), False, 6),      # HD rows: a wide row group of 2 waves (960 = 8 15 8)
    ((1, 1, 256, 1280), None, True, 6),                # 720p rows (wide, 640 = 10 8 8) beside power-of-two columns
    # the training row plans (MRowT) at every length where a training kernel takes one (§7c rule)
    ((1, 1, 128, 640), None, True, 6),                 # 320 (VGA rows): every pass on the 1-wave training plan
    ((1, 2, 128, 960), ("motion", 5), False, 6),       # 480: reverse passes on the 2-wave training plan
    ((1, 1, 128, 1080), None, True, 6),                # 540 (4-column blocks: N = 540)
    ((1, 1, 128, 1600), None, True, 5),                # 800: forward and reverse on the 4-wave training plan
    ((1, 1, 64, 2560), ("gauss:1.5", 5), False, 5),    # 1280 (QHD rows): both on the training plan
    ((1, 1, 240, 1440), None, False, 5),               # 720: both on the inference plan (no 4-wave widening)
]


@pytest.mark.parametrize("shape,psf,iso,it", TRAIN_CASES)
def test_mixed_training_gradients_vs_oracle(cuda_dev, monkeypatch, shape, psf, iso, it):
    """Training at smooth sizes runs on the mixed kernels (forward with history: k_pass_a_m / k_iso_norm_m
    with HIST; backward: the inference column pass + k_bwd_pass_a_m / k_bwd_iso_q_m): output, x, lambda
    and rho gradients against the fp64 oracle's autograd (deconv.py:103-115), and against the same training
    step on the generic kernels (the A/B build, ADMM_MIXED=0)."""
    from admmtor import _native
    from admmtor.eops.deconv import fft_admm_tv
    from admmtor.synth import blurred_batch, make_psf
    from oracle.admm_oracle import solve_fourier
    assert _native.load().admm_tv_supported(shape[2], shape[3]) == 3
    k = make_psf(*psf) if psf else None
    x = blurred_batch(*shape, k if k is not None else torch.empty(0), seed=sum(shape) + 3)
    cot = torch.randn(x.shape, generator=torch.Generator().manual_seed(1))

    def hip():
        xg = x.to(cuda_dev).requires_grad_(True)
        lam = torch.tensor([0.03], device=cuda_dev, requires_grad=True)
        rho = torch.tensor([0.05], device=cuda_dev, requires_grad=True)
        kk = k.to(cuda_dev) if k is not None else torch.empty(0, device=cuda_dev)
        out = fft_admm_tv(xg, lam, rho, kk, iso, it)
        g = torch.autograd.grad(out, (xg, lam, rho), cot.to(cuda_dev))
        torch.cuda.synchronize()
        return [out.detach().cpu()] + [v.cpu() for v in g]
    got = hip()
    monkeypatch.setenv("ADMM_MIXED", "0")
    with _native.ab_library():
        gen = hip()
    xr = x.double().requires_grad_(True)
    lr = torch.tensor([0.03], dtype=torch.float64, requires_grad=True)
    rr = torch.tensor([0.05], dtype=torch.float64, requires_grad=True)
    kr = k.double() if k is not None else torch.empty(0, dtype=torch.float64)
    ref = solve_fourier(xr, lr, rr, kr, iso, it)
    want = [ref.detach()] + list(torch.autograd.grad(ref, (xr, lr, rr), cot.double()))
    e = [rel(a, b) for a, b in zip(got, want)]
    eg = [rel(a, b) for a, b in zip(gen, want)]
    # the rho gradient is a sum of large cancelling terms (and, aniso, of shrink masks that one fp32 ulp
    # can flip): one fp32 evaluation lands 1e-7..3e-4 from fp64 depending on the rounding pattern
    # (test_gpu_sharded._rho_grad_noise).  Its gate is 1e-4 or, where this input is that sensitive, 3x the
    # spread of the reference formulation's own fp32 evaluation on it (the oracle in fp32, on the CPU) --
    # never a term measured on a HIP path (the generic kernels' error is printed only)
    lr32 = torch.tensor([0.03], requires_grad=True)
    rr32 = torch.tensor([0.05], requires_grad=True)
    ref32 = solve_fourier(x, lr32, rr32, k if k is not None else torch.empty(0), iso, it)
    noise32 = rel(torch.autograd.grad(ref32, rr32, cot)[0], want[3])
    rho_gate = max(1e-4, 3 * noise32)
    print(shape, psf, "iso" if iso else "aniso", it, "mixed (out, x, lam, rho):", ["%.2e" % v for v in e],
          "generic:", ["%.2e" % v for v in eg], "oracle fp32 rho: %.2e (rho gate %.2e)" % (noise32, rho_gate))
    assert e[0] <= TOL_REF64 and max(e[1:3]) <= 1e-4 and e[3] <= rho_gate
    # the training solve ran on the mixed kernels: the library's own answer for this descriptor (not an
    # inference from rounding differences)
    assert _native.path(_native.desc(*shape, k.shape[-1] if k is not None else 0, iso, it), train=True) \
        == "fused mixed-radix"


def test_mixed_size_psf_gradient_uses_generic_history(cuda_dev):
    """A PSF gradient at a smooth size keeps the generic training path (its column-spectrum history):
    x, lambda, rho and PSF gradients against the fp64 oracle's autograd."""
    from admmtor.eops.deconv import fft_admm_tv
    from admmtor.synth import blurred_batch, make_psf
    from oracle.admm_oracle import solve_spatial  # the reference's op sequence: autograd reaches the PSF
    k = make_psf("motion", 5)
    x = blurred_batch(1, 1, 240, 480, k, seed=9)
    cot = torch.randn(x.shape, generator=torch.Generator().manual_seed(2))
    xg = x.to(cuda_dev).requires_grad_(True)
    lam = torch.tensor([0.03], device=cuda_dev, requires_grad=True)
    rho = torch.tensor([0.05], device=cuda_dev, requires_grad=True)
    kg = k.to(cuda_dev).requires_grad_(True)
    out = fft_admm_tv(xg, lam, rho, kg, False, 6)
    got = [out.detach().cpu()] + [v.cpu() for v in torch.autograd.grad(out, (xg, lam, rho, kg), cot.to(cuda_dev))]
    xr = x.double().requires_grad_(True)
    lr = torch.tensor([0.03], dtype=torch.float64, requires_grad=True)
    rr = torch.tensor([0.05], dtype=torch.float64, requires_grad=True)
    kr = k.double().requires_grad_(True)
    ref = solve_spatial(xr, lr, rr, kr, False, 6)
    want = [ref.detach()] + list(torch.autograd.grad(ref, (xr, lr, rr, kr), cot.double()))
    e = [rel(a, b) for a, b in zip(got, want)]
    print("240x480 PSF gradient:", ["%.2e" % v for v in e])
    assert e[0] <= TOL_REF64 and max(e[1:]) <= 1e-3

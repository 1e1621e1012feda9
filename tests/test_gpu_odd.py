"""The two-launch iteration at odd row lengths (odd_kernels.hpp; admm_tv_supported == 4):
the generic column pass, then ONE row pass -- inverse rows, the step, forward rows, in one wave per strip
of six rows -- instead of the generic path's three launches.  BSD's 481-point rows (13 * 37, prime-factor
transforms).  The reference runs every H, W through one op sequence (deconv.py:42,104-106); each case here
is checked against the fp64 oracle (north-star gate 1e-5) and against the generic kernels' solve of the
same input (the A/B build with ADMM_ODD=0: the same algorithm with other roundings)."""
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


def test_odd_path_codes():
    """The size class and the path each entry point takes (admm_tv_path, host-only)."""
    from admmtor import _native
    lib = _native.load()
    assert [lib.admm_tv_supported(*hw) for hw in ((321, 481), (1, 481), (4096, 481), (17, 481))] == [4] * 4
    assert [lib.admm_tv_supported(*hw) for hw in ((481, 321), (481, 1), (481, 17))] == [4] * 3  # transposed
    assert [lib.admm_tv_supported(*hw) for hw in ((509, 509), (1080, 1921), (321, 321))] == [2] * 3
    assert lib.admm_tv_supported(481, 481) == 4  # 481-point rows (the landscape path itself)
    assert _native.path(_native.desc(1, 3, 481, 321, 9, False, 10)) == "fused odd-length"
    assert _native.path(_native.desc(1, 3, 481, 321, 9, False, 10), train=True) == "generic"
    d = _native.desc(2, 3, 321, 481, 9, False, 10)
    assert _native.path(d) == "fused odd-length" and _native.path(d, train=True) == "generic"
    assert _native.path(_native.desc(2, 3, 321, 481, 9, True, 10)) == "generic"  # iso: the generic kernels


CASES = [
    # (B, C, H, W), psf, iterations
    ((2, 3, 321, 481), ("gauss:1.5", 9), 30),   # BSD landscape frames: 53 strips of 6 rows + one of 3
    ((1, 2, 480, 481), ("motion", 9), 12),      # even H, 80 full strips; non-centrosymmetric PSF
    ((1, 1, 17, 481), ("gauss:1.0", 5), 15),    # strips of 6, 6, 5 rows (an odd last strip)
    ((3, 1, 7, 481), None, 10),                 # one strip of 6 + one of 1; no PSF
    ((1, 1, 2, 481), None, 8),                  # one strip of 2 rows: its halo rows are its own rows
    ((2, 1, 1, 481), None, 6),                  # a one-row image: every halo row is the row itself
    ((1, 1, 321, 481), ("random", 7), 1),       # one iteration (the first pass A only)
    ((1, 2, 1000, 481), ("gauss:2", 11), 6),    # 1000 = 2^3 5^3 columns (LDS column pass, not the MFMA one)
]


@pytest.mark.parametrize("shape,psf,it", CASES)
def test_odd_vs_oracle_and_generic(cuda_dev, monkeypatch, shape, psf, it):
    from admmtor import _native
    from admmtor.synth import blurred_batch, make_psf
    assert _native.path(_native.desc(*shape, 0, False, it)) == "fused odd-length"
    k = make_psf(*psf) if psf else None
    x = blurred_batch(*shape, k if k is not None else torch.empty(0), seed=sum(shape) + it)
    got = solve(x, k, False, it, cuda_dev)
    ref = oracle(x, k, False, it)
    monkeypatch.setenv("ADMM_ODD", "0")  # the same solve on the generic kernels (an A/B knob)
    with _native.ab_library() as ab:
        assert ab.admm_tv_supported(shape[2], shape[3]) == 2
        gen = solve(x, k, False, it, cuda_dev)
    e_ref, e_gen, e_gen_ref = rel(got, ref), rel(got, gen), rel(gen, ref)
    print(shape, psf, it, f"odd vs fp64 oracle {e_ref:.2e}, vs generic {e_gen:.2e} (generic vs oracle {e_gen_ref:.2e})")
    assert e_ref <= TOL_REF64
    assert e_gen <= 2 * max(e_gen_ref, 1e-7) + e_ref


def test_odd_planes_independent_and_streams(cuda_dev, monkeypatch):
    """aniso planes are independent: a plane solved inside a batch matches the plane solved alone to the
    fp32 level (1e-5: the solve's setup and last row transforms, generic_kernels.hpp, pair real rows over the
    whole batch, so with an odd H a plane's last row meets another partner than alone, and that rounding
    difference grows through the shrink like any other -- measured 3.5e-6 after 10 iterations, the level of
    either solve against the fp64 oracle), and the two-stream plane split
    equals one stream bit for bit (the parts split at even row counts; the row pass's strips never straddle
    planes)."""
    from admmtor.synth import blurred_batch, make_psf
    k = make_psf("gauss:1.5", 9)
    x = blurred_batch(3, 3, 321, 481, k, seed=5)
    full = solve(x, k, False, 10, cuda_dev)
    for b, c in ((1, 1), (1, 2), (2, 2)):
        one = solve(x[b:b + 1, c:c + 1].contiguous(), k, False, 10, cuda_dev)
        assert rel(full[b:b + 1, c:c + 1], one) <= TOL_REF64, (b, c)
    monkeypatch.setenv("ADMM_GEN_STREAMS", "1")
    assert torch.equal(solve(x, k, False, 10, cuda_dev), full)


def test_odd_graph_capture(cuda_dev):
    """The odd-length solve enqueues only asynchronous work: captured in a HIP graph and replayed, it gives
    the eager result bit for bit."""
    from admmtor.eops.deconv import fft_admm_tv
    from admmtor.synth import blurred_batch, make_psf
    k = make_psf("gauss:1.5", 9).to(cuda_dev)
    static_x = blurred_batch(2, 3, 321, 481, k.cpu(), seed=7).to(cuda_dev)
    eager = fft_admm_tv(static_x, 0.01, 0.02, k, False, 8)
    s = torch.cuda.Stream(cuda_dev)
    s.wait_stream(torch.cuda.current_stream(cuda_dev))
    with torch.cuda.stream(s):
        fft_admm_tv(static_x, 0.01, 0.02, k, False, 8)
    torch.cuda.current_stream(cuda_dev).wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        static_out = fft_admm_tv(static_x, 0.01, 0.02, k, False, 8)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(static_out, eager)


def test_odd_size_iso_and_training_keep_generic(cuda_dev):
    """iso and training at an odd size run on the generic kernels (admm_tv_path): still against the fp64
    oracle, including the gradients of a short training solve."""
    from admmtor.eops.deconv import fft_admm_tv
    from admmtor.synth import blurred_batch, make_psf
    from oracle.admm_oracle import solve_fourier
    k = make_psf("gauss:1.5", 7)
    x = blurred_batch(1, 2, 41, 481, k, seed=3)
    assert rel(solve(x, k, True, 10, cuda_dev), oracle(x, k, True, 10)) <= TOL_REF64
    xg = x.to(cuda_dev).requires_grad_(True)
    lam = torch.tensor([0.02], device=cuda_dev, requires_grad=True)
    out = fft_admm_tv(xg, lam, 0.05, k.to(cuda_dev), False, 6)
    cot = torch.randn(x.shape, generator=torch.Generator().manual_seed(4))
    got = torch.autograd.grad(out, (xg, lam), cot.to(cuda_dev))
    xr = x.double().requires_grad_(True)
    lr = torch.tensor([0.02], dtype=torch.float64, requires_grad=True)
    ref = solve_fourier(xr, lr, 0.05, k.double(), False, 6)
    want = torch.autograd.grad(ref, (xr, lr), cot.double())
    assert rel(out.detach().cpu(), ref.detach()) <= TOL_REF64
    assert rel(got[0].cpu(), want[0]) <= 1e-3 and rel(got[1].cpu(), want[1]) <= 1e-3


@pytest.mark.parametrize("shape,psf,it", [((2, 3, 481, 321), ("gauss:1.5", 9), 20), ((1, 2, 481, 17), ("motion", 5), 10),
                                          ((1, 1, 481, 1), None, 6)])
def test_odd_transposed_orientation(cuda_dev, monkeypatch, shape, psf, it):
    """A portrait odd-width image (H = 481, the BSD portrait frames) runs as its transpose on the odd-length
    iteration (Layout::tr): the solve commutes with transposing the image and the PSF (Dx and Dy trade
    places), so the result is the landscape solve of the transposed input, transposed back -- bit for bit --
    and within the gate of the fp64 oracle and of the generic kernels."""
    from admmtor import _native
    from admmtor.synth import blurred_batch, make_psf
    k = make_psf(*psf) if psf else None
    x = blurred_batch(*shape, k if k is not None else torch.empty(0), seed=sum(shape) + it)
    got = solve(x, k, False, it, cuda_dev)
    kt = k.transpose(-1, -2).contiguous() if k is not None else None
    land = solve(x.transpose(-1, -2).contiguous(), kt, False, it, cuda_dev)
    assert torch.equal(got, land.transpose(-1, -2))
    ref = oracle(x, k, False, it)
    monkeypatch.setenv("ADMM_ODD", "0")
    with _native.ab_library():
        gen = solve(x, k, False, it, cuda_dev)
    e_ref, e_gen, e_gen_ref = rel(got, ref), rel(got, gen), rel(gen, ref)
    print(shape, psf, it, f"transposed odd vs fp64 oracle {e_ref:.2e}, vs generic {e_gen:.2e} (generic {e_gen_ref:.2e})")
    assert e_ref <= TOL_REF64 and e_gen <= 2 * max(e_gen_ref, 1e-7) + e_ref

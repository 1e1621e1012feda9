"""Second-order autograd through the HIP solver vs the reference's own fp64 second-order gradients.

Objective (tests/golden/make_golden_second_order.py, run on deconv.py:35-117 in fp64):
``g = d<cot, fft_admm_tv(x, lam, rho, psf)>/d(x, lam, rho, psf)`` with ``create_graph=True``,
``P = <sx, g_x> + sl g_lam + sr g_rho + <sk, g_psf>``, then ``dP/d(cot, x, lam, rho, psf)``.
On the device: the first-order gradient is the native ``admm_tv_backward`` (fp64 kernels for fp64
inputs), the second-order terms come from the backward op's autograd formula (admmtor._unrolled).
Gates: fp64 1e-9 (both sides fp64; the reference is exact to ~1e-14 on these sizes), fp32 2e-3
(second-order terms of an fp32 solve; the first-order fp32 gate of the suite is 1e-4).
"""
import pytest
import torch

from conftest import load_golden
from oracle.admm_oracle import rel_l2

pytestmark = pytest.mark.gpu

CASES = ["aniso_psf", "iso_psf", "aniso_nopsf"]


def _case(tag, dev, dt):
    g = load_golden("g12_second_order")
    d = {k.split("/", 1)[1]: torch.from_numpy(v) for k, v in g.items() if k.startswith(tag + "/")}
    B, C, H, W, k, kgrad, iso, maxit = (int(v) for v in d["meta"])
    lam0, rho0, sl, sr = (float(v) for v in d["scal"])
    T = lambda t: t.to(device=dev, dtype=dt)  # noqa: E731
    psf = T(d["psf"]) if "psf" in d else torch.empty(0, device=dev, dtype=dt)
    return d, T, psf, bool(kgrad), bool(iso), maxit, sl, sr


def _second_order(d, T, psf, kgrad, iso, maxit, sl, sr):
    from admmtor.eops.deconv import fft_admm_tv
    x = T(d["x"]).requires_grad_(True)
    lam = T(d["lam"]).requires_grad_(True)
    rho = T(d["rho"]).requires_grad_(True)
    cot = T(d["cot"]).requires_grad_(True)
    k = psf.clone().requires_grad_(kgrad)
    y = fft_admm_tv(x, lam, rho, k, iso, maxit)
    prims = [x, lam, rho] + ([k] if kgrad else [])
    g = torch.autograd.grad(y, prims, cot, create_graph=True)
    pen = (T(d["sx"]) * g[0]).sum() + sl * g[1].sum() + sr * g[2].sum()
    if kgrad:
        pen = pen + (T(d["sk"]) * g[3]).sum()
    h = torch.autograd.grad(pen, [cot] + prims)
    return y, g, h


@pytest.mark.parametrize("tag", CASES)
@pytest.mark.parametrize("dt,gate", [(torch.float64, 1e-9), (torch.float32, 2e-3)])
def test_second_order_vs_reference(cuda_dev, tag, dt, gate):
    d, T, psf, kgrad, iso, maxit, sl, sr = _case(tag, cuda_dev, dt)
    y, g, h = _second_order(d, T, psf, kgrad, iso, maxit, sl, sr)
    first = 1e-12 if dt == torch.float64 else 1e-4
    assert rel_l2(y.detach().cpu(), d["out"]) <= first
    assert rel_l2(g[0].detach().cpu(), d["gx"]) <= first * 10
    keys = ["hcot", "hx", "hlam", "hrho"] + (["hpsf"] if kgrad else [])
    errs = {key: rel_l2(v.detach().cpu(), d[key]) for key, v in zip(keys, h)}
    print(tag, dt, {k: f"{v:.2e}" for k, v in errs.items()})
    assert all(v <= gate for v in errs.values()), errs


def test_hessian_vector_product_module(cuda_dev):
    """A gradient penalty on ADMMDeconv's parameters (lambda, rho): the double backward reaches the
    module parameters and agrees with central finite differences of the fp64 first-order gradient."""
    from admmtor.eops.deconv import fft_admm_tv
    d, T, psf, kgrad, iso, maxit, sl, sr = _case("aniso_nopsf", cuda_dev, torch.float64)
    x = T(d["x"])
    cot = T(d["cot"])

    def grad_lam(rho_v):
        lam = T(d["lam"]).requires_grad_(True)
        rho = torch.tensor([rho_v], device=cuda_dev, dtype=torch.float64)
        y = fft_admm_tv(x, lam, rho, psf, iso, maxit)
        return torch.autograd.grad(y, lam, cot)[0]

    lam = T(d["lam"]).requires_grad_(True)
    rho = T(d["rho"]).requires_grad_(True)
    y = fft_admm_tv(x, lam, rho, psf, iso, maxit)
    (gl,) = torch.autograd.grad(y, lam, cot, create_graph=True)
    (hlr,) = torch.autograd.grad(gl.sum(), rho)  # d^2 <cot, y> / d lam d rho
    r0, eps = float(d["rho"][0]), 1e-6
    fd = (grad_lam(r0 + eps) - grad_lam(r0 - eps)) / (2 * eps)
    assert abs(float(hlr) - float(fd)) <= 1e-5 * max(1.0, abs(float(fd))), (float(hlr), float(fd))


def test_grouped_modules_second_order(cuda_dev):
    """fft_admm_tv_grouped (two modules sharing x, one native call) differentiates twice like the two
    separate solves: a gradient penalty on x reaching both modules' lambda / rho."""
    from admmtor.eops.deconv import fft_admm_tv, fft_admm_tv_grouped
    from admmtor.synth import blurred_batch, make_psf
    psf = make_psf("motion", 5).to(cuda_dev)
    x0 = blurred_batch(2, 3, 32, 64, psf.cpu(), seed=4).to(cuda_dev)

    def run(grouped):
        x = x0.clone().requires_grad_(True)
        lams = [torch.tensor([0.02], device=cuda_dev, requires_grad=True),
                torch.tensor([0.01], device=cuda_dev, requires_grad=True)]
        rhos = [torch.tensor([0.05], device=cuda_dev, requires_grad=True),
                torch.tensor([0.04], device=cuda_dev, requires_grad=True)]
        if grouped:
            outs = fft_admm_tv_grouped(x, lams, rhos, psf, True, 6)
        else:
            outs = [fft_admm_tv(x, l, r, psf, True, 6) for l, r in zip(lams, rhos)]
        loss = sum((o * o).sum() for o in outs)
        (gx,) = torch.autograd.grad(loss, x, create_graph=True)
        pen = (gx * gx).sum()
        return torch.autograd.grad(pen, [x] + lams + rhos)

    hg, hs = run(True), run(False)
    for a, b in zip(hg, hs):
        assert rel_l2(a.detach().cpu(), b.detach().cpu()) <= 1e-5


def test_double_backward_memory_bounded(cuda_dev, monkeypatch):
    """A double backward at 4x3x512^2, 100 iterations (iso, learnable lambda / rho, the config-5 regime):
    the default formulation (the tangent solve along the seeds, reverse pass through checkpointed
    segments of ~sqrt(maxit) iterations; admmtor._unrolled._double_backward_tangent) against the unrolled
    create_graph formulation (ADMM_SO_UNROLLED=1, round 3's): same second-order gradients (fp64, 1e-9)
    at <= 1/5 of its peak memory above the first-order state."""
    from admmtor.eops.deconv import fft_admm_tv
    from admmtor.synth import blurred_batch
    x0 = blurred_batch(4, 3, 512, 512, torch.empty(0), seed=17).double().to(cuda_dev)
    cot = torch.randn(x0.shape, generator=torch.Generator().manual_seed(3), dtype=torch.float64).to(cuda_dev)
    k = torch.empty(0, device=cuda_dev, dtype=torch.float64)

    def run():
        x = x0.clone().requires_grad_(True)
        lam = torch.tensor([0.02], device=cuda_dev, dtype=torch.float64, requires_grad=True)
        rho = torch.tensor([0.05], device=cuda_dev, dtype=torch.float64, requires_grad=True)
        y = fft_admm_tv(x, lam, rho, k, True, 100)
        gx, gl = torch.autograd.grad(y, (x, lam), cot, create_graph=True)
        pen = gx.square().sum() + 10.0 * gl.sum()
        torch.cuda.synchronize()
        torch.cuda.reset_peak_memory_stats(cuda_dev)
        base = torch.cuda.memory_allocated(cuda_dev)
        h = torch.autograd.grad(pen, (x, lam, rho))
        torch.cuda.synchronize()
        peak = torch.cuda.max_memory_allocated(cuda_dev) - base
        return [t.detach().cpu() for t in h], peak

    h_t, peak_t = run()
    monkeypatch.setenv("ADMM_SO_UNROLLED", "1")
    h_u, peak_u = run()
    errs = [rel_l2(a, b) for a, b in zip(h_t, h_u)]
    print(f"double backward 4x3x512^2 x 100 it: peak {peak_t / 2**30:.2f} GiB (tangent, checkpointed) vs "
          f"{peak_u / 2**30:.2f} GiB (unrolled create_graph); rel diff {errs}")
    assert all(e <= 1e-9 for e in errs), errs
    assert peak_t * 5 <= peak_u


def test_second_order_through_a_nonlinear_loss(cuda_dev):
    """gout itself depends on x (L = sum y^2, so gout = 2 y): the double backward's local derivatives take
    gout as a leaf and the engine carries the path through gout -- every path counted once, as in the
    reference's plain autograd through the unrolled iteration (deconv.py:103-115; here
    admmtor._unrolled.unrolled_solve, fp64)."""
    from admmtor._unrolled import unrolled_solve
    from admmtor.eops.deconv import fft_admm_tv
    from admmtor.synth import blurred_batch, make_psf
    k = make_psf("motion", 5).double().to(cuda_dev)
    x0 = blurred_batch(2, 2, 32, 48, k.float().cpu(), seed=4).double().to(cuda_dev)
    res = []
    for solver in ("native", "unrolled"):
        x = x0.clone().requires_grad_(True)
        lam = torch.tensor([0.02], device=cuda_dev, dtype=torch.float64, requires_grad=True)
        rho = torch.tensor([0.05], device=cuda_dev, dtype=torch.float64, requires_grad=True)
        y = fft_admm_tv(x, lam, rho, k, False, 12) if solver == "native" else unrolled_solve(x, lam, rho, k, False, 12)
        gx, gr = torch.autograd.grad(y.square().sum(), (x, rho), create_graph=True)
        pen = gx.square().sum() + gr.sum()
        res.append([t.detach().cpu() for t in torch.autograd.grad(pen, (x, lam, rho))])
    errs = [rel_l2(a, b) for a, b in zip(*res)]
    print("second order through L = sum y^2 (native vs unrolled autograd):", errs)
    assert all(e <= 1e-9 for e in errs), errs

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

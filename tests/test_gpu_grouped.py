"""Grouped solves (desc.groups): G modules sharing the input, own lambda / rho,
one native pass sequence.  Must equal G separate fft_admm_tv calls: aniso bit for bit (every
plane's arithmetic is the same), iso to fp32 reassociation (the per-module norm sums planes in
different group sizes), gradients likewise (lambda / rho per module, x summed over modules).
Power-of-two sizes run the modules in every launch; smooth sizes (720x1280, 240x480) one module
after another inside one call (inference)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.double().cpu().reshape(-1), b.double().cpu().reshape(-1)
    return (torch.linalg.vector_norm(a - b) / torch.linalg.vector_norm(b)).item()


@pytest.mark.parametrize("iso,psf,shape", [(False, None, (2, 3, 64, 128)), (True, None, (4, 3, 64, 64)),
                                           (False, ("gauss:1.0", 5), (1, 3, 128, 64)),
                                           (True, ("motion", 7), (2, 2, 32, 256)),
                                           # smooth sizes (mixed-radix kernels): inference grouped in one
                                           # call, training one call per module
                                           (False, ("gauss:1.5", 9), (2, 3, 720, 1280)),
                                           (True, ("motion", 7), (2, 3, 240, 480))])
def test_grouped_equals_separate(cuda_dev, iso, psf, shape):
    from admmtor.eops.deconv import fft_admm_tv, fft_admm_tv_grouped
    from admmtor.synth import blurred_batch, make_psf
    k = make_psf(*psf).to(cuda_dev) if psf else torch.empty(0, device=cuda_dev)
    x = blurred_batch(*shape, k.cpu(), seed=3).to(cuda_dev)
    lams, rhos = [0.01, 0.03, 0.02], [0.02, 0.05, 0.08]
    cot = [torch.randn(shape, generator=torch.Generator().manual_seed(i)).to(cuda_dev) for i in range(3)]
    # forward, inference
    sep = [fft_admm_tv(x, l, r, k, iso, 12) for l, r in zip(lams, rhos)]
    grp = fft_admm_tv_grouped(x, lams, rhos, k, iso, 12)
    for a, b in zip(grp, sep):
        if iso:
            assert rel(a, b) <= 1e-6
        else:
            assert torch.equal(a, b)
    # gradients
    def run(grouped):
        xr = x.clone().requires_grad_(True)
        lt = [torch.tensor([v], device=cuda_dev, requires_grad=True) for v in lams]
        rt = [torch.tensor([v], device=cuda_dev, requires_grad=True) for v in rhos]
        outs = fft_admm_tv_grouped(xr, lt, rt, k, iso, 12) if grouped else \
            [fft_admm_tv(xr, l, r, k, iso, 12) for l, r in zip(lt, rt)]
        sum((o * c).sum() for o, c in zip(outs, cot)).backward()
        return xr.grad, torch.cat([t.grad for t in lt]), torch.cat([t.grad for t in rt])
    g_sep, g_grp = run(False), run(True)
    errs = [rel(a, b) for a, b in zip(g_grp, g_sep)]
    print("grouped vs separate grads (x, lam, rho):", errs)
    assert errs[0] <= 1e-6 and errs[1] <= 1e-5 and errs[2] <= 1e-5

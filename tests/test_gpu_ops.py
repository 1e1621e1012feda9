"""The dispatcher ops admm_hip::*  on the GPU.

* torch.library.opcheck on the three ops (schema, fake kernels vs the real ones, autograd
  registration, AOT dispatch);
* torch.compile(ADMMDeconv, fullgraph=True) -- the solver is one graph node, no graph break --
  with the aot_eager backend (this build ships no Triton code; inductor would generate it for the
  surrounding elementwise ops), same bits as eager, forward and backward;
* double backward (create_graph=True, then a backward of the gradient) runs through the backward
  op's own autograd formula; retain_graph=True gives the same gradients twice.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _inputs(dev, B=2, C=3, H=32, W=32, k=5, seed=0):
    from admmtor.synth import blurred_batch, make_psf
    psf = make_psf("motion", k) if k else torch.empty(0)
    x = blurred_batch(B, C, H, W, psf, seed=seed).to(dev)
    return x, psf.to(dev)


@pytest.mark.parametrize("iso", [False, True])
def test_opcheck_forward(cuda_dev, iso):
    import admmtor._ops  # noqa: F401
    x, k = _inputs(cuda_dev)
    lam = torch.tensor([0.01], device=cuda_dev)
    rho = torch.tensor([0.02], device=cuda_dev)
    torch.library.opcheck(torch.ops.admm_hip.fft_admm_tv_fwd.default, (x, lam, rho, k, iso, 7))


@pytest.mark.parametrize("iso,psf_grad", [(False, True), (True, False), (True, True)])
def test_opcheck_train_and_backward(cuda_dev, iso, psf_grad):
    import admmtor._ops  # noqa: F401
    x, k = _inputs(cuda_dev, H=16, W=32)
    x.requires_grad_(True)
    lam = torch.tensor([0.01], device=cuda_dev, requires_grad=True)
    rho = torch.tensor([0.02], device=cuda_dev, requires_grad=True)
    k = k.clone().requires_grad_(psf_grad)
    # the dynamic-shape AOT test needs a static history size; the other checks run
    torch.library.opcheck(torch.ops.admm_hip.fft_admm_tv_fwd_train.default, (x, lam, rho, k, iso, 5, psf_grad),
                          test_utils=("test_schema", "test_autograd_registration", "test_faketensor",
                                      "test_aot_dispatch_static"))
    out, hist = torch.ops.admm_hip.fft_admm_tv_fwd_train(x.detach(), lam.detach(), rho.detach(), k.detach(),
                                                          iso, 5, psf_grad)
    g = torch.randn_like(out)
    torch.library.opcheck(torch.ops.admm_hip.fft_admm_tv_bwd.default,
                          (g, x.detach(), lam.detach(), rho.detach(), k.detach(), hist, iso, 5, psf_grad,
                           True, True, psf_grad))


@pytest.mark.parametrize("iso,kern", [(False, (3, 3)), (True, ())])
def test_torch_compile_fullgraph_matches_eager(cuda_dev, iso, kern):
    from admmtor.elayers.admmdeconv import ADMMDeconv
    torch.manual_seed(11)
    m = ADMMDeconv(kern, 12, iso=iso).to(cuda_dev)
    x, _ = _inputs(cuda_dev, k=0, seed=3)
    x1 = x.clone().requires_grad_(True)
    x2 = x.clone().requires_grad_(True)
    torch._dynamo.reset()
    explain = torch._dynamo.explain(m)(x1)
    assert explain.graph_break_count == 0 and explain.graph_count == 1, explain.break_reasons
    cm = torch.compile(m, backend="aot_eager", fullgraph=True)
    ye = m(x1)
    yc = cm(x2)
    assert torch.equal(ye, yc)
    g = torch.randn_like(ye)
    ge = torch.autograd.grad(ye, [x1] + [p for p in m.parameters()], g)
    gc = torch.autograd.grad(yc, [x2] + [p for p in m.parameters()], g)
    for a, b in zip(ge, gc):
        assert torch.equal(a, b)


def test_double_backward_through_the_op(cuda_dev):
    """The backward op has an autograd formula: a gradient penalty differentiates (values are checked
    against the reference's fp64 second-order gradients in tests/test_gpu_second_order.py)."""
    from admmtor.eops.deconv import fft_admm_tv
    x, k = _inputs(cuda_dev)
    x.requires_grad_(True)
    y = fft_admm_tv(x, 0.01, 0.02, k, True, 5)
    (gx,) = torch.autograd.grad(y.square().sum(), x, create_graph=True)
    gx.square().sum().backward()
    assert x.grad is not None and torch.isfinite(x.grad).all()


def test_retain_graph_second_backward_same(cuda_dev):
    from admmtor.eops.deconv import fft_admm_tv
    x, k = _inputs(cuda_dev)
    x.requires_grad_(True)
    lam = torch.tensor([0.01], device=cuda_dev, requires_grad=True)
    y = fft_admm_tv(x, lam, 0.02, k, False, 6).square().sum()
    g1 = torch.autograd.grad(y, (x, lam), retain_graph=True)
    g2 = torch.autograd.grad(y, (x, lam))
    for a, b in zip(g1, g2):
        assert torch.equal(a, b)

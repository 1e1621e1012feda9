"""Host-side boundary of the MI355X build (no GPU needed).

* the error classes fft_admm_tv raises match the reference's (tests/golden/errors.json,
  recorded by running the reference)
* host tensors are refused loudly: there is no CPU fallback of the product path
* ADMMDeconv keeps the reference's constructor, parameter/buffer names, shapes,
  registration order and seeded initial values (tests/golden/module_init.json)
"""
import json
import os

import pytest
import torch

from conftest import GOLDEN, golden_errors


def _cases():
    x4 = torch.rand(1, 1, 16, 16)
    return {
        "input_3d": lambda f: f(torch.rand(1, 16, 16), 0.01, 0.02, torch.empty(0), False, 2),
        "input_5d": lambda f: f(torch.rand(1, 1, 1, 16, 16), 0.01, 0.02, torch.empty(0), False, 2),
        "kernel_nonsquare": lambda f: f(x4, 0.01, 0.02, torch.rand(1, 1, 3, 5), False, 2),
        "kernel_dtype_mismatch": lambda f: f(x4, 0.01, 0.02, torch.rand(1, 1, 3, 3).double(), False, 2),
        "input_bf16": lambda f: f(x4.bfloat16(), 0.01, 0.02, torch.empty(0), False, 2),
        "input_fp16": lambda f: f(x4.half(), 0.01, 0.02, torch.empty(0), False, 2),
        "kernel_2ch": lambda f: f(torch.rand(1, 2, 16, 16), 0.01, 0.02, torch.rand(1, 2, 3, 3), False, 2),
        "kernel_2d": lambda f: f(x4, 0.01, 0.02, torch.rand(3, 3), False, 2),
    }


@pytest.mark.parametrize("case", sorted(_cases()))
def test_error_classes_match_reference(case):
    from admmtor.eops.deconv import fft_admm_tv
    expected = golden_errors()[case]
    assert expected is not None
    with pytest.raises(Exception) as ei:
        _cases()[case](fft_admm_tv)
    assert type(ei.value).__name__ == expected, (case, type(ei.value).__name__, str(ei.value))


def test_host_tensors_have_no_fallback():
    from admmtor.eops.deconv import fft_admm_tv
    with pytest.raises(RuntimeError, match="ROCm device"):
        fft_admm_tv(torch.rand(1, 1, 16, 16), 0.01, 0.02, torch.empty(0), False, 0)


def test_public_helpers_semantics():
    from admmtor.eops import deconv as d
    x = torch.tensor([[[[-2.0, -0.5, 0.0, 0.3, 1.5]]]])
    assert torch.equal(d.soft_thresh(x, 0.5), torch.tensor([[[[-1.5, -0.0, 0.0, 0.0, 1.0]]]]))
    assert torch.equal(d.hard_thresh(x, 0.5), torch.tensor([[[[-2.0, 0.0, 0.0, 0.0, 1.5]]]]))
    assert torch.equal(d.torch_abs2(torch.tensor([3.0 + 4.0j])), torch.tensor([25.0]))
    assert d.identity(x) is x
    y = torch.rand(2, 3, 4, 5)
    n = d.pixelnorm(y)
    assert n.shape == (4, 5) and torch.allclose(n, torch.sqrt((y * y).sum((0, 1)) + 1e-15))
    bt = d.block_thresh(y, torch.tensor([0.3]))
    assert torch.allclose(bt, torch.clamp_min(1 - 0.3 / (n + 1e-15), 0) * y)
    w = torch.ones(3, 1, 2, 2)
    assert d.conv_circular(y, w, (1, 0, 1, 0), 3).shape == y.shape


def test_admmdeconv_matches_reference_construction():
    from admmtor.elayers.admmdeconv import ADMMDeconv
    with open(os.path.join(GOLDEN, "module_init.json")) as f:
        cases = json.load(f)
    for i, c in enumerate(cases):
        kw = dict(c["kwargs"])
        kw["kern_size"] = tuple(kw["kern_size"])
        torch.manual_seed(100 + i)
        m = ADMMDeconv(**kw)
        sd = m.state_dict()
        assert list(sd.keys()) == c["keys"]
        assert [n for n, _ in m.named_parameters()] == c["params"]
        assert [n for n, _ in m.named_buffers()] == c["buffers"]
        for k, v in sd.items():
            assert list(v.shape) == c["shapes"][k]
            assert v.flatten().tolist() == pytest.approx(c["values"][k], abs=0, rel=0), k


def test_admmdeconv_loads_reference_style_checkpoint():
    from admmtor.elayers.admmdeconv import ADMMDeconv
    src = ADMMDeconv((3, 3), 5, iso=False)
    dst = ADMMDeconv((3, 3), 5, iso=False)
    dst.load_state_dict(src.state_dict())
    for k in ("w", "lmbda", "rho", "b"):
        assert torch.equal(getattr(src, k), getattr(dst, k))


def test_reference_checkpoint_loads():
    """a checkpoint written by the reference's ADMMDeconv (saver.py:49-54 layout) loads into this
    build's module with the safe loader (weights_only=True), values intact."""
    from admmtor.elayers.admmdeconv import ADMMDeconv
    ck = torch.load(os.path.join(GOLDEN, "ref_admmdeconv_ckpt.tar"), weights_only=True, map_location="cpu")
    m = ADMMDeconv((5, 5), max_iters=7, iso=False, bias=True)
    m.load_state_dict(ck["model_state_dict"])
    assert m.lmbda.item() == pytest.approx(0.031) and m.rho.item() == pytest.approx(0.047)
    assert m.b.item() == pytest.approx(0.25) and m.w.shape == (1, 1, 5, 5)
    assert torch.equal(m.w.detach(), ck["model_state_dict"]["w"])


def test_clamp_regularisers():
    from admmtor.elayers.admmdeconv import ADMMDeconv
    from admmtor.modelbuild.eregularizers import ADMMClipper, ADMMWeightClipper, WeightClipper
    m = torch.nn.Sequential(ADMMDeconv((3, 3), 5), ADMMDeconv((), 5))
    with torch.no_grad():
        m[0].lmbda.fill_(-1.0)
        m[0].rho.fill_(9.0)
        m[0].w.fill_(3.0)
        m[1].lmbda.fill_(0.0)
    m.apply(ADMMClipper(2.0))
    assert m[0].lmbda.item() == pytest.approx(1e-9, rel=1e-6) and m[0].rho.item() == 2.0
    assert m[1].lmbda.item() == pytest.approx(1e-9, rel=1e-6)
    m.apply(ADMMWeightClipper((-0.5, 0.5)))
    assert m[0].w.max().item() == 0.5
    with torch.no_grad():
        m[0].rho.fill_(9.0)
    m.apply(WeightClipper())
    assert m[0].rho.item() == 5.0

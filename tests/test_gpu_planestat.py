"""GPU parity of the whole-plane median / mode kernels (include/admm_chanstat.h, admm_planestat_*)
that replace ChannelWiseAttention's amedian / amodes (reference elayers/cwa.py): the selected flat
indices and values are bit-exact against torch's CPU kernels (the reference's tie rules), the
introsort depth-limit fallback against the oracle, the gradient against torch's CPU autograd.
"""
import numpy as np
import pytest
import torch

from oracle.chanpool_oracle import mode_of

pytestmark = pytest.mark.gpu


def _inputs(shape, dt, kind, seed):
    g = torch.Generator().manual_seed(seed)
    if kind == "gauss":
        return torch.randn(shape, generator=g).to(dt)
    k = {"few": 3, "many": 60}[kind]
    return (torch.randint(-k, k + 1, shape, generator=g).double() / 8).to(dt)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("shape", [(2, 3, 3, 3), (1, 2, 4, 4), (2, 3, 17, 31), (2, 4, 64, 64), (1, 3, 256, 256)])
def test_median_mode_vs_torch_cpu(cuda_dev, dt, shape):
    from admmtor.elayers.cwa import plane_select_native
    for kind in ("few", "many", "gauss"):
        x = _inputs(shape, dt, kind, sum(shape))
        P = shape[0] * shape[1]
        flat = x.reshape(P, -1)
        mi = plane_select_native(x.to(cuda_dev), "median").cpu()
        oi = plane_select_native(x.to(cuda_dev), "mode").cpu()
        med, mod = flat.median(dim=1), flat.mode(dim=1)
        assert torch.equal(mi, med.indices), (kind, "median")
        assert torch.equal(oi, mod.indices), (kind, "mode")
        assert torch.equal(flat.gather(1, oi[:, None]).squeeze(1), mod.values)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16, torch.float32])
def test_median_nan_signed_zero_inf(cuda_dev, dt):
    # torch.median's CPU rules: a plane holding NaN gives its first NaN; -0 and +0 tie (flat
    # order decides); infinities order as numbers
    from admmtor.elayers.cwa import plane_select_native
    g = torch.Generator().manual_seed(21)
    x = (torch.randint(-3, 4, (4, 1, 16, 33), generator=g).double() / 2).to(dt)
    x[0, 0, 3, 5] = float("nan")
    x[0, 0, 9, 1] = float("nan")
    x[1, 0, 0, :8] = -0.0
    x[1, 0, 2, :8] = float("inf")
    x[2, 0, 1, :30] = float("-inf")
    x[3].fill_(-0.0)
    x[3, 0, ::2, ::3] = 0.0
    flat = x.reshape(4, -1)
    mi = plane_select_native(x.to(cuda_dev), "median").cpu()
    assert torch.equal(mi, flat.median(dim=1).indices)


def test_fp32_median_low_bits(cuda_dev):
    # codes that share their high 16 bits and differ only in the low ones (the radix select's
    # second pass), with ties, at a 512x512 plane size
    from admmtor.elayers.cwa import plane_select_native
    g = torch.Generator().manual_seed(22)
    k = torch.randint(0, 40, (3, 2, 512, 512), generator=g).double()
    x = (1.0 + k * 2.0 ** -20).float()
    x[1] = -x[1]
    flat = x.reshape(6, -1)
    mi = plane_select_native(x.to(cuda_dev), "median").cpu()
    assert torch.equal(mi, flat.median(dim=1).indices)


def test_unique_values_and_small_planes(cuda_dev):
    from admmtor.elayers.cwa import plane_select_native
    x = torch.randperm(10, generator=torch.Generator().manual_seed(1)).to(torch.bfloat16).reshape(1, 1, 2, 5)
    assert plane_select_native(x.to(cuda_dev), "mode").item() == x.reshape(-1).mode().indices.item()
    assert plane_select_native(x.to(cuda_dev), "median").item() == x.reshape(-1).median(0).indices.item()
    x1 = torch.full((1, 1, 1, 1), 2.0, dtype=torch.bfloat16)
    assert plane_select_native(x1.to(cuda_dev), "mode").item() == 0


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("depth", [0, 1, 3])
def test_depth_limited_vs_oracle(cuda_dev, depth, dt):
    from admmtor.elayers.cwa import plane_select_native
    x = _inputs((1, 2, 20, 30), dt, "few", 7 + depth)
    got = plane_select_native(x.to(cuda_dev), "mode", depth_limit=depth).cpu().numpy()
    for p in range(2):
        col = x.reshape(2, -1)[p].double().numpy()
        assert got[p] == mode_of(col, depth_limit=depth)[1]


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_gradient_vs_torch_cpu(cuda_dev, dt):
    from admmtor.elayers.cwa import amedian, amodes
    x = _inputs((2, 3, 32, 32), dt, "many", 11)
    w = torch.randn(2, 3, generator=torch.Generator().manual_seed(12)).to(dt)
    xg = x.to(cuda_dev).requires_grad_(True)
    (amedian(xg) * w.to(cuda_dev) + amodes(xg) * 2 * w.to(cuda_dev)).sum().backward()
    xc = x.clone().requires_grad_(True)
    f = xc.reshape(2, 3, -1)
    (f.median(dim=-1).values * w + f.mode(dim=-1).values * 2 * w).sum().backward()
    assert torch.equal(xg.grad.cpu(), xc.grad)


def test_cwa_module_uses_native_and_matches_cpu(cuda_dev):
    from admmtor.elayers.cwa import ChannelWiseAttention
    torch.manual_seed(0)
    m = ChannelWiseAttention(8)
    x = _inputs((2, 8, 16, 16), torch.bfloat16, "many", 13).float()
    ref = m.double()(x.double().to(torch.bfloat16).double())
    # the statistics on bf16 inputs: the module on the GPU in bf16 vs the same ops on the CPU in bf16
    mg = ChannelWiseAttention(8)
    mg.load_state_dict(m.state_dict())
    xb = x.to(torch.bfloat16)
    vals_gpu = [f(xb.to(cuda_dev)).cpu() for f in mg.compress_methods]
    vals_cpu = [f(xb) for f in mg.compress_methods]
    for a, b in zip(vals_gpu[1:3], vals_cpu[1:3]):  # median, mode: exact
        assert torch.equal(a, b)
    assert torch.isfinite(ref).all()

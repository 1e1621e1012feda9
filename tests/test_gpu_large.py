"""Batches past 2^31 pixels (MI355X: 288 GB of HBM per GPU holds them): 64-bit addressing end to end.

One call over more than 2^31 pixels (8.6 GB of fp32 input; ~80-100 GB with output and workspace), on
the fused path (1024^2 planes, config 3's size) and on the generic path (321 x 481, the BSD size).
Inputs are distinct seeded noise planes, so a plane read through a wrapped 32-bit offset could not
pass as its neighbour.  Checks, around the plane whose first pixel is element 2^31 and at the end of
the batch:
* bit-exact against the same planes solved in a small batch (planes are independent in aniso mode,
  and the kernels' results do not depend on the batch -- tests/test_gpu_0_parity.py);
* two of them against the fp64 oracle at the 1e-5 gate.
"""
import pytest
import torch

from oracle.admm_oracle import rel_l2, solve_fourier

pytestmark = pytest.mark.gpu

IT = 3


def _noise(P, H, W, dev, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    return torch.rand((P, 1, H, W), generator=g, device=dev)


@pytest.mark.parametrize("P,H,W", [(2100, 1024, 1024), (14100, 321, 481)])
def test_batch_past_2_31_pixels(cuda_dev, P, H, W):
    from admmtor.eops.deconv import fft_admm_tv
    from admmtor.synth import make_psf
    assert P * H * W > 2 ** 31
    free, _ = torch.cuda.mem_get_info(cuda_dev)
    if free < 140e9:
        pytest.skip(f"needs ~100 GB of free device memory, {free / 1e9:.0f} GB free")
    psf = make_psf("gauss:1.5", 9).to(cuda_dev)
    x = _noise(P, H, W, cuda_dev, seed=11)
    x = x.reshape(P // 3, 3, H, W)
    out = fft_admm_tv(x, 0.01, 0.02, psf, False, IT)
    torch.cuda.synchronize()
    flat_out = out.reshape(P, H, W)
    b31 = 2 ** 31 // (H * W)  # the plane holding element 2^31
    # 6 planes from an even plane index hold plane b31 (the generic row kernels pair real rows by their
    # index in the launch: with odd H an even first plane keeps every row's partner, hence the bits)
    lo = max(0, (b31 - 2) // 2 * 2)
    for p0 in (lo, P - 6):  # 6 planes = 2 images around 2^31, and the last two images
        small = fft_admm_tv(x.reshape(P, H, W)[p0:p0 + 6].reshape(2, 3, H, W).contiguous(), 0.01, 0.02, psf,
                            False, IT)
        torch.cuda.synchronize()
        assert torch.equal(small.reshape(6, H, W), flat_out[p0:p0 + 6]), (P, H, W, p0)
    for p in (b31, P - 1):
        xp = x.reshape(P, H, W)[p].reshape(1, 1, H, W).double().cpu()
        ref = solve_fourier(xp, 0.01, 0.02, psf.double().cpu(), False, IT)
        e = rel_l2(flat_out[p].reshape(1, 1, H, W).cpu(), ref)
        print(f"{P}x{H}x{W} plane {p}: rel-L2 vs fp64 oracle {e:.2e}")
        assert e <= 1e-5
    del out, flat_out, x
    torch.cuda.empty_cache()

"""Checkpoint compatibility on the GPU: a checkpoint written by the reference's
ADMMDeconv (saver.py:49-54 layout) loads with the safe loader (``weights_only=True``, as
scripts/train.py:75-78 loads it) into this build's module, and the HIP forward on the device
matches the reference's own output for that state (tests/golden/g11_ckpt.npz, made by
tests/golden/make_golden_ckpt.py): <= 1e-5 relative L2 against the reference's fp64 run."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, load_golden

pytestmark = pytest.mark.gpu


def test_reference_checkpoint_forward_on_gpu(cuda_dev):
    from admmtor.elayers.admmdeconv import ADMMDeconv
    g = load_golden("g11_ckpt")
    ck = torch.load(os.path.join(GOLDEN, "ref_admmdeconv_ckpt.tar"), weights_only=True, map_location="cpu")
    m = ADMMDeconv((5, 5), max_iters=7, iso=False, bias=True)
    m.load_state_dict(ck["model_state_dict"])
    m = m.to(cuda_dev)
    with torch.no_grad():
        out = m(torch.from_numpy(g["x"]).to(cuda_dev))
    assert out.is_cuda
    ref = g["out64"].astype(np.float64)
    e = float(np.linalg.norm(out.cpu().double().numpy() - ref) / np.linalg.norm(ref))
    print(f"checkpoint forward: {e:.3e} (reference fp32: {float(g['ref32_err']):.3e})")
    assert e <= 1e-5
    # and a training step from the loaded state runs through the native backward
    x = torch.from_numpy(g["x"]).to(cuda_dev)
    m(x).square().mean().backward()
    for n, p in m.named_parameters():
        assert p.grad is not None and torch.isfinite(p.grad).all(), n

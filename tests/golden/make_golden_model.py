"""Golden fixtures for the config-5 caller: the REFERENCE's DivergentRestorer
at reduced width, forward and backward, run in this build container.

Run from the repo root (build container only; nothing at test time reads /root/reference):

    PYTHONDONTWRITEBYTECODE=1 PYTHONPATH=/root/reference/src python tests/golden/make_golden_model.py

It imports the reference package alone (the build's own ``admmtor`` is NOT on the path, the two
share a name) and stores data only: the seeded initial state_dict, inputs, outputs and fp64
gradients of every parameter (plus the reference's fp32 run, the floor for an fp32 build).

  g8_model_admm   DivergentRestorer([2, 4, 4], 3, 3, 8, 8, 2, Sigmoid, admms = 2 x iso, no PSF,
                  10 it) on 2x3x32^2 -- the train.py architecture at reduced width / depth
  g8_model_plain  same without the ADMM modules (admms=None): the CNN alone, checkable on CPU
"""
import os
import sys

import numpy as np
import torch

sys.dont_write_bytecode = True
from admmtor.modelbuild.denoiser import DivergentRestorer  # noqa: E402  (the reference's)

OUT = os.path.dirname(os.path.abspath(__file__))
SEED = 20251205 + 5


def build(admms):
    torch.manual_seed(SEED)
    return DivergentRestorer([2, 4, 4], 3, 3, 8, 8, 2, output_activation=torch.nn.Sigmoid(), admms=admms)


def smooth_batch(g):
    """Smooth random images (sums of Gaussian bumps): the TV solve then has no flat plateaus, so
    the median / mode statistics downstream select the same element in fp32 and fp64."""
    yy, xx = torch.meshgrid(torch.arange(32, dtype=torch.float64), torch.arange(32, dtype=torch.float64),
                            indexing="ij")
    x = torch.zeros(2, 3, 32, 32, dtype=torch.float64)
    for b in range(2):
        for c in range(3):
            p = torch.rand(6, 4, generator=g, dtype=torch.float64)
            for cy, cx, s, a in p:
                x[b, c] += (0.2 + a) * torch.exp(-((yy - 32 * cy) ** 2 + (xx - 32 * cx) ** 2) / (2 * (2 + 6 * s) ** 2))
            x[b, c] += 0.01 * (yy + 2 * xx) / 32
    return x


def make(name, admms):
    model = build(admms)
    init = {k: v.detach().clone() for k, v in model.state_dict().items()}
    g = torch.Generator().manual_seed(SEED + 1)
    if admms is not None:
        # the seeded uniform(0, 1) lambda / rho give tau up to ~100 (everything flattened);
        # run at a moderate tau = lambda / rho instead (stored: "sd/" is the state the run used)
        with torch.no_grad():
            for i, m in enumerate(model.blocks[0].admms):
                m.lmbda.fill_(0.002 * (i + 1))
                m.rho.fill_(0.05)
    x = smooth_batch(g)
    cot = torch.randn(2, 3, 32, 32, generator=g, dtype=torch.float64)
    # the reference's own fp32 run: the noise floor an fp32 implementation is judged against
    x32 = x.float().clone().requires_grad_(True)
    out32 = model(x32)
    (out32 * cot.float()).sum().backward()
    fp32 = {"out32": out32.detach().numpy(), "gx32": x32.grad.numpy()}
    for k, p in model.named_parameters():
        if p.grad is not None:
            fp32["grad32/" + k] = p.grad.numpy().copy()
    model.zero_grad(set_to_none=True)
    model = model.double()
    x_req = x.clone().requires_grad_(True)
    out = model(x_req)
    (out * cot).sum().backward()
    data = {"x": x.numpy(), "cot": cot.numpy(), "out": out.detach().numpy(), "gx": x_req.grad.numpy()}
    data.update(fp32)
    for k, v in init.items():
        data["init/" + k] = v.numpy()
    for k, v in model.state_dict().items():
        data["sd/" + k] = v.float().numpy()
    for k, p in model.named_parameters():
        if p.grad is not None:
            data["grad/" + k] = p.grad.numpy()
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **data)
    print(name, out.shape, len(init), "state entries,",
          sum(1 for k in data if k.startswith("grad/")), "grads")


if __name__ == "__main__":
    admm = {"kern_size": (), "max_iters": 10, "iso": True}
    make("g8_model_admm", [dict(admm), dict(admm)])
    make("g8_model_plain", None)

"""Write tests/golden/g9_chanpool.npz: ChannelPool's statistics from PyTorch's own CPU kernels.

The reference's ChannelPool (/root/reference/src/admmtor/elayers/attentions.py:44-47) is
`cat(x.std(1), x.median(1).values, x.mode(1).values)`; its arithmetic (and the tie rules for the
returned indices, which decide where the gradient goes) lives in torch's CPU kernels, which are
importable here.  Inputs are heavy-tie integer grids (so the mode / median index rules matter)
and Gaussian values rounded to the dtype.  Stored per case: the input (as float32 values of the
dtype), std/median/mode values and median/mode indices, and the gradient of
sum(out * cot) w.r.t. x for a fixed cotangent (fp64 autograd on the same values).

  python tests/golden/make_golden_chanpool.py
"""
import os

import numpy as np
import torch

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "g9_chanpool.npz")

CASES = [  # name, dtype, B, C, H, W, kind
    ("c3_bf16", torch.bfloat16, 2, 3, 5, 6, "int"),
    ("c16_bf16", torch.bfloat16, 2, 16, 4, 5, "int"),
    ("c17_f32", torch.float32, 2, 17, 4, 5, "int"),
    ("c86_bf16", torch.bfloat16, 2, 86, 6, 6, "int"),
    ("c86_bf16_gauss", torch.bfloat16, 2, 86, 6, 6, "gauss"),
    ("c86_f32", torch.float32, 2, 86, 4, 4, "int"),
    ("c129_f16", torch.float16, 1, 129, 4, 4, "int"),
    ("c200_bf16", torch.bfloat16, 1, 200, 3, 4, "int"),
]


def main():
    g = torch.Generator().manual_seed(20251205)
    arrays = {}
    for name, dt, B, C, H, W, kind in CASES:
        if kind == "int":
            x = (torch.randint(-5, 6, (B, C, H, W), generator=g).to(torch.float64) * 0.25).to(dt)
        else:
            x = torch.randn((B, C, H, W), generator=g).to(dt)
        sd = x.std(dim=1)
        med = x.median(dim=1)
        mod = x.mode(dim=1)
        xd = x.double().requires_grad_(True)
        outd = torch.cat((xd.std(dim=1, keepdim=True), xd.median(dim=1, keepdim=True).values,
                          xd.mode(dim=1, keepdim=True).values), dim=1)
        cot = torch.randn(outd.shape, generator=g, dtype=torch.float64)
        (outd * cot).sum().backward()
        arrays[f"{name}/x"] = x.float().numpy()
        arrays[f"{name}/std"] = sd.float().numpy()
        arrays[f"{name}/median"] = med.values.float().numpy()
        arrays[f"{name}/median_idx"] = med.indices.numpy().astype(np.int16)
        arrays[f"{name}/mode"] = mod.values.float().numpy()
        arrays[f"{name}/mode_idx"] = mod.indices.numpy().astype(np.int16)
        arrays[f"{name}/cot"] = cot.numpy()
        arrays[f"{name}/grad64"] = xd.grad.numpy()
        # the fp64 run picks its indices on the same values: they must agree with the dtype run
        assert torch.equal(xd.median(dim=1).indices, med.indices) and torch.equal(xd.mode(dim=1).indices, mod.indices)
    arrays["dtypes"] = np.array([str(c[1]).replace("torch.", "") for c in CASES])
    arrays["names"] = np.array([c[0] for c in CASES])
    arrays["torch_version"] = np.array(torch.__version__)
    np.savez_compressed(OUT, **arrays)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()

"""GPU diagnostics for the config-5 model parity (where does the fp32 GPU run leave the fp64 reference?)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "torch-admm-deconv_amd"), os.path.join(ROOT, "tests")]
from conftest import load_golden  # noqa: E402
from admmtor.modelbuild.denoiser import DivergentRestorer  # noqa: E402
from admmtor.elayers.cwa import ChannelWiseAttention  # noqa: E402

dev = torch.device("cuda:0")
# 1. torch.mode tie-break for all-distinct values, CPU vs GPU
v = torch.stack([torch.randperm(256).float() for _ in range(4)])
print("mode cpu", v.mode(-1).values.tolist(), "gpu", v.to(dev).mode(-1).values.cpu().tolist())
print("median cpu", v.median(-1).values.tolist(), "gpu", v.to(dev).median(-1).values.cpu().tolist())

g = load_golden("g8_model_admm")
ADMM = {"kern_size": (), "max_iters": 10, "iso": True}
m = DivergentRestorer([2, 4, 4], 3, 3, 8, 8, 2, output_activation=torch.nn.Sigmoid(), admms=[ADMM, ADMM])
m.load_state_dict({k[3:]: torch.from_numpy(g[k]) for k in g if k.startswith("sd/")})
m = m.to(dev)
dups = []
captured = {}


def cwa_hook(mod, inp):
    x = inp[0].detach().reshape(inp[0].shape[0], inp[0].shape[1], -1)
    for b in range(x.shape[0]):
        for c in range(x.shape[1]):
            dups.append(x[b, c].numel() - torch.unique(x[b, c]).numel())


for mod in m.modules():
    if isinstance(mod, ChannelWiseAttention):
        mod.register_forward_pre_hook(cwa_hook)
for i, a in enumerate(m.blocks[0].admms):
    a.register_forward_hook(lambda mod, inp, out, i=i: captured.__setitem__(i, out.detach().cpu()))
x = torch.from_numpy(g["x"]).float().to(dev)
out = m(x).detach().cpu().double()
print("planes with duplicates in CWA inputs:", sum(d > 0 for d in dups), "of", len(dups), "max dup", max(dups))
ref = torch.from_numpy(g["out"])
print("gpu vs ref64", ((out - ref).norm() / ref.norm()).item())
# 2. same ADMM outputs, CNN on CPU in fp64 and fp32
for dt in (torch.float64, torch.float32):
    mc = DivergentRestorer([2, 4, 4], 3, 3, 8, 8, 2, output_activation=torch.nn.Sigmoid(), admms=[ADMM, ADMM])
    mc.load_state_dict({k[3:]: torch.from_numpy(g[k]) for k in g if k.startswith("sd/")})
    mc = mc.to(dt)
    for i, a in enumerate(mc.blocks[0].admms):
        a.forward = (lambda xx, i=i: captured[i].to(dt))
    oc = mc(torch.from_numpy(g["x"]).to(dt)).detach().double()
    print(dt, "cpu CNN on gpu ADMM outputs vs gpu", ((oc - out).norm() / out.norm()).item(),
          "vs ref64", ((oc - ref).norm() / ref.norm()).item())

import os, sys, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "torch-admm-deconv_amd")]
from admmtor.eops.deconv import fft_admm_tv
from admmtor.synth import blurred_batch, make_psf
from oracle.admm_oracle import solve_spatial
dev = torch.device("cuda:0")
def rel(a, b):
    if a is None or b is None: return None
    return ((a.double().cpu() - b.double().cpu()).norm() / b.double().cpu().norm()).item()
cases = [(("random", 9), (2, 3, 128, 128), 15), (("random", 9), (1, 6, 128, 128), 15), (("random", 9), (6, 1, 128, 128), 15),
         (("random", 9), (1, 3, 128, 128), 15), (("random", 9), (1, 4, 128, 128), 15), (("random", 9), (2, 3, 128, 128), 3)]
for psf, shape, it in cases:
    k = make_psf(*psf); x = blurred_batch(*shape, k, seed=13)
    kk = k if k.numel() else torch.empty(0)
    cot = torch.randn(x.shape, generator=torch.Generator().manual_seed(3))
    xg = x.to(dev).requires_grad_(True)
    lg = torch.tensor([0.02], device=dev, requires_grad=True); rg = torch.tensor([0.05], device=dev, requires_grad=True)
    o = fft_admm_tv(xg, lg, rg, kk.to(dev), False, it)
    gs = torch.autograd.grad(o, (xg, lg, rg), cot.to(dev), allow_unused=True)
    xd = x.double().requires_grad_(True)
    ld = torch.tensor([0.02], dtype=torch.float64, requires_grad=True); rd = torch.tensor([0.05], dtype=torch.float64, requires_grad=True)
    od = solve_spatial(xd, ld, rd, kk.double(), False, it)
    gd = torch.autograd.grad(od, (xd, ld, rd), cot.double(), allow_unused=True)
    pl = [rel(gs[0][:, :, :, :][b, c], gd[0][b, c]) for b in range(shape[0]) for c in range(shape[1])]
    print(psf, shape, it, "out", rel(o.detach(), od.detach()), "gx", rel(gs[0], gd[0]), "per-plane gx", pl,
          "glam", rel(gs[1], gd[1]), "grho", rel(gs[2], gd[2]), flush=True)

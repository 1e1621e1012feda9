import os, sys, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "torch-admm-deconv_amd")]
from admmtor.eops.deconv import fft_admm_tv
from admmtor.synth import blurred_batch, make_psf
from oracle.admm_oracle import solve_fourier, rel_l2
dev = torch.device("cuda:0")
k = make_psf("motion", 9)
x = blurred_batch(2, 3, 256, 256, k, seed=2)
ref = solve_fourier(x.double(), 0.01, 0.02, k.double(), False, 6)
outs = {}
for R in ("16", "16", "8", "4", "2", "32", "256"):
    os.environ["ADMM_PASSA_R"] = R
    o = fft_admm_tv(x.to(dev), 0.01, 0.02, k.to(dev), False, 6).cpu()
    torch.cuda.synchronize()
    e = rel_l2(o, ref)
    if R in outs:
        print("R", R, "repeat bitwise equal:", torch.equal(o, outs[R]))
    outs[R] = o
    d = (o.double() - ref).abs().amax(dim=(0, 1, 3))  # per row max error
    print("R", R, "rel vs oracle", e, "rows with max err: ", torch.topk(d, 6).indices.tolist(), torch.topk(d, 6).values.tolist())
for it in (1, 2, 3):
    for R in ("16", "8"):
        os.environ["ADMM_PASSA_R"] = R
        o = fft_admm_tv(x.to(dev), 0.01, 0.02, k.to(dev), False, it).cpu()
        r = solve_fourier(x.double(), 0.01, 0.02, k.double(), False, it)
        d = (o.double() - r).abs().amax(dim=(0, 1, 3))
        print("it", it, "R", R, "rel", rel_l2(o, r), "worst rows", torch.topk(d, 4).indices.tolist())

import sys, os
sys.path[:0] = ["/root/repo", "/root/repo/tests", "/root/repo/torch-admm-deconv_amd"]
os.chdir(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch, numpy as np
from conftest import load_golden
import test_gpu_model as T
dev = torch.device("cuda:0")
g = load_golden("g8_model_admm")
m = T._model(g, dev)
x = torch.from_numpy(g["x"]).float().to(dev)
with torch.no_grad():
    outs = [m(x).cpu() for _ in range(3)]
print("forward bitwise repeatable:", all(torch.equal(outs[0], o) for o in outs[1:]))
print("e_out", T.rel(outs[0], g["out"]))
# the statistics alone, repeated on a large random input
from admmtor.elayers.attentions import _chanstat_native
from admmtor.elayers.cwa import plane_select_native
xr = torch.randn(4, 86, 256, 256, device=dev).to(torch.bfloat16)
a = [_chanstat_native(xr)[1].cpu() for _ in range(3)]
b = [plane_select_native(xr, "mode").cpu() for _ in range(3)]
c = [plane_select_native(xr.float(), "mode").cpu() for _ in range(3)]
print("chanstat repeatable:", all(torch.equal(a[0], t) for t in a), "plane mode:", all(torch.equal(b[0], t) for t in b),
      "plane mode f32:", all(torch.equal(c[0], t) for t in c))

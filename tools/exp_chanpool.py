import os, sys
sys.path.insert(0, "torch-admm-deconv_amd"); sys.path.insert(0, "tools")
import torch
from admmtor import _native
from admmtor.elayers.attentions import _chanstat_native
from ab_chanpool import timed, data
dev = torch.device("cuda:0"); gen = torch.Generator().manual_seed(0)
with _native.ab_library():
    for kind in ("gauss", "gelu"):
        x = data(kind, (16, 86, 512, 512), torch.bfloat16, gen).to(dev)
        for e in (0, 1, 2, 4, 8, 1 | 2 | 4, 1 | 2 | 4 | 8):
            os.environ["ADMM_CHANPOOL_EXP"] = str(e)
            print(f"{kind} exp={e:2d}: {timed(lambda: _chanstat_native(x)):.3f} ms", flush=True)
    os.environ["ADMM_CHANPOOL_EXP"] = "0"

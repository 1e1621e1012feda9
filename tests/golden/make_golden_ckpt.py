"""Golden for the checkpoint round trip on the GPU, made by running the REFERENCE
in this container (nothing at test time reads /root/reference):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_ckpt.py

The reference's ADMMDeconv((5,5), max_iters=7, iso=False, bias=True) loads the reference-written
checkpoint tests/golden/ref_admmdeconv_ckpt.tar (saver.py:49-54 layout, read with
``weights_only=True`` as scripts/train.py:75-78 would load it) and runs on a synthetic batch in
fp64 and fp32.  Stored (g11_ckpt.npz): the input, the fp64 output (rounded to fp32) and the fp32
run's distance to it.
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "torch-admm-deconv_amd"))
from admmtor.synth import blurred_batch, make_psf  # noqa: E402

CKPT = os.path.join(ROOT, "tests", "golden", "ref_admmdeconv_ckpt.tar")
OUT = os.path.join(ROOT, "tests", "golden", "g11_ckpt.npz")

REF_CODE = r"""
import sys, numpy as np, torch
from admmtor.elayers.admmdeconv import ADMMDeconv
x = torch.from_numpy(np.load(sys.argv[1])["x"])
ck = torch.load(sys.argv[3], weights_only=True, map_location="cpu")
o = {}
for tag, dt in (("64", torch.float64), ("32", torch.float32)):
    m = ADMMDeconv((5, 5), max_iters=7, iso=False, bias=True)
    m.load_state_dict(ck["model_state_dict"])
    m = m.to(dt)
    with torch.no_grad():
        o["out" + tag] = m(x.to(dt)).numpy()
np.savez(sys.argv[2], **o)
"""


def main():
    x = blurred_batch(2, 3, 64, 64, make_psf("gauss:1.5", 9), seed=4711).numpy()
    with tempfile.TemporaryDirectory() as td:
        fin, fout = os.path.join(td, "in.npz"), os.path.join(td, "out.npz")
        np.savez(fin, x=x)
        env = dict(os.environ, PYTHONPATH="/root/reference/src", PYTHONDONTWRITEBYTECODE="1")
        subprocess.run([sys.executable, "-c", REF_CODE, fin, fout, CKPT], env=env, check=True, cwd=td)
        o = dict(np.load(fout))
    err = np.linalg.norm(o["out32"] - o["out64"]) / np.linalg.norm(o["out64"])
    np.savez_compressed(OUT, x=x, out64=o["out64"].astype(np.float32), ref32_err=np.float64(err))
    print("ref32 vs ref64", err, "size", os.path.getsize(OUT))


if __name__ == "__main__":
    main()

"""In-process tuning sweep of the HIP passes (ADMM_PASSB_C / ADMM_PASSA_R env knobs).
The knobs are read only by an A/B build of the library (csrc/knobs.hpp): bash tools/build_variant.sh ab,
then run with ADMMTOR_LIB_OVERRIDE=tools/_variants/ab.so (read here, by the tool: the package
itself never reads it; this calls admmtor._native.use_library).

usage: python tools/sweep.py [--config c3] [--steps 3] VAR=v1,v2 [VAR2=...]
Prints per-kernel average launch time and GB/s (algorithmic bytes) for each setting.
"""
import argparse
import itertools
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "torch-admm-deconv_amd")]
import torch  # noqa: E402

from bench import CONFIGS, PASS_A_BYTES, PASS_B_BYTES  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--maxit", type=int, default=0)
    ap.add_argument("knobs", nargs="*")
    a = ap.parse_args()
    from admmtor import _native
    if os.environ.get("ADMMTOR_LIB_OVERRIDE"):
        _native.use_library(os.environ["ADMMTOR_LIB_OVERRIDE"])
    from admmtor.eops.deconv import fft_admm_tv
    from admmtor.synth import blurred_batch, make_psf
    B, C, H, W, kind, k, maxit, iso, _ = CONFIGS[a.config]
    maxit = a.maxit or maxit
    dev = torch.device("cuda:0")
    psf = make_psf(kind, k).to(dev) if k else torch.empty(0, device=dev)
    x = blurred_batch(B, C, H, W, psf.cpu(), seed=1, device=dev)
    npx = B * C * H * W
    knobs = [kv.split("=") for kv in a.knobs]
    names = [k for k, _ in knobs]
    grid = list(itertools.product(*[v.split(",") for _, v in knobs])) or [()]
    ref = None
    for vals in grid:
        for n, v in zip(names, vals):
            os.environ[n] = v
        out = fft_admm_tv(x, 0.01, 0.02, psf, iso, maxit)  # warm-up
        torch.cuda.synchronize()
        if ref is None:
            ref = out
        diff = ((out - ref).norm() / ref.norm()).item()
        _native.profile_reset()
        _native.profile_enable(True)
        t0 = time.perf_counter()
        for _ in range(a.steps):
            fft_admm_tv(x, 0.01, 0.02, psf, iso, maxit)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        _native.profile_enable(False)
        ms, cnt = _native.profile_read()
        res = {"knobs": dict(zip(names, vals)), "it_s": maxit * a.steps / dt,
               "A_ms": ms[0] / max(cnt[0], 1), "A_GBs": PASS_A_BYTES * npx / (ms[0] / max(cnt[0], 1)) / 1e6,
               "B_ms": ms[1] / max(cnt[1], 1), "B_GBs": PASS_B_BYTES * npx / (ms[1] / max(cnt[1], 1)) / 1e6,
               "iso_ms": ms[2] / max(cnt[2], 1), "setup_ms": ms[3] / a.steps, "diff_vs_first": diff}
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

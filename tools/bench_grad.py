"""Training-path timing: forward with history + native backward (x, lambda, rho gradients).

usage: python tools/bench_grad.py [--config c3|c2|c5fwd] [--maxit N] [--steps K]
Prints per-kernel-class time (HIP events: 0 row pass, 1 column pass, 2 iso, 3 setup) for the
forward-train and the backward separately, and the backward's row-pass bandwidth on its
algorithmic bytes (r^ spectrum 4 + a_k 8 + a_{k-1} 8 + a^ in 8 + a^ out 8 + b^ rw 8 + x^ out 4
= 48 B/px; iso adds N, Q maps which stay in L2).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "torch-admm-deconv_amd")]
import torch  # noqa: E402

from bench import CONFIGS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--maxit", type=int, default=0)
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    from admmtor import _native
    from admmtor.eops.deconv import fft_admm_tv
    from admmtor.synth import blurred_batch, make_psf
    B, C, H, W, kind, k, maxit, iso, _ = CONFIGS[a.config]
    maxit = a.maxit or maxit
    dev = torch.device("cuda:0")
    psf = make_psf(kind, k).to(dev) if k else torch.empty(0, device=dev)
    x = blurred_batch(B, C, H, W, psf.cpu(), seed=1, device=dev).requires_grad_(True)
    lam = torch.tensor([0.01], device=dev, requires_grad=True)
    rho = torch.tensor([0.02], device=dev, requires_grad=True)
    cot = torch.randn(x.shape, device=dev)

    def step():
        out = fft_admm_tv(x, lam, rho, psf, iso, maxit)
        torch.cuda.synchronize()
        t_f = time.perf_counter()
        ms_f, _ = _native.profile_read()
        out.backward(cot)
        torch.cuda.synchronize()
        return t_f, list(ms_f)

    step()
    x.grad = lam.grad = rho.grad = None
    tot = {"fwd": 0.0, "bwd": 0.0}
    kf = [0.0] * 4
    kb = [0.0] * 4
    nb = [0] * 4
    for _ in range(a.steps):
        _native.profile_reset()
        _native.profile_enable(True)
        t0 = time.perf_counter()
        t_f, ms_f = step()
        t1 = time.perf_counter()
        ms_all, cnt_all = _native.profile_read()
        _native.profile_enable(False)
        tot["fwd"] += t_f - t0
        tot["bwd"] += t1 - t_f
        for i in range(4):
            kf[i] += ms_f[i]
            kb[i] += ms_all[i] - ms_f[i]
            nb[i] = cnt_all[i]
        x.grad = lam.grad = rho.grad = None
    K = a.steps
    npx = B * C * H * W
    bwd_row_ms = kb[0] / K / maxit
    print(json.dumps({
        "config": a.config, "maxit": maxit, "iso": iso,
        "fwd_ms": tot["fwd"] / K * 1e3, "bwd_ms": tot["bwd"] / K * 1e3,
        "fwd_kernel_ms": [v / K for v in kf], "bwd_kernel_ms": [v / K for v in kb],
        "bwd_row_pass_ms_per_it": bwd_row_ms,
        "bwd_row_pass_GBps_48B": 48 * npx / (bwd_row_ms * 1e-3) / 1e9 if bwd_row_ms > 0 else None,
        "peak_mem_GiB": torch.cuda.max_memory_allocated(dev) / 2**30}))


if __name__ == "__main__":
    main()

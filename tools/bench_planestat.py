"""Whole-plane median / mode (ChannelWiseAttention's statistics) time: the HIP kernels vs
PyTorch's GPU median/mode at the config-5 shape (16 x 86 planes of 512^2, bf16).
  python tools/bench_planestat.py [--native-only]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torch-admm-deconv_amd"))
import torch  # noqa: E402

from admmtor.elayers.cwa import plane_select_native  # noqa: E402


def timed(fn, n):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    for B, C, H, W, dt in ((16, 86, 512, 512, torch.bfloat16), (16, 86, 128, 128, torch.bfloat16),
                           (16, 86, 512, 512, torch.float32)):
        x = torch.randn((B, C, H, W), device=dev, generator=g).to(dt)
        med = timed(lambda: plane_select_native(x, "median"), 5)
        mod = timed(lambda: plane_select_native(x, "mode"), 5)
        line = f"{B}x{C}x{H}x{W} {str(dt)[6:]}: native median {med:.2f} ms, mode {mod:.2f} ms"
        if "--native-only" not in sys.argv:
            f = x.reshape(B, C, -1)
            tmed = timed(lambda: f.median(dim=-1), 1)
            tmod = timed(lambda: f.mode(dim=-1), 1)
            line += f"; torch median {tmed:.1f} ms, mode {tmod:.1f} ms"
        print(line, flush=True)


if __name__ == "__main__":
    main()

"""Small-problem latency of fft_admm_tv (launch-bound sizes, e.g. C1 = 1x1x256^2, 9x9 PSF, 30 it).

Per shape: wall time per call (host launch + GPU, synchronised), and the same with the
per-kernel profile on to split GPU work from launch gaps.
  python tools/bench_small.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torch-admm-deconv_amd"))
import torch  # noqa: E402

from admmtor.eops.deconv import fft_admm_tv  # noqa: E402
from admmtor.synth import blurred_batch, make_psf  # noqa: E402

SHAPES = [  # B, C, H, W, psf, k, maxit, iso
    (1, 1, 256, 256, "gauss:1.5", 9, 30, False),
    (1, 3, 256, 256, "gauss:1.5", 9, 30, False),
    (1, 3, 512, 512, "motion", 15, 50, False),
    (4, 3, 256, 256, "gauss:1.5", 9, 100, True),
    (1, 3, 321, 481, "gauss:1.5", 9, 50, False),
]


def main():
    dev = torch.device("cuda:0")
    for B, C, H, W, kind, k, maxit, iso in SHAPES:
        psf = make_psf(kind, k).to(dev)
        x = blurred_batch(B, C, H, W, psf.cpu(), seed=3).to(dev)
        for _ in range(5):
            fft_admm_tv(x, 0.01, 0.02, psf, iso, maxit)
        torch.cuda.synchronize()
        n = 50
        t0 = time.perf_counter()
        for _ in range(n):
            fft_admm_tv(x, 0.01, 0.02, psf, iso, maxit)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / n * 1e3
        # host-side enqueue time alone (no sync inside the loop)
        t0 = time.perf_counter()
        for _ in range(n):
            fft_admm_tv(x, 0.01, 0.02, psf, iso, maxit)
        host = (time.perf_counter() - t0) / n * 1e3
        torch.cuda.synchronize()
        # the same call captured once in a HIP graph (torch.cuda.CUDAGraph) and replayed
        st = torch.cuda.Stream(dev)
        st.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(st):
            fft_admm_tv(x, 0.01, 0.02, psf, iso, maxit)
        torch.cuda.current_stream(dev).wait_stream(st)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fft_admm_tv(x, 0.01, 0.02, psf, iso, maxit)
        g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            g.replay()
        torch.cuda.synchronize()
        graph = (time.perf_counter() - t0) / n * 1e3
        print(f"{B}x{C}x{H}x{W} k{k} {'iso' if iso else 'aniso'} {maxit} it: {wall:.3f} ms/call "
              f"({maxit / wall * 1e3:.0f} it/s), host enqueue {host:.3f} ms/call; graph replay {graph:.3f} ms/call "
              f"({maxit / graph * 1e3:.0f} it/s)", flush=True)


if __name__ == "__main__":
    main()

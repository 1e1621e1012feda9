"""ChannelPool forward / backward time: the HIP kernels (include/admm_chanstat.h) vs PyTorch's
sort-based std/median/mode (the reference's op sequence) at the config-5 caller's shapes.
  python tools/bench_chanpool.py [--native-only]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torch-admm-deconv_amd"))
import torch  # noqa: E402

from admmtor.elayers.attentions import _ChannelPoolFn, channel_pool_reference_ops  # noqa: E402


def timed(fn, n=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    for B, C, H, W in ((16, 86, 512, 512), (16, 86, 256, 256), (16, 86, 128, 128)):
        x = torch.randn((B, C, H, W), device=dev, generator=g).to(torch.bfloat16)
        xr = x.clone().requires_grad_(True)
        cot = torch.randn((B, 3, H, W), device=dev, generator=g).to(torch.bfloat16)
        fwd_native = timed(lambda: _ChannelPoolFn.apply(x))
        if "--native-only" in sys.argv:
            print(f"{B}x{C}x{H}x{W} bf16: forward native {fwd_native:.3f} ms", flush=True)
            continue
        fwd_torch = timed(lambda: channel_pool_reference_ops(x), n=3)

        def fb_native():
            xr.grad = None
            _ChannelPoolFn.apply(xr).backward(cot)

        def fb_torch():
            xr.grad = None
            channel_pool_reference_ops(xr).backward(cot)

        fb_n = timed(fb_native)
        fb_t = timed(fb_torch, n=3)
        gb = B * H * W * (C + 3 + 2) * 2 / 1e9
        print(f"{B}x{C}x{H}x{W} bf16: forward native {fwd_native:.3f} ms ({gb / fwd_native * 1e3:.0f} GB/s of compulsory "
              f"traffic) vs torch {fwd_torch:.2f} ms ({fwd_torch / fwd_native:.0f}x); forward+backward native "
              f"{fb_n:.3f} ms vs torch {fb_t:.2f} ms ({fb_t / fb_n:.0f}x)", flush=True)


if __name__ == "__main__":
    main()

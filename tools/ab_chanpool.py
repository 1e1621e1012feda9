"""ChannelPool forward: the one-pixel-per-lane kernel (16-bit types, C <= 128) against the
one-pixel-per-wave kernel it replaced (the A/B build's ADMM_CHANPOOL_WAVE=1), bit-exact on several
value distributions, and both timed at the config-5 caller's shape.
  python tools/ab_chanpool.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torch-admm-deconv_amd"))
import torch  # noqa: E402

from admmtor import _native  # noqa: E402
from admmtor.elayers.attentions import _chanstat_native  # noqa: E402


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


def data(kind, shape, dt, gen):
    if kind == "gauss":
        return torch.randn(shape, generator=gen).to(dt)
    if kind == "gelu":  # activation-like: many near-zero values, so many ties
        return torch.nn.functional.gelu(torch.randn(shape, generator=gen) * 2).to(dt)
    k = 3 if kind == "few" else 40
    return (torch.randint(-k, k + 1, shape, generator=gen).double() / 4).to(dt)


def run(x, wave, depth=None):
    os.environ["ADMM_CHANPOOL_WAVE"] = "1" if wave else "0"
    return _chanstat_native(x, depth)


def main():
    dev = torch.device("cuda:0")
    gen = torch.Generator().manual_seed(0)
    bad = 0
    with _native.ab_library():
        for dt in (torch.bfloat16, torch.float16):
            for C in (1, 2, 17, 33, 64, 65, 86, 127, 128):
                for kind in ("gauss", "gelu", "few", "many"):
                    x = data(kind, (3, C, 33, 47), dt, gen).to(dev)
                    if kind == "many" and C > 2:
                        x[0, 1, 0, :5] = float("nan")
                        x[1, :, 3, 3] = float("nan")
                        x[2, 0, 5, 5] = -0.0
                    for depth in ((None, 0, 2) if C == 86 else (None,)):
                        ow, iw = run(x, True, depth)
                        ol, il = run(x, False, depth)
                        same = torch.equal(iw, il) and torch.equal(ow.view(torch.int16), ol.view(torch.int16))
                        if not same:
                            bad += 1
                            d = (iw != il).nonzero()[:3].tolist()
                            print(f"MISMATCH {dt} C={C} {kind} depth={depth}: idx diffs at {d}", flush=True)
        print(f"bit-exact checks: {bad} mismatches", flush=True)
        for kind in ("gauss", "gelu", "few"):
            x = data(kind, (16, 86, 512, 512), torch.bfloat16, gen).to(dev)
            tw = timed(lambda: run(x, True))
            tl = timed(lambda: run(x, False))
            same = all(torch.equal(a, b) for a, b in zip(run(x, True), run(x, False)))
            print(f"16x86x512x512 bf16 {kind}: wave kernel {tw:.3f} ms, lane kernel {tl:.3f} ms "
                  f"({tw / tl:.1f}x), bit-exact {same}", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()

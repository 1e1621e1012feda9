"""Benchmark of the MI355X ADMM-TV solver on BASELINE.json's metric.

metric : ADMM iterations/sec, batch-64 1024x1024x3, 50 iters (BASELINE.json "metric").
step   : one fft_admm_tv call over the rank's batch-64 shard (64x3x1024^2, 21x21
         Gaussian PSF sigma 3, lambda 0.01, rho 0.02, aniso, 50 iterations), inputs
         resident in HBM; PSF / lambda / rho broadcast from rank 0 over RCCL each step.
value  : whole-job batch-64 ADMM iterations per second = n_gpus * 50 * K / T
         (T = max over ranks of the K-step wall time; weak scaling: 64 images per GPU).

Launch: python bench.py [--gpus N --steps K --warmup W].  N > 1 runs one process per GPU (RCCL
over xGMI): under torch.distributed.run (the driver's launch; --gpus must equal WORLD_SIZE, else
the bench exits with status 2), or, started without it, the bench starts torch.distributed.run
itself as a child process before anything touches the GPU and exits with its status.  Rank 0 prints ONE
JSON line with the roofline of the dominant kernel (HIP events on the launch
stream inside the timed region) and the CPU baseline (the oracle, i.e. the
reference's op sequence restated, timed on a bounded sample on the host cores).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "torch-admm-deconv_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
MFMA_F32_PEAK_TFLOPS = 157.3  # dense f32-input MFMA peak (v_mfma_f32_16x16x4_f32, MI355X_MICROARCH.md)


def mm_col_flops(H, Wh, P):
    """Matrix-core flops per launch of the generic column pass (csrc/gcol_mm.hpp) for columns H = S * R
    (R odd in [17, 127], the largest such factor with S <= 8): per column sequence of R complex values,
    forward and inverse, the cosine and sine products of the (h+1)-point real matrices (h = (R-1)/2),
    padded to 16-row tiles and 4-deep k-steps, on the real and imaginary parts; None without such a plan."""
    Rs = [r for r in range(127, 16, -2) if H % r == 0 and H // r <= 8]
    if not Rs:
        return None
    R = Rs[0]
    S, h = H // R, (R - 1) // 2
    M, K = -(-(h + 1) // 16) * 16, -(-(h + 1) // 4) * 4
    return P * Wh * S * (2 * 2 * 2 * M * K * 2)

CONFIGS = {
    # name: (B, C, H, W, psf kind, k, maxit, iso, description)
    "c3": (64, 3, 1024, 1024, "gauss:3", 21, 50, False,
           "C3/metric: batch-64 1024x1024x3, 21x21 Gaussian PSF (sigma 3), lambda 0.01, rho 0.02, aniso, 50 iters"),
    "c3x100": (64, 3, 1024, 1024, "gauss:3", 21, 100, False,
               "C3 at 100 iters (SURVEY §8 d1): batch-64 1024x1024x3, 21x21 Gaussian PSF, aniso"),
    "c3iso": (64, 3, 1024, 1024, "gauss:3", 21, 50, True,
              "C3 with block (iso) shrinkage, the ADMMDeconv default: batch-64 1024x1024x3, 21x21 PSF, 50 iters"),
    "bsd": (32, 3, 321, 481, "gauss:1.5", 9, 50, False,
            "BSD image size (row f4): batch-32 481x321x3, 9x9 Gaussian PSF, aniso, 50 iters"),
    "hd": (8, 3, 1080, 1920, "gauss:1.5", 9, 50, False,
           "HD frame (row f4): batch-8 1080x1920x3, 9x9 Gaussian PSF, aniso, 50 iters"),
    "uhd": (2, 3, 2160, 3840, "gauss:2", 11, 50, False,
            "4K UHD frame (row f4): batch-2 2160x3840x3, 11x11 Gaussian PSF, aniso, 50 iters"),
    "p720": (16, 3, 720, 1280, "gauss:1.5", 9, 50, False,
             "720p frame (row f4): batch-16 720x1280x3, 9x9 Gaussian PSF, aniso, 50 iters"),
    "vga": (32, 3, 480, 640, "gauss:1.5", 9, 50, False,
            "VGA frame (row f4): batch-32 480x640x3, 9x9 Gaussian PSF, aniso, 50 iters"),
    "sd": (32, 3, 360, 720, "gauss:1.5", 9, 50, False,
           "360x720 frame (row f4): batch-32 360x720x3, 9x9 Gaussian PSF, aniso, 50 iters"),
    "c2": (32, 3, 512, 512, "motion", 15, 50, False,
           "C2: batch-32 512x512x3, 15x15 motion PSF, lambda 0.01, rho 0.02, aniso, 50 iters"),
    "c5fwd": (16, 3, 512, 512, "none", 0, 100, True,
              "C5 forward (one ADMM module): batch-16 512x512x3, no PSF, iso, 100 iters"),
    "c5": (16, 3, 512, 512, "none", 0, 100, True,
           "C5 training step: DivergentRestorer([2,8,32],3,3,86,86,8, Sigmoid, 2 x ADMM-TV iso 100 it) "
           "(scripts/train.py:70-73), batch-16 512x512x3, bf16 autocast, L1 loss, AdamW"),
}

# algorithmic HBM bytes per pixel per launch: pass A reads the x row
# spectrum (4), u_x/u_y (8), b (4) and writes u (8) and the r row spectrum (4); the
# first iteration reads no u.  Pass B reads and writes the spectrum (4 + 4).
PASS_A_BYTES = 28
PASS_A_FIRST_BYTES = 20
PASS_B_BYTES = 8
ISO_NORM_BYTES = 12
# generic sizes: the column pass (half spectra in and out, 8) and the inverse row transform that
# follows it in the same timer (half spectra in 4, x image out 4)
GEN_COL_BYTES = 16
# training backward, reverse row pass (admm_backward.hpp k_bwd_pass_a) per reverse step k: reads the
# r^ spectrum 4, a^_k 8, a_k 8, a_{k-1} 8, b^ 4; writes b^ 4, a^_{k-1} 8, the x^ spectrum 4 = 48;
# k = K reads no a^ and no b^ (36); k = 1 reads no a_{k-1} and writes no a^ / x^ (28)
BWD_ROW_BYTES, BWD_ROW_LAST_BYTES, BWD_ROW_FIRST_BYTES = 48, 36, 28


def path_of(H, W, iso=False, k=0):
    """The kernel path an inference solve of this size takes, from the library (admm_tv_path, host-only):
    "fused", "fused mixed-radix", "fused odd-length" or "generic"."""
    from admmtor import _native
    return _native.path(_native.desc(1, 1, H, W, k, iso, 1))


def labelled(desc, path):
    """A workload label names the kernel path it ran on, taken from the library at run time (never
    written into CONFIGS, where it could go stale)."""
    return f"{desc} [{path} path]"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks, one per GPU (default: WORLD_SIZE under torch.distributed.run, else 1)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-extras", action="store_true",
                    help="c3: skip the extra measurements after the timed region (C3 at 100 iterations, C3 iso, "
                         "the generic-size bsd / hd workloads, the training step)")
    ap.add_argument("--no-c5-extra", action="store_true",
                    help="c3: skip the whole C5 model step after the other extras (its first step compiles MIOpen's "
                         "kernels: minutes on a fresh box)")
    ap.add_argument("--cpu-planes", type=int, default=6, help="CPU baseline sample: planes of 1024^2")
    ap.add_argument("--cpu-iters", type=int, default=36, help="CPU baseline sample: timed iterations")
    ap.add_argument("--batch", type=int, default=None,
                    help="override the per-GPU batch (launch rehearsals only: the line then names a reduced "
                         "workload, config.reduced_batch)")
    ap.add_argument("--c5-batch", type=int, default=None, help="C5 only: override the per-GPU batch")
    ap.add_argument("--c5-no-ckpt", action="store_true", help="C5 only: keep all branch activations")
    ap.add_argument("--c5-channels-last", action="store_true", help="C5 only: NHWC activations (MIOpen NHWC convs)")
    ap.add_argument("--c5-conv-benchmark", action="store_true", help="C5 only: MIOpen find (cudnn.benchmark)")
    return ap.parse_args()


def pmc_traffic(config: str, kernel: str, launches: int, steps: int, build_hash: str):
    """Per-launch HBM traffic of `kernel` from a committed rocprofv3 PMC summary
    (profiles/*_pmc_summary.json, made by tools/pmc/run_rdreq.sh + summarize_rdreq.py: separate
    --pmc passes of the memory-side request-size counters) taken on THIS build: the summary records
    the library's admm_tv_build_hash and names the kernels by role, so a summary of another build
    (other kernels, other template arguments) is never reported.  -> (bytes or None, source)."""
    import glob
    if config not in ("c3", "c3x100"):
        return None, "no PMC summary for this config"
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_summary.json")), reverse=True):
        with open(path) as f:
            summ = json.load(f)
        if summ.get("build_hash") != build_hash or "roles" not in summ:
            continue
        kern, roles = summ["kernels"], summ["roles"]
        src = os.path.relpath(path, ROOT)
        if kernel == "pass_a":
            first = kern.get(roles.get("pass_a_first", ""), {}).get("traffic_bytes")
            rest = kern.get(roles.get("pass_a", ""), {}).get("traffic_bytes")
            if first is None or rest is None or launches < steps:
                return None, src + " (pass A roles missing)"
            return (first * steps + rest * (launches - steps)) / launches, src
        if kernel == "pass_b":
            v = kern.get(roles.get("pass_b", ""), {}).get("traffic_bytes")
            return v, src
        return None, src
    return None, f"no PMC summary of build {build_hash} under profiles/"


def c3_extras(x, psf, lam, rho, no_parity, steps=3):
    """The other C3 figures of SURVEY §8 d1, measured after the headline's timed region on the same
    resident inputs, so one run of the default bench records them all: C3 at 100 iterations
    (BASELINE configs[2]) with its rel-L2 vs the fp64 oracle, and C3 with block (iso) shrinkage,
    the ADMMDeconv default.  One warm-up call, then `steps` calls between synchronisations."""
    from admmtor.eops.deconv import fft_admm_tv
    out = {}
    for key, iso, maxit in (("c3_100it", False, 100), ("c3iso", True, 50)):
        fft_admm_tv(x, lam, rho, psf, iso, maxit)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            o = fft_admm_tv(x, lam, rho, psf, iso, maxit)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        e = {"value": maxit * steps / dt, "unit": "iterations/s", "ms_per_step": dt / steps * 1e3, "steps": steps,
             "maxit": maxit, "iso": iso, "workload": f"batch-{x.shape[0]} 1024x1024x3, 21x21 Gaussian PSF, "
                                                     f"{'iso' if iso else 'aniso'}, {maxit} iters"}
        if not no_parity and not iso:
            from oracle.admm_oracle import rel_l2, solve_fourier
            ref = solve_fourier(x[:1, :1].double().cpu(), 0.01, 0.02, psf.double().cpu(), False, maxit)
            e["rel_l2"] = rel_l2(o[:1, :1].cpu(), ref)
            e["rel_l2_vs"] = "fp64 CPU oracle, plane (0,0)"
        out[key] = e
    return out


def generic_extras(dev, no_parity, keys=("bsd", "hd")):
    """Generic-size path figures on the default line: for each workload one warm-up
    solve, then timed solves on the default two-stream schedule (iterations/s, us per iteration per
    Mpx), the rel-L2 of plane (0, 0) vs the fp64 oracle, and a one-stream profiling pass (ADMM_GEN_STREAMS=1:
    the two streams' launches overlap) for the per-kernel achieved GB/s of the algorithmic bytes."""
    from admmtor import _native
    from admmtor.eops.deconv import fft_admm_tv
    from admmtor.synth import CONFIG_SEED, blurred_batch, make_psf
    out = {}
    for key in keys:
        B, C, H, W, kind, k, maxit, iso, desc = CONFIGS[key]
        psf = make_psf(kind, k).to(dev)
        x = blurred_batch(B, C, H, W, psf.cpu(), seed=CONFIG_SEED + 10, device=dev)
        lam = torch.tensor([0.01], device=dev)
        rho = torch.tensor([0.02], device=dev)
        o = fft_admm_tv(x, lam, rho, psf, iso, maxit)
        torch.cuda.synchronize()
        steps = 10 if B * C * H * W < 20e6 else 4
        t0 = time.perf_counter()
        for _ in range(steps):
            o = fft_admm_tv(x, lam, rho, psf, iso, maxit)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        npx = B * C * H * W
        path = path_of(H, W, iso, k)
        e = {"value": maxit / dt, "unit": "iterations/s", "ms_per_step": dt * 1e3, "steps": steps,
             "us_per_iter_per_Mpx": dt / maxit / (npx / 1e6) * 1e6, "workload": labelled(desc, path), "path": path}
        if not no_parity:
            from oracle.admm_oracle import rel_l2, solve_fourier
            ref = solve_fourier(x[:1, :1].double().cpu(), 0.01, 0.02, psf.double().cpu(), iso, maxit)
            e["rel_l2"] = rel_l2(o[:1, :1].cpu(), ref)
            e["rel_l2_vs"] = "fp64 CPU oracle, plane (0,0)"
        old = os.environ.get("ADMM_GEN_STREAMS")
        os.environ["ADMM_GEN_STREAMS"] = "1"
        try:
            _native.profile_reset()
            _native.profile_enable(True)
            for _ in range(2):
                fft_admm_tv(x, lam, rho, psf, iso, maxit)
            torch.cuda.synchronize()
            _native.profile_enable(False)
            ms, cnt = _native.profile_read()
        finally:
            if old is None:
                del os.environ["ADMM_GEN_STREAMS"]
            else:
                os.environ["ADMM_GEN_STREAMS"] = old
        generic = e["path"] == "generic"  # the fused paths (power-of-two and mixed-radix) keep pass A / B bytes
        ba = (2 * PASS_A_FIRST_BYTES + (cnt[0] - 2) * PASS_A_BYTES) * npx
        bb = cnt[1] * (GEN_COL_BYTES if generic else PASS_B_BYTES) * npx
        per = {}
        for name, t, n, b in (("row_step" if generic else "pass_a", ms[0], cnt[0], ba),
                              ("column_pass" if generic else "pass_b", ms[1], cnt[1], bb)):
            gbs = b / (t / 1e3) / 1e9 if t > 0 else None
            per[name] = {"avg_launch_ms": t / max(n, 1), "launches": n, "algorithmic_bytes_per_launch": b / max(n, 1),
                         "GBps": gbs, "frac": gbs / HBM_PEAK_GBS if gbs else None}
        mm = mm_col_flops(H, W // 2 + 1, B * C) if e["path"] == "fused odd-length" else None
        if mm and per["pass_b"]["avg_launch_ms"] > 0:
            # the matrix-core column pass's own bound: its R-point DFT products on the f32 MFMA
            tf = mm / (per["pass_b"]["avg_launch_ms"] / 1e3) / 1e12
            per["pass_b"]["mfma"] = {"flops_per_launch": mm, "TFLOPs": tf, "peak": MFMA_F32_PEAK_TFLOPS,
                                     "frac": tf / MFMA_F32_PEAK_TFLOPS}
        e["roofline_one_stream"] = {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s", "per_kernel": per,
                                    "timing": "HIP events, 2 solves on one stream after the timed solves"}
        out[key] = e
        del x, o
    return out


def train_extra(dev, steps=3):
    """The training path (BASELINE configs[4]: autograd through the HIP op; reference: plain autograd
    through deconv.py:103-115): one ADMMDeconv module at the C5 shape (batch-16 512x512x3, iso, no PSF,
    100 iterations, learnable lambda / rho, seeded init), forward with history (admm_tv_forward_train) +
    backward (admm_tv_backward) per step, timed with HIP events on torch's stream (where the op launches);
    the reverse row pass's achieved GB/s from the library's per-launch events against its algorithmic
    bytes (BWD_ROW_*)."""
    from admmtor import _native
    from admmtor.elayers.admmdeconv import ADMMDeconv
    from admmtor.synth import CONFIG_SEED, blurred_batch
    B, C, H, W, K = 16, 3, 512, 512, 100
    torch.manual_seed(CONFIG_SEED + 5)
    m = ADMMDeconv((), max_iters=K, iso=True).to(dev)
    x = blurred_batch(B, C, H, W, torch.empty(0), seed=CONFIG_SEED + 5, device=dev).requires_grad_(True)
    v = torch.randn(x.shape, generator=torch.Generator(device=dev).manual_seed(3), device=dev)
    fwd_ms, bwd_ms = [], []
    prof = None
    for i in range(1 + steps):
        m.zero_grad(set_to_none=True)
        x.grad = None
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record()
        out = m(x)
        loss = (out * v).sum()
        e1.record()
        if i == steps:  # the last step's backward with the library's per-launch events
            _native.profile_reset()
            _native.profile_enable(True)
        loss.backward()
        e2.record()
        torch.cuda.synchronize()
        if i == steps:
            _native.profile_enable(False)
            prof = _native.profile_read()
        if i > 0:
            fwd_ms.append(e0.elapsed_time(e1))
            bwd_ms.append(e1.elapsed_time(e2))
    ms, cnt = prof
    npx = B * C * H * W
    nrow = cnt[0]
    brow = ((nrow - 2) * BWD_ROW_BYTES + BWD_ROW_LAST_BYTES + BWD_ROW_FIRST_BYTES) * npx if nrow >= 2 else 0
    gbs = brow / (ms[0] / 1e3) / 1e9 if ms[0] > 0 else None
    f, b = sum(fwd_ms) / steps, sum(bwd_ms) / steps
    return {"train": {"workload": "one ADMMDeconv module at the C5 shape: batch-16 512x512x3, iso, no PSF, 100 iters, "
                                  "learnable lambda/rho, fp32 solve; forward with history + backward",
                      "ms_per_step": f + b, "fwd_train_ms": f, "bwd_ms": b, "steps": steps,
                      "steps_per_s": 1e3 / (f + b),
                      "bwd_row_pass": {"avg_launch_ms": ms[0] / max(nrow, 1), "launches": nrow,
                                       "algorithmic_bytes_per_launch": brow / max(nrow, 1), "GBps": gbs,
                                       "frac": gbs / HBM_PEAK_GBS if gbs else None, "bound": "hbm"},
                      "bwd_kernel_ms": {"row_pass": ms[0], "column_pass": ms[1], "iso_q": ms[2]},
                      "grads_finite": bool(torch.isfinite(x.grad).all() and torch.isfinite(m.lmbda.grad).all()
                                           and torch.isfinite(m.rho.grad).all())}}


def cpu_baseline(cfg, planes, iters):
    """Oracle (reference op sequence: circular pad + depthwise conv operators, H_t
    recomputed every iteration, torch.fft x-update) on a bounded sample, on host cores."""
    from oracle.admm_oracle import solve_spatial
    from admmtor.synth import blurred_batch, make_psf
    B, C, H, W, kind, k, maxit, iso, _ = cfg
    ncores = len(os.sched_getaffinity(0))
    torch.set_num_threads(min(ncores, int(os.environ.get("OMP_NUM_THREADS", ncores))))
    psf = make_psf(kind, k)
    nb = max(1, planes // C)
    x = blurred_batch(nb, C, H, W, psf, seed=99)
    solve_spatial(x, 0.01, 0.02, psf, iso, 1)  # warm-up
    t0 = time.perf_counter()
    solve_spatial(x, 0.01, 0.02, psf, iso, iters)
    dt = time.perf_counter() - t0
    it_s_sample = iters / dt
    # the metric's unit is iterations/s for the whole batch: scale by the plane ratio
    value = it_s_sample * (nb * C) / (B * C)
    cpu = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": value, "unit": "batch-equivalent ADMM iterations/s", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": f"{nb}x{C}x{H}x{W} ({nb * C} of {B * C} planes), {iters} iterations after 1 warm-up, "
                      f"{dt:.1f} s; oracle/admm_oracle.py solve_spatial (reference op sequence), "
                      f"value scaled by planes {nb * C}/{B * C}; CPU: {cpu}"}


def cpu_baseline_c5(H=128, B=1, steps=2):
    """C5 on the host cores: the same training step (DivergentRestorer, two learnable iso ADMM
    modules of 100 iterations, L1 loss, AdamW) in fp32 on a bounded sample, with the solver
    routed to the oracle's restatement of the reference op sequence (solve_spatial, autograd
    through it, as the reference trains) -- the reference's CPU path.  Scaled by pixels to the
    C5 batch (16 x 3 x 512^2)."""
    import admmtor.elayers.admmdeconv as admmdeconv
    from admmtor.modelbuild.denoiser import DivergentRestorer
    from admmtor.synth import CONFIG_SEED, clean_images
    from oracle.admm_oracle import solve_spatial
    ncores = len(os.sched_getaffinity(0))
    torch.set_num_threads(min(ncores, int(os.environ.get("OMP_NUM_THREADS", ncores))))
    Bc, C, Hc, Wc, _, _, maxit, _, _ = CONFIGS["c5"]
    solver = admmdeconv.fft_admm_tv
    admmdeconv.fft_admm_tv = lambda x, l, r, k, iso, it: solve_spatial(x, l, r, k, iso, it)
    try:
        deconv = {"kern_size": (), "max_iters": maxit, "iso": True}
        torch.manual_seed(CONFIG_SEED + 5)
        model = DivergentRestorer([2, 8, 32], 3, 3, 86, 86, 8, output_activation=torch.nn.Sigmoid(),
                                  admms=[dict(deconv), dict(deconv)])
        opt = torch.optim.AdamW(model.parameters(), 8.8e-4, betas=(0.9, 0.9))
        y = clean_images(B, C, H, H, seed=CONFIG_SEED + 5)
        x = (y + 0.06 * torch.randn(y.shape, generator=torch.Generator().manual_seed(5))).clamp_(0, 1)

        def step():
            opt.zero_grad(set_to_none=True)
            loss = (model(x) - y).abs().mean()
            loss.backward()
            opt.step()
        step()  # warm-up
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        dt = (time.perf_counter() - t0) / steps
    finally:
        admmdeconv.fft_admm_tv = solver
    scale = (B * H * H) / (Bc * Hc * Wc)
    return {"value": scale / dt, "unit": "C5-equivalent training steps/s", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": f"{B}x{C}x{H}x{H} fp32, {steps} steps after 1 warm-up, {dt:.2f} s/step; solver = "
                      f"oracle/admm_oracle.py solve_spatial (reference op sequence, autograd), CNN = this "
                      f"build's state-dict-compatible modules on the CPU; value scaled by pixels "
                      f"{B * H * H}/{Bc * Hc * Wc}"}


def c5_session(dev, B, rank=0, world=1, ckpt=True, channels_last=False, conv_benchmark=False):
    """The config-5 training step (scripts/train.py:70-73): DivergentRestorer with two learnable iso ADMM-TV
    modules of 100 iterations, bf16 autocast, L1 loss, AdamW; autograd through the HIP solver.  Returns
    step() -> loss.  ckpt: the 8- and 32-branch levels recompute their branches in the backward (exact;
    without it the activations of batch 16 at 512^2 exceed 288 GB -- measured: OOM at 282 GiB allocated)."""
    from admmtor.modelbuild.blocks import set_branch_checkpointing
    from admmtor.modelbuild.denoiser import DivergentRestorer
    from admmtor.synth import CONFIG_SEED, clean_images
    _, C, H, W, _, _, maxit, _, _ = CONFIGS["c5"]
    deconv = {"kern_size": (), "max_iters": maxit, "iso": True}
    torch.manual_seed(CONFIG_SEED + 5)
    model = DivergentRestorer([2, 8, 32], 3, 3, 86, 86, 8, output_activation=torch.nn.Sigmoid(),
                              admms=[dict(deconv), dict(deconv)]).to(dev)
    if ckpt:
        set_branch_checkpointing(model, True)
    if channels_last:
        model = model.to(memory_format=torch.channels_last)
    if world > 1:
        model = torch.nn.parallel.DistributedDataParallel(model, device_ids=[dev.index],
                                                          find_unused_parameters=True)
    opt = torch.optim.AdamW(model.parameters(), 8.8e-4, betas=(0.9, 0.9))
    y = clean_images(B, C, H, W, seed=CONFIG_SEED + 5 + 1000 * rank, device=dev)
    g = torch.Generator(device=dev).manual_seed(CONFIG_SEED + 5 + rank)
    x = (y + 0.06 * torch.randn(y.shape, generator=g, device=dev)).clamp_(0, 1)
    if conv_benchmark:
        torch.backends.cudnn.benchmark = True
    if channels_last:
        x = x.contiguous(memory_format=torch.channels_last)
        y = y.contiguous(memory_format=torch.channels_last)

    def step():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = model(x)
        loss = (out.float() - y).abs().mean()
        loss.backward()
        opt.step()
        return loss
    return step


def heartbeat(tag):
    """stderr progress every 30 s (the first C5 step compiles MIOpen's kernels: minutes on a fresh box)."""
    import threading
    t_start = time.time()

    def beat():
        while True:
            time.sleep(30)
            print(f"{tag} alive {time.time() - t_start:.0f} s", file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()


def c5_extra(dev, steps=2, warmup=1):
    """The whole config-5 model step on the default line: steps/s, the ADMM kernels'
    share of it (the library's per-launch events) and the peak memory, at the full 16x3x512^2 shape, after
    the other extras (their tensors freed)."""
    from admmtor import _native
    B, C, H, W, _, _, maxit, _, desc = CONFIGS["c5"]
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats(dev)
    step = c5_session(dev, B)
    heartbeat("c5 extra")
    t0 = time.perf_counter()
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t_warm = time.perf_counter() - t0
    _native.profile_reset()
    _native.profile_enable(True)
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    torch.cuda.synchronize()
    T = time.perf_counter() - t0
    _native.profile_enable(False)
    ms, cnt = _native.profile_read()
    return {"c5": {"workload": desc, "value": steps / T, "unit": "steps/s", "ms_per_step": T / steps * 1e3,
                   "steps": steps, "warmup": warmup, "warmup_s": t_warm, "dtype": "bf16 autocast (ADMM solve f32)",
                   "admm_share": {"ms_per_step_in_admm_kernels": sum(ms) / steps,
                                  "fraction": sum(ms) / 1e3 / T, "launches_per_step": sum(cnt) / steps},
                   "peak_mem_GiB": torch.cuda.max_memory_allocated(dev) / 2**30,
                   "loss_finite": bool(torch.isfinite(loss.detach()))}}


def run_c5(args, world, rank, dev):
    """Config 5: one training step of the reference's training model
    (scripts/train.py:70-73: two learnable iso ADMM-TV modules, 100 iterations each, then the
    attention CNN), autograd through the HIP solver.  The reference trains with an SSIM-Lab loss
    from its metrics package (out of scope); the step here uses L1 -- the loss is a few
    elementwise ops next to the model.  N > 1: DDP over RCCL (gradient all-reduce, a real exchange
    step), weak scaling (batch 16 per GPU)."""
    from admmtor import _native
    B, C, H, W, _, _, maxit, _, desc = CONFIGS["c5"]
    reduced = (args.c5_batch or args.batch) is not None and (args.c5_batch or args.batch) != B
    B = args.c5_batch or args.batch or B
    if reduced:  # launch rehearsals only; the line names the reduced workload
        desc += f" [REDUCED: batch {B} per GPU]"
    step = c5_session(dev, B, rank, world, not args.c5_no_ckpt, args.c5_channels_last, args.c5_conv_benchmark)
    if rank == 0:
        heartbeat("c5")
    for i in range(args.warmup):
        step()
        torch.cuda.synchronize()
        if rank == 0:
            print(f"c5 warmup step {i + 1}/{args.warmup} done", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    _native.profile_reset()
    _native.profile_enable(True)
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = step()
        if rank == 0:  # progress for long runs (host-side only: no sync inside the timed region)
            print(f"c5 step {i + 1}/{args.steps} enqueued", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    _native.profile_enable(False)
    ms, cnt = _native.profile_read()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    T = elapsed.item()
    K = args.steps
    if rank == 0:
        admm_ms = sum(ms)
        print(json.dumps({
            "metric": "C5 training steps/sec", "value": world * K / T, "unit": "steps/s", "n_gpus": world,
            "steps": K, "warmup": args.warmup, "ms_per_step": T / K * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16 autocast (ADMM solve f32)",
            "data": "synthetic (piecewise-constant shapes + AWGN 0.06, seeded per rank); random-init weights",
            "config": {"workload": desc, "batch_per_gpu": B, "reduced_batch": reduced, "H": H, "W": W,
                       "branch_checkpointing": not args.c5_no_ckpt,
                       "channels_last": bool(args.c5_channels_last), "conv_benchmark": bool(args.c5_conv_benchmark),
                       "parallelism": f"ddp{world}" if world > 1 else "single"},
            "admm_share": {"ms_per_step_in_admm_kernels": admm_ms / K, "fraction": admm_ms / 1e3 / T,
                           "launches_per_step": sum(cnt) / K},
            "peak_mem_GiB": torch.cuda.max_memory_allocated(dev) / 2**30,
            "loss": float(loss.detach()),
            "cpu_baseline": cpu_baseline_c5() if (world == 1 and not args.no_cpu_baseline) else None}),
              flush=True)


def resolve_world(gpus, env):
    """(world size, launch ranks?) from --gpus and the environment, before any GPU call.
    Under torch.distributed.run WORLD_SIZE is set and --gpus (if given) must equal it; without it,
    --gpus N > 1 means this process launches the N ranks.  A mismatch raises SystemExit(2)."""
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if gpus is not None and gpus != int(ws):
            print(f"bench.py: --gpus {gpus} but WORLD_SIZE={ws} (torch.distributed.run --nproc-per-node); "
                  "they must be equal", file=sys.stderr, flush=True)
            raise SystemExit(2)
        return int(ws), False
    n = 1 if gpus is None else gpus
    if n < 1:
        print(f"bench.py: --gpus {n} must be >= 1", file=sys.stderr, flush=True)
        raise SystemExit(2)
    return n, n > 1


def launch_cmd(n, argv, port):
    """The child that runs the N ranks: torch.distributed.run on this same script, on 127.0.0.1."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def launch_ranks(n, argv):
    """Start the N rank processes as ONE child process tree (torch.distributed.run) and return its
    exit status.  Called before this process touches the GPU (torch.cuda.device_count() does not
    initialise it on this image), and the ranks are children, never an exec of this process."""
    import socket
    import subprocess
    rehearsal = bool(os.environ.get("ADMM_BENCH_REHEARSAL"))
    ndev = torch.cuda.device_count()
    if not rehearsal and n > ndev:
        print(f"bench.py: --gpus {n} but {ndev} GPU(s) visible", file=sys.stderr, flush=True)
        return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ)
    print(f"bench.py: launching {n} ranks (torch.distributed.run, port {port})", file=sys.stderr, flush=True)
    return subprocess.run(launch_cmd(n, argv, port), env=env).returncode


def rocfft_rank_cache(local_rank):
    """Give this rank its own rocFFT kernel cache before anything touches the GPU.

    rocFFT keeps the kernels it compiles at run time in a per-user sqlite database (WAL journal) that every
    process of the user opens.  In the round-5 rehearsal the ranks stalled at their first device FFT when the
    parent process (a pytest run) had used rocFFT before launching them: a process that keeps the database
    open holds its read snapshot, and a writer's WAL checkpoint then waits for it.  Each rank now uses a
    cache file of its own (ROCFFT_RTC_CACHE_PATH, unless the caller set one); the shipped read-only system
    cache is unaffected."""
    if "ROCFFT_RTC_CACHE_PATH" not in os.environ:
        import tempfile
        os.environ["ROCFFT_RTC_CACHE_PATH"] = os.path.join(
            tempfile.gettempdir(), f"admmtor_rocfft_uid{os.getuid()}_rank{local_rank}.db")


def main():
    args = parse()
    world, launch = resolve_world(args.gpus, os.environ)
    if launch:
        sys.exit(launch_ranks(world, sys.argv[1:]))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        rocfft_rank_cache(local)
        # rehearsal on a 1-GPU box (never set by the driver): every rank on cuda:0 over gloo
        if os.environ.get("ADMM_BENCH_REHEARSAL"):
            local = 0
        torch.cuda.set_device(local)
        dist.init_process_group("gloo" if os.environ.get("ADMM_BENCH_REHEARSAL") else "nccl")
    dev = torch.device("cuda", local)
    if args.config == "c5":
        run_c5(args, world, rank, dev)
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return
    cfg = CONFIGS[args.config]
    if args.batch is not None:  # launch rehearsals only; the line names the reduced workload
        cfg = (args.batch,) + cfg[1:8] + (cfg[8] + f" [REDUCED: batch {args.batch} per GPU]",)
    B, C, H, W, kind, k, maxit, iso, desc = cfg

    from admmtor import _native
    lib_override = os.environ.get("ADMMTOR_LIB_OVERRIDE")  # A/B tooling (tools/gpu_ab_env.sh) only
    if lib_override:
        _native.use_library(lib_override)
    from admmtor.sharded import sharded_fft_admm_tv
    from admmtor.synth import CONFIG_SEED, blurred_batch, make_psf

    def progress(msg):  # multi-rank runs: rank 0's stages on stderr (a slow start stays visible)
        if world > 1 and rank == 0:
            print(f"bench rank 0/{world}: {msg}", file=sys.stderr, flush=True)

    progress("process group up")
    # rank-local shard of synthetic blurred images: in HBM directly at N = 1; with N > 1 synthesised on the
    # host and copied in, so the ranks run no torch.fft of their own.  Round 6 synthesised on the device
    # with a rocFFT kernel cache per rank (rocfft_rank_cache, still set): the 8-rank rehearsal passed once,
    # then stalled again after "inputs generated" with ranks missing at the next collective.
    psf = make_psf(kind, k).to(dev) if k else torch.empty(0, device=dev)
    syn_dev = dev if world == 1 else torch.device("cpu")
    x = blurred_batch(B, C, H, W, psf.cpu(), seed=CONFIG_SEED + 2 + 1000 * rank, device=syn_dev).to(dev)
    lam = torch.tensor([0.01], device=dev)
    rho = torch.tensor([0.02], device=dev)
    torch.cuda.synchronize()
    progress("inputs generated")

    # N > 1: the north star's final gather of the whole output over xGMI runs on a side stream and its
    # own process group (its own RCCL communicator / stream), so step k's all_gather overlaps step
    # k+1's solve (pipelined; every gather completes inside the timed region); double-buffered.
    gather_pg = dist.new_group(list(range(world))) if world > 1 else None
    comm = torch.cuda.Stream(device=dev) if world > 1 else None
    gbufs = [torch.empty((world * B, C, H, W), dtype=torch.float32, device=dev) for _ in range(2)] \
        if world > 1 else None
    rehearsal = bool(os.environ.get("ADMM_BENCH_REHEARSAL"))
    nstep = [0]

    def step():
        # RCCL broadcast of PSF / lambda / rho from rank 0 (no-op at N=1), then the local shard
        out = sharded_fft_admm_tv(x, lam, rho, psf, iso, maxit)
        if world > 1:
            buf = gbufs[nstep[0] % 2]
            nstep[0] += 1
            comm.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(comm):
                if rehearsal:  # gloo: list all_gather
                    dist.all_gather(list(buf.chunk(world, 0)), out, group=gather_pg)
                else:
                    dist.all_gather_into_tensor(buf, out, group=gather_pg)
            out.record_stream(comm)
        return out

    progress("inputs ready")
    for _ in range(args.warmup):
        out = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    progress("warm-up done")
    _native.profile_reset()
    _native.profile_enable(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    _native.profile_enable(False)
    ms, cnt = _native.profile_read()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    T = elapsed.item()
    progress(f"timed region done ({T:.2f} s)")

    P = B * C
    npx = P * H * W
    K = args.steps
    lib = _native.load()
    build_hash = lib.admm_tv_build_hash().decode()
    path = path_of(H, W, iso, k)
    generic = path == "generic"
    odd = path == "fused odd-length"
    # The generic aniso inference solve runs two plane halves on two streams (ADMM_GEN_STREAMS): the
    # event times of its launches overlap and do not add up to kernel durations.  Its roofline then
    # comes from a separate profiling pass of the same solve on one stream (after the timed region;
    # the headline value is the timed region's).
    two_stream = (generic or odd) and not iso and P >= 2 and os.environ.get("ADMM_GEN_STREAMS", "2") != "1"
    roof_steps, roof_note = K, "HIP events of every launch inside the timed region"
    if two_stream:
        roof_steps = min(K, 5)
        os.environ["ADMM_GEN_STREAMS"] = "1"
        try:
            _native.profile_reset()
            _native.profile_enable(True)
            for _ in range(roof_steps):
                sharded_fft_admm_tv(x, lam, rho, psf, iso, maxit)
            torch.cuda.synchronize()
            _native.profile_enable(False)
            ms, cnt = _native.profile_read()
        finally:
            del os.environ["ADMM_GEN_STREAMS"]
        roof_note = (f"HIP events of a one-stream profiling pass ({roof_steps} solves, ADMM_GEN_STREAMS=1) after the "
                     "timed region: the timed solves run two plane halves on two streams, whose launches overlap")
    # roofline of the dominant kernel: algorithmic bytes of all its launches / its event time.
    # Fused path: pass A (row pass) and pass B (column pass).  Generic path: the row pass with the
    # fused step (same 28 / 20 B/px) and the column pass with the inverse row transform (16 B/px).
    na = cnt[0]
    bytes_a = ((roof_steps * PASS_A_FIRST_BYTES + (na - roof_steps) * PASS_A_BYTES) * npx if na >= roof_steps
               else na * PASS_A_BYTES * npx)
    gen_col = GEN_COL_BYTES
    bytes_b = cnt[1] * (gen_col if generic else PASS_B_BYTES) * npx
    names = ("row_step", "column_pass") if generic else ("pass_a", "pass_b")
    kern = {
        names[0]: (ms[0], na, bytes_a),
        names[1]: (ms[1], cnt[1], bytes_b),
    }
    if iso:
        kern["iso_norm"] = (ms[2], cnt[2], cnt[2] * ISO_NORM_BYTES * npx)
    dom = max(kern, key=lambda n: kern[n][0])
    dms, dn, dbytes = kern[dom]
    achieved = (dbytes / (dms / 1e3)) / 1e9 if dms > 0 else 0.0

    traffic, traffic_src = pmc_traffic(args.config, dom, dn, roof_steps, build_hash)
    parity = None
    if rank == 0 and not args.no_parity:
        from oracle.admm_oracle import rel_l2, solve_fourier
        ref = solve_fourier(x[:1, :1].double().cpu(), 0.01, 0.02, psf.double().cpu(), iso, maxit) \
            if not iso else None
        if ref is not None:
            parity = {"rel_l2": rel_l2(out[:1, :1].cpu(), ref),
                      "vs": "fp64 CPU oracle (pinned to the reference), plane (0,0) of the last step"}
    extras = {}
    if rank == 0 and world == 1 and args.config == "c3" and not args.no_extras:
        extras = c3_extras(x, psf, lam, rho, args.no_parity)
        del out, x  # free the C3 batch before the other workloads
        torch.cuda.empty_cache()
        extras.update(generic_extras(dev, args.no_parity))
        extras.update(train_extra(dev))
        if not args.no_c5_extra:
            extras.update(c5_extra(dev))
    result = None
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(cfg, args.cpu_planes, args.cpu_iters)
        value = world * maxit * K / T
        it_bytes = (PASS_A_BYTES + (gen_col if generic else PASS_B_BYTES) + (ISO_NORM_BYTES if iso else 0)) * npx
        result = {
            "metric": "ADMM iterations/sec, batch-64 1024x1024x3, 50 iters; rel-L2 vs CPU ref"
            if args.config == "c3" else f"ADMM iterations/sec ({args.config})",
            "value": value,
            "unit": "iterations/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": T / K * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (piecewise-constant shapes, circular blur, AWGN 0.01; seeded per rank)",
            "config": {"workload": labelled(desc, path), "path": path, "batch_per_gpu": B, "reduced_batch": args.batch is not None, "channels": C, "H": H, "W": W, "psf": f"{kind}/{k}",
                       "maxit": maxit, "iso": iso,
                       "parallelism": (f"shard{world} (batch sharded; RCCL broadcast of PSF/lambda/rho per step and "
                                       "the final all_gather of every step's output inside the timed region, on a "
                                       "side stream overlapping the next step's solve"
                                       + (", per-iteration all_reduce of the iso norms" if iso else "") + ")")
                       if world > 1 else "shard1 (single GPU, no collective)"},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_unit": "bytes/launch",
                         "traffic_source": traffic_src, "build_hash": build_hash, "timing": roof_note,
                         "library": os.path.relpath(_native.lib_path(), ROOT),
                         "launches": dn, "avg_launch_ms": dms / max(dn, 1),
                         "algorithmic_bytes_per_launch": dbytes / max(dn, 1),
                         "per_kernel": {n: {"ms_total": v[0], "launches": v[1],
                                            "GBps": (v[2] / (v[0] / 1e3) / 1e9) if v[0] > 0 else None}
                                        for n, v in kern.items()}},
            "iteration_roofline": {"bytes_per_iter": it_bytes, "it_s_at_peak": HBM_PEAK_GBS * 1e9 / it_bytes},
            "parity": parity,
            "cpu_baseline": cpu,
        }
        result.update(extras)
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

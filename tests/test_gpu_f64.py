"""fp64 inputs are solved in fp64 (ADMM_TV_FLAG_F64), as the reference computes in xin.dtype
(/root/reference/src/admmtor/eops/deconv.py:49,61-67,104-106; its notebook feeds fp64 tensors,
test_torch_admm.ipynb:249).

The fp64 solve runs on the generic kernels' double instantiation (include/admm_tv.h *_f64 entry
points).  Gates (relative L2):
  * 1e-12 against the reference's own fp64 outputs where the goldens store them in fp64 (g4, g5,
    g6, g7) and against the fp64 oracle (pinned to the reference at <= 1e-10 by
    tests/test_oracle_golden.py; its restatement of the reference is exact to ~1e-14) where the
    goldens keep the fp64 result rounded to fp32 (g1, g2, g3, g10) -- those are checked at 2e-7, the
    rounding of their storage;
  * gradients (x, lambda, rho, PSF) vs the reference's fp64 autograd: 1e-9.
"""
import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu

TOL64 = 1e-12
TOL64_GRAD = 1e-9
TOL_STORED32 = 2e-7  # an fp64 reference stored rounded to fp32


def rel(a, b):
    a = torch.as_tensor(a).double().cpu().reshape(-1)
    b = torch.as_tensor(b).double().cpu().reshape(-1)
    return (torch.linalg.vector_norm(a - b) / torch.linalg.vector_norm(b)).item()


def solve64(x, psf, lam, rho, iso, it, dev):
    from admmtor.eops.deconv import fft_admm_tv
    x = torch.as_tensor(x).double().to(dev)
    k = torch.as_tensor(psf).double().to(dev) if psf is not None else torch.empty(0, dtype=torch.float64, device=dev)
    out = fft_admm_tv(x, lam, rho, k, iso, it)
    torch.cuda.synchronize()
    assert out.dtype == torch.float64 and out.device == x.device
    return out


def oracle64(x, psf, lam, rho, iso, it):
    from oracle.admm_oracle import solve_fourier
    x = torch.as_tensor(x).double().cpu()
    k = torch.as_tensor(psf).double() if psf is not None else torch.empty(0, dtype=torch.float64)
    return solve_fourier(x, lam, rho, k, iso, it)


def test_f64_g1_g2_g3(cuda_dev):
    g = load_golden("g1_c1")
    out = solve64(g["x"], g["psf"], 0.01, 0.02, False, 30, cuda_dev)
    e_o, e_r = rel(out, oracle64(g["x"], g["psf"], 0.01, 0.02, False, 30)), rel(out, g["ref64"])
    print("g1 fp64: vs oracle", e_o, "vs stored ref64", e_r)
    assert e_o <= TOL64 and e_r <= TOL_STORED32
    g = load_golden("g2_motion")
    for iso in (False, True):
        out = solve64(g["x"], g["psf"], 0.01, 0.02, iso, 50, cuda_dev)
        e_o = rel(out, oracle64(g["x"], g["psf"], 0.01, 0.02, iso, 50))
        e_r = rel(out, g["ref64_iso" if iso else "ref64_aniso"])
        print("g2 fp64 iso" if iso else "g2 fp64 aniso", e_o, e_r)
        assert e_o <= TOL64 and e_r <= TOL_STORED32
    g = load_golden("g3_c3")
    out = solve64(g["x"], g["psf"], 0.01, 0.02, False, 100, cuda_dev)
    e_o, e_r = rel(out, oracle64(g["x"], g["psf"], 0.01, 0.02, False, 100)), rel(out, g["ref64"])
    print("g3 fp64 100 it", e_o, e_r)
    assert e_o <= TOL64 and e_r <= TOL_STORED32


def test_f64_g6_first_iterations(cuda_dev):
    g = load_golden("g6_inter")
    for it, key in ((1, "x_it1"), (2, "x_it2")):
        out = solve64(g["x"], g["psf"], 0.01, 0.02, False, it, cuda_dev)
        e = rel(out, g[key])
        print("g6 fp64", key, e)
        assert e <= TOL64, key


def test_f64_g7_edges(cuda_dev):
    e = load_golden("g7_edges")
    out0 = solve64(e["m0_x"], e["m0_psf"], 0.01, 0.02, False, 0, cuda_dev)
    assert torch.count_nonzero(out0).item() == 0
    cases = [("m1", e["m0_x"], e["m0_psf"], 0.01, 0.02, False, 1, e["m1_out"]),
             ("odd 15x17, 4x4 PSF", e["odd_x"], e["odd_psf"], 0.01, 0.02, False, 20, e["odd_out"]),
             ("no PSF iso", e["noPSF_iso_x"], None, 0.03, 0.05, True, 40, e["noPSF_iso_out"]),
             ("even 4x4 PSF", e["even4_x"], e["even4_psf"], 0.01, 0.02, False, 25, e["even4_out"]),
             ("rect aniso", e["rect_x"], e["rect_psf"], 0.01, 0.02, False, 30, e["rect_out_aniso"]),
             ("rect iso", e["rect_x"], e["rect_psf"], 0.01, 0.02, True, 30, e["rect_out_iso"])]
    for name, x, k, lam, rho, iso, it, ref in cases:
        out = solve64(x, k, lam, rho, iso, it, cuda_dev)
        err = rel(out, ref)
        print("g7 fp64", name, err)
        assert err <= TOL64, name


def _grads64(x, psf, lam, rho, iso, it, cot, dev, psf_grad=False):
    from admmtor.eops.deconv import fft_admm_tv
    x = torch.as_tensor(x).double().to(dev).requires_grad_(True)
    lam_t = torch.tensor([float(np.asarray(lam).reshape(-1)[0])], dtype=torch.float64, device=dev, requires_grad=True)
    rho_t = torch.tensor([float(np.asarray(rho).reshape(-1)[0])], dtype=torch.float64, device=dev, requires_grad=True)
    k = torch.as_tensor(psf).double().to(dev) if psf is not None else torch.empty(0, dtype=torch.float64, device=dev)
    if psf_grad:
        k.requires_grad_(True)
    out = fft_admm_tv(x, lam_t, rho_t, k, iso, it)
    inputs = (x, lam_t, rho_t) + ((k,) if psf_grad else ())
    grads = torch.autograd.grad(out, inputs, torch.as_tensor(cot).double().to(dev))
    torch.cuda.synchronize()
    assert all(gr.dtype == torch.float64 for gr in grads)
    return (out.detach(),) + tuple(grads)


def test_f64_g4_train_config_grads(cuda_dev):
    g = load_golden("g4_train_grad")
    out, gx, gl, gr = _grads64(g["x"], None, g["lam"], g["rho"], True, 100, g["cot"], cuda_dev)
    e = (rel(out, g["out"]), rel(gx, g["gx"]), rel(gl, g["glam"]))
    print("g4 fp64 out/gx/glam", e, "grho", gr.item(), g["grho"])
    assert e[0] <= TOL64 and e[1] <= TOL64_GRAD and e[2] <= TOL64_GRAD
    # rho's gradient is ~1e-10-size in this config: absolute
    assert abs(gr.item() - float(g["grho"][0])) <= 1e-9 * max(1.0, abs(gl.item()))


@pytest.mark.parametrize("iso", [False, True])
def test_f64_g5_psf_grads(cuda_dev, iso):
    g = load_golden("g5_psf_grad")
    tag = "iso" if iso else "aniso"
    out, gx, gl, gr, gk = _grads64(g["x"], g["psf"], g["lam"], g["rho"], iso, 20, g[f"cot_{tag}"], cuda_dev,
                                   psf_grad=True)
    e = (rel(out, g[f"out_{tag}"]), rel(gx, g[f"gx_{tag}"]), rel(gl, g[f"glam_{tag}"]), rel(gr, g[f"grho_{tag}"]),
         rel(gk, g[f"gpsf_{tag}"]))
    print("g5 fp64", tag, "out/gx/glam/grho/gpsf", e)
    assert e[0] <= TOL64
    assert max(e[1:]) <= TOL64_GRAD


@pytest.mark.parametrize("shape,psf,iso", [
    ((2, 3, 64, 128), ("gauss:2", 9), False),    # power of two: fp64 runs on the generic kernels too
    ((1, 2, 97, 101), ("motion", 7), True),      # primes (the any-prime stage)
    ((1, 1, 5, 7), ("gauss:1.0", 3), False),
    ((2, 1, 1, 64), ("none", 0), True),          # one-row planes
    ((1, 1, 121, 250), ("gauss:1.5", 9), False),
])
def test_f64_shapes_vs_oracle(cuda_dev, shape, psf, iso):
    from admmtor.synth import blurred_batch, make_psf
    k = make_psf(psf[0], psf[1], dtype=torch.float64)
    x = blurred_batch(*shape, k.float(), seed=8).double()
    kk = k if k.numel() else None
    out = solve64(x, kk, 0.01, 0.02, iso, 25, cuda_dev)
    e = rel(out, oracle64(x, kk, 0.01, 0.02, iso, 25))
    print(shape, psf, iso, e)
    assert e <= TOL64


def test_f64_notebook_host_call(cuda_dev):
    """test_torch_admm.ipynb:249 with fp64 host tensors (numpy-derived): fp64 back on the host."""
    from admmtor.eops.deconv import fft_admm_tv
    g = load_golden("g10_notebook")
    x = torch.from_numpy(g["nb249_x"].astype(np.float64))
    k = torch.from_numpy(g["nb249_k"].astype(np.float64))
    out = fft_admm_tv(x, 0.02, 0.02, k, True, 300)
    assert out.dtype == torch.float64 and out.device.type == "cpu"
    e_o, e_r = rel(out, oracle64(x, k, 0.02, 0.02, True, 300)), rel(out, g["nb249_ref64"])
    print("notebook 249 fp64: vs oracle", e_o, "vs stored ref64", e_r)
    assert e_o <= TOL64 and e_r <= TOL_STORED32


def test_f64_module_and_fp32_unchanged(cuda_dev):
    """ADMMDeconv on fp64 inputs (parameters cast with the input, as torch modules do with .double()),
    and fp32 inputs still take the fp32 kernels (their result is not the fp64 one)."""
    from admmtor.elayers.admmdeconv import ADMMDeconv
    from admmtor.synth import blurred_batch, make_psf
    torch.manual_seed(3)
    m = ADMMDeconv((5, 5), max_iters=20, lmbda=0.02, rho=0.04, iso=False).to(cuda_dev).double()
    x = blurred_batch(2, 3, 48, 40, make_psf("gauss:1.5", 5), seed=2).double().to(cuda_dev)
    out = m(x)
    assert out.dtype == torch.float64
    # the module's lambda / rho buffers hold 0.02 / 0.04 as created (fp32-rounded, then cast)
    ref = oracle64(x.cpu(), m.w.detach().cpu(), m.lmbda.item(), m.rho.item(), False, 20) + m.b.item()
    assert rel(out, ref) <= TOL64
    out32 = m.float()(x.float())
    assert out32.dtype == torch.float32 and 1e-10 < rel(out32, ref) <= 1e-5

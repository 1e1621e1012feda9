"""Second-order autograd (double backward) on the CPU: the host logic of admm_hip::fft_admm_tv_bwd's
autograd formula (admmtor._unrolled) and the oracle, both against the reference's own fp64
second-order gradients (tests/golden/g12_second_order.npz, made by make_golden_second_order.py from
deconv.py:35-117 with create_graph=True).

The GPU test of the same objective through the native ops is tests/test_gpu_second_order.py.
"""
import numpy as np
import pytest
import torch

from conftest import load_golden
from admmtor._unrolled import double_backward, unrolled_solve
from oracle.admm_oracle import rel_l2, solve_spatial

CASES = ["aniso_psf", "iso_psf", "aniso_nopsf"]


def case(tag):
    g = load_golden("g12_second_order")
    d = {k.split("/", 1)[1]: torch.from_numpy(v) for k, v in g.items() if k.startswith(tag + "/")}
    B, C, H, W, k, kgrad, iso, maxit = (int(v) for v in d["meta"])
    lam0, rho0, sl, sr = (float(v) for v in d["scal"])
    psf = d.get("psf", torch.empty(0, dtype=torch.float64))
    return d, psf, bool(kgrad), bool(iso), maxit, sl, sr


@pytest.mark.parametrize("tag", CASES)
def test_unrolled_solve_matches_reference_fp64(tag):
    d, psf, kgrad, iso, maxit, _, _ = case(tag)
    out = unrolled_solve(d["x"], d["lam"], d["rho"], psf, iso, maxit)
    assert rel_l2(out, d["out"]) <= 1e-12


@pytest.mark.parametrize("tag", CASES)
def test_double_backward_matches_reference_fp64(tag):
    d, psf, kgrad, iso, maxit, sl, sr = case(tag)
    seeds = (d["sx"], torch.tensor([sl], dtype=torch.float64), torch.tensor([sr], dtype=torch.float64),
             d["sk"] if kgrad else None)
    with torch.no_grad():  # as the autograd engine calls it for a plain (not create_graph) second backward
        h = double_backward(d["cot"], d["x"], d["lam"], d["rho"], psf, iso, maxit,
                            (True, True, True, kgrad), seeds, (True, True, True, True, kgrad))
    assert rel_l2(h[0], d["hcot"]) <= 1e-10
    assert rel_l2(h[1], d["hx"]) <= 1e-10
    assert rel_l2(h[2], d["hlam"]) <= 1e-10
    assert rel_l2(h[3], d["hrho"]) <= 1e-10
    if kgrad:
        assert rel_l2(h[4], d["hpsf"]) <= 1e-10
    else:
        assert h[4] is None


def test_double_backward_partial_seeds_and_targets():
    """Only the lam seed given and only x wanted: the other slots come back None."""
    d, psf, kgrad, iso, maxit, sl, sr = case("aniso_nopsf")
    h = double_backward(d["cot"], d["x"], d["lam"], d["rho"], psf, iso, maxit, (True, True, True, False),
                        (None, torch.ones(1, dtype=torch.float64), None, None), (False, True, False, False, False))
    assert h[0] is None and h[2] is None and h[3] is None and h[4] is None
    x = d["x"].clone().requires_grad_(True)
    lam = d["lam"].clone().requires_grad_(True)
    y = unrolled_solve(x, lam, d["rho"], psf, iso, maxit)
    (gl,) = torch.autograd.grad(y, lam, d["cot"], create_graph=True)
    (hx,) = torch.autograd.grad(gl.sum(), x)
    assert rel_l2(h[1], hx) <= 1e-12


def test_double_backward_third_order_graph():
    """With grad mode on (create_graph in the double backward) the result carries a graph."""
    d, psf, kgrad, iso, maxit, sl, sr = case("aniso_nopsf")
    rho = d["rho"].clone().requires_grad_(True)
    with torch.enable_grad():
        h = double_backward(d["cot"], d["x"], d["lam"], rho, psf, iso, maxit, (True, True, True, False),
                            (d["sx"], None, None, None), (False, False, False, True, False))
    assert h[3] is not None and h[3].requires_grad
    (t,) = torch.autograd.grad(h[3].sum(), rho)
    assert torch.isfinite(t).all()


@pytest.mark.parametrize("tag", ["aniso_psf", "iso_psf"])
def test_oracle_second_order_matches_reference(tag):
    """The oracle's spatial restatement differentiates twice to the same values (pins the oracle the
    GPU test compares against)."""
    d, psf, kgrad, iso, maxit, sl, sr = case(tag)
    x = d["x"].clone().requires_grad_(True)
    lam = d["lam"].clone().requires_grad_(True)
    rho = d["rho"].clone().requires_grad_(True)
    k = psf.clone().requires_grad_(True)
    cot = d["cot"].clone().requires_grad_(True)
    y = solve_spatial(x, lam, rho, k, iso, maxit)
    g = torch.autograd.grad(y, (x, lam, rho, k), cot, create_graph=True)
    pen = (d["sx"] * g[0]).sum() + sl * g[1].sum() + sr * g[2].sum() + (d["sk"] * g[3]).sum()
    h = torch.autograd.grad(pen, (cot, x, lam, rho, k))
    for got, key in zip(h, ("hcot", "hx", "hlam", "hrho", "hpsf")):
        assert rel_l2(got, d[key]) <= 1e-10, key


def test_unrolled_solve_grouped_modules():
    """G modules sharing xin (fft_admm_tv_grouped's layout): module-major output, each module its own
    lambda / rho and, with iso, its own norm over its (B, C) -- equal to the separate solves."""
    d, psf, kgrad, iso, maxit, sl, sr = case("iso_psf")
    lam = torch.tensor([0.02, 0.05], dtype=torch.float64)
    rho = torch.tensor([0.05, 0.03], dtype=torch.float64)
    both = unrolled_solve(d["x"], lam, rho, psf, True, maxit)
    B = d["x"].shape[0]
    for g in range(2):
        one = unrolled_solve(d["x"], lam[g:g + 1], rho[g:g + 1], psf, True, maxit)
        assert torch.equal(both[g * B:(g + 1) * B], one)


@pytest.mark.parametrize("flat", [True, False])
@pytest.mark.parametrize("iso", [False, True])
def test_tangent_solve_matches_jvp_of_unrolled_lam0(flat, iso):
    """tangent_solve (the default second-order path) is the directional derivative torch's forward
    mode takes through unrolled_solve, also with lam = 0 on flat regions (a = 0 and tau = 0: the soft
    threshold passes its clamp, and torch's derivative of sign(a)*clamp_min(|a|-tau, 0) is 0 there)."""
    from admmtor._unrolled import tangent_solve
    g = torch.Generator().manual_seed(11)
    x = torch.zeros(2, 2, 12, 16, dtype=torch.float64)
    if not flat:
        x = torch.rand(x.shape, generator=g, dtype=torch.float64)
    tx = torch.randn(x.shape, generator=g, dtype=torch.float64)
    lam = torch.tensor([0.0], dtype=torch.float64)
    rho = torch.tensor([0.05], dtype=torch.float64)
    tl, tr = torch.tensor([0.3], dtype=torch.float64), torch.tensor([0.01], dtype=torch.float64)
    psf = torch.empty(0, dtype=torch.float64)
    y, ydot = tangent_solve(x, lam, rho, psf, iso, 6, (tx, tl, tr, None))
    y2, ydot2 = torch.func.jvp(lambda a, b, c: unrolled_solve(a, b, c, psf, iso, 6), (x, lam, rho), (tx, tl, tr))
    assert torch.equal(y, y2)
    assert rel_l2(ydot, ydot2) <= 1e-12

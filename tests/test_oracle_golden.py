"""Pin the CPU oracle (oracle/admm_oracle.py) to the reference's own outputs.

The golden vectors were produced by running the reference solver
(/root/reference/src/admmtor/eops/deconv.py) in the build container
(tests/golden/make_golden.py).  Both oracle restatements must reproduce the
reference's fp64 results to rounding (fp64 fixtures: 1e-10; fixtures whose
fp64 output is stored rounded to fp32: 2e-7), including gradients (autograd
through the spatial restatement vs the reference's autograd).
"""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle.admm_oracle import apply_psf_transpose, rel_l2, solve_fourier, solve_spatial, wiener_factor

ROUND32 = 2e-7  # fp64 reference stored as fp32


def T(a, dt=torch.float64):
    return torch.from_numpy(np.asarray(a)).to(dt)


@pytest.mark.parametrize("solver", [solve_fourier, solve_spatial])
def test_g1_c1(solver):
    g = load_golden("g1_c1")
    out = solver(T(g["x"]), 0.01, 0.02, T(g["psf"]), False, 30)
    assert rel_l2(out, T(g["ref64"])) <= ROUND32
    # the reference's own fp32 output against its fp64 output: the fp32 noise floor
    assert 1e-7 < rel_l2(T(g["ref32"]), T(g["ref64"])) < 1e-5


@pytest.mark.parametrize("iso", [False, True])
def test_g2_motion(iso):
    g = load_golden("g2_motion")
    out = solve_fourier(T(g["x"]), 0.01, 0.02, T(g["psf"]), iso, 50)
    assert rel_l2(out, T(g["ref64_iso" if iso else "ref64_aniso"])) <= ROUND32


def test_g3_c3_reduced():
    g = load_golden("g3_c3")
    out = solve_fourier(T(g["x"]), 0.01, 0.02, T(g["psf"]), False, 100)
    assert rel_l2(out, T(g["ref64"])) <= ROUND32
    out50 = solve_fourier(T(g["x"]), 0.01, 0.02, T(g["psf"]), False, 50)
    assert rel_l2(out50, T(g["ref64_it50"])) <= ROUND32


def test_g4_train_config_grads():
    g = load_golden("g4_train_grad")
    x = T(g["x"]).requires_grad_(True)
    lam = T(g["lam"]).requires_grad_(True)
    rho = T(g["rho"]).requires_grad_(True)
    out = solve_spatial(x, lam, rho, torch.empty(0, dtype=torch.float64), True, 100)
    assert rel_l2(out, T(g["out"])) <= 1e-10
    gx, gl, gr = torch.autograd.grad(out, (x, lam, rho), T(g["cot"]))
    assert rel_l2(gx, T(g["gx"])) <= 1e-8
    assert rel_l2(gl, T(g["glam"])) <= 1e-8
    assert abs(gr.item() - float(g["grho"][0])) <= 1e-8 * max(1.0, abs(float(g["grho"][0])))


@pytest.mark.parametrize("iso", [False, True])
def test_g5_psf_grads(iso):
    g = load_golden("g5_psf_grad")
    tag = "iso" if iso else "aniso"
    x = T(g["x"]).requires_grad_(True)
    k = T(g["psf"]).requires_grad_(True)
    lam = torch.tensor([0.02], dtype=torch.float64, requires_grad=True)
    rho = torch.tensor([0.05], dtype=torch.float64, requires_grad=True)
    out = solve_spatial(x, lam, rho, k, iso, 20)
    assert rel_l2(out, T(g[f"out_{tag}"])) <= 1e-10
    gx, gl, gr, gk = torch.autograd.grad(out, (x, lam, rho, k), T(g[f"cot_{tag}"]))
    for got, key in ((gx, "gx"), (gl, "glam"), (gr, "grho"), (gk, "gpsf")):
        assert rel_l2(got, T(g[f"{key}_{tag}"])) <= 1e-8, key


def test_g6_intermediates():
    g = load_golden("g6_inter")
    fc = wiener_factor(64, 64, T(g["psf"]), 0.02)
    assert rel_l2(fc, T(g["freq_c"])) <= 1e-12
    b = apply_psf_transpose(T(g["x"]), T(g["psf"]))
    assert rel_l2(b, T(g["b"])) <= 1e-12
    for it, key in ((1, "x_it1"), (2, "x_it2")):
        assert rel_l2(solve_fourier(T(g["x"]), 0.01, 0.02, T(g["psf"]), False, it), T(g[key])) <= 1e-12


def test_g7_edges():
    e = load_golden("g7_edges")
    z = solve_fourier(T(e["m0_x"]), 0.01, 0.02, T(e["m0_psf"]), False, 0)
    assert torch.count_nonzero(z).item() == 0 and np.abs(e["m0_out"]).max() == 0
    assert rel_l2(solve_fourier(T(e["m0_x"]), 0.01, 0.02, T(e["m0_psf"]), False, 1), T(e["m1_out"])) <= 1e-12
    # odd 15x17 image with an even 4x4 PSF (anchor ceil((k-1)/2))
    for solver in (solve_fourier, solve_spatial):
        o = solver(T(e["odd_x"]), 0.01, 0.02, T(e["odd_psf"]), False, 20)
        assert rel_l2(o, T(e["odd_out"])) <= 1e-10
    o = solve_fourier(T(e["noPSF_iso_x"]), 0.03, 0.05, torch.empty(0, dtype=torch.float64), True, 40)
    assert rel_l2(o, T(e["noPSF_iso_out"])) <= 1e-10
    o = solve_spatial(T(e["even4_x"]), 0.01, 0.02, T(e["even4_psf"]), False, 25)
    assert rel_l2(o, T(e["even4_out"])) <= 1e-10
    for iso, key in ((False, "rect_out_aniso"), (True, "rect_out_iso")):
        o = solve_fourier(T(e["rect_x"]), 0.01, 0.02, T(e["rect_psf"]), iso, 30)
        assert rel_l2(o, T(e[key])) <= 1e-10


def test_iso_couples_the_batch():
    """block shrink: the norm runs over batch AND channel, so solving one image alone differs."""
    e = load_golden("g7_edges")
    x = T(e["noPSF_iso_x"])
    full = solve_fourier(x, 0.03, 0.05, torch.empty(0, dtype=torch.float64), True, 40)
    one = solve_fourier(x[:1], 0.03, 0.05, torch.empty(0, dtype=torch.float64), True, 40)
    assert rel_l2(one, full[:1]) > 1e-4


def test_forward_mode_oracle_pinned_by_reference_gradients():
    """oracle.solve_fourier_jvp (the forward-mode checker of the full-shape config-5 gradient test) is
    pinned to the reference's own fp64 autograd (g4: train config, iso, 100 iterations): with the
    reference's vector-Jacobian products gx, glam, grho for the cotangent c, <c, J t> = <gx, t_x> +
    glam t_lam + grho t_rho for every direction t."""
    from oracle.admm_oracle import solve_fourier_jvp
    g = load_golden("g4_train_grad")
    x = T(g["x"])
    gen = torch.Generator().manual_seed(5)
    tx = torch.zeros((3,) + tuple(x.shape), dtype=torch.float64)
    tx[0] = torch.randn(x.shape, generator=gen, dtype=torch.float64)
    y, yd = solve_fourier_jvp(x, float(g["lam"][0]), float(g["rho"][0]), torch.empty(0, dtype=torch.float64), True,
                              int(g["maxit"]), tx, torch.tensor([0.0, 1.0, 0.0]), torch.tensor([0.0, 0.0, 1.0]))
    assert rel_l2(y, T(g["out"])) <= 1e-10
    c = T(g["cot"]).flatten()
    got = [torch.dot(c, yd[i].flatten()).item() for i in range(3)]
    want = [torch.dot(T(g["gx"]).flatten(), tx[0].flatten()).item(), float(g["glam"][0]), float(g["grho"][0])]
    for a, b in zip(got, want):
        assert abs(a - b) <= 1e-9 * max(1.0, abs(b)), (got, want)


@pytest.mark.parametrize("iso", [False, True])
def test_forward_mode_oracle_is_torch_jvp(iso):
    """solve_fourier_jvp's written-out tangents equal torch.func.jvp through solve_fourier (PSF and
    no PSF), all three tangent kinds at once."""
    from oracle.admm_oracle import solve_fourier_jvp
    gen = torch.Generator().manual_seed(1)
    for kern in (torch.empty(0, dtype=torch.float64), torch.rand(1, 1, 5, 5, generator=gen, dtype=torch.float64)):
        x = torch.rand(2, 3, 24, 20, generator=gen, dtype=torch.float64)
        lam, rho = torch.tensor(0.05, dtype=torch.float64), torch.tensor(0.3, dtype=torch.float64)
        tx = torch.stack([torch.randn(x.shape, generator=gen, dtype=torch.float64), torch.zeros_like(x),
                          torch.randn(x.shape, generator=gen, dtype=torch.float64)])
        tl = torch.tensor([0.0, 1.0, 0.4], dtype=torch.float64)
        tr = torch.tensor([0.0, 0.0, -0.7], dtype=torch.float64)
        y, yd = solve_fourier_jvp(x, lam, rho, kern, iso, 12, tx, tl, tr)

        def f(tt):
            return torch.func.jvp(lambda a, lm, r: solve_fourier(a, lm, r, kern, iso, 12), (x, lam, rho), tt)[1]
        ref = torch.vmap(f)((tx, tl, tr))
        assert rel_l2(y, solve_fourier(x, lam, rho, kern, iso, 12)) <= 1e-14
        for i in range(3):
            assert rel_l2(yd[i], ref[i]) <= 1e-12

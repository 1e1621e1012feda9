"""The matrix-core transforms (csrc/gcol_mm.hpp): column lengths H = S * R with an odd R in
[17, 127] that carries H's largest prime factor run their R-point transforms as cosine / sine matrix
products on v_mfma_f32_16x16x4_f32 (k_gcol_mm; BSD: 321 = 3 * 107), and so do the row inverses of
row lengths W = S * R (k_grow_inv_mm; BSD: 481 = 13 * 37).

Parity as for the rest of the generic path (test_gpu_generic.py): rel-L2 <= 1e-5 against the fp64
oracle, which is pinned to the reference (tests/test_oracle_golden.py); the reference's own x-update is
deconv.py:104-106.  The LDS column pass (ADMM_GCOL_MM=0) is the same transform with other roundings:
both meet the gate and agree to ~1e-6.
"""
import pytest
import torch

from admmtor import _native
from test_gpu_generic import TOL_REF64, oracle, rel, solve

pytestmark = pytest.mark.gpu

# (B, C, H, W): H = S * R for every kernel instance S and 1-4 row tiles of the (h + 1)-row matrices
MM_SHAPES = [
    ((2, 2, 17, 40), ("gauss:1.0", 5), False),    # S 1, R 17: one row tile, 3 k-steps
    ((1, 2, 107, 64), ("gauss:1.5", 7), True),    # S 1, R 107
    ((1, 1, 127, 50), ("motion", 7), False),      # S 1, R 127: h + 1 = 64 rows, 16 k-steps
    ((1, 1, 93, 70), ("gauss:2", 9), False),      # S 1, R 93 = 3 * 31 (not prime): 3 row tiles
    ((1, 1, 214, 90), ("gauss:1.5", 9), True),    # S 2, R 107
    ((1, 3, 321, 481), ("gauss:1.5", 9), False),  # S 3, R 107: the BSD image (bench.py --config bsd)
    ((2, 1, 123, 45), ("motion", 5), False),      # S 3, R 41: 2 row tiles
    ((1, 2, 148, 33), ("gauss:1.0", 5), True),    # S 4, R 37
    ((1, 1, 115, 77), ("gauss:1.5", 7), False),   # S 5, R 23
    ((1, 1, 114, 60), ("motion", 9), False),      # S 6, R 19 (table-twiddle 6-point butterflies)
    ((1, 1, 136, 28), ("gauss:1.0", 5), False),   # S 8, R 17
    ((1, 2, 107, 1), None, False),                # one column (Wh = 1: a block of one valid column)
    ((1, 1, 321, 2000), ("gauss:2", 11), False),  # Wh = 1,001 columns
]


def _x(shape, psf, seed):
    from admmtor.synth import blurred_batch, make_psf
    k = make_psf(*psf) if psf else None
    return blurred_batch(*shape, k if k is not None else torch.empty(0), seed=seed), k


@pytest.mark.parametrize("shape,psf,iso", MM_SHAPES)
def test_mm_column_pass_vs_oracle(cuda_dev, shape, psf, iso, monkeypatch):
    x, k = _x(shape, psf, sum(shape))
    it = 20 if shape[2] * shape[3] < 200_000 else 10
    ref = oracle(x, k, 0.01, 0.02, iso, it)
    got = solve(x, k, 0.01, 0.02, iso, it, cuda_dev)
    monkeypatch.setenv("ADMM_GCOL_MM", "0")
    with _native.ab_library():  # the LDS pass: an A/B knob
        lds = solve(x, k, 0.01, 0.02, iso, it, cuda_dev)
    e, e_lds, d = rel(got, ref), rel(lds, ref), rel(got, lds)
    print(shape, psf, "iso" if iso else "aniso", f"matrix-core {e:.3e}  LDS pass {e_lds:.3e}  between {d:.3e}")
    assert e <= TOL_REF64
    assert e <= 2 * e_lds + 1e-6
    assert not torch.equal(got, lds)  # the two passes round differently: the matrix-core one ran


# row lengths W = S * R for the matrix-core row inverse (k_grow_inv_mm); odd row counts leave the last
# line of a batch with one real row
ROW_SHAPES = [
    ((1, 2, 9, 107), ("gauss:1.0", 5), False),    # S 1, R 107 (odd row count: 18 rows)
    ((2, 1, 7, 214), ("gauss:1.5", 7), True),     # S 2
    ((1, 3, 20, 321), ("gauss:1.5", 9), False),   # S 3
    ((1, 1, 15, 148), ("motion", 7), False),      # S 4, R 37
    ((1, 1, 12, 115), ("gauss:1.0", 5), True),    # S 5, R 23
    ((1, 1, 11, 136), ("gauss:1.5", 9), False),   # S 8, R 17
    ((1, 3, 33, 481), ("gauss:1.5", 9), False),   # S 13, R 37: the BSD rows
    ((1, 1, 5, 221), ("motion", 5), True),        # S 13, R 17
    ((1, 1, 13, 127), ("gauss:2", 9), False),     # S 1, R 127: 4 row tiles
    ((3, 1, 1, 93), None, False),                 # one-row planes, R 93 = 3 * 31
]


@pytest.mark.parametrize("shape,psf,iso", ROW_SHAPES)
def test_mm_row_inverse_vs_oracle(cuda_dev, shape, psf, iso, monkeypatch):
    x, k = _x(shape, psf, sum(shape) + 1)
    ref = oracle(x, k, 0.01, 0.02, iso, 15)
    got = solve(x, k, 0.01, 0.02, iso, 15, cuda_dev)
    monkeypatch.setenv("ADMM_GROW_MM", "0")
    with _native.ab_library():
        lds = solve(x, k, 0.01, 0.02, iso, 15, cuda_dev)
    e, e_lds = rel(got, ref), rel(lds, ref)
    print(shape, psf, "iso" if iso else "aniso", f"matrix-core rows {e:.3e}  LDS rows {e_lds:.3e}")
    assert e <= TOL_REF64
    assert e <= 2 * e_lds + 1e-6
    assert not torch.equal(got, lds)


def test_mm_bsd_batch_sampled_planes(cuda_dev):
    """The bench's BSD workload (32 x 3 x 321 x 481, 9x9 PSF, 50 iterations): two planes of the full
    batch against the fp64 oracle (the planes are independent in the aniso solve)."""
    from admmtor.synth import blurred_batch, make_psf
    k = make_psf("gauss:1.5", 9)
    x = blurred_batch(32, 3, 321, 481, k, seed=11)
    got = solve(x, k, 0.01, 0.02, False, 50, cuda_dev)
    for b, c in ((0, 0), (31, 2)):
        e = rel(got[b:b + 1, c:c + 1], oracle(x[b:b + 1, c:c + 1], k, 0.01, 0.02, False, 50))
        print("BSD plane", (b, c), e)
        assert e <= TOL_REF64


def test_mm_two_streams_bit_identical(cuda_dev, monkeypatch):
    """The solve's plane parts on 1 or 2 streams give the same bits with the matrix-core pass."""
    x, k = _x((4, 3, 321, 96), ("gauss:1.5", 9), 5)
    monkeypatch.setenv("ADMM_GEN_STREAMS", "1")
    a = solve(x, k, 0.01, 0.02, False, 10, cuda_dev)
    monkeypatch.setenv("ADMM_GEN_STREAMS", "2")
    b = solve(x, k, 0.01, 0.02, False, 10, cuda_dev)
    assert torch.equal(a, b)


@pytest.mark.parametrize("shape,iso,psf", [((1, 2, 107, 30), False, ("gauss:1.0", 5)),
                                           ((2, 1, 123, 20), True, ("motion", 5))])
def test_mm_grads_vs_oracle(cuda_dev, shape, iso, psf):
    """Training forward (the column pass dumps the forward column spectra for the PSF gradient) and the
    backward through it, at matrix-core column lengths."""
    from oracle.admm_oracle import kink_margins
    from test_gpu_grad import hip_grads, oracle_grads
    x, k = _x(shape, psf, 9)
    cot = torch.randn(x.shape, generator=torch.Generator().manual_seed(2))
    o1, gx1, gl1, gr1 = hip_grads(x, k, 0.03, 0.07, iso, 5, cot, cuda_dev)
    o2, gx2, gl2, gr2 = oracle_grads(x, k, 0.03, 0.07, iso, 5, cot)
    e = (rel(o1, o2), rel(gx1, gx2), rel(gl1, gl2), rel(gr1, gr2))
    print(shape, iso, "out/gx/glam/grho rel:", e)
    assert e[0] <= TOL_REF64
    margins = None if iso else kink_margins(x.double(), 0.03, 0.07, k.double(), 5)
    if margins is None or float(margins.min()) >= 1e-5:
        assert max(e[1:]) <= 1e-3


def test_mm_psf_gradient_vs_oracle(cuda_dev):
    from admmtor.synth import blurred_batch, make_psf
    from oracle.admm_oracle import solve_spatial
    from test_gpu_grad import hip_grads_psf
    k = make_psf("gauss:1.0", 5)
    x = blurred_batch(1, 2, 107, 30, k, seed=5)
    cot = torch.randn(x.shape, generator=torch.Generator().manual_seed(4))
    _, gx1, gl1, gr1, gk1 = hip_grads_psf(x, k, 0.02, 0.05, False, 6, cot, cuda_dev)
    xd = x.double().requires_grad_(True)
    kd = k.double().requires_grad_(True)
    ld = torch.tensor([0.02], dtype=torch.float64, requires_grad=True)
    rd = torch.tensor([0.05], dtype=torch.float64, requires_grad=True)
    g = torch.autograd.grad(solve_spatial(xd, ld, rd, kd, False, 6), (xd, ld, rd, kd), cot.double())
    e = (rel(gx1, g[0]), rel(gl1, g[1]), rel(gr1, g[2]), rel(gk1, g[3]))
    print("mm psf grad (x, lam, rho, psf)", e)
    assert max(e) <= 1e-3

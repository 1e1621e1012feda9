"""The fused generic row pass (csrc/gfused_mm.hpp, k_grow_fused_mm): for row lengths W = S * R with an
odd R in [17, 127] carrying W's large prime factor, an aniso inference iteration runs the row inverse,
the ADMM step and the row forward transform in one kernel over strips of rows (halo rows re-transformed,
neighbours wrapping inside each plane), instead of the step pass + a separate row inverse.  The
reference runs every size through the same loop body (deconv.py:104-115).  Measured slower than the two
kernels it replaces, so it is an A/B option (ADMM_GEN_FUSED=1), tested here.

Each case: rel-L2 <= 1e-5 against the fp64 oracle (pinned to the reference, tests/test_oracle_golden.py),
and the unfused generic solve of the same input (ADMM_GEN_FUSED=0: the same algorithm with other
roundings) agrees to fp32 noise.
"""
import pytest
import torch

from test_gpu_generic import TOL_REF64, oracle, rel, solve

pytestmark = pytest.mark.gpu


def _x(shape, psf, seed):
    from admmtor.synth import blurred_batch, make_psf
    k = make_psf(*psf) if psf else None
    return blurred_batch(*shape, k if k is not None else torch.empty(0), seed=seed), k


CASES = [
    # (B, C, H, W), psf, iterations
    ((1, 3, 321, 481), ("gauss:1.5", 9), 12),   # the BSD image: S 13, R 37, 21 strips of 15-16 rows
    ((2, 1, 33, 481), ("motion", 7), 8),        # 3 strips of 11 rows
    ((3, 1, 1, 481), None, 6),                  # one-row planes: both halos are the row itself
    ((2, 2, 2, 481), None, 5),                  # two-row planes
    ((1, 2, 3, 107), None, 7),                  # S 1, R 107, three-row planes
    ((2, 1, 7, 214), ("gauss:1.5", 7), 9),      # S 2, R 107
    ((1, 3, 20, 321), ("gauss:1.5", 9), 8),     # S 3, R 107: strips of 10 rows
    ((1, 1, 15, 148), ("motion", 7), 10),       # S 4, R 37
    ((1, 1, 12, 115), ("gauss:1.0", 5), 10),    # S 5, R 23
    ((1, 1, 32, 136), ("gauss:1.5", 9), 6),     # S 8, R 17: two full 16-row strips
    ((1, 1, 13, 127), ("gauss:2", 9), 7),       # S 1, R 127: 4 row tiles, 7-line strips
    ((1, 2, 5, 1651), ("gauss:1.0", 5), 5),    # S 13, R 127, long rows: fewer lines per strip (LDS)
    ((1, 1, 40, 93), None, 1),                  # one iteration (no fused pass runs)
    ((1, 1, 40, 93), ("motion", 5), 2),         # R 93 = 3 * 31; one fused pass (the first)
]


@pytest.mark.parametrize("shape,psf,it", CASES)
def test_fused_row_pass_vs_oracle(cuda_dev, monkeypatch, shape, psf, it):
    x, k = _x(shape, psf, sum(shape) + it)
    ref = oracle(x, k, 0.01, 0.02, False, it)
    monkeypatch.setenv("ADMM_GEN_FUSED", "1")
    got = solve(x, k, 0.01, 0.02, False, it, cuda_dev)
    monkeypatch.setenv("ADMM_GEN_FUSED", "0")
    unf = solve(x, k, 0.01, 0.02, False, it, cuda_dev)
    e, e_unf, d = rel(got, ref), rel(unf, ref), rel(got, unf)
    print(shape, psf, it, f"fused {e:.3e}  unfused {e_unf:.3e}  between {d:.3e}")
    assert e <= TOL_REF64
    assert e <= 2 * e_unf + 1e-6
    if it > 1:
        assert not torch.equal(got, unf)  # the fused pass ran (other transform roundings)


@pytest.mark.parametrize("nl", ["1", "3", "5"])
def test_fused_strip_heights(cuda_dev, monkeypatch, nl):
    """Strips of at most 2 NLf rows for every NLf (ADMM_GEN_FUSED_NL): all within the gate."""
    x, k = _x((1, 2, 37, 481), ("gauss:1.5", 9), 3)
    monkeypatch.setenv("ADMM_GEN_FUSED", "1")
    monkeypatch.setenv("ADMM_GEN_FUSED_NL", nl)
    got = solve(x, k, 0.01, 0.02, False, 8, cuda_dev)
    e = rel(got, oracle(x, k, 0.01, 0.02, False, 8))
    print("NLf", nl, e)
    assert e <= TOL_REF64


def test_fused_planes_independent_and_streams(cuda_dev, monkeypatch):
    """A plane solved inside a batch equals the plane solved alone, bit for bit, and one or two streams
    give the same bits (the strips never cross planes; an even H, since the final row inverse pairs
    rows across the batch)."""
    x, k = _x((3, 2, 46, 481), ("gauss:1.5", 9), 4)
    monkeypatch.setenv("ADMM_GEN_FUSED", "1")
    full = solve(x, k, 0.01, 0.02, False, 10, cuda_dev)
    one = solve(x[1:2, 1:2].contiguous(), k, 0.01, 0.02, False, 10, cuda_dev)
    assert torch.equal(full[1:2, 1:2], one)
    monkeypatch.setenv("ADMM_GEN_STREAMS", "1")
    single = solve(x, k, 0.01, 0.02, False, 10, cuda_dev)
    assert torch.equal(full, single)

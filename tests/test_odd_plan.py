"""CPU check of the fused odd-length row pass's plan (odd_kernels.hpp k_pass_a_odd), before and beside the
GPU tests: a numpy restatement of what one launch does -- strips of 6 rows, the halo line (rows r0 - 1 and
r0 + nr), the prime-factor index maps (pixel n at (nA mod W1, nB mod W2), frequency k at (k mod W1,
k mod W2)), the Hermitian completion, the step walked row by row one row behind, the zeroed missing row of
an odd strip and the split into half spectra -- against the same iteration step written the plain way
(irfft rows, the per-pixel step with circular neighbours, rfft rows: generic_kernels.hpp's sequence, the
reference's deconv.py:104-115 between two column passes).  Exact arithmetic (fp64 DFT matrices): a wrong
index map, halo or strip boundary shows as an O(1) error."""
import numpy as np
import pytest

W1, W2 = 13, 37
W = W1 * W2
WH = (W + 1) // 2


def _inv(a, m):
    return next(i for i in range(1, m) if a * i % m == 1)


A, B = _inv(W2 % W1, W1), _inv(W1 % W2, W2)
N = np.arange(W)
KPOS = (N % W1) * W2 + N % W2                 # frequency k -> position in the W1 x W2 image
NPOS = ((N * A) % W1) * W2 + (N * B) % W2     # pixel n -> position
F1 = {d: np.exp(d * 2j * np.pi * np.outer(np.arange(W1), np.arange(W1)) / W1) for d in (-1, 1)}
F2 = {d: np.exp(d * 2j * np.pi * np.outer(np.arange(W2), np.arange(W2)) / W2) for d in (-1, 1)}


def _dft2(line, d):  # W1-point DFTs along the first axis, W2-point along the second (unnormalised)
    return (F1[d] @ line.reshape(W1, W2) @ F2[d].T).reshape(-1)


def _soft(a, t):
    return np.sign(a) * np.maximum(np.abs(a) - t, 0)


def _plain(S, ux, uy, b, tau, rho):
    H = S.shape[0]
    full = np.zeros((H, W), complex)
    full[:, :WH] = S
    full[:, 0] = full[:, 0].real
    full[:, WH:] = np.conj(S[:, 1:][:, ::-1])
    x = np.real(np.fft.ifft(full, axis=1) * W)
    ax = x - np.roll(x, 1, 1) + ux
    ay = x - np.roll(x, 1, 0) + uy
    zx, zy = _soft(ax, tau), _soft(ay, tau)
    nux, nuy = ax - zx, ay - zy
    wx, wy = zx - nux, zy - nuy
    r = rho * ((wx - np.roll(wx, -1, 1)) + (wy - np.roll(wy, -1, 0))) + b
    return np.fft.fft(r, axis=1)[:, :WH], nux, nuy


def _kernel(S, ux, uy, b, tau, rho, RS=6):
    H = S.shape[0]
    Sout, uxo, uyo = np.zeros_like(S), np.zeros_like(ux), np.zeros_like(uy)
    for r0 in range(0, H, RS):
        nr = min(RS, H - r0)
        nlf = (nr + 1) // 2
        g = lambda ro: (r0 + ro) % H  # noqa: E731
        X = np.zeros((nlf + 1, W), complex)
        for l in range(nlf + 1):
            ra, rb = (g(-1), g(nr)) if l == 0 else (g(2 * l - 2), g(2 * l - 1))
            ca = S[ra].copy()
            cb = S[rb].copy() if (l == 0 or 2 * l - 1 < nr) else np.zeros(WH, complex)
            ca[0], cb[0] = ca[0].real, cb[0].real
            k = np.arange(WH)
            X[l, KPOS[k]] = ca + 1j * cb
            X[l, KPOS[W - k[1:]]] = np.conj(ca[1:]) + 1j * np.conj(cb[1:])
            X[l] = _dft2(X[l], +1)

        def line(ro):
            return (0, 0) if ro < 0 else (0, 1) if ro >= nr else (1 + ro // 2, ro & 1)

        def get(ro):
            l, c = line(ro)
            v = X[l, NPOS]
            return v.real.copy() if c == 0 else v.imag.copy()

        def put(ro, val):
            l, c = line(ro)
            v = X[l, NPOS]
            X[l, NPOS] = (val + 1j * v.imag) if c == 0 else (v.real + 1j * val)

        for ro in range(nr + 1):
            gr = g(ro)
            x, xu = get(ro), get(ro - 1)
            ax = (x - np.roll(x, 1)) + ux[gr]
            ay = (x - xu) + uy[gr]
            zx, zy = _soft(ax, tau), _soft(ay, tau)
            nux, nuy = ax - zx, ay - zy
            wx, wy = zx - nux, zy - nuy
            if ro < nr:
                uxo[gr], uyo[gr] = nux, nuy
            if ro > 0:  # r of the row above, one row behind
                put(ro - 1, rho * ((wxp - np.roll(wxp, -1)) + (wyp - wy)) + bp)
            wxp, wyp, bp = wx, wy, (b[gr] if ro < nr else None)
        if nr & 1:
            l = 1 + (nr - 1) // 2
            X[l] = X[l].real
        for m in range(nlf):
            Z = _dft2(X[1 + m], -1)
            z, mz = Z[KPOS[:WH]], Z[KPOS[(W - np.arange(WH)) % W]]
            ra = g(2 * m)
            Sout[ra] = 0.5 * (z.real + mz.real) + 0.5j * (z.imag - mz.imag)
            if 2 * m + 1 < nr:
                Sout[ra + 1] = 0.5 * (z.imag + mz.imag) + 0.5j * (mz.real - z.real)
    return Sout, uxo, uyo


@pytest.mark.parametrize("H", [1, 2, 7, 13, 17, 24])
def test_odd_row_pass_plan_matches_plain_step(H):
    rng = np.random.default_rng(H)
    S = rng.standard_normal((H, WH)) + 1j * rng.standard_normal((H, WH))
    ux, uy, b = (rng.standard_normal((H, W)) for _ in range(3))
    tau, rho = 0.3 / 0.7, 0.7
    want = _plain(S, ux, uy, b, tau, rho)
    got = _kernel(S, ux, uy, b, tau, rho)
    assert np.abs(got[0] - want[0]).max() <= 1e-11 * np.abs(want[0]).max()
    assert np.abs(got[1] - want[1]).max() <= 1e-11 and np.abs(got[2] - want[2]).max() <= 1e-11


def test_prime_factor_maps_are_permutations():
    assert sorted(KPOS) == list(range(W)) and sorted(NPOS) == list(range(W))
    # the 2-D DFT on the maps is the W-point DFT
    x = np.random.default_rng(1).standard_normal(W) + 0j
    img = np.zeros(W, complex)
    img[NPOS] = x
    assert np.allclose(_dft2(img, -1)[KPOS], np.fft.fft(x), atol=1e-9)

"""CPU check of every mixed-radix transform plan compiled into the library (csrc/mixed_kernels.hpp
MRow<N> / MRowT<N> / MCol<H> specialisations): each schedule is run through an exact-arithmetic simulation of the
guarded Stockham stages (csrc/mixed_fft.hpp mstage: butterflies t + L q over L lanes, the lanes past the
last butterfly idle, registers q + Q k, LDS exchange between stages) and compared with numpy's DFT.

Rows: the inverse schedule maps the spectrum layout (Es values over Ls lanes) to the pixel layout (Ep
over Lp) and the forward schedule back.  Columns: the forward schedule maps layout(Ec) to the edge layout
of its last radix (where the Wiener factor is applied), the inverse schedule maps that layout back.  The
GPU tests (tests/test_gpu_mixed.py) check the same plans end to end against the fp64 oracle; this pins
each plan's index mapping without a GPU.
"""
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "torch-admm-deconv_amd", "csrc", "mixed_kernels.hpp")
DEFAULTS = {"ADMM_TPLAN_320": 1, "ADMM_M960_V": 0, "ADMM_M1080_V": 2, "ADMM_M2160_V": 1, "ADMM_M360_V": 1, "ADMM_MROW_V": 1, "ADMM_MCOL_C": 8}


def _preprocess(text):
    """The header's #if NAME == V / #elif / #else / #endif blocks with the build's default knob values."""
    out, stack = [], []  # stack of (taking, taken_any)
    for line in text.splitlines():
        s = line.strip()
        m = re.match(r"#(el)?if\s+(\w+)\s*==\s*(\d+)", s)
        if m and m.group(1) is None:
            cond = DEFAULTS.get(m.group(2), 0) == int(m.group(3))
            stack.append([cond, cond])
            continue
        if m:
            cond = not stack[-1][1] and DEFAULTS.get(m.group(2), 0) == int(m.group(3))
            stack[-1] = [cond, stack[-1][1] or cond]
            continue
        if s.startswith("#else") and stack:
            stack[-1] = [not stack[-1][1], True]
            continue
        if s.startswith("#endif") and stack:
            stack.pop()
            continue
        if all(t for t, _ in stack):
            out.append(line)
    return "\n".join(out)


def _plans(kind):
    text = _preprocess(open(HDR).read())
    plans = []
    for m in re.finditer(r"template <> struct %s<(\d+)> \{(.*?)\n\};" % kind, text, re.S):
        body = m.group(2)
        vals = {k: v for k, v in re.findall(r"(\w+) = (\w+)", body)}
        fwd = tuple(int(r) for r in re.search(r"using Fwd = Sched<([^>]*)>", body).group(1).split(","))
        inv = tuple(int(r) for r in re.search(r"using Inv = Sched<([^>]*)>", body).group(1).split(","))
        plans.append((int(m.group(1)), vals, fwd, inv))
    return plans


def _regs(N, L, R):
    return R * ((N // R + L - 1) // L)


def _run(N, L, sched, v, DIR):
    """The guarded Stockham stages of mstage on per-lane register lists v[t] (in place)."""
    buf = np.zeros(N, complex)
    NS = 1
    for si, R in enumerate(sched):
        NB, Q = N // R, (N // R + L - 1) // L
        if si:
            for t in range(L):
                for q in range(Q):
                    vt = t + L * q
                    if vt < NB:
                        for k in range(R):
                            v[t][q + Q * k] = buf[vt + k * NB]
        Wm = np.exp(DIR * 2j * np.pi * np.outer(np.arange(R), np.arange(R)) / R)
        for t in range(L):
            for q in range(Q):
                vt = t + L * q
                m = vt % NS
                a = np.array([v[t][q + Q * k] * np.exp(DIR * 2j * np.pi * m * k / (NS * R)) for k in range(R)])
                y = Wm @ a
                for k in range(R):
                    v[t][q + Q * k] = y[k]
        if si < len(sched) - 1:
            for t in range(L):
                for q in range(Q):
                    vt = t + L * q
                    if vt < NB:
                        base = (vt // NS) * NS * R + vt % NS
                        for k in range(R):
                            buf[base + k * NS] = v[t][q + Q * k]
        NS *= R
    return v


def _natural_in(x, L, lanes, e, EM):
    return [[x[t + lanes * j] for j in range(e)] + [0j] * (EM - e) if t < lanes else [0j] * EM for t in range(L)]


def _natural_out(v, N, lanes, e):
    got = np.zeros(N, complex)
    for t in range(lanes):
        for j in range(e):
            got[t + lanes * j] = v[t][j]
    return got


ROWS = _plans("MRow")
TRAIN_ROWS = _plans("MRowT")  # the training backward's row plans
COLS = _plans("MCol")


def test_header_has_the_plans():
    assert {n for n, *_ in ROWS} >= {960, 640, 1920, 2048, 1024, 480, 540, 360, 320, 240, 400, 720, 800, 1280}
    assert {n for n, *_ in TRAIN_ROWS} >= {240, 320, 360, 400, 480, 540, 640, 720, 800, 960, 1280}
    assert all(int(v["Ep"]) <= 5 for _, v, *_ in TRAIN_ROWS)
    assert {h for h, *_ in COLS} >= {1080, 2160, 720, 960, 540, 480, 360, 240, 600, 768, 800, 1200, 1440, 1536}


@pytest.mark.parametrize("N,vals,fwd,inv", ROWS + TRAIN_ROWS,
                         ids=[str(p[0]) for p in ROWS] + ["T%d" % p[0] for p in TRAIN_ROWS])
def test_row_plan_exact(N, vals, fwd, inv):
    Lg, Lp, Ep, Ls, Es = (int(vals[k]) for k in ("Lg", "Lp", "Ep", "Ls", "Es"))
    assert Lp * Ep == N and Ls * Es == N and Lp <= Lg and Ls <= Lg and Lg <= 256
    assert int(np.prod(fwd)) == N and int(np.prod(inv)) == N
    EM = max(max(_regs(N, Lg, R) for R in inv), max(_regs(N, Lg, R) for R in fwd))
    x = np.random.default_rng(N).standard_normal(N) + 1j * np.random.default_rng(N + 1).standard_normal(N)
    # inverse: spectrum layout(Es) over Ls lanes -> pixel layout(Ep) over Lp lanes, unnormalised
    got = _natural_out(_run(N, Lg, inv, _natural_in(x, Lg, Ls, Es, EM), +1), N, Lp, Ep)
    ref = np.fft.ifft(x) * N
    assert np.abs(got - ref).max() <= 1e-11 * np.abs(ref).max()
    # forward: pixel layout -> spectrum layout
    got = _natural_out(_run(N, Lg, fwd, _natural_in(x, Lg, Lp, Ep, EM), -1), N, Ls, Es)
    ref = np.fft.fft(x)
    assert np.abs(got - ref).max() <= 1e-11 * np.abs(ref).max()


@pytest.mark.parametrize("H,vals,fwd,inv", COLS, ids=[str(p[0]) for p in COLS])
def test_column_plan_exact(H, vals, fwd, inv):
    Lc, Ec = int(vals["Lc"]), int(vals["Ec"])
    assert Lc * Ec == H and int(np.prod(fwd)) == H and tuple(inv) == tuple(fwd[::-1])
    EM = max(max(_regs(H, Lc, R) for R in fwd), max(_regs(H, Lc, R) for R in inv))
    x = np.random.default_rng(H).standard_normal(H) + 1j * np.random.default_rng(H + 1).standard_normal(H)
    v = _run(H, Lc, fwd, _natural_in(x, Lc, Lc, Ec, EM), -1)
    # the forward result sits in the last radix's edge layout: register q + Qz k of lane t holds frequency
    # t + Lc q + NBz k (mixed_kernels.hpp k_pass_b_m, where the factor is applied)
    Rz = fwd[-1]
    NBz, Qz = H // Rz, (H // Rz + Lc - 1) // Lc
    spec = np.full(H, np.nan + 0j)
    for t in range(Lc):
        for q in range(Qz):
            if t + Lc * q < NBz:
                for k in range(Rz):
                    spec[t + Lc * q + NBz * k] = v[t][q + Qz * k]
    ref = np.fft.fft(x)
    assert np.abs(spec - ref).max() <= 1e-11 * np.abs(ref).max()
    # the inverse schedule from that layout returns the column (x H) in layout(Ec)
    back = _natural_out(_run(H, Lc, inv, v, +1), H, Lc, Ec)
    assert np.abs(back - H * x).max() <= 1e-11 * H * np.abs(x).max()

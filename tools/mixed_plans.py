"""Search transform plans for the mixed-radix fused kernels (csrc/mixed_kernels.hpp) and check them.

Rows (N = W / 2 complex points): a row group of Lg lanes (16 ... 256), pixels in layout(Ep) over
Lp = N / Ep lanes, spectra in layout(Es) over Ls = N / Es lanes, inverse schedule Es ... Ep.
Columns (H points): Lc threads per column in layout(Ec), forward schedule Ec ... Rz, inverse reversed.
Every candidate is verified with an exact-arithmetic simulation of the guarded Stockham stages
(mixed_fft.hpp mstage), then printed as C++ specialisations.
usage: python tools/mixed_plans.py rows 384 400 ... | cols 768 600 ...
"""
import itertools
import sys

import numpy as np

RADICES = (2, 3, 4, 5, 6, 8, 9, 10, 12, 15, 16)


def regs(N, L, R):
    return R * ((N // R + L - 1) // L)


def schedules(N, first, last, maxlen=4):
    mid = N // (first * last) if N % (first * last) == 0 else 0
    if not mid:
        return
    if mid == 1:
        yield (first, last)
        return
    for n in range(1, maxlen - 1):
        for combo in itertools.product(RADICES, repeat=n):
            if np.prod(combo) == mid:
                yield (first,) + combo + (last,)


def simulate(N, L, sched, lin, ein, lout, eout, DIR):
    rng = np.random.default_rng(0)
    x = rng.standard_normal(N) + 1j * rng.standard_normal(N)
    EM = max(regs(N, L, R) for R in sched)
    v = [[x[t + lin * j] for j in range(ein)] + [0] * (EM - ein) if t < lin else [0] * EM for t in range(L)]
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
        W = np.exp(DIR * 2j * np.pi * np.outer(np.arange(R), np.arange(R)) / R)
        for t in range(L):
            for q in range(Q):
                vt = t + L * q
                m = vt % NS
                a = np.array([v[t][q + Q * k] * np.exp(DIR * 2j * np.pi * m * k / (NS * R)) for k in range(R)])
                y = W @ a
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
    ref = np.fft.fft(x) if DIR < 0 else np.fft.ifft(x) * N
    got = np.zeros(N, complex)
    for t in range(lout):
        for j in range(eout):
            got[t + lout * j] = v[t][j]
    return np.abs(got - ref).max() / np.abs(ref).max()


def edge_ok(N, L, R, Lx):
    return ((N // R + L - 1) // L == 1 and N // R == Lx) or (L == Lx and (N // R) % L == 0)


def row_plans(N):
    out = []
    for Lg in (16, 32, 64, 128, 256):
        for Ep in RADICES:
            if N % Ep or not (5 <= Ep <= 9 or Ep == 16 and N // Ep == Lg) or N // Ep > Lg:
                continue
            Lp = N // Ep
            for Es in RADICES:
                if N % Es or N // Es > Lg:
                    continue
                Ls = N // Es
                for inv in schedules(N, Es, Ep):
                    if not (edge_ok(N, Lg, inv[0], Ls) and edge_ok(N, Lg, inv[-1], Lp)):
                        continue
                    EM = max(regs(N, Lg, R) for R in inv)
                    if EM > 16:
                        continue
                    # cost: pixel state (registers), lanes idle at the pixel edge, exchanges (more when wide)
                    waves = max(1, Lg // 64)
                    cost = 4 * Ep + EM + 6 * (1 - Lp / Lg) * 10 + (len(inv) - 1) * (3 if waves > 1 else 1) \
                        + (4 if waves > 1 else 0)
                    out.append((cost, Lg, Lp, Ep, Ls, Es, inv, EM))
    return sorted(out)[:3]


def col_plans(H):
    out = []
    for Ec in RADICES:
        if H % Ec:
            continue
        Lc = H // Ec
        if Lc > 512:
            continue
        for fwd in itertools.chain(*(schedules(H, Ec, z) for z in RADICES)):
            if not edge_ok(H, Lc, fwd[0], Lc):
                continue
            inv = fwd[::-1]
            if not edge_ok(H, Lc, inv[-1], Lc):
                continue
            EM = max(max(regs(H, Lc, R) for R in fwd), max(regs(H, Lc, R) for R in inv))
            if EM > 16:
                continue
            C = 8 if 8 * Lc <= 1024 else 4 if 4 * Lc <= 1024 else 2
            cost = EM + 2 * len(fwd) + (8 - C)
            out.append((cost, Lc, Ec, C, fwd, inv, EM))
    return sorted(out)[:3]


def main():
    kind, sizes = sys.argv[1], [int(v) for v in sys.argv[2:]]
    for n in sizes:
        plans = row_plans(n) if kind == "rows" else col_plans(n)
        if not plans:
            print(f"// {kind} {n}: no plan")
            continue
        p = plans[0]
        if kind == "rows":
            _, Lg, Lp, Ep, Ls, Es, inv, EM = p
            fwd = inv[::-1]
            e1 = simulate(n, Lg, inv, Ls, Es, Lp, Ep, +1)
            e2 = simulate(n, Lg, fwd, Lp, Ep, Ls, Es, -1)
            print(f"template <> struct MRow<{n}> {{  // W = {2 * n}  (EM {EM}; simulated {max(e1, e2):.1e})")
            print(f"    static constexpr int Lg = {Lg}, Lp = {Lp}, Ep = {Ep}, Ls = {Ls}, Es = {Es};")
            print(f"    using Inv = Sched<{', '.join(map(str, inv))}>;")
            print(f"    using Fwd = Sched<{', '.join(map(str, fwd))}>;")
            print("};")
        else:
            _, Lc, Ec, C, fwd, inv, EM = p
            e = simulate(n, Lc, fwd, Lc, Ec, Lc, Ec, -1) if fwd[-1] == Ec and (n // Ec) % Lc == 0 else None
            print(f"template <> struct MCol<{n}> {{  // (EM {EM})")
            print(f"    static constexpr int Lc = {Lc}, Ec = {Ec}, C = {C};")
            print(f"    using Fwd = Sched<{', '.join(map(str, fwd))}>;")
            print(f"    using Inv = Sched<{', '.join(map(str, inv))}>;")
            print("};")


if __name__ == "__main__":
    main()

"""CPU tests of the one-pixel-per-lane ChannelPool forward's logic (csrc/chanpool_lane.hpp).

The kernel's per-pixel function ``lane_pixel`` compiles for the host too: ``tests/native/
chanpool_lane_host.cpp`` runs it with plain memory accessors (clang++, for the kernel's 16-bit vector
types), and this file compares its std, median channel and mode channel with torch's CPU
``std``/``median``/``mode`` (the reference's kernels, attentions.py:44-47) on many pixels, and with the
oracle's libstdc++ restatement under a forced depth budget (the heapsort fallback).  No GPU: this pins
the packed sort network, the scans and the chunked introsort trace before any device run.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest
import torch

from conftest import ROOT
from oracle.chanpool_oracle import channel_pool

CLANG = "/opt/rocm/lib/llvm/bin/clang++"
SRC = os.path.join(ROOT, "tests", "native", "chanpool_lane_host.cpp")

pytestmark = pytest.mark.skipif(not os.path.exists(CLANG) and shutil.which("clang++") is None,
                                reason="clang++ (ext_vector_type) not available")


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    d = tmp_path_factory.mktemp("lanehost")
    exe = str(d / "chanpool_lane_host")
    cc = CLANG if os.path.exists(CLANG) else shutil.which("clang++")
    subprocess.run([cc, "-O2", "-std=c++17", "-o", exe, SRC], check=True)
    return exe, d


def _run(harness, x, depth=-1):
    exe, d = harness
    B, C, H, W = x.shape
    kind = "bf16" if x.dtype == torch.bfloat16 else "f16"
    xc = x.permute(1, 0, 2, 3).reshape(C, -1).contiguous().view(torch.int16).numpy()
    n = xc.shape[1]
    fin, fout = str(d / "in.u16"), str(d / "out.bin")
    xc.tofile(fin)
    subprocess.run([exe, kind, str(C), str(n), str(depth), fin, fout], check=True)
    o = np.fromfile(fout, dtype=np.int32)
    return o[:n].view(np.float32), o[n:2 * n], o[2 * n:]


def _data(kind, shape, dt, gen):
    if kind == "gauss":
        return torch.randn(shape, generator=gen).to(dt)
    if kind == "gelu":
        return torch.nn.functional.gelu(torch.randn(shape, generator=gen) * 2).to(dt)
    k = {"few": 3, "many": 40}[kind]
    return (torch.randint(-k, k + 1, shape, generator=gen).double() / 4).to(dt)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("C", [1, 2, 16, 17, 33, 64, 65, 86, 127, 128])
def test_lane_pixel_vs_torch_cpu(harness, dt, C):
    gen = torch.Generator().manual_seed(7000 + C)
    for kind in ("gauss", "gelu", "few", "many"):
        x = _data(kind, (2, C, 23, 29), dt, gen)
        if kind == "many" and C > 2:
            x[0, 0, 0, 0] = -0.0
            x[1, :, 2, 3] = 0.0
            x[1, : C // 2, 4, 5] = -0.0
        sd, mi, oi = _run(harness, x)
        med, mod = x.median(dim=1), x.mode(dim=1)
        np.testing.assert_array_equal(mi, med.indices.reshape(-1).numpy(), err_msg=f"{kind} median")
        np.testing.assert_array_equal(oi, mod.indices.reshape(-1).numpy(), err_msg=f"{kind} mode")
        if C > 1:
            ref = x.double().std(dim=1).reshape(-1).numpy()
            got = sd.astype(np.float64)
            assert np.all(np.abs(got - ref) <= 1e-6 * np.abs(ref) + 1e-30), (kind, np.abs(got - ref).max())


def test_lane_pixel_config5_volume(harness):
    # the config-5 caller's channel count on 2 x 128 x 128 pixels of each value distribution
    gen = torch.Generator().manual_seed(5)
    for kind in ("gauss", "gelu"):
        x = _data(kind, (2, 86, 128, 128), torch.bfloat16, gen)
        _, mi, oi = _run(harness, x)
        med, mod = x.median(dim=1), x.mode(dim=1)
        assert (mi == med.indices.reshape(-1).numpy()).all() and (oi == mod.indices.reshape(-1).numpy()).all(), kind


def test_lane_pixel_nan_median_rule(harness):
    gen = torch.Generator().manual_seed(31)
    x = (torch.randint(-3, 4, (2, 86, 4, 9), generator=gen).double() / 2).to(torch.bfloat16)
    x[0, 5, 0, 0] = x[0, 40, 0, 0] = float("nan")
    x[1, :, 2, 2] = float("nan")
    sd, mi, _ = _run(harness, x)
    np.testing.assert_array_equal(mi, x.median(dim=1).indices.reshape(-1).numpy())
    nan_cols = x.isnan().any(dim=1).reshape(-1).numpy()
    assert np.isnan(sd[nan_cols]).all() and not np.isnan(sd[~nan_cols]).any()


@pytest.mark.parametrize("depth", [0, 1, 3])
def test_lane_pixel_depth_limited_vs_oracle(harness, depth):
    gen = torch.Generator().manual_seed(depth)
    x = torch.randint(0, 7, (1, 86, 8, 16), generator=gen).to(torch.bfloat16)
    _, mi, oi = _run(harness, x, depth)
    _, _, omi, _, ooi = channel_pool(x.double().numpy(), depth_limit=depth)
    np.testing.assert_array_equal(oi, ooi.reshape(-1))
    np.testing.assert_array_equal(mi, omi.reshape(-1))

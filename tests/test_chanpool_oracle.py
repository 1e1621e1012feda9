"""CPU tests of the channel-statistics oracle (oracle/chanpool_oracle.py) and the C ABI of
include/admm_chanstat.h (exports only; no kernel launches without a GPU).

Pins: the oracle against the committed fixture from torch's CPU kernels (g9_chanpool.npz), against
torch's CPU median/mode live on fresh heavy-tie inputs, and its heapsort fallback against
std::make_heap + std::sort_heap compiled here with g++.
"""
import os
import re
import shutil
import subprocess

import numpy as np
import pytest
import torch

from conftest import ROOT, load_golden
from oracle.chanpool_oracle import channel_pool, channel_pool_backward, heap_sort, std_sort

HEADER = os.path.join(ROOT, "include", "admm_chanstat.h")


def _cases():
    g = load_golden("g9_chanpool")
    return g, [str(n) for n in g["names"]]


def test_oracle_matches_fixture():
    g, names = _cases()
    for name in names:
        x = g[f"{name}/x"].astype(np.float64)
        std, mv, mi, ov, oi = channel_pool(x)
        np.testing.assert_array_equal(mv, g[f"{name}/median"], err_msg=name)
        np.testing.assert_array_equal(mi, g[f"{name}/median_idx"], err_msg=name)
        np.testing.assert_array_equal(ov, g[f"{name}/mode"], err_msg=name)
        np.testing.assert_array_equal(oi, g[f"{name}/mode_idx"], err_msg=name)
        ref = g[f"{name}/std"].astype(np.float64)
        # the fixture's std is rounded to the dtype: within half an ulp of the dtype
        assert np.all(np.abs(std - ref) <= 2.0 ** -8 * np.abs(ref)), name
        gx = channel_pool_backward(x, std, mi, oi, g[f"{name}/cot"])
        np.testing.assert_allclose(gx, g[f"{name}/grad64"], rtol=1e-10, atol=1e-12, err_msg=name)


@pytest.mark.parametrize("C", [2, 15, 16, 17, 18, 31, 64, 86, 100, 129, 256])
def test_oracle_mode_index_matches_torch_cpu(C):
    g = torch.Generator().manual_seed(C)
    for alphabet in (2, 5, 40):
        x = torch.randint(0, alphabet, (3, C, 4, 5), generator=g).to(torch.float32)
        _, mv, mi, ov, oi = channel_pool(x.double().numpy())
        m = x.mode(dim=1)
        d = x.median(dim=1)
        np.testing.assert_array_equal(oi, m.indices.numpy())
        np.testing.assert_array_equal(ov, m.values.numpy())
        np.testing.assert_array_equal(mi, d.indices.numpy())
        np.testing.assert_array_equal(mv, d.values.numpy())


def test_signed_zero_ties():
    # -0.0 == +0.0 for the comparator: one run of four zeros; the returned value is the stored element
    x = torch.tensor([0.0, -0.0, 1.0, -0.0, 0.0, 2.0]).reshape(1, 6, 1, 1)
    _, mv, mi, ov, oi = channel_pool(x.double().numpy())
    m = x.mode(dim=1)
    assert oi.item() == m.indices.item() and ov.item() == 0.0


_HEAP_CPP = r"""
#include <algorithm>
#include <cstdio>
#include <utility>
#include <vector>
int main() {
    int n;
    while (std::scanf("%d", &n) == 1) {
        std::vector<std::pair<int, int>> v(n);
        for (int i = 0; i < n; ++i) { std::scanf("%d", &v[i].first); v[i].second = i; }
        auto cmp = [](const std::pair<int, int>& a, const std::pair<int, int>& b) { return a.first < b.first; };
        std::make_heap(v.begin(), v.end(), cmp);
        std::sort_heap(v.begin(), v.end(), cmp);
        for (int i = 0; i < n; ++i) std::printf("%d ", v[i].second);
        std::printf("\n");
    }
}
"""


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ absent")
def test_heapsort_matches_libstdcxx(tmp_path):
    src = tmp_path / "heap.cpp"
    exe = tmp_path / "heap"
    src.write_text(_HEAP_CPP)
    subprocess.run(["g++", "-O1", "-o", str(exe), str(src)], check=True)
    rng = np.random.default_rng(5)
    cols = [rng.integers(0, k, size=n) for n in (2, 3, 17, 40, 86, 129) for k in (2, 4, 30)]
    inp = "".join(f"{len(c)} " + " ".join(map(str, c)) + "\n" for c in cols)
    out = subprocess.run([str(exe)], input=inp, capture_output=True, text=True, check=True).stdout.splitlines()
    for c, line in zip(cols, out):
        pairs = [(float(v), i) for i, v in enumerate(c)]
        heap_sort(pairs, 0, len(pairs))
        assert [p[1] for p in pairs] == [int(t) for t in line.split()]


def test_depth_limited_sort_still_sorts():
    rng = np.random.default_rng(7)
    for depth in (0, 1, 2, 3):
        col = rng.integers(0, 6, size=86)
        stats = {"heapsort": 0}
        pairs = std_sort([(float(v), i) for i, v in enumerate(col)], depth, stats)
        assert [p[0] for p in pairs] == sorted(float(v) for v in col)
        assert stats["heapsort"] >= 1


def _declared():
    txt = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    return sorted(set(re.findall(r"\b(admm_(?:chanstat|planestat)_\w+)\s*\(", txt)))


def test_chanstat_header_binding_and_exports():
    from admmtor import _native
    assert _declared() == sorted(_native.EXPORTED_CHANSTAT)
    so = _native.lib_path()
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    assert set(_declared()) <= set(re.findall(r"\sT\s(admm_(?:chanstat|planestat)_\w+)", out))
    lib = _native.load()
    assert lib.admm_chanstat_max_channels(_native.CHANSTAT_F32) == 128
    assert lib.admm_chanstat_max_channels(_native.CHANSTAT_BF16) == 256
    assert lib.admm_chanstat_max_channels(_native.CHANSTAT_F16) == 256
    assert lib.admm_chanstat_max_channels(7) == 0
    # argument checks run on the host before any launch
    assert lib.admm_chanstat_pool(_native.CHANSTAT_F32, None, 1, 3, 4, None, None, None) == _native.ADMM_TV_EINVAL
    assert lib.admm_chanstat_pool(_native.CHANSTAT_F32, 8, 1, 129, 4, 8, None, None) == _native.ADMM_TV_EUNSUPPORTED
    assert lib.admm_chanstat_pool(_native.CHANSTAT_BF16, 8, 0, 86, 4, 8, None, None) == 0  # empty batch: no launch
    assert lib.admm_chanstat_pool_depth(_native.CHANSTAT_BF16, 8, 1, 86, 4, 8, None, 17, None) == _native.ADMM_TV_EINVAL
    import ctypes
    n = ctypes.c_size_t(0)
    assert lib.admm_planestat_workspace_size(1376, 512 * 512, ctypes.byref(n)) == 0
    assert n.value >= 1376 * 24 * 512 * 512
    # plane statistics: fp32 takes the median only, workspace checked before any launch
    assert lib.admm_planestat_median_mode(_native.CHANSTAT_F32, 8, 2, 16, None, 8, 8, 1 << 20, -1, None) \
        == _native.ADMM_TV_EUNSUPPORTED
    assert lib.admm_planestat_median_mode(_native.CHANSTAT_F32, 8, 2, 16, 8, None, 8, 16, -1, None) \
        == _native.ADMM_TV_EWORKSPACE
    assert lib.admm_planestat_median_mode(_native.CHANSTAT_BF16, 8, 2, 16, None, None, 8, 16, -1, None) \
        == _native.ADMM_TV_EWORKSPACE
    assert lib.admm_planestat_median_mode(_native.CHANSTAT_BF16, 8, 0, 16, None, None, None, 0, -1, None) == 0


def test_channel_pool_module_cpu_is_reference_ops():
    from admmtor.elayers.attentions import ChannelPool, native_channel_pool_applies
    x = torch.randn(2, 8, 5, 5, dtype=torch.float64)
    assert not native_channel_pool_applies(x)
    ref = torch.cat((x.std(1, keepdim=True), x.median(1, keepdim=True).values, x.mode(1, keepdim=True).values), 1)
    assert torch.equal(ChannelPool()(x), ref)

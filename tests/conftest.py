"""Shared test setup: import paths, the `gpu` marker, golden-fixture loading.

CPU tests (-m "not gpu") cover the oracle against the reference's golden vectors,
the host-side boundary logic and the C-ABI library exports.  GPU tests (-m gpu)
are the parity tests proper: the HIP path (through the C ABI) vs the golden
vectors and the oracle.
"""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "torch-admm-deconv_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")

# A/B test runs of a library variant (tools/gpu_ab_variant.sh): the test harness, not the package, reads
# the override and hands it to admmtor._native.use_library before any native call
if os.environ.get("ADMMTOR_LIB_OVERRIDE"):
    from admmtor import _native as _nat
    _nat.use_library(os.environ["ADMMTOR_LIB_OVERRIDE"])


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm device); parity tests of the HIP path")
    config.addinivalue_line("markers", "slow: long-running")


def load_golden(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


def golden_errors():
    with open(os.path.join(GOLDEN, "errors.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def cuda_dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda:0")

"""bench.py plumbing on the CPU: the PMC traffic lookup and the CPU-baseline leg (which times the
oracle's reference op sequence on a bounded sample).  The GPU run itself is the driver's."""
import json
import os

import pytest

import bench


def test_configs_name_the_metric_workload():
    assert bench.CONFIGS["c3"][:8] == (64, 3, 1024, 1024, "gauss:3", 21, 50, False)
    for name, cfg in bench.CONFIGS.items():
        assert len(cfg) == 9 and isinstance(cfg[8], str) and cfg[8], name


def test_pmc_traffic_reads_committed_summary():
    traffic, src = bench.pmc_traffic("c3", "pass_a", 490, 10)
    if src is None:
        pytest.skip("no committed PMC summary")
    summ = json.load(open(os.path.join(bench.ROOT, src)))["kernels"]
    rest = summ["k_pass_a<512, false, false, false>"]
    assert 0.9 * rest["algorithmic_bytes"] < traffic < 1.2 * rest["algorithmic_bytes"]
    assert bench.pmc_traffic("c2", "pass_a", 10, 1) == (None, None)


def test_cpu_baseline_leg_small_sample():
    import torch
    torch.set_num_threads(2)
    cfg = (2, 3, 64, 64, "gauss:3", 21, 5, False, "tiny")
    res = bench.cpu_baseline(cfg, planes=3, iters=2)
    assert res["kind"] == "port" and res["value"] > 0 and res["cores"] >= 1
    assert "planes 3/6" in res["sample"] and res["unit"] == "batch-equivalent ADMM iterations/s"

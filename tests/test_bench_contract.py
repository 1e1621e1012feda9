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


def test_pmc_traffic_is_keyed_by_build_hash(tmp_path, monkeypatch):
    """The roofline's traffic comes only from a PMC summary of the SAME build (its recorded
    admm_tv_build_hash), looked up by kernel role; any other build gives traffic None."""
    summ = {"build_hash": "abc", "workload": "c3",
            "roles": {"pass_a_first": "k_pass_a<512, false, true, false, true>",
                      "pass_a": "k_pass_a<512, false, false, false, true>", "pass_b": "k_pass_b<1024, 8, 0>"},
            "kernels": {"k_pass_a<512, false, true, false, true>": {"traffic_bytes": 4.0e9},
                        "k_pass_a<512, false, false, false, true>": {"traffic_bytes": 6.0e9},
                        "k_pass_b<1024, 8, 0>": {"traffic_bytes": 1.7e9}}}
    (tmp_path / "profiles").mkdir()
    (tmp_path / "profiles" / "r99_pmc_summary.json").write_text(json.dumps(summ))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    traffic, src = bench.pmc_traffic("c3", "pass_a", 490, 10, "abc")
    assert src == os.path.join("profiles", "r99_pmc_summary.json")
    assert traffic == pytest.approx((4.0e9 * 10 + 6.0e9 * 480) / 490)
    assert bench.pmc_traffic("c3", "pass_b", 500, 10, "abc")[0] == 1.7e9
    traffic, src = bench.pmc_traffic("c3", "pass_a", 490, 10, "other")
    assert traffic is None and "other" in src
    assert bench.pmc_traffic("c2", "pass_a", 10, 1, "abc")[0] is None


def test_committed_pmc_summaries_name_their_build():
    """Every summary bench.py may report carries the build hash and the kernel roles."""
    import glob
    for path in glob.glob(os.path.join(bench.ROOT, "profiles", "*_pmc_summary.json")):
        summ = json.load(open(path))
        if "roles" not in summ:  # rounds 1-2: never reported (no build hash)
            continue
        assert len(summ["build_hash"]) == 16
        for role in ("pass_a_first", "pass_a", "pass_b"):
            assert summ["roles"][role] in summ["kernels"], (path, role)


def test_cpu_baseline_leg_small_sample():
    import torch
    torch.set_num_threads(2)
    cfg = (2, 3, 64, 64, "gauss:3", 21, 5, False, "tiny")
    res = bench.cpu_baseline(cfg, planes=3, iters=2)
    assert res["kind"] == "port" and res["value"] > 0 and res["cores"] >= 1
    assert "planes 3/6" in res["sample"] and res["unit"] == "batch-equivalent ADMM iterations/s"


def test_world_from_gpus_and_env():
    """--gpus N without torch.distributed.run launches N ranks; under it, --gpus must equal WORLD_SIZE."""
    assert bench.resolve_world(None, {}) == (1, False)
    assert bench.resolve_world(1, {}) == (1, False)
    assert bench.resolve_world(8, {}) == (8, True)
    assert bench.resolve_world(None, {"WORLD_SIZE": "4"}) == (4, False)
    assert bench.resolve_world(4, {"WORLD_SIZE": "4"}) == (4, False)
    for gpus, env in ((8, {"WORLD_SIZE": "1"}), (2, {"WORLD_SIZE": "4"}), (0, {})):
        with pytest.raises(SystemExit) as e:
            bench.resolve_world(gpus, env)
        assert e.value.code == 2


def test_launch_cmd_is_torchrun_on_loopback():
    cmd = bench.launch_cmd(8, ["--gpus", "8", "--steps", "3"], 29511)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29511"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"] and cmd[-5].endswith("bench.py")


def test_gpus_mismatch_exits_before_any_gpu_call():
    """A torchrun rank whose --gpus differs from WORLD_SIZE exits with status 2 at once (no JSON line)."""
    import subprocess
    import sys
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(bench.ROOT, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 2, p.stderr
    assert p.stdout.strip() == "" and "WORLD_SIZE=2" in p.stderr


def test_workload_labels_agree_with_the_path():
    """No CONFIGS label hard-codes a kernel path (round 5's `hd` label said "generic-size path" while the
    solve ran on the mixed-radix kernels): the path is appended at run time from the library's own answer
    for the solve's descriptor (admm_tv_path, a host-only query), so a label always names the path its
    solve takes."""
    for name, cfg in bench.CONFIGS.items():
        B, C, H, W, kind, k, maxit, iso, desc = cfg
        assert "path" not in desc.lower(), (name, desc)
        path = bench.path_of(H, W, iso, k)
        assert bench.labelled(desc, path).endswith(f"[{path} path]")
    assert bench.path_of(1024, 1024) == "fused" and bench.path_of(1080, 1920) == "fused mixed-radix"
    assert bench.path_of(15, 17) == "generic" and bench.path_of(321, 481) == "fused odd-length"
    assert bench.path_of(321, 481, iso=True) == "generic"  # iso keeps the generic kernels there


def test_rocfft_rank_cache(monkeypatch):
    """Each rank gets its own rocFFT kernel-cache file unless the caller chose one."""
    monkeypatch.delenv("ROCFFT_RTC_CACHE_PATH", raising=False)
    bench.rocfft_rank_cache(3)
    path = os.environ["ROCFFT_RTC_CACHE_PATH"]
    assert path.endswith("_rank3.db") and f"uid{os.getuid()}" in path
    monkeypatch.setenv("ROCFFT_RTC_CACHE_PATH", "/somewhere/mine.db")
    bench.rocfft_rank_cache(5)
    assert os.environ["ROCFFT_RTC_CACHE_PATH"] == "/somewhere/mine.db"


def test_mm_col_flops_plan():
    # BSD columns 321 = 3 * 107: h = 53 -> 64-row tiles, 56-deep k; forward + inverse, cos + sin, re + im
    import bench
    assert bench.mm_col_flops(321, 241, 96) == 96 * 241 * 3 * (2 * 2 * 2 * 64 * 56 * 2)
    assert bench.mm_col_flops(1024, 513, 1) is None  # no odd factor in [17, 127]

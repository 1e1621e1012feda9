"""bench.py --gpus N started without torch.distributed.run launches N rank processes itself and
rank 0 reports n_gpus = N.  Rehearsed on the 1-GPU box: ADMM_BENCH_REHEARSAL puts every rank on
cuda:0 over gloo (the driver's 8-GPU node runs RCCL), with a reduced batch and one timed step, so
this checks the launch and the multi-rank reporting, not throughput."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run_bench(n, tmo=150, config="c3"):  # below the box's 180 s silence limit
    env = dict(os.environ, ADMM_BENCH_REHEARSAL="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "ROCFFT_RTC_CACHE_PATH"):
        env.pop(k, None)
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--batch", "1", "--steps", "1",
           "--warmup", "0", "--no-cpu-baseline", "--no-parity", "--no-extras", "--config", config]
    # stderr (torchrun's and the ranks' progress lines) streams through, so a slow start stays visible
    p = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, text=True, timeout=tmo, cwd=ROOT)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p, lines


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 8])
def test_bench_gpus_n_launches_n_ranks(cuda_dev, n):
    p, lines = _run_bench(n)
    assert p.returncode == 0, p.stdout[-3000:]
    assert len(lines) == 1, p.stdout[-3000:]  # rank 0 only
    res = json.loads(lines[0])
    print(f"bench --gpus {n}: n_gpus={res['n_gpus']} value={res['value']:.1f} {res['config']['parallelism'][:40]}")
    assert res["n_gpus"] == n
    assert res["config"]["reduced_batch"] is True and res["config"]["batch_per_gpu"] == 1
    assert res["config"]["parallelism"].startswith(f"shard{n} ")
    assert res["value"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 8])
def test_ranks_after_parent_used_rocfft(cuda_dev, n):
    """the ranks' first device FFT stalled when the parent process had used rocFFT.
    This parent runs device FFTs of the BSD sizes (run-time compiled Bluestein kernels) and keeps rocFFT
    loaded; then N rehearsal ranks (each with its own rocFFT cache, bench.rocfft_rank_cache; shards
    synthesised on the host) solve their BSD shards, and the run completes."""
    import torch
    x = torch.rand(2, 3, 321, 481, device=cuda_dev)
    y = torch.fft.irfftn(torch.fft.rfftn(x, dim=(2, 3)), s=(321, 481), dim=(2, 3))
    torch.cuda.synchronize()
    assert torch.allclose(x, y, atol=1e-5)
    p, lines = _run_bench(n, config="bsd")
    assert p.returncode == 0, p.stdout[-3000:]
    res = json.loads(lines[-1])
    print(f"bsd --gpus {n} after a parent rocFFT: n_gpus={res['n_gpus']} value={res['value']:.1f}")
    assert res["n_gpus"] == n and res["config"]["path"] == "fused odd-length"

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


def _run_bench(n, tmo=280):
    env = dict(os.environ, ADMM_BENCH_REHEARSAL="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--batch", "1", "--steps", "1",
           "--warmup", "0", "--no-cpu-baseline", "--no-parity", "--no-extras"]
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

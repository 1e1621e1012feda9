"""Config 4 (BASELINE configs[3]: batch-512 1024x1024x3 sharded over 8 GPUs) on the one-GPU box.

* test_c4_full_size_world8_gloo: the full C4 batch, 8 ranks (processes) on cuda:0 over gloo, 64 images
  of 1024^2 x 3 per rank (21x21 Gaussian sigma 3, lambda 0.01, rho 0.02, aniso, 50 iterations, the bench's
  per-rank seeds), ~7 GB of HBM per rank.  Every rank's sharded solve (parameters broadcast from rank 0)
  must equal a single-process solve of its shard bit for bit; planes (0, 0) and (63, 2) of ranks 0 and 7
  are checked against the fp64 oracle (<= 1e-5, the north-star gate; aniso planes are independent, so a
  plane is its own oracle input).
* test_rccl_world1_collectives: the RCCL calls of the multi-GPU path executed on hardware -- one process,
  init_process_group("nccl", world_size=1), every collective forced on (sharded._FORCE_COLLECTIVES):
  the packed parameter broadcast, the iso all-reduce hook in the forward and the backward (deconv.py:19-24,
  the batch coupling it carries) under a side torch stream, and gather="all" through
  all_gather_into_tensor.  World size 1 makes each collective an identity, so the result must equal the
  solve without torch.distributed bit for bit.

RCCL refuses two ranks on one device, so the 8-rank topology runs over gloo here; the 8-GPU RCCL run
is the driver's (SCALE).
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _paths():
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "torch-admm-deconv_amd")]


C4_PLANES = ((0, 0), (63, 2))


def _c4_worker(rank, world, port, q):
    _paths()
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from admmtor.eops.deconv import fft_admm_tv
        from admmtor.sharded import sharded_fft_admm_tv
        from admmtor.synth import CONFIG_SEED, blurred_batch, make_psf
        dev = torch.device("cuda:0")
        psf = make_psf("gauss:3", 21)
        x = blurred_batch(64, 3, 1024, 1024, psf, seed=CONFIG_SEED + 2 + 1000 * rank, device=dev)
        # non-source ranks pass a wrong PSF / lambda / rho: the broadcast from rank 0 must replace them
        kern = psf.to(dev) if rank == 0 else torch.rand(1, 1, 21, 21, device=dev)
        lam, rho = (0.01, 0.02) if rank == 0 else (3.0, 5.0)
        print(f"c4 rank {rank}: shard generated", flush=True)
        out = sharded_fft_admm_tv(x, lam, rho, kern, False, 50)
        single = fft_admm_tv(x, 0.01, 0.02, psf.to(dev), False, 50)
        torch.cuda.synchronize()
        print(f"c4 rank {rank}: solved", flush=True)
        same = torch.equal(out, single)
        planes = None
        if rank in (0, world - 1):
            # numpy arrays travel by value: torch CPU tensors on a queue are shared through a file
            # descriptor server in this process, gone if it exits before the parent reads (r06e)
            planes = [(b, c, x[b, c].cpu().numpy().copy(), out[b, c].cpu().numpy().copy()) for b, c in C4_PLANES]
        del x, out, single
        torch.cuda.empty_cache()
        q.put((rank, same, planes))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_c4_full_size_world8_gloo(cuda_dev):
    from oracle.admm_oracle import rel_l2, solve_fourier
    from admmtor.synth import make_psf
    world = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_c4_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, same, planes = q.get(timeout=600)
        res[rank] = (same, planes)
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert sorted(res) == list(range(world))
    assert all(res[r][0] for r in range(world)), {r: res[r][0] for r in range(world)}
    psf = make_psf("gauss:3", 21).double()
    for r in (0, world - 1):
        for b, c, xin, got in res[r][1]:
            xin, got = torch.from_numpy(xin), torch.from_numpy(got)
            ref = solve_fourier(xin.double().reshape(1, 1, 1024, 1024), 0.01, 0.02, psf, False, 50)
            e = rel_l2(got.reshape(1, 1, 1024, 1024), ref)
            print(f"C4 rank {r} plane ({b},{c}): rel-L2 vs fp64 oracle {e:.3e}")
            assert e <= 1e-5


def _rccl_worker(port, q):
    _paths()
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        from admmtor import sharded
        from admmtor.eops.deconv import fft_admm_tv
        from admmtor.synth import blurred_batch, make_psf
        assert dist.get_backend() == "nccl"
        sharded._FORCE_COLLECTIVES = True
        k = make_psf("motion", 7).to(dev)
        x = blurred_batch(3, 3, 64, 128, k.cpu(), seed=31).to(dev)
        cot = torch.randn(x.shape, generator=torch.Generator().manual_seed(2)).to(dev)
        results = {}
        for iso in (True, False):
            # without torch.distributed: the plain solve + gradients
            xr = x.clone().requires_grad_(True)
            lr = torch.tensor([0.02], device=dev, requires_grad=True)
            rr = torch.tensor([0.05], device=dev, requires_grad=True)
            ref = fft_admm_tv(xr, lr, rr, k, iso, 12)
            (ref * cot).sum().backward()
            # the sharded path with every collective on RCCL, inside a side torch stream
            xs = x.clone().requires_grad_(True)
            ls = torch.tensor([0.02], device=dev, requires_grad=True)
            rs = torch.tensor([0.05], device=dev, requires_grad=True)
            st = torch.cuda.Stream(dev)
            st.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(st):
                out = sharded.sharded_fft_admm_tv(xs, ls, rs, k, iso, 12)
                (out * cot).sum().backward()
                # float lambda / rho (the packed broadcast carries them) and the output all-gather
                # (all_gather_into_tensor; not differentiable, as in the multi-GPU bench)
                out2 = sharded.sharded_fft_admm_tv(x, 0.02, 0.05, k, iso, 12, gather="all")
            st.synchronize()
            torch.cuda.synchronize()
            results[iso] = (torch.equal(out, ref.detach()), torch.equal(out2, ref.detach()),
                            torch.equal(xs.grad, xr.grad), torch.equal(ls.grad, lr.grad), torch.equal(rs.grad, rr.grad),
                            tuple(out.shape))
        q.put(results)
    finally:
        dist.destroy_process_group()


def test_rccl_world1_collectives(cuda_dev):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_port(), q))
    p.start()
    res = q.get(timeout=300)
    p.join(60)
    assert p.exitcode == 0
    for iso, (o, o2, gx, gl, gr, shape) in res.items():
        print("iso" if iso else "aniso", "out/out2/gx/glam/grho bit-exact:", o, o2, gx, gl, gr, shape)
        assert shape == (3, 3, 64, 128)
        assert o and o2 and gx and gl and gr

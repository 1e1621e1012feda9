"""Concurrency and autograd-contract tests of the HIP solver.

* b5: "safe for concurrent calls on different streams, since each call has its own workspace":
  two host threads, each on its own HIP stream, run aniso and iso solves (forward and the native
  backward) at the same time; every result is bit-identical to the same call run alone.  The
  library keeps no per-solve global state (ABI v4 carries the all-reduce hook in the descriptor;
  the profiler totals sit behind a lock), and the Python binding binds each call's hook to that
  call's buffers only.
* a9: a gradient taken with create_graph=True keeps the native backward's values and can be
  differentiated again (values: tests/test_gpu_second_order.py); a second backward through the same
  graph with retain_graph=True gives the same gradient.
"""
import threading

import pytest
import torch

pytestmark = pytest.mark.gpu


def _case(dev, iso, seed, generic=False):
    from admmtor.synth import blurred_batch, make_psf
    k = make_psf("motion", 9)
    x = blurred_batch(3, 3, 128, 256, k, seed=seed).to(dev)
    if generic:  # a generic size: the aniso inference solve runs as two plane halves on two streams
        x = x[..., :120, :250].contiguous()
    return x, k.to(dev), iso


def _run(x, k, iso, grad):
    from admmtor.eops.deconv import fft_admm_tv
    if not grad:
        return (fft_admm_tv(x, 0.01, 0.02, k, iso, 25),)
    xg = x.clone().requires_grad_(True)
    lam = torch.tensor([0.01], device=x.device, requires_grad=True)
    out = fft_admm_tv(xg, lam, 0.02, k, iso, 25)
    (out * out).sum().backward()
    return out.detach(), xg.grad, lam.grad


def test_two_threads_two_streams_bit_identical(cuda_dev):
    cases = [(_case(cuda_dev, False, 1), False), (_case(cuda_dev, True, 2), True),
             (_case(cuda_dev, False, 3), True), (_case(cuda_dev, True, 4), False),
             # generic-size aniso inference on both threads: the fork / join of the two-stream
             # solve runs concurrently, each caller stream with its own auxiliary stream
             (_case(cuda_dev, False, 7, True), False), (_case(cuda_dev, False, 8, True), False)]
    serial = [_run(*c, grad) for c, grad in cases]
    torch.cuda.synchronize()
    results = [[None] * len(cases) for _ in range(2)]
    errors = []

    def worker(t):
        try:
            s = torch.cuda.Stream(device=cuda_dev)
            with torch.cuda.stream(s):
                for rep in range(3):  # interleave many launches of both threads
                    for i in range(t, len(cases), 2):
                        c, grad = cases[i]
                        results[t][i] = _run(*c, grad)
            s.synchronize()
        except BaseException as e:  # noqa: BLE001
            errors.append(e)

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(2)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(120)
    torch.cuda.synchronize()
    assert not errors, errors
    for i in range(len(cases)):
        got = results[i % 2][i]
        assert got is not None
        for a, b in zip(got, serial[i]):
            assert torch.equal(a, b), f"case {i} differs from its serial run"


def test_profiler_totals_under_threads(cuda_dev):
    """the process-wide pass timers count every launch of every thread"""
    from admmtor import _native
    x, k, _ = _case(cuda_dev, False, 5)
    _native.profile_reset()
    _native.profile_enable(True)
    ths = [threading.Thread(target=lambda: _run(x, k, False, False)) for _ in range(3)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(60)
    torch.cuda.synchronize()
    _native.profile_enable(False)
    ms, n = _native.profile_read()
    assert n[1] == 3 * 25 and n[0] == 3 * 24  # column pass every iteration, row pass all but the last
    assert all(v >= 0 for v in ms)


def test_create_graph_first_order_values_native(cuda_dev):
    """A gradient taken with create_graph=True has the native backward's values bit for bit (the
    double-backward formula only adds a graph, admmtor._unrolled), can be differentiated again,
    and a second backward with retain_graph=True reuses the kept history: same gradient."""
    from admmtor.eops.deconv import fft_admm_tv
    x, k, _ = _case(cuda_dev, True, 6)
    xg = x.clone().requires_grad_(True)
    out = fft_admm_tv(xg, 0.01, 0.02, k, True, 10)
    (g,) = torch.autograd.grad(out.square().sum(), xg, create_graph=True)
    out0 = fft_admm_tv(xg, 0.01, 0.02, k, True, 10)
    (g0,) = torch.autograd.grad(out0.square().sum(), xg)
    assert torch.equal(g.detach(), g0)
    assert g.requires_grad
    (h,) = torch.autograd.grad(g.sum(), xg)
    assert torch.isfinite(h).all()
    out = fft_admm_tv(xg, 0.01, 0.02, k, True, 10)
    loss = out.square().sum()
    (g1,) = torch.autograd.grad(loss, xg, retain_graph=True)
    (g2,) = torch.autograd.grad(loss, xg)
    assert torch.equal(g1, g2)


@pytest.mark.parametrize("iso,generic", [(False, False), (True, False), (False, True)])
def test_solver_is_graph_capturable(cuda_dev, iso, generic):
    """The solve enqueues only asynchronous work on the current stream (no host synchronisation,
    workspace from the caching allocator): it can be captured in a HIP graph (torch.cuda.CUDAGraph)
    and replayed, giving the eager result bit for bit (include/admm_tv.h: graph-capturable)."""
    from admmtor.eops.deconv import fft_admm_tv
    x, k, _ = _case(cuda_dev, iso, 6)
    if generic:  # the generic-size path (two plane halves on two streams when not captured)
        x = x[..., :120, :250].contiguous()
    static_x = x.clone()
    eager = fft_admm_tv(static_x, 0.01, 0.02, k, iso, 12)
    s = torch.cuda.Stream(cuda_dev)
    s.wait_stream(torch.cuda.current_stream(cuda_dev))
    with torch.cuda.stream(s):  # warm-up on the side stream, as torch.cuda.graphs recommends
        fft_admm_tv(static_x, 0.01, 0.02, k, iso, 12)
    torch.cuda.current_stream(cuda_dev).wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        static_out = fft_admm_tv(static_x, 0.01, 0.02, k, iso, 12)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(static_out, eager)
    static_x.copy_(x.flip(-1))  # new input, same buffers
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(static_out, fft_admm_tv(x.flip(-1), 0.01, 0.02, k, iso, 12))


@pytest.mark.parametrize("B,C,H,W", [(1, 3, 321, 481), (3, 1, 121, 250), (1, 2, 45, 64), (5, 3, 33, 40)])
def test_two_stream_split_matches_one_stream(cuda_dev, monkeypatch, B, C, H, W):
    """The generic row kernels transform real rows in pairs: the two-stream split of an aniso
    inference solve puts an even number of rows in its first half (odd H: an even plane count), so
    the eager two-stream solve equals the one-stream solve (ADMM_GEN_STREAMS=1, also what a
    captured solve runs) bit for bit -- odd H with P = 3 included (the BSD image, 1x3x321x481)."""
    from admmtor.eops.deconv import fft_admm_tv
    from admmtor.synth import blurred_batch, make_psf
    k = make_psf("gauss:1.5", 9)
    x = blurred_batch(B, C, H, W, k, seed=11).to(cuda_dev)
    two = fft_admm_tv(x, 0.01, 0.02, k.to(cuda_dev), False, 8)
    monkeypatch.setenv("ADMM_GEN_STREAMS", "1")
    one = fft_admm_tv(x, 0.01, 0.02, k.to(cuda_dev), False, 8)
    monkeypatch.setenv("ADMM_GEN_STREAMS", "4")
    four = fft_admm_tv(x, 0.01, 0.02, k.to(cuda_dev), False, 8)
    torch.cuda.synchronize()
    assert torch.equal(two, one) and torch.equal(four, one)


def test_input_on_another_device_than_current(cuda_dev):
    """A solve of tensors on cuda:1 while the current device is cuda:0 runs on cuda:1: the library
    takes the device from the caller's stream (two-stream generic solve, fused solve, backward)."""
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two ROCm devices")
    from admmtor.eops.deconv import fft_admm_tv
    d1 = torch.device("cuda:1")
    torch.cuda.set_device(0)
    for generic in (True, False):
        x, k, _ = _case(torch.device("cpu"), False, 9, generic)
        ref = fft_admm_tv(x.to(cuda_dev), 0.01, 0.02, k.to(cuda_dev), False, 10).cpu()
        out = fft_admm_tv(x.to(d1), 0.01, 0.02, k.to(d1), False, 10)
        assert out.device == d1 and torch.cuda.current_device() == 0
        assert torch.equal(out.cpu(), ref)
        xg = x.to(d1).requires_grad_(True)
        fft_admm_tv(xg, 0.01, 0.02, k.to(d1), True, 6).square().sum().backward()
        assert xg.grad.device == d1 and torch.isfinite(xg.grad).all()

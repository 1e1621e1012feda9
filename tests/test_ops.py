"""The dispatcher ops admm_hip::* on the CPU: registration, fake kernels, and a
dynamo trace of ADMMDeconv with no graph break (meta tensors: shapes only, nothing runs).  The
real kernels are checked with torch.library.opcheck on the GPU (tests/test_gpu_ops.py)."""
import pytest
import torch


def test_ops_registered():
    import admmtor._ops  # noqa: F401
    for name in ("fft_admm_tv_fwd", "fft_admm_tv_fwd_train", "fft_admm_tv_bwd"):
        assert hasattr(torch.ops.admm_hip, name)


def test_fake_kernels_shapes():
    import admmtor._ops  # noqa: F401
    from torch._subclasses.fake_tensor import FakeTensorMode
    from admmtor import _native
    with FakeTensorMode():
        x = torch.empty(2, 3, 64, 32)
        lam = torch.empty(2)  # two modules solved together
        k = torch.empty(1, 1, 5, 5)
        assert torch.ops.admm_hip.fft_admm_tv_fwd(x, lam, lam, k, False, 10).shape == (4, 3, 64, 32)
        out, hist = torch.ops.admm_hip.fft_admm_tv_fwd_train(x, lam, lam, k, True, 10, False)
        assert out.shape == (4, 3, 64, 32) and hist.dtype == torch.uint8
        want = _native.history_size(_native.desc(2, 3, 64, 32, 5, True, 10, 0, 2))
        assert hist.shape == (want,)
        gx, gl, gr, gk = torch.ops.admm_hip.fft_admm_tv_bwd(out, x, lam, lam, k, hist, True, 10, False,
                                                             True, True, False)
        assert gx.shape == x.shape and gl.shape == (2,) and gr.shape == (2,) and gk.numel() == 0


def test_ops_refuse_host_tensors():
    import admmtor._ops  # noqa: F401
    x = torch.rand(1, 1, 16, 16)
    with pytest.raises(RuntimeError, match="ROCm device"):
        torch.ops.admm_hip.fft_admm_tv_fwd(x, torch.ones(1), torch.ones(1), torch.empty(0), False, 2)


@pytest.mark.parametrize("iso,kern", [(False, (5, 5)), (True, ())])
def test_admmdeconv_traces_as_one_graph(iso, kern):
    from admmtor.elayers.admmdeconv import ADMMDeconv
    torch._dynamo.reset()
    m = ADMMDeconv(kern, 10, iso=iso).to("meta")
    x = torch.empty(2, 3, 64, 64, device="meta", requires_grad=True)
    ex = torch._dynamo.explain(m)(x)
    assert ex.graph_count == 1 and ex.graph_break_count == 0, ex.break_reasons
    code = ex.graphs[0].code
    assert "admm_hip.fft_admm_tv_fwd_train" in code
    y = torch.compile(m, backend="aot_eager", fullgraph=True)(x)
    assert y.shape == x.shape
    y.sum().backward()
    assert x.grad.shape == x.shape


def test_history_gradient_is_not_materialised():
    """The training forward's second output (the uint8 history) never has a gradient; with autograd's
    default grad materialisation a history-sized zero tensor (10 GB at the C5 shape) was allocated and
    filled before every backward.  _setup_context turns materialisation off, and _backward returns no
    gradients when the solve's output gradient is absent."""
    from admmtor import _ops

    class Ctx:
        needs_input_grad = (True, True, True, False, False, False, False)

        def set_materialize_grads(self, v):
            self.materialize = v

        def save_for_backward(self, *t):
            self.saved = t

    ctx = Ctx()
    x = torch.rand(1, 1, 8, 8)
    hist = torch.empty(16, dtype=torch.uint8)
    _ops._setup_context(ctx, (x, torch.ones(1), torch.ones(1), torch.empty(0), False, 3, False),
                        (torch.empty_like(x), hist))
    assert ctx.materialize is False
    assert _ops._backward(ctx, None, None) == (None,) * 7


def test_inference_tensor_input_is_copied_not_versioned():
    """An image made under torch.inference_mode() and then solved with a learnable lambda / rho: an inference
    tensor has no version counter (reading x._version raises), so the forward keeps a private copy of it
    instead of a versioned reference, and the backward sees that copy."""
    from admmtor import _ops

    class Ctx:
        needs_input_grad = (False, True, True, False, False, False, False)

        def set_materialize_grads(self, v):
            self.materialize = v

        def save_for_backward(self, *t):
            self.saved = t

    with torch.inference_mode():
        x = torch.rand(1, 1, 8, 8)
    assert x.is_inference()
    ctx = Ctx()
    _ops._setup_context(ctx, (x, torch.ones(1), torch.ones(1), torch.empty(0), False, 3, False),
                        (torch.empty_like(x), torch.empty(16, dtype=torch.uint8)))
    xs = ctx.saved[0]
    assert ctx.xref is None and not xs.is_inference() and torch.equal(xs, x)
    # an ordinary tensor is still only referenced (no copy) with its version
    y = torch.rand(1, 1, 8, 8)
    _ops._setup_context(ctx, (y, torch.ones(1), torch.ones(1), torch.empty(0), False, 3, False),
                        (torch.empty_like(y), torch.empty(16, dtype=torch.uint8)))
    assert ctx.saved[0].numel() == 0 and ctx.xref[0].data_ptr() == y.data_ptr()

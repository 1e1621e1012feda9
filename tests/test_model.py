"""Config-5 caller: DivergentRestorer / DivergentAttention rebuilt as plain
PyTorch modules around the HIP ADMM solver, pinned to the reference's own model
(tests/golden/make_golden_model.py: reduced width, seeded init, fp64 forward + backward).

CPU: same seed -> the same state_dict (names, order, values, bit for bit); the CNN alone
(admms=None) reproduces the reference's fp64 output and every parameter gradient.
"""
import numpy as np
import pytest
import torch

from conftest import load_golden

from admmtor.modelbuild.blocks import DivergentAttention, _branch_plan, set_branch_checkpointing
from admmtor.modelbuild.denoiser import DivergentRestorer

SEED = 20251205 + 5
ADMM = {"kern_size": (), "max_iters": 10, "iso": True}


def build(admms):
    torch.manual_seed(SEED)
    return DivergentRestorer([2, 4, 4], 3, 3, 8, 8, 2, output_activation=torch.nn.Sigmoid(), admms=admms)


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


@pytest.mark.parametrize("name,admms", [("g8_model_plain", None), ("g8_model_admm", [ADMM, ADMM])])
def test_seeded_init_matches_reference(name, admms):
    g = load_golden(name)
    sd = build(admms).state_dict()
    ref_keys = [k[5:] for k in g if k.startswith("init/")]
    assert list(sd.keys()) == ref_keys
    for k, v in sd.items():
        assert np.array_equal(v.numpy(), g["init/" + k]), k


def test_plain_forward_backward_matches_reference_fp64():
    g = load_golden("g8_model_plain")
    model = build(None).double()
    x = torch.from_numpy(g["x"]).requires_grad_(True)
    out = model(x)
    assert rel(out.detach(), g["out"]) <= 1e-12
    (out * torch.from_numpy(g["cot"])).sum().backward()
    assert rel(x.grad, g["gx"]) <= 1e-10
    grads = {k: p.grad for k, p in model.named_parameters() if p.grad is not None}
    assert sorted(grads) == sorted(k[5:] for k in g if k.startswith("grad/"))
    # a conv bias feeding an instance norm has an analytically zero gradient: compare it
    # absolutely (rounding noise ~1e-15 on both sides)
    zero = {k for k in grads if np.linalg.norm(g["grad/" + k]) < 1e-12}
    assert all(grads[k].norm() < 1e-12 for k in zero)
    assert all(k.endswith("spatial.conv.bias") for k in zero)
    worst = max(rel(v, g["grad/" + k]) for k, v in grads.items() if k not in zero)
    assert worst <= 1e-9, worst


def test_branch_plan_follows_reference_zip():
    # no ADMM: 2b conv outputs, b attentions -> outs[0:b/2] and outs[b:3b/2] are used
    assert _branch_plan(8, 4) == ([(0, 0), (1, 1)], [(2, 4), (3, 5)])
    # with b ADMM modules: zip(convs, admms) keeps b outputs, all used
    assert _branch_plan(2, 2) == ([(0, 0)], [(1, 1)])


def test_unused_branches_get_no_gradient():
    torch.manual_seed(0)
    blk = DivergentAttention(4, 3, 8, 8, 8, 2).double()
    blk(torch.rand(1, 3, 16, 16, dtype=torch.float64)).sum().backward()
    used = {n.split(".")[1] for n, p in blk.named_parameters() if n.startswith("convs.") and p.grad is not None}
    assert used == {"0", "1", "4", "5"}


def test_admm_model_refuses_host_tensors():
    with pytest.raises(RuntimeError):
        build([ADMM, ADMM])(torch.rand(1, 3, 32, 32))


def test_branch_checkpointing_is_exact():
    g = load_golden("g8_model_plain")
    res = []
    for ckpt in (False, True):
        model = build(None).double()
        assert set_branch_checkpointing(model, ckpt) == 3
        x = torch.from_numpy(g["x"]).requires_grad_(True)
        out = model(x)
        (out * torch.from_numpy(g["cot"])).sum().backward()
        res.append((out.detach(), x.grad, [p.grad for p in model.parameters()]))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    assert all((a is None and b is None) or torch.equal(a, b) for a, b in zip(res[0][2], res[1][2]))

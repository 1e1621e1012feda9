"""Batch-sharded ADMM-TV over the GPUs of a node (one process per GPU, RCCL over xGMI).

SURVEY.md §8 e1: with soft shrinkage (iso=False) every (b, c) plane is an
independent problem, so a batch is split across ranks with NO per-iteration
communication.  The only collectives are a broadcast of the PSF, lambda and rho
from rank 0 (a few KB: every rank then builds its own Wiener factor) and,
optionally, a final gather of the outputs.  iso=True couples the whole batch
through the per-pixel (B, C) norm: it is sharded with a per-iteration SUM
all-reduce of the 2*H*W per-pixel sums (RCCL), handed to the library per call in the
descriptor (``admm_tv_desc.allreduce``; also the cross-plane products Q in the backward).  A rank
whose shard is empty (B < world) still takes part in every one of those reductions.

The reference has no distributed code at all; this module is the
multi-GPU layer of the MI355X build.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch
import torch.distributed as dist

__all__ = ["shard_bounds", "broadcast_params", "sharded_fft_admm_tv", "make_host_group"]

# Test-only switch: run every collective of the sharded path (the parameter broadcast, the iso
# all-reduce hook, the output gather) also at world size 1, where they are identities -- so a
# single-GPU box can execute the RCCL calls of the multi-GPU path (tests/test_gpu_c4.py).
_FORCE_COLLECTIVES = False


def _world(group) -> int:
    return dist.get_world_size(group) if (dist.is_available() and dist.is_initialized()) else 1


def _collectives(group) -> bool:
    return _world(group) > 1 or (_FORCE_COLLECTIVES and dist.is_available() and dist.is_initialized())


def shard_bounds(total: int, world: int, rank: int):
    """Contiguous near-equal split of `total` items: the [start, stop) of `rank`."""
    base, rem = divmod(total, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def _as_tensor(v, device, dtype=torch.float64):
    if isinstance(v, torch.Tensor):
        return v.detach().reshape(-1)[:1].to(device=device, dtype=dtype).clone()
    return torch.tensor([float(v)], device=device, dtype=dtype)


def broadcast_params(kern: torch.Tensor, lmbd, rho, group=None, src: int = 0, device=None):
    """Broadcast (kern, lambda, rho) from `src` to every rank of `group` (one packed collective).

    Non-source ranks only need to pass a kern of the right size (its values are
    overwritten).  Tensors that require grad are trainable parameters replicated by
    the training framework (DDP keeps them identical): they are returned unchanged so
    autograd reaches them.  Returns kern (1,1,k,k) or empty, lambda (1,), rho (1,).
    """
    device = device or (kern.device if kern.numel() else torch.device("cpu"))

    def trainable(v):
        return isinstance(v, torch.Tensor) and v.requires_grad

    # the PSF keeps its dtype (fp64 callers solve in fp64); lambda / rho travel as fp64 scalars
    kdt = kern.dtype if (kern.numel() and kern.is_floating_point()) else torch.float32
    k = kern if trainable(kern) else (kern.detach().to(device=device, dtype=kdt).contiguous().clone()
                                      if kern.numel() else torch.empty(0, device=device))
    lam = lmbd if trainable(lmbd) else _as_tensor(lmbd, device)
    rh = rho if trainable(rho) else _as_tensor(rho, device)
    if _collectives(group):
        parts = [t for t in (lam, rh, k) if not trainable(t)]
        if parts:
            packed = torch.cat([t.reshape(-1).to(torch.float64) for t in parts])  # one collective, exact
            dist.broadcast(packed, src=src, group=group)
            off = 0
            out = []
            for t in (lam, rh, k):
                if trainable(t):
                    out.append(t)
                else:
                    out.append(packed[off:off + t.numel()].reshape(t.shape).to(t.dtype))
                    off += t.numel()
            lam, rh, k = out
    return k, lam, rh


def sharded_fft_admm_tv(x_local: torch.Tensor, lmbd, rho, kern: torch.Tensor, iso: bool = False, maxit: int = 100,
                        *, group=None, gather: Optional[str] = None, total_batch: Optional[int] = None,
                        solver: Optional[Callable] = None) -> torch.Tensor:
    """Solve this rank's batch shard; optionally all-gather the full output.

    x_local      (b_r, C, H, W) shard owned by this rank (see shard_bounds)
    gather       None -> return the local result; "all" -> every rank gets the
                 full (B, C, H, W) output (all_gather over RCCL, shards padded
                 to equal size internally)
    solver       defaults to admmtor.eops.deconv.fft_admm_tv (the HIP path)
    """
    world = _world(group)
    coll = _collectives(group)
    if solver is None:
        from admmtor import _native
        from admmtor.eops.deconv import _fft_admm_tv_impl
        hook = _native.AllReduceHook(group) if (iso and coll) else None

        def solver(x, l, r, k, i, m):
            return _fft_admm_tv_impl(x, l, r, k, i, m, hook=hook)
    k, lam, rh = broadcast_params(kern, lmbd, rho, group=group, device=x_local.device)
    out = solver(x_local, lam, rh, k, iso, maxit)
    if gather is None or not coll:
        return out
    if gather != "all":
        raise ValueError("gather must be None or 'all'")
    sizes = shard_sizes(x_local.shape[0], group=group, total_batch=total_batch)
    B, per = sum(sizes), max(sizes)
    if out.shape[0] == per:
        src = out.contiguous()
    else:  # a short shard (B not divisible by the world size) is padded to the common size
        src = torch.zeros((per,) + tuple(out.shape[1:]), dtype=out.dtype, device=out.device)
        src[: out.shape[0]] = out
    full = torch.empty((world * per,) + tuple(out.shape[1:]), dtype=out.dtype, device=out.device)
    if hasattr(dist, "all_gather_into_tensor") and dist.get_backend(group) != "gloo":
        dist.all_gather_into_tensor(full, src, group=group)  # one RCCL collective, no staging copies
    else:
        dist.all_gather(list(full.chunk(world, 0)), src, group=group)
    if per * world == B:  # equal shards: the gathered buffer is the output
        return full
    return torch.cat([full[r * per: r * per + sizes[r]] for r in range(world)], 0)


_size_groups = {}


def _group_key(group):
    """Cache key of a process group: its global ranks (an ``id()`` can be reused by a later group
    after the first is garbage-collected, which would hand back a gloo group over other ranks)."""
    return tuple(range(dist.get_world_size())) if group is None else tuple(dist.get_process_group_ranks(group))


def make_host_group(group=None):
    """The CPU (gloo) group over the ranks of `group` that ``shard_sizes`` exchanges sizes on.

    The world (``group=None`` or a group over every rank) gets an ordinary ``new_group``: a
    collective of all ranks, named from torch's group counter, which advances on every rank alike.
    A true subgroup is created with ``use_local_synchronization=True``, so only its members enter
    the creation (a plain ``new_group`` is a collective over the whole world, and a subgroup's first
    gather would hang waiting for the ranks outside it).  torch names such a group by hashing its
    ranks with the number of groups the calling rank already knows, so two members that have seen
    different groups before would rendezvous under different names: create subgroup host groups up
    front, right after the subgroups themselves, in the same order on every rank (calling this
    function on each member).  Cached per rank set; ``shard_sizes`` otherwise creates it on first use."""
    key = _group_key(group)
    if key not in _size_groups:
        if key == tuple(range(dist.get_world_size())):
            _size_groups[key] = dist.new_group(backend="gloo")
        else:
            _size_groups[key] = dist.new_group(ranks=list(key), backend="gloo", use_local_synchronization=True)
    return _size_groups[key]


def _host_group(group):
    """A CPU (gloo) process group over the same ranks as `group`, for host-side metadata: exchanging
    shard sizes there needs no device synchronisation (an RCCL collective of a size tensor would
    need a .item() host sync, which breaks the no-sync / graph-capturable contract of b3/b5).
    A gloo `group` is used as it is; for any other backend see ``make_host_group``."""
    if dist.get_backend(group) == "gloo":
        return group
    return make_host_group(group)


def shard_sizes(local: int, group=None, total_batch: Optional[int] = None):
    """Every rank's shard size along the batch.  With `total_batch` the shards are the contiguous
    split of shard_bounds (no communication); otherwise the sizes are exchanged on the host over
    a CPU group (no device synchronisation), so any split -- also an uneven or empty shard -- works."""
    world = dist.get_world_size(group)
    if total_batch is not None:
        sizes = [e - s for s, e in (shard_bounds(int(total_batch), world, r) for r in range(world))]
        if sizes[dist.get_rank(group)] != local:
            raise ValueError(f"total_batch={total_batch}: this rank holds {local} items, shard_bounds gives "
                             f"{sizes[dist.get_rank(group)]}")
        return sizes
    t = torch.tensor([int(local)], dtype=torch.int64)
    parts = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(parts, t, group=_host_group(group))
    return [int(p[0]) for p in parts]

"""Collectives of the data-parallel step (reference DDP, train.py:300; cfg-5 global negatives).

On the product backend (``nccl`` = RCCL over xGMI) each helper is the one native collective.
Under ``gloo`` (the CPU tests, and the 1-GPU rehearsal where several ranks share one device,
which RCCL refuses) device tensors are staged through host memory, because gloo's device
support does not cover every collective; the arithmetic and the rank order are the same.

* ``all_gather_into(out, inp)``  — out = cat over ranks of inp (rank order).
* ``reduce_scatter_sum(out, inp)`` — out = Σ_ranks inp[rank·n : (rank+1)·n] (owner's slice).
* ``all_reduce_sum(t, async_op)`` — in place; returns the work handle when ``async_op``.
* ``broadcast(t, src)`` — in place.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

Tensor = torch.Tensor


def world_size(group=None) -> int:
    return dist.get_world_size(group) if dist.is_initialized() else 1


def rank(group=None) -> int:
    return dist.get_rank(group) if dist.is_initialized() else 0


def _staged(t: Tensor, group) -> bool:
    """True when the collective must run on a host copy of ``t`` (gloo + device tensor)."""
    return t.is_cuda and dist.get_backend(group) == "gloo"


class _HostWork:
    """Completed-work stand-in for staged (synchronous) collectives."""

    def wait(self) -> bool:
        return True


def all_gather_into(out: Tensor, inp: Tensor, group=None) -> None:
    if world_size(group) == 1:
        out.copy_(inp)
        return
    if _staged(inp, group):
        h = torch.empty(out.shape, dtype=out.dtype)
        dist.all_gather_into_tensor(h, inp.cpu(), group=group)
        out.copy_(h)
        return
    dist.all_gather_into_tensor(out, inp, group=group)


def reduce_scatter_sum(out: Tensor, inp: Tensor, group=None) -> None:
    if world_size(group) == 1:
        out.copy_(inp)
        return
    if _staged(inp, group):
        h = torch.empty(out.shape, dtype=out.dtype)
        dist.reduce_scatter_tensor(h, inp.cpu(), op=dist.ReduceOp.SUM, group=group)
        out.copy_(h)
        return
    dist.reduce_scatter_tensor(out, inp, op=dist.ReduceOp.SUM, group=group)


def all_reduce_sum(t: Tensor, group=None, async_op: bool = False):
    if world_size(group) == 1:
        return _HostWork() if async_op else None
    if _staged(t, group):
        h = t.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
        t.copy_(h)
        return _HostWork() if async_op else None
    return dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group, async_op=async_op)


def broadcast(t: Tensor, src: int = 0, group=None) -> None:
    if world_size(group) == 1:
        return
    if _staged(t, group):
        h = t.cpu()
        dist.broadcast(h, src=src, group=group)
        t.copy_(h)
        return
    dist.broadcast(t, src=src, group=group)


def group_src(src: int, group=None) -> int:
    """Global rank of ``src`` within ``group`` (dist.broadcast takes global ranks)."""
    if group is None or not dist.is_initialized():
        return src
    return dist.get_global_rank(group, src)


__all__ = ["world_size", "rank", "all_gather_into", "reduce_scatter_sum", "all_reduce_sum",
           "broadcast", "group_src"]

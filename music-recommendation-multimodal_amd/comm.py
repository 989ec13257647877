"""Collectives of the data-parallel step (reference DDP, train.py:300; cfg-5 global negatives).

On the product backend (``nccl`` = RCCL over xGMI) each helper is the one native collective.
Under ``gloo`` (the CPU tests, and the 1-GPU rehearsal where several ranks share one device,
which RCCL refuses) device tensors are staged through host memory, because gloo's device
support does not cover every collective; the arithmetic and the rank order are the same.

* ``all_gather_into(out, inp)``  — out = cat over ranks of inp (rank order).
* ``reduce_scatter_sum(out, inp)`` — out = Σ_ranks inp[rank·n : (rank+1)·n] (owner's slice).
* ``all_reduce_sum(t, async_op)`` — in place; returns the work handle when ``async_op``.
* ``broadcast(t, src)`` — in place.

``force_dp()`` (env ``TTMI_FORCE_DP=1``) makes a world-size-1 process group run the
data-parallel schedule: every helper then calls the real collective instead of returning early,
so RCCL itself executes (and can be timed and graph-captured) on a one-GPU box.  At world size 1
every collective is the identity, so the forced schedule must reproduce the single-process
step bit for bit (tests/test_gpu_rccl.py).

``capturable(group)``: the backend's collectives can be recorded inside a HIP graph (RCCL can;
gloo's host-side collectives cannot), so TrainStep captures the whole data-parallel step as one
graph with the all-reduces as graph nodes on RCCL's stream instead of cutting it into segments.

A staged ``all_reduce_sum(..., async_op=True)`` does not block the caller: an event recorded on
the current stream orders a device→pinned-host copy on a side stream; one worker thread per
process waits for that copy and runs the gloo reduction; ``wait()`` joins it and queues the
host→device copy on the caller's current stream.  The worker is FIFO, so ranks that issue
their buckets in the same order reduce them in the same order; every other helper (and a
synchronous all-reduce) first drains the pending staged work, so no collective overtakes one
already issued.  This is what makes the overlap of the gradient all-reduce with the rest of the
backward real under gloo (TrainStep's layer-1 cut, train.py GradSync).
"""
from __future__ import annotations

import concurrent.futures
import os
import queue
import threading

import torch
import torch.distributed as dist

Tensor = torch.Tensor


def world_size(group=None) -> int:
    return dist.get_world_size(group) if dist.is_initialized() else 1


def rank(group=None) -> int:
    return dist.get_rank(group) if dist.is_initialized() else 0


_FORCE_DP = os.environ.get("TTMI_FORCE_DP", "0") == "1"


def force_dp(on: bool = True) -> None:
    """Run the data-parallel schedule (and its collectives) even at world size 1."""
    global _FORCE_DP
    _FORCE_DP = bool(on)


def dp_active(group=None) -> bool:
    """True when the step must run its collectives: a process group of world size > 1, or any
    initialised group under ``force_dp``."""
    if not dist.is_initialized():
        return False
    return dist.get_world_size(group) > 1 or _FORCE_DP


def capturable(group=None) -> bool:
    """The group's collectives can be recorded in a HIP graph: RCCL (``nccl``) only;
    ``TTMI_CAPTURE_COLLECTIVES=0`` keeps the segmented schedule (host cuts)."""
    if not dist.is_initialized() or os.environ.get("TTMI_CAPTURE_COLLECTIVES", "1") == "0":
        return False
    return dist.get_backend(group) == "nccl"


def quiesce_before_capture(seconds: float = 0.3) -> None:
    """Call after a device synchronize, before a capture that records collectives.  torch's
    process-group watchdog polls its finished collectives about every 100 ms before retiring
    them.  The first collective recorded in a capture joins the group's stream to that capture.
    A finished collective still listed from before then has its event queried on a capturing
    stream: HIP refuses the query (hipErrorCapturedEvent) and the watchdog aborts the process.
    This was seen once in the GPU suite with thread-local capture.  Waiting a few polls lets
    the watchdog retire every earlier collective first."""
    import time
    time.sleep(seconds)


def _staged(t: Tensor, group) -> bool:
    """True when the collective must run on a host copy of ``t`` (gloo + device tensor)."""
    return t.is_cuda and dist.get_backend(group) == "gloo"


class _HostWork:
    """Completed-work stand-in (world size 1)."""

    def wait(self) -> bool:
        return True


class _Stager:
    """The asynchronous gloo staging of device tensors (module docstring).  Pinned host
    buffers are cached per (device pointer, bytes): a bucket's buffer is reused every step."""

    def __init__(self):
        self.pool = None
        self.lock = threading.Lock()
        self.pending = []
        self.host = {}
        self.side = {}
        # set when a staged reduction timed out: its worker thread may still be stuck in it
        # (and may later write the pinned buffer), so neither is used again
        self.broken = None

    def _executor(self):
        if self.pool is None:
            self.pool = _FifoWorker()
        return self.pool

    def _buffer(self, t: Tensor) -> Tensor:
        key = (t.data_ptr(), t.numel(), t.dtype)
        h = self.host.get(key)
        if h is None:
            h = torch.empty(t.shape, dtype=t.dtype, pin_memory=t.is_cuda and torch.cuda.is_available())
            self.host[key] = h
        return h.view(t.shape)

    def all_reduce(self, t: Tensor, group) -> "_StagedWork":
        self.check()
        h = self._buffer(t)
        ev = None
        if t.is_cuda:
            ready = torch.cuda.Event()
            ready.record()                                   # the gradient slice is final here
            side = self.side.get(t.device)
            if side is None:
                side = self.side[t.device] = torch.cuda.Stream(device=t.device)
            with torch.cuda.stream(side):
                side.wait_event(ready)
                h.copy_(t, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
        else:
            h.copy_(t)

        def run():
            if ev is not None:
                ev.synchronize()
            dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
        w = _StagedWork(self, t, h, self._executor().submit(run))
        with self.lock:
            self.pending.append(w)
        return w

    def check(self) -> None:
        if self.broken is not None:
            raise RuntimeError(f"comm: a staged gloo all-reduce timed out earlier ({self.broken}); "
                               "the staging worker is unusable for the rest of this process")

    def drain(self) -> None:
        with self.lock:
            works, self.pending = self.pending, []
        for w in works:
            w.wait()


class _FifoWorker:
    """One daemon thread running submitted reductions in order (a ThreadPoolExecutor's worker is
    joined at interpreter exit, so a reduction stuck on a dead peer would block the exit)."""

    def __init__(self):
        self.q = queue.Queue()
        threading.Thread(target=self._loop, name="ttmi-gloo", daemon=True).start()

    def _loop(self) -> None:
        while True:
            fut, fn = self.q.get()
            if not fut.set_running_or_notify_cancel():
                continue
            try:
                fut.set_result(fn())
            except BaseException as exc:                     # handed to the waiter
                fut.set_exception(exc)

    def submit(self, fn) -> concurrent.futures.Future:
        fut = concurrent.futures.Future()
        self.q.put((fut, fn))
        return fut


# seconds a staged reduction may take before wait() gives up (a peer that never joins)
STAGED_TIMEOUT_S = float(os.environ.get("TTMI_GLOO_TIMEOUT", "600"))


class _StagedWork:
    def __init__(self, stager: _Stager, t: Tensor, h: Tensor, fut):
        self.stager, self.t, self.h, self.fut = stager, t, h, fut
        self.done = False

    def is_completed(self) -> bool:
        return self.done or self.fut.done()

    def wait(self) -> bool:
        if self.done:
            return True
        self.stager.check()
        try:       # re-raises a failed reduction once; it leaves `pending` either way
            self.fut.result(timeout=STAGED_TIMEOUT_S)
        except concurrent.futures.TimeoutError:
            self.stager.broken = f"no result after {STAGED_TIMEOUT_S:.0f} s"
            raise
        finally:
            with self.stager.lock:
                if self in self.stager.pending:
                    self.stager.pending.remove(self)
        # ordered on the caller's stream ahead of every later consumer; the pinned buffer is
        # only rewritten by a later start, whose copy waits for an event recorded after this
        self.t.copy_(self.h, non_blocking=self.t.is_cuda)
        self.done = True
        return True


_STAGER = _Stager()


def drain() -> None:
    """Complete every pending staged all-reduce (in issue order)."""
    if _STAGER.pending:
        _STAGER.drain()


def all_gather_into(out: Tensor, inp: Tensor, group=None) -> None:
    drain()
    if not dp_active(group):
        out.copy_(inp)
        return
    if _staged(inp, group):
        h = torch.empty(out.shape, dtype=out.dtype)
        dist.all_gather_into_tensor(h, inp.cpu(), group=group)
        out.copy_(h)
        return
    dist.all_gather_into_tensor(out, inp, group=group)


def reduce_scatter_sum(out: Tensor, inp: Tensor, group=None) -> None:
    drain()
    if not dp_active(group):
        out.copy_(inp)
        return
    if _staged(inp, group):
        h = torch.empty(out.shape, dtype=out.dtype)
        dist.reduce_scatter_tensor(h, inp.cpu(), op=dist.ReduceOp.SUM, group=group)
        out.copy_(h)
        return
    dist.reduce_scatter_tensor(out, inp, op=dist.ReduceOp.SUM, group=group)


def all_reduce_sum(t: Tensor, group=None, async_op: bool = False):
    if not dp_active(group):
        return _HostWork() if async_op else None
    if _staged(t, group) or (_FORCE_STAGE and async_op):
        w = _STAGER.all_reduce(t, group)
        if async_op:
            return w
        drain()
        return None
    drain()
    return dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group, async_op=async_op)


# tests: stage host tensors too, so the asynchronous path runs on a CPU-only gloo world
_FORCE_STAGE = False


def broadcast(t: Tensor, src: int = 0, group=None) -> None:
    drain()
    if not dp_active(group):
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
           "broadcast", "group_src", "drain", "force_dp", "dp_active", "capturable"]

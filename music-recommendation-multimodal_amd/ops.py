"""Torch-tensor wrappers over the libttmi C ABI (include/ttmi.h).

Every wrapper launches on ``torch.cuda.current_stream()`` and returns immediately; none
allocates inside the library (outputs come from the torch caching allocator), so a whole
step can be captured into a HIP graph.  Shapes are checked here and again in C.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import warnings
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from . import lib as _L
from .lib import (BF16, F32, BnBwdDesc, ConvDesc, DisAttnDesc, FoldDesc, GemmDesc, LnBwdDesc,
                  UserHeadBwdDesc, UserHeadDesc, ItemHeadBwdDesc, ItemHeadDesc, WgradDesc, call)

Tensor = torch.Tensor
# Dropout spec: (p, seed) where seed is a 1-element int64 DEVICE tensor holding the 64-bit
# seed bits (a view into a per-step seed table), or None when p == 0.
Drop = Tuple[float, Optional[Tensor]]
NO_DROP: Drop = (0.0, None)

_DT = {torch.float32: F32, torch.bfloat16: BF16}


def code(dtype: torch.dtype) -> int:
    try:
        return _DT[dtype]
    except KeyError:
        raise TypeError(f"unsupported dtype {dtype} (float32 / bfloat16)") from None


def _p(t: Optional[Tensor]):
    return None if t is None else t.data_ptr()


def _s():
    return torch.cuda.current_stream().cuda_stream


def _dev(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise ValueError("libttmi ops need GPU tensors")


# ----------------------------------------------------------------------------- id range flags
# The reference's nn.Embedding lookups raise IndexError for an id outside the table
# (user_tower.py:26,30-31; the DeBERTa word embedding; the catalogue assignment
# evaluate_metrics.py:102).  The device lookups never index outside a table (include/ttmi.h
# TTMI_IDERR_*): they clamp / skip and set a flag in two places (ABI 22): a device int32[8] that
# the fused AdamW reads (``skip_if``: a step that met a bad id updates no parameter, as the
# reference raises before optimizer.step()) and that TrainStep clears when it stages a batch; and
# a host-mapped int32[8] (hipHostMalloc, mapped + coherent), so reading them needs no device
# sync and costs the step nothing: check_id_errors() raises once the flagging launch has run
# (the next step / forward, or any point after a sync).
ID_ERR_KEYS = ("history_ids", "user_gender", "user_country", "target_input_ids", "target_id")
_IDERR_HEAD_POLL = 7        # TTMI_IDERR_HEAD_POLL: not an id, the co-launched head's poll timed out
_N_IDERR = 8


def _hip_runtime():
    """The HIP runtime torch has loaded (found in this process's mappings, whatever its soname
    version), opened without loading a second copy; None if there is none."""
    paths = []
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                i = line.find("/")
                if i >= 0 and "libamdhip64.so" in line[i:]:
                    paths.append(line[i:].strip())
    except OSError:
        pass
    for name in dict.fromkeys(paths + ["libamdhip64.so", "libamdhip64.so.7", "libamdhip64.so.6"]):
        try:
            return ctypes.CDLL(name, mode=os.RTLD_NOLOAD)
        except OSError:
            continue
    return None


_WARNED_NO_HOST_MAP = [False]


class _IdFlags:
    """The id_err block of one device (include/ttmi.h, ABI 22): ``dev`` int32[16] on the device —
    flags [0, 8) and, at byte 32, the device address of the host-mapped int32[8] ``host`` — and
    ``dptr`` (what the kernels get).  If the runtime refuses the host mapping, the pointer slot
    stays NULL and the device flags are read on sync only (warned once).  The 32-byte pinned
    block lives as long as the process (one per device; never freed)."""

    def __init__(self, device: torch.device):
        self.host = None
        self.dev = torch.zeros(16, dtype=torch.int32, device=device)
        self.zeros = torch.zeros(_N_IDERR, dtype=torch.int32, device=device)
        self.dptr = self.dev.data_ptr()
        hip = _hip_runtime()
        if hip is not None:
            ptr, dptr = ctypes.c_void_p(), ctypes.c_void_p()
            flags = 0x1 | 0x2 | 0x40000000      # hipHostMallocPortable | Mapped | Coherent
            with torch.cuda.device(device):
                if hip.hipHostMalloc(ctypes.byref(ptr), ctypes.c_size_t(4 * _N_IDERR),
                                     ctypes.c_uint(flags)) == 0 and \
                        hip.hipHostGetDevicePointer(ctypes.byref(dptr), ptr, ctypes.c_uint(0)) == 0:
                    self.host = (ctypes.c_int32 * _N_IDERR).from_address(ptr.value)
                    for i in range(_N_IDERR):
                        self.host[i] = 0
                    self.dev.view(torch.int64)[4] = dptr.value
        if self.host is None and not _WARNED_NO_HOST_MAP[0]:
            _WARNED_NO_HOST_MAP[0] = True
            warnings.warn("libttmi: no host-mapped id-range flags (HIP runtime not found or the "
                          "mapping was refused); out-of-table ids are reported only by "
                          "check_id_errors(sync=True) / TrainStep.check()", RuntimeWarning)

    def take(self, sync: bool) -> List[int]:
        """Indices of the raised flags (cleared).  A flag raised again between the read and the
        clear is lost, which only drops a duplicate report: the caller raises for the first."""
        if self.host is not None:
            vals = list(self.host)
            for i, v in enumerate(vals):
                if v:
                    self.host[i] = 0
        elif sync:
            vals = self.dev[:_N_IDERR].tolist()
            if any(vals):
                self.dev[:_N_IDERR].zero_()
        else:
            return []
        return [i for i, v in enumerate(vals) if v]


_IDF: Dict[int, _IdFlags] = {}


def _id_flags(t: Tensor) -> _IdFlags:
    idx = t.device.index if t.device.index is not None else torch.cuda.current_device()
    f = _IDF.get(idx)
    if f is None:
        if torch.cuda.is_current_stream_capturing():
            # the block's zero fill and pointer write would be recorded, not run
            raise RuntimeError("libttmi: the id-range flag block is first needed inside a graph "
                               "capture; run the captured ops once eagerly first (a warm-up)")
        f = _IDF[idx] = _IdFlags(torch.device("cuda", idx))
    return f


def id_err_ptr(t: Tensor) -> int:
    """Device pointer of the id_err block of ``t``'s device (allocated on first use); also
    AdamW's ``skip_if``."""
    return _id_flags(t).dptr


def id_err_flags(t: Tensor) -> Tensor:
    """The device half of the id_err block of ``t``'s device: int32[8], a raised flag holds the
    bit pattern of 1.0f (include/ttmi.h)."""
    return _id_flags(t).dev[:_N_IDERR]


def id_err_step_reset(t: Tensor):
    """(dst, src) for batch_copy: zeroes the device flags of ``t``'s device (the per-step half
    that AdamW's skip_if reads; TrainStep does this in its staging launch)."""
    f = _id_flags(t)
    return f.dev[:_N_IDERR], f.zeros


def check_id_errors(sync: bool = False) -> None:
    """Raise IndexError (as nn.Embedding does) if a device lookup has met an id outside its
    table since the last check; the flags are cleared.  sync=True first waits for the device,
    so every launch issued so far is covered; otherwise only launches that have finished."""
    if not _IDF:
        return
    if sync:
        torch.cuda.synchronize()
    for f in _IDF.values():
        bad = f.take(sync)
        if _IDERR_HEAD_POLL in bad:
            raise RuntimeError("ttmi_user_item_head_fwd_ac: the item head's stage-C poll timed out "
                               "(TTMI_HEAD_AC=1); that step's item embeddings are invalid")
        if bad:
            keys = ", ".join(ID_ERR_KEYS[i] if i < len(ID_ERR_KEYS) else f"flag {i}" for i in bad)
            raise IndexError(f"index out of range in self: {keys} held an id outside its embedding "
                             f"table (the device lookup was clamped)")


# ----------------------------------------------------------------------------- GEMM
def gemm(A: Tensor, B: Tensor, C: Tensor, M: int, N: int, K: int, *, lda: int, a_kmajor: bool,
         ldb: int, b_kmajor: bool, ldc: int, accumulate: bool = False, alpha: float = 1.0,
         bias: Optional[Tensor] = None, act: int = 0, drop: Drop = NO_DROP, ld_drop: int = 0,
         gate: Optional[Tensor] = None, ld_gate: int = 0, gate_scale: float = 1.0,
         residual: Optional[Tensor] = None, ld_res: int = 0, colsum: Optional[Tensor] = None,
         split_k: int = 1, drop_rows: Optional[Tensor] = None,
         rowsum_a: Optional[Tensor] = None, pre_out: Optional[Tensor] = None) -> Tensor:
    """C = epi(alpha · A·Bᵀ) (include/ttmi.h ttmi_gemm).  pre_out (bf16, with act 2): also
    store the pre-activation there, same row stride as C."""
    _dev(A, B, C)
    if pre_out is not None and (pre_out.dtype != torch.bfloat16 or pre_out.device != C.device):
        raise TypeError("gemm: pre_out must be a bf16 tensor on C's device")
    if A.dtype != B.dtype:
        raise TypeError(f"gemm operands differ in dtype: {A.dtype} vs {B.dtype}")
    d = GemmDesc()
    d.dtype = code(A.dtype)
    d.M, d.N, d.K = M, N, K
    d.A, d.lda, d.a_kmajor = _p(A), lda, int(a_kmajor)
    d.B, d.ldb, d.b_kmajor = _p(B), ldb, int(b_kmajor)
    d.C, d.ldc, d.c_dtype, d.c_mode = _p(C), ldc, code(C.dtype), int(accumulate)
    d.alpha = alpha
    d.bias = _p(bias)
    d.act = act
    d.drop_p, d.drop_seed, d.ld_drop = float(drop[0]), _p(drop[1]), ld_drop
    d.gate, d.gate_dtype, d.ld_gate, d.gate_scale = (
        _p(gate), code(gate.dtype) if gate is not None else 0, ld_gate, gate_scale)
    d.residual, d.ld_res = _p(residual), ld_res
    d.colsum = _p(colsum)
    d.split_k = split_k
    d.drop_rows = _p(drop_rows)
    d.rowsum_a = _p(rowsum_a)
    d.pre_out = _p(pre_out)
    call("ttmi_gemm", ctypes.byref(d), _s())
    return C


def linear(x: Tensor, w: Tensor, bias: Optional[Tensor], out: Tensor, *, act: int = 0,
           drop: Drop = NO_DROP, residual: Optional[Tensor] = None,
           drop_rows: Optional[Tensor] = None, gate: Optional[Tensor] = None,
           gate_scale: float = 1.0) -> Tensor:
    """out[M,N] = epi(x[M,K] · w[N,K]ᵀ + bias)  (nn.Linear forward; with w = Wᵀ mirror and a
    gate, the input grad of a ReLU/dropout-gated Linear); dropout indices use drop_rows[m]
    (int32) as the row when given (pruned last layer)."""
    M, K = x.shape
    N = w.shape[0]
    return gemm(x, w, out, M, N, K, lda=K, a_kmajor=True, ldb=K, b_kmajor=True, ldc=N,
                bias=bias, act=act, drop=drop, ld_drop=N, residual=residual, ld_res=N,
                drop_rows=drop_rows, gate=gate, ld_gate=N, gate_scale=gate_scale)


def linear_dx(dy: Tensor, w: Tensor, out: Tensor, *, gate: Optional[Tensor] = None,
              gate_scale: float = 1.0, colsum: Optional[Tensor] = None) -> Tensor:
    """out[M,K] = (dy[M,N] · w[N,K]) ⊙ gate-mask  (nn.Linear input grad)."""
    M, N = dy.shape
    K = w.shape[1]
    return gemm(dy, w, out, M, K, N, lda=N, a_kmajor=True, ldb=K, b_kmajor=False, ldc=K,
                gate=gate, ld_gate=K, gate_scale=gate_scale, colsum=colsum)


class WgradPending:
    """Parameter gradients still to be completed: weight-gradient GEMMs recorded but not yet
    launched (their operands kept alive here) and LayerNorm weight/bias sums whose
    per-workgroup partials sit in workspaces (ttmi_linear_ln_bwd with sum_ws).  ``flush()``
    runs every recorded GEMM as one grouped launch and folds all partials in a fixed order
    (ttmi_wgrad_batch: two launches per flush)."""

    def __init__(self, defer_fold: bool = False):
        self.items = []
        self.folds = []
        self.slots: Dict[str, int] = {}
        # defer_fold (ABI 19, one process): the flush runs the grouped GEMMs only and leaves
        # the partials to the optimizer (``plan`` for adamw(fold_plan=...); ``keep`` holds the
        # partials' workspaces and operands until that update has been issued)
        self.defer_fold = defer_fold
        self.plan = None
        self.keep: list = []
        self.side = None          # launch_early's stream, joined by flush()
        self.side_flushed = None  # flush_on's stream, joined by join()
        self.hold_join = False    # flush() leaves the join to the caller (join())

    def slot(self, key: str) -> int:
        """Index of the next persistent zero workspace for ``key`` within this block: calls
        whose partials wait for the same flush must not share one (the k-th call of a step
        always gets slot k, so graph replays reuse the same buffers)."""
        k = self.slots.get(key, 0)
        self.slots[key] = k + 1
        return k

    def launch_early(self, side: "torch.cuda.Stream") -> bool:
        """defer_fold only: run the GEMMs recorded so far now, as one grouped launch on ``side``
        (after the current stream's work), so they overlap what the current stream does next;
        their fold segments join the folds' at flush(), which also joins ``side``.  Nothing may
        be recorded after this call but LayerNorm sums / fixed-point folds."""
        if not self.defer_fold or self.plan is not None or not self.items:
            return False
        arr = (ctypes.POINTER(WgradDesc) * len(self.items))(*[ctypes.pointer(d) for d, *_ in self.items])
        side.wait_stream(torch.cuda.current_stream(side.device))
        self.plan = _L.FoldPlan()
        with torch.cuda.stream(side):
            call("ttmi_wgrad_batch_plan", len(self.items), arr, 0, (FoldDesc * 1)(),
                 ctypes.byref(self.plan), _s())
        self.keep = self.keep + self.items
        self.items = []
        self.side = side
        return True

    def join(self) -> None:
        """The current stream waits for launch_early's GEMMs and flush_on's work (no-op when
        neither ran)."""
        for st in (self.side, self.side_flushed):
            if st is not None:
                torch.cuda.current_stream(st.device).wait_stream(st)
        self.side = None
        self.side_flushed = None

    def flush_on(self, side: "torch.cuda.Stream") -> None:
        """Complete every weight gradient and fold recorded so far on ``side`` (after the current
        stream's work): the data-parallel step's first bucket, whose all-reduce then follows on
        ``side`` while the current stream goes on with the rest of the backward.  Operands are
        kept alive until join()."""
        if self.side is not None or self.plan is not None:
            raise RuntimeError("WgradPending.flush_on: after launch_early")
        side.wait_stream(torch.cuda.current_stream(side.device))
        with torch.cuda.stream(side):
            if self.items or self.folds:
                arr = (ctypes.POINTER(WgradDesc) * max(len(self.items), 1))(
                    *[ctypes.pointer(d) for d, *_ in self.items])
                farr = (FoldDesc * max(len(self.folds), 1))(*[f for f, *_ in self.folds])
                call("ttmi_wgrad_batch", len(self.items), arr, len(self.folds), farr, _s())
        self.keep = self.keep + self.items + self.folds
        self.items = []
        self.folds = []
        self.slots = {}
        self.side_flushed = side

    def flush(self) -> None:
        if self.side is not None:         # launch_early ran: plan the folds, join the GEMMs
            if self.items:
                raise RuntimeError("WgradPending: weight gradients recorded after launch_early")
            if self.folds:
                farr = (FoldDesc * len(self.folds))(*[f for f, *_ in self.folds])
                p2 = _L.FoldPlan()
                call("ttmi_wgrad_batch_plan", 0, (ctypes.POINTER(WgradDesc) * 1)(), len(self.folds), farr,
                     ctypes.byref(p2), _s())
                call("ttmi_fold_plan_merge", ctypes.byref(self.plan), ctypes.byref(p2), _s())
                self.keep = self.keep + self.folds
            if not self.hold_join:
                self.join()
            self.folds = []
            self.slots = {}
            return
        if not self.items and not self.folds:
            return
        arr = (ctypes.POINTER(WgradDesc) * max(len(self.items), 1))(
            *[ctypes.pointer(d) for d, *_ in self.items])
        farr = (FoldDesc * max(len(self.folds), 1))(*[f for f, *_ in self.folds])
        if self.defer_fold and self.plan is None:
            self.plan = _L.FoldPlan()
            call("ttmi_wgrad_batch_plan", len(self.items), arr, len(self.folds), farr,
                 ctypes.byref(self.plan), _s())
            self.keep = self.keep + self.items + self.folds
        else:
            call("ttmi_wgrad_batch", len(self.items), arr, len(self.folds), farr, _s())
        self.items = []
        self.folds = []
        self.slots = {}


_PENDING: List[WgradPending] = []


@contextlib.contextmanager
def deferred_wgrad(defer_fold: bool = False):
    """Inside the block, bf16 ``linear_dw`` calls (and the fused LN-backward's weight sums)
    are deferred to the yielded WgradPending (flushed, at the latest, on exit): a backward's
    weight gradients become one grouped GEMM launch plus one fold launch.  ``defer_fold``:
    the last flush leaves the fold to ``adamw(fold_plan=pend.plan)`` (one process only)."""
    pend = WgradPending(defer_fold)
    _PENDING.append(pend)
    try:
        yield pend
    finally:
        _PENDING.pop()
        pend.flush()


_WG_SIDE: Dict[str, "torch.cuda.Stream"] = {}
_WG_EARLY = os.environ.get("TTMI_WGRAD_EARLY", "1") != "0"


def wgrad_side_stream(dev) -> "torch.cuda.Stream":
    """The per-device side stream of the weight-gradient GEMMs (created on first use, i.e. in an
    eager step before any graph capture)."""
    key = str(dev)
    if key not in _WG_SIDE:
        _WG_SIDE[key] = torch.cuda.Stream(dev)
    return _WG_SIDE[key]


def fold_plan_run(plan) -> None:
    """Fold a WgradPending plan's segments now (ttmi_fold_plan_run): the data-parallel step
    completes its gradient before the all-reduce instead of folding inside AdamW."""
    call("ttmi_fold_plan_run", ctypes.byref(plan), _s())


def wgrad_launch_early() -> bool:
    """Inside ``deferred_wgrad(defer_fold=True)``: launch the weight-gradient GEMMs recorded so
    far on a side stream (created per device on first use, i.e. in an eager step before any
    graph capture) so they overlap the rest of the backward (``TTMI_WGRAD_EARLY=0``: at the
    block's exit, as before).  Results are unchanged: same GEMMs, same fold order."""
    if not (_WG_EARLY and _PENDING):
        return False
    pend = _PENDING[-1]
    if not pend.defer_fold or not pend.items:
        return False
    return pend.launch_early(wgrad_side_stream(pend.items[0][2].device))


def linear_dw(dy: Tensor, x: Tensor, gw: Tensor, gb: Optional[Tensor] = None,
              split_k: int = 0, defer: bool = True) -> Tensor:
    """gw[N,K] += dy[M,N]ᵀ · x[M,K]; gb[N] += Σ_m dy[m,:] (nn.Linear weight and bias grads,
    accumulated).  bf16 operands: ttmi_wgrad (split partials summed in a fixed order: the
    result is bit-reproducible); fp32 operands: the generic split-K GEMM.  Inside
    ``deferred_wgrad()`` the GEMM runs at the block's flush (grouped with the others) unless
    ``defer=False`` (callers that read gw right away); dy and x must not change before then."""
    M, N = dy.shape
    K = x.shape[1]
    if dy.dtype != torch.bfloat16 or x.dtype != torch.bfloat16:
        return gemm(dy, x, gw, N, K, M, lda=dy.stride(0), a_kmajor=False, ldb=x.stride(0),
                    b_kmajor=False, ldc=gw.stride(0), accumulate=True, split_k=split_k,
                    rowsum_a=gb)
    _dev(dy, x, gw)
    if gw.dtype != torch.float32 or (gb is not None and gb.dtype != torch.float32):
        raise TypeError("linear_dw: weight / bias gradients must be fp32")
    _L.load()
    d = WgradDesc()
    d.R, d.M, d.N = M, N, K
    d.dy, d.ld_dy = _p(dy), dy.stride(0)
    d.x, d.ld_x = _p(x), x.stride(0)
    d.dw, d.ld_dw = _p(gw), gw.stride(0)
    d.db = _p(gb)
    d.alpha = 1.0
    d.accumulate = 1
    nbytes = int(_L._lib.ttmi_wgrad_workspace(M, N, K, d.ld_dy, d.ld_x))
    ws = torch.empty(nbytes, device=dy.device, dtype=torch.uint8) if nbytes else None
    d.workspace, d.workspace_bytes = _p(ws), nbytes
    pend = _PENDING[-1] if (_PENDING and defer) else None
    if pend is not None:                 # computed, with the block's others, at the flush
        pend.items.append((d, ws, dy, x, gw, gb))
        return gw
    d.defer = 0
    call("ttmi_wgrad", ctypes.byref(d), _s())
    return gw


def linear_ln_bwd(dh: Tensor, wt: Tensor, x: Tensor, mean: Tensor, rstd: Tensor, ln_w: Tensor,
                  dx: Tensor, ln_dw: Optional[Tensor], ln_db: Optional[Tensor], *,
                  res: Optional[Tensor] = None, next_: Optional[Tensor] = None,
                  drop: Drop = NO_DROP, drop_rows: Optional[Tensor] = None,
                  res_rows: Optional[Tensor] = None, res_L: int = 0,
                  dy_add: Optional[Tensor] = None) -> Tensor:
    """dx = LN'(dh · wtᵀ) + res; ln_dw/ln_db += LN param grads; next_ = bf16(dropout(dx))
    (one kernel: the Linear input grad, LayerNorm backward and dropout backward).  res_rows:
    res is [M / res_L, N] and its row b is added only to row res_rows[b] (b = m / res_L);
    dy_add (fp32 [M / res_L, N], with res_rows): its row b joins dh·wtᵀ of row res_rows[b]
    before the LayerNorm backward (ABI 21)."""
    if dy_add is not None and (res_rows is None or tuple(dy_add.shape) != (res_rows.shape[0], wt.shape[0])):
        raise ValueError("linear_ln_bwd: dy_add needs res_rows and shape [M / res_L, N]")
    if res_rows is not None and (res is None or res_L <= 0 or res.shape[0] * res_L != dh.shape[0]):
        raise ValueError("linear_ln_bwd: res_rows needs res [M / res_L, N]")
    _dev(dh, wt, x, dx)
    M, K = dh.shape
    N = wt.shape[0]
    d = LnBwdDesc()
    d.M, d.N, d.K = M, N, K
    d.dh, d.ld_dh = _p(dh), dh.stride(0)
    d.wt, d.ld_wt = _p(wt), wt.stride(0)
    d.x, d.ldx = _p(x), x.stride(0)
    d.mean, d.rstd, d.ln_w = _p(mean), _p(rstd), _p(ln_w)
    d.res, d.ld_res = _p(res), (res.stride(0) if res is not None else 0)
    d.dx, d.lddx = _p(dx), dx.stride(0)
    d.next, d.ld_next = _p(next_), (next_.stride(0) if next_ is not None else 0)
    d.drop_p, d.drop_seed, d.ld_drop = float(drop[0]), _p(drop[1]), N
    d.drop_rows = _p(drop_rows)
    d.res_rows, d.res_L = _p(res_rows), int(res_L)
    d.dy_add, d.ld_add = _p(dy_add), (dy_add.stride(0) if dy_add is not None else 0)
    d.ln_dw, d.ln_db = _p(ln_dw), _p(ln_db)
    folds = []
    if ln_dw is not None or ln_db is not None:
        # per-workgroup sums, folded in workgroup order (with the step's weight gradients
        # inside deferred_wgrad, else right after the launch): bit-reproducible
        _L.load()
        G = int(_L._lib.ttmi_linear_ln_bwd_sum_blocks_n(M, N))
        ws = torch.empty(G * 2 * N, device=dx.device, dtype=torch.float32)
        d.sum_ws = _p(ws)
        for j, g in enumerate((ln_dw, ln_db)):
            if g is not None:
                f = FoldDesc()
                f.part, f.S, f.s_stride, f.M, f.N = ws.data_ptr() + 4 * N * j, G, 2 * N, 1, N
                f.C, f.ldc, f.accumulate, f.fx_shift = _p(g), N, 1, 0
                folds.append((f, ws, g))
    call("ttmi_linear_ln_bwd", ctypes.byref(d), _s())
    _run_folds(folds)
    return dx


def linear_res_ln(x: Tensor, w: Tensor, bias: Optional[Tensor], residual: Tensor, out: Tensor,
                  ln_w: Tensor, ln_b: Tensor, y: Tensor, mean: Tensor, rstd: Tensor, *,
                  eps: float = 1e-5, drop: Drop = NO_DROP) -> Tensor:
    """out = residual + dropout(x·wᵀ + bias) (fp32), y = bf16(LN(out)·ln_w + ln_b), mean/rstd:
    a residual sub-block's end and the following LayerNorm in one kernel (N = 128, or N = 256
    with K in {256, 512, 768, 1024}: the streamed-W panel, ABI 19)."""
    _dev(x, w, residual, out, y)
    M, K = x.shape
    N = w.shape[0]
    d = _L.ResLnDesc()
    d.M, d.N, d.K = M, N, K
    d.x, d.ldx = _p(x), x.stride(0)
    d.w, d.ldw = _p(w), w.stride(0)
    d.bias = _p(bias)
    d.drop_p, d.drop_seed, d.ld_drop = float(drop[0]), _p(drop[1]), N
    d.residual, d.ld_res = _p(residual), residual.stride(0)
    d.out, d.ld_out = _p(out), out.stride(0)
    d.ln_w, d.ln_b, d.eps = _p(ln_w), _p(ln_b), float(eps)
    d.y, d.ldy = _p(y), y.stride(0)
    d.mean, d.rstd = _p(mean), _p(rstd)
    call("ttmi_linear_res_ln", ctypes.byref(d), _s())
    return out


# ----------------------------------------------------------------------------- cfg 5 pieces
def l2norm_fwd(x: Tensor, y: Tensor, norms: Tensor) -> Tensor:
    _dev(x, y, norms)
    n, D = x.shape
    call("ttmi_l2norm_fwd", n, D, _p(x), _p(y), _p(norms), _s())
    return y


def l2norm_bwd(y: Tensor, norms: Tensor, dy: Tensor, dx: Tensor,
               dy2: Optional[Tensor] = None) -> Tensor:
    n, D = y.shape
    call("ttmi_l2norm_bwd", n, D, _p(y), _p(norms), _p(dy), _p(dy2), _p(dx), _s())
    return dx


def rowce_fwd(q: Tensor, k: Tensor, uid_q: Optional[Tensor], uid_k: Optional[Tensor], row0: int,
              inv_tau: float, logits: Tensor, lse: Tensor, ce: Tensor) -> Tensor:
    """logits = q·kᵀ·inv_tau (collision-masked), lse, ce per row; positives at row0 + i."""
    _dev(q, k, logits)
    R, D = q.shape
    C = k.shape[0]
    call("ttmi_rowce_fwd", R, C, D, _p(q), _p(k), _p(uid_q), _p(uid_k), row0, inv_tau,
         _p(logits), _p(lse), _p(ce), _s())
    return logits


def rowce_bwd(q: Tensor, k: Tensor, logits: Tensor, lse: Tensor, uid_q: Optional[Tensor],
              uid_k: Optional[Tensor], row0: int, inv_tau: float, dloss: Optional[Tensor],
              scale: float, dq: Tensor, dk: Tensor) -> None:
    R, D = q.shape
    C = k.shape[0]
    _L.load()
    ws = torch.empty(int(_L._lib.ttmi_rowce_workspace(R, C)), device=q.device,
                     dtype=torch.uint8)
    call("ttmi_rowce_bwd", R, C, D, _p(q), _p(k), _p(logits), _p(lse), _p(uid_q), _p(uid_k),
         row0, inv_tau, _p(dloss), scale, _p(dq), _p(dk), _p(ws), _s())


def sum_scaled(x: Tensor, scale: float, out: Tensor) -> Tensor:
    call("ttmi_sum_scaled", x.numel(), _p(x), scale, _p(out), _s())
    return out


# ----------------------------------------------------------------------------- convolution
FWD, DGRAD, WGRAD = 0, 1, 2


def conv_out_hw(H: int, W: int, k: int, stride: int, pad: int):
    return (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1


CONV_STAT_REPS = 16    # TTMI_CONV_STAT_REPS: BatchNorm column stats are [16][C] int64 replica rows
ATTN_LMAX = 2048       # TTMI_ATTN_LMAX: longest sequence the attention kernels take


def conv2d(mode: int, N: int, H: int, W: int, C: int, Cin: int, Co: int, k: int, stride: int,
           pad: int, *, x: Optional[Tensor] = None, dy: Optional[Tensor] = None,
           w: Optional[Tensor] = None, out: Tensor, addend: Optional[Tensor] = None,
           colsum: Optional[Tensor] = None, colsumsq: Optional[Tensor] = None,
           bn: Optional[Tuple[Optional[Tensor], Tensor, Tensor, Tensor, Tensor]] = None) -> Tensor:
    """Implicit-GEMM conv (include/ttmi.h ttmi_conv2d): FWD y = conv(x), DGRAD dx, WGRAD dW.
    DGRAD ``bn`` = (gate, x, mean, rstd, sums): the backward reduction of the BatchNorm(+ReLU)
    that produced the conv input, fused into the epilogue (out then holds the gated g)."""
    Ho, Wo = conv_out_hw(H, W, k, stride, pad)
    xn = N * (H // 2) * (W // 2) * C if mode in (STEM_FWD, STEM_WGRAD) else N * H * W * C
    need = {"x": (x, xn), "dy": (dy, N * Ho * Wo * Co),
            "colsum": (colsum, CONV_STAT_REPS * Co), "colsumsq": (colsumsq, CONV_STAT_REPS * Co)}
    if mode == STEM_FWD:
        need.update(w=(w, Co * 16 * C), out=(out, N * Ho * Wo * Co))
    elif mode == FWD:
        need.update(w=(w, Co * k * k * C), out=(out, N * Ho * Wo * Co))
    elif mode == DGRAD:
        need.update(w=(w, C * k * k * Co), out=(out, N * H * W * C), addend=(addend, N * H * W * C))
    else:
        need.update(out=(out, Co * Cin * k * k))
    for name, (t, n) in need.items():       # an undersized buffer would fault the GPU
        if t is not None and t.numel() < n:
            raise ValueError(f"conv2d: {name} has {t.numel()} elements, needs {n}")
    for t in (colsum, colsumsq):
        if t is not None and t.dtype != torch.int64:
            raise TypeError("conv2d: colsum / colsumsq are int64 fixed-point replica rows")
    d = ConvDesc()
    d.mode, d.N, d.H, d.W, d.C, d.Cin, d.Co = mode, N, H, W, C, Cin, Co
    d.KH = d.KW = k
    d.stride, d.pad = stride, pad
    d.x, d.dy, d.w, d.out, d.addend = _p(x), _p(dy), _p(w), _p(out), _p(addend)
    d.colsum, d.colsumsq = _p(colsum), _p(colsumsq)
    if bn is not None:
        if mode != DGRAD:
            raise ValueError("conv2d: bn (fused BatchNorm-backward reduction) is a DGRAD option")
        gate, bx, bmean, brstd, bsums = bn
        n_in = N * H * W * C
        if bx.numel() < n_in or (gate is not None and gate.numel() < n_in):
            raise ValueError("conv2d: bn gate / x smaller than the DGRAD output")
        if bsums.numel() < 2 * CONV_STAT_REPS * C or bsums.dtype != torch.int64:
            raise ValueError(f"conv2d: bn sums needs [{CONV_STAT_REPS}][{2 * C}] int64 replica rows")
        d.bn_gate, d.bn_x, d.bn_mean, d.bn_rstd, d.bn_sums = _p(gate), _p(bx), _p(bmean), _p(brstd), _p(bsums)
    ws = None
    if mode in (WGRAD, STEM_WGRAD):
        _L.load()
        nb = int(_L._lib.ttmi_conv2d_workspace(ctypes.byref(d)))
        if nb < 0:
            raise _L.TTMIError(_L._lib.ttmi_last_error().decode())
        ws = torch.empty(max(nb, 16), device=out.device, dtype=torch.uint8)
        d.workspace, d.workspace_bytes = ws.data_ptr(), nb
    call("ttmi_conv2d", ctypes.byref(d), _s())
    return out


def conv_weight_prep(w: Tensor, Cp: int, wf: Tensor, wd: Optional[Tensor] = None) -> None:
    """bf16 GEMM mirrors of a torch Conv2d weight [Co, Cin, k, k]: wf [Co, k, k, Cp],
    wd [Cin, k, k, Co]."""
    Co, Cin, KH, KW = w.shape
    call("ttmi_conv_weight_prep", Co, Cin, Cp, KH, KW, _p(w), _p(wf), _p(wd), _s())


def conv_weight_prep_batch(items) -> None:
    """All mirrors in one launch (ttmi_conv_weight_prep_batch): items = [(w, Cp, wf, wd, s2d)]
    with w torch's fp32 [Co, Cin, k, k]; s2d: the stem's 4x4 space-to-depth mirror."""
    arr = (_L.ConvWPrep * max(1, len(items)))()
    for i, (w, Cp, wf, wd, s2d) in enumerate(items):
        Co, Cin, KH, KW = w.shape
        n = Co * (16 if s2d else KH * KW) * Cp
        if wf.numel() < n or (wd is not None and wd.numel() < Co * Cin * KH * KW) or not w.is_contiguous():
            raise ValueError(f"conv_weight_prep_batch: item {i} buffers / layout")
        arr[i] = _L.ConvWPrep(Co, Cin, Cp, KH, KW, int(s2d), w.data_ptr(), wf.data_ptr(), _p(wd) or 0)
    call("ttmi_conv_weight_prep_batch", len(items), ctypes.addressof(arr), _s())


def nchw_to_nhwc(x: Tensor, Cp: int, y: Tensor) -> Tensor:
    N, Cin, H, W = x.shape
    call("ttmi_nchw_to_nhwc", N, Cin, H, W, Cp, _p(x), _p(y), _s())
    return y


STEM_FWD, STEM_WGRAD = 3, 4     # ttmi_conv2d modes of the 7x7/2 stem on a space-to-depth input


def stem_s2d(x: Tensor, Cp: int, y: Tensor) -> Tensor:
    """Space-to-depth stem input (include/ttmi.h ttmi_stem_s2d): x fp32 NCHW [N, Cin, H, W]
    -> y bf16 [N, H/2, W/2, Cp], channel (ph*2 + pw)*Cin + ci."""
    N, Cin, H, W = x.shape
    if y.numel() < N * (H // 2) * (W // 2) * Cp:
        raise ValueError("stem_s2d: y too small")
    call("ttmi_stem_s2d", N, Cin, H, W, Cp, _p(x), _p(y), _s())
    return y


def stem_weight_prep(w: Tensor, Cp: int, wf: Tensor) -> None:
    """The 7x7 stem weight [Co, Cin, 7, 7] fp32 as the 4x4 kernel over stem_s2d's input:
    wf bf16 [Co, 4, 4, Cp]."""
    Co, Cin, KH, KW = w.shape
    if (KH, KW) != (7, 7) or wf.numel() < Co * 16 * Cp:
        raise ValueError("stem_weight_prep: needs a 7x7 weight and a [Co, 4, 4, Cp] mirror")
    call("ttmi_stem_weight_prep", Co, Cin, Cp, _p(w), _p(wf), _s())


def bn2d_fwd(x: Tensor, colsum: Optional[Tensor], colsumsq: Optional[Tensor], w: Tensor, b: Tensor, y: Tensor,
             save_mean: Tensor, save_rstd: Tensor, *, running_mean: Optional[Tensor] = None,
             running_var: Optional[Tensor] = None, num_batches: Optional[Tensor] = None,
             residual: Optional[Tensor] = None, relu: bool = False, eps: float = 1e-5,
             momentum: float = 0.1) -> Tensor:
    C = x.shape[-1]
    M = x.numel() // C
    for name, t in (("colsum", colsum), ("colsumsq", colsumsq)):
        if t is not None and (t.numel() < CONV_STAT_REPS * C or t.dtype != torch.int64):
            raise ValueError(f"bn2d_fwd: {name} needs [{CONV_STAT_REPS}][{C}] int64 replica rows")
    if y.numel() < x.numel() or (residual is not None and residual.numel() < x.numel()):
        raise ValueError("bn2d_fwd: y / residual smaller than x")
    call("ttmi_bn2d_fwd", M, C, _p(x), _p(colsum), _p(colsumsq), _p(w), _p(b), eps, momentum,
         _p(running_mean), _p(running_var), _p(num_batches), _p(residual), int(relu), _p(y),
         _p(save_mean), _p(save_rstd), _s())
    return y


def bn2d_bwd(dy: Tensor, x: Tensor, mean: Tensor, rstd: Tensor, w: Tensor, sums: Tensor,
             dx: Tensor, dw: Optional[Tensor], db: Optional[Tensor], *,
             gate: Optional[Tensor] = None, g_out: Optional[Tensor] = None) -> Tensor:
    C = x.shape[-1]
    M = x.numel() // C
    if sums.numel() < 2 * CONV_STAT_REPS * C or sums.dtype != torch.int64:
        raise ValueError(f"bn2d_bwd: sums needs [{CONV_STAT_REPS}][{2 * C}] int64 replica rows")
    for name, t in (("dy", dy), ("dx", dx), ("gate", gate), ("g_out", g_out)):
        if t is not None and t.numel() < x.numel():
            raise ValueError(f"bn2d_bwd: {name} smaller than x")
    call("ttmi_bn2d_bwd", M, C, _p(dy), _p(gate), _p(x), _p(mean), _p(rstd), _p(w), _p(sums),
         _p(g_out), _p(dx), _p(dw), _p(db), _s())
    return dx


def stem_pool_fwd(x: Tensor, colsum: Optional[Tensor], colsumsq: Optional[Tensor], w: Tensor, b: Tensor,
                  y: Tensor, idx: Tensor, save_mean: Tensor, save_rstd: Tensor, *,
                  running_mean: Optional[Tensor] = None, running_var: Optional[Tensor] = None,
                  num_batches: Optional[Tensor] = None, eps: float = 1e-5, momentum: float = 0.1) -> Tensor:
    """resnet18 stem tail bn1 → ReLU → maxpool(3, 2, 1) without storing the BN output
    (include/ttmi.h ttmi_stem_pool_fwd): x [N, H, W, C] conv output -> y [N, Ho, Wo, C] + idx."""
    N, H, W, C = x.shape
    Ho, Wo = conv_out_hw(H, W, 3, 2, 1)
    for name, t in (("colsum", colsum), ("colsumsq", colsumsq)):
        if t is not None and (t.numel() < CONV_STAT_REPS * C or t.dtype != torch.int64):
            raise ValueError(f"stem_pool_fwd: {name} needs [{CONV_STAT_REPS}][{C}] int64 replica rows")
    if y.numel() < N * Ho * Wo * C or idx.numel() < N * Ho * Wo * C:
        raise ValueError("stem_pool_fwd: y / idx too small")
    call("ttmi_stem_pool_fwd", N, H, W, C, _p(x), _p(colsum), _p(colsumsq), _p(w), _p(b), eps, momentum,
         _p(running_mean), _p(running_var), _p(num_batches), _p(y), _p(idx), _p(save_mean), _p(save_rstd), _s())
    return y


def stem_pool_bwd(dy: Tensor, idx: Tensor, x: Tensor, mean: Tensor, rstd: Tensor, w: Tensor, b: Tensor,
                  sums: Tensor, dx: Tensor, dw: Optional[Tensor], db: Optional[Tensor]) -> Tensor:
    """Backward of stem_pool_fwd (include/ttmi.h ttmi_stem_pool_bwd): dx at the conv output."""
    N, H, W, C = x.shape
    Ho, Wo = conv_out_hw(H, W, 3, 2, 1)
    if sums.numel() < 2 * CONV_STAT_REPS * C or sums.dtype != torch.int64:
        raise ValueError(f"stem_pool_bwd: sums needs [{CONV_STAT_REPS}][{2 * C}] int64 replica rows")
    if dy.numel() < N * Ho * Wo * C or idx.numel() < N * Ho * Wo * C or dx.numel() < x.numel():
        raise ValueError("stem_pool_bwd: dy / idx / dx too small")
    call("ttmi_stem_pool_bwd", N, H, W, C, _p(dy), _p(idx), _p(x), _p(mean), _p(rstd), _p(w), _p(b),
         _p(sums), _p(dx), _p(dw), _p(db), _s())
    return dx


def bn2d_bwd_apply(g: Tensor, x: Tensor, mean: Tensor, rstd: Tensor, w: Tensor, sums: Tensor,
                   dx: Tensor, dw: Optional[Tensor], db: Optional[Tensor]) -> Tensor:
    """Second pass of bn2d_bwd on an already-gated g whose sums were accumulated elsewhere
    (conv2d(..., bn=...)): dx = w·rstd·(g − Σg/M − x̂·Σgx̂/M); dw, db += the sums."""
    C = x.shape[-1]
    M = x.numel() // C
    if sums.numel() < 2 * CONV_STAT_REPS * C or sums.dtype != torch.int64:
        raise ValueError(f"bn2d_bwd_apply: sums needs [{CONV_STAT_REPS}][{2 * C}] int64 replica rows")
    if g.numel() < x.numel() or dx.numel() < x.numel():
        raise ValueError("bn2d_bwd_apply: g / dx smaller than x")
    call("ttmi_bn2d_bwd_apply", M, C, _p(g), None, _p(x), _p(mean), _p(rstd), _p(w), _p(sums), _p(dx),
         _p(dw), _p(db), _s())
    return dx


def maxpool_fwd(x: Tensor, k: int, stride: int, pad: int, y: Tensor, idx: Tensor) -> Tensor:
    N, H, W, C = x.shape
    call("ttmi_maxpool_fwd", N, H, W, C, k, stride, pad, _p(x), _p(y), _p(idx), _s())
    return y


def maxpool_bwd(dy: Tensor, idx: Tensor, k: int, stride: int, pad: int, dx: Tensor) -> Tensor:
    N, H, W, C = dx.shape
    call("ttmi_maxpool_bwd", N, H, W, C, k, stride, pad, _p(dy), _p(idx), _p(dx), _s())
    return dx


def avgpool_fwd(x: Tensor, y: Tensor) -> Tensor:
    N, H, W, C = x.shape
    call("ttmi_avgpool_fwd", N, H * W, C, _p(x), _p(y), _s())
    return y


def avgpool_bwd(dy: Tensor, dx: Tensor, gate: Optional[Tensor] = None) -> Tensor:
    N, H, W, C = dx.shape
    call("ttmi_avgpool_bwd", N, H * W, C, _p(dy), code(dy.dtype), _p(gate), _p(dx), _s())
    return dx


# ----------------------------------------------------------------------------- norms
def layernorm_fwd(x: Tensor, w: Tensor, b: Tensor, y: Tensor, mean: Tensor, rstd: Tensor, *,
                  eps: float = 1e-5, relu: bool = False, drop: Drop = NO_DROP) -> Tensor:
    _dev(x, y)
    M, D = x.shape
    call("ttmi_layernorm_fwd", M, D, _p(x), D, _p(w), _p(b), eps, int(relu), float(drop[0]),
         _p(drop[1]), _p(y), code(y.dtype), D, _p(mean), _p(rstd), _s())
    return y


def layernorm_bwd(dy: Tensor, x: Tensor, mean: Tensor, rstd: Tensor, w: Tensor, dx: Tensor,
                  dw: Optional[Tensor], db: Optional[Tensor], *, gate: Optional[Tensor] = None,
                  gate_scale: float = 1.0, res: Optional[Tensor] = None,
                  dx16: Optional[Tensor] = None, drop: Drop = NO_DROP) -> Tensor:
    """LayerNorm backward (+ gate, + residual); dx16 (bf16) optionally receives
    bf16(dropout(dx)) (drop: the residual branch's dropout, keep index m*D + n).  The weight /
    bias sums go through int64 fixed-point replicas (bit-reproducible), folded with the
    deferred weight gradients inside ``deferred_wgrad`` (else right away)."""
    M, D = x.shape
    sums = dw is not None or db is not None
    defer = bool(_PENDING) and sums
    slot = _PENDING[-1].slot(f"ln{D}") if defer else 0
    ws = _zero_ws("ttmi_layernorm_bwd_workspace", (D,), x.device, slot) if sums else None
    if dx16 is not None and dx16.dtype != torch.bfloat16:
        raise ValueError("layernorm_bwd: dx16 must be bf16")
    call("ttmi_layernorm_bwd", M, D, _p(dy), D, _p(x), D, _p(mean), _p(rstd), _p(w), _p(gate),
         code(gate.dtype) if gate is not None else 0, D, gate_scale, _p(res), _p(dx), D, _p(dw),
         _p(db), _p(ws), _p(dx16), dx16.stride(0) if dx16 is not None else 0, float(drop[0]),
         _p(drop[1]), int(defer), _s())
    if defer:
        out = (FoldDesc * 2)()
        call("ttmi_layernorm_bwd_folds", D, _p(ws), _p(dw), _p(db), out)
        n = (dw is not None) + (db is not None)
        _PENDING[-1].folds.extend((out[j], ws, dw, db) for j in range(n))
    return dx


def seq_embed_fwd(ids: Tensor, E: Tensor, P: Tensor, w: Tensor, b: Tensor, x: Tensor,
                  mean: Tensor, rstd: Tensor, *, eps: float = 1e-5, drop: Drop = NO_DROP,
                  norm1: Optional[Tuple[Tensor, Tensor, float, Tensor, Tensor, Tensor]] = None):
    """x = dropout(LN(E[ids] + P)); with norm1 = (w1, b1, eps1, y1, mean1, rstd1) also
    y1 = bf16(LN1(x)) (the first encoder layer's norm1, fused)."""
    B, L = ids.shape
    V, D = E.shape
    w1, b1, eps1, y1, m1, r1 = norm1 if norm1 is not None else (None, None, 0.0, None, None, None)
    if y1 is not None and y1.dtype != torch.bfloat16:
        raise ValueError("seq_embed_fwd: norm1 output must be bf16")
    call("ttmi_seq_embed_fwd", B, L, D, _p(ids), _p(E), V, _p(P), _p(w), _p(b), eps,
         float(drop[0]), _p(drop[1]), _p(x), _p(mean), _p(rstd), _p(w1), _p(b1), float(eps1),
         _p(y1), _p(m1), _p(r1), id_err_ptr(ids), _s())
    return x


_ZERO_WS: Dict[tuple, Tensor] = {}


def _zero_ws(sizer: str, args: tuple, device, slot: int = 0) -> Tensor:
    """Persistent zero workspace of the kernels whose column sums go through replicas
    (ttmi_seq_embed_bwd, ttmi_layernorm_bwd): zero on entry and left zero by every call, so
    one buffer per (device, entry point, sizes) serves every call and every graph replay on a
    stream.  Allocated on first use (the warm-up step, before any capture)."""
    key = (str(device), sizer, slot) + tuple(args)
    ws = _ZERO_WS.get(key)
    if ws is None:
        _L.load()
        nb = int(getattr(_L._lib, sizer)(*args))
        ws = _ZERO_WS[key] = torch.zeros(max(nb // 4, 1), device=device, dtype=torch.float32)
    return ws


_FX_ZERO: Dict[tuple, Tensor] = {}
FX_GRAD_SHIFT = 36      # TTMI_FX_GRAD_SHIFT (include/ttmi.h)


def _fx_zero(name: str, numel: int, device) -> Tensor:
    """Persistent zero int64 fixed-point accumulator (one per (device, name, size) and, inside
    ``deferred_wgrad``, per call of the block); the fold that converts it (fx_folds) leaves it
    zero again, so graph replays reuse it."""
    slot = _PENDING[-1].slot("fx:" + name) if _PENDING else 0
    key = (str(device), name, int(numel), slot)
    t = _FX_ZERO.get(key)
    if t is None:
        t = _FX_ZERO[key] = torch.zeros(max(int(numel), 2), device=device, dtype=torch.int64)
    return t


def _run_folds(folds) -> None:
    """(FoldDesc, keep-alive...) tuples: deferred to the open ``deferred_wgrad`` block's flush,
    else launched now."""
    if not folds:
        return
    pend = _PENDING[-1] if _PENDING else None
    if pend is not None:
        pend.folds.extend(folds)
        return
    farr = (FoldDesc * len(folds))(*[f for f, *_ in folds])
    call("ttmi_wgrad_batch", 0, (ctypes.POINTER(WgradDesc) * 1)(), len(folds), farr, _s())


def fx_folds(pairs) -> None:
    """Convert int64 fixed-point accumulators into fp32 gradients (added; accumulators left
    zero): pairs of (acc, grad) with acc shaped like grad (None pairs skipped)."""
    folds = []
    for acc, g in pairs:
        if acc is None or g is None:
            continue
        N = g.shape[-1]
        M = g.numel() // N
        f = FoldDesc()
        f.part, f.S, f.s_stride, f.M, f.N = acc.data_ptr(), 1, M * N, M, N
        f.C, f.ldc, f.accumulate, f.fx_shift = _p(g), N, 3, FX_GRAD_SHIFT
        folds.append((f, acc, g))
    _run_folds(folds)


def seq_embed_bwd(ids: Tensor, E: Tensor, P: Tensor, w: Tensor, mean: Tensor, rstd: Tensor,
                  dx: Tensor, dE: Tensor, dP: Tensor, dw: Tensor, db: Tensor, *,
                  drop: Drop = NO_DROP, padding_idx: int = 0):
    """SASRec input-block backward (ttmi_seq_embed_bwd): the embedding-row scatter and the
    position / LayerNorm sums accumulate in int64 fixed point (bit-reproducible), converted
    by folds that run with the deferred weight gradients (else right away)."""
    B, L = ids.shape
    V, D = E.shape
    defer = bool(_PENDING)
    slot = _PENDING[-1].slot("seq_embed") if defer else 0
    ws = _zero_ws("ttmi_seq_embed_bwd_workspace", (V, L, D), dx.device, slot)
    call("ttmi_seq_embed_bwd", B, L, D, V, _p(ids), _p(E), _p(P), _p(w), _p(mean), _p(rstd),
         float(drop[0]), _p(drop[1]), _p(dx), _p(dE), _p(dP), _p(dw), _p(db), padding_idx,
         _p(ws), int(defer), _s())
    if defer:       # the four conversions fold with the deferred weight gradients (ws left zero)
        out = (FoldDesc * 4)()
        call("ttmi_seq_embed_bwd_folds", V, L, D, _p(ws), _p(dE), _p(dP), _p(dw), _p(db), out)
        first = 0
        if _FX_SINK and not _FX_SINK[-1]:     # dE stays fixed point: AdamW converts it
            _FX_SINK[-1].append((ws.view(torch.int64)[:V * D], dE))
            first = 1
        _PENDING[-1].folds.extend((out[j], ws, dE, dP, dw, db) for j in range(first, 4))


# ----------------------------------------------------------------------------- attention
def mha_fwd(qkv: Tensor, key_valid: Tensor, B: int, L: int, H: int, ctx: Tensor, lse: Tensor,
            drop: Drop = NO_DROP):
    Dh = qkv.shape[1] // (3 * H)
    _q1_batch_check("mha_fwd", B, L, H, drop)
    call("ttmi_mha_fwd", code(qkv.dtype), B, L, H, Dh, _p(qkv), _p(key_valid), float(drop[0]),
         _p(drop[1]), _p(ctx), _p(lse), _s())
    return ctx


def mha_tuned_supported(L: int, Dh: int) -> bool:
    """Whether ttmi_mha_fwd / _bwd (and the fused and one-query attention kernels) serve this
    shape: L <= TTMI_ATTN_LMAX and Dh a multiple of 8 up to 64.  Other shapes run
    mha_generic_fwd / _bwd."""
    return 0 < L <= ATTN_LMAX and 0 < Dh <= 64 and Dh % 8 == 0


def mha_generic_fwd(qkv: Tensor, key_valid: Tensor, B: int, L: int, H: int, ctx: Tensor, lse: Tensor,
                    drop: Drop = NO_DROP) -> Tensor:
    """ttmi_mha_generic_fwd: mha_fwd for any L and head widths up to 512 (ABI 22)."""
    _dev(qkv, key_valid, ctx, lse)
    Dh = qkv.shape[1] // (3 * H)
    call("ttmi_mha_generic_fwd", code(qkv.dtype), B, L, H, Dh, _p(qkv), _p(key_valid), float(drop[0]),
         _p(drop[1]), _p(ctx), _p(lse), _s())
    return ctx


def mha_generic_bwd(qkv: Tensor, key_valid: Tensor, lse: Tensor, ctx: Tensor, dctx: Tensor, B: int, L: int,
                    H: int, dqkv: Tensor, drop: Drop = NO_DROP) -> Tensor:
    """ttmi_mha_generic_bwd: mha_bwd for the shapes mha_generic_fwd serves; needs the forward's
    ctx rows."""
    _dev(qkv, key_valid, lse, ctx, dctx, dqkv)
    Dh = qkv.shape[1] // (3 * H)
    ws = torch.empty(max(B * H * L, 1), device=qkv.device, dtype=torch.float32)
    call("ttmi_mha_generic_bwd", code(qkv.dtype), B, L, H, Dh, _p(qkv), _p(key_valid), _p(lse), _p(ctx),
         _p(dctx), float(drop[0]), _p(drop[1]), _p(ws), _p(dqkv), _s())
    return dqkv


_QA_OK: Dict[Tuple[int, int, int, int], bool] = {}


def qkv_attn_supported(dtype: torch.dtype, L: int, H: int, Dh: int) -> bool:
    """Whether ttmi_qkv_attn_fwd serves this shape (bf16, H·Dh = 128, Dh = 32, L <= 64)."""
    if dtype not in _DT:
        return False
    key = (code(dtype), L, H, Dh)
    if key not in _QA_OK:
        _QA_OK[key] = bool(_L.load().ttmi_qkv_attn_supported(*key))
    return _QA_OK[key]


def qkv_attn_fwd(a: Tensor, w: Tensor, b: Tensor, key_valid: Tensor, B: int, L: int, H: int,
                 qkv: Tensor, ctx: Tensor, lse: Tensor, drop: Drop = NO_DROP) -> Tensor:
    """in_proj + attention in one launch: qkv = a·wᵀ + b (kept for the backward), then
    ctx / lse as mha_fwd — bit-identical to linear() (from M = 2048 rows, its panel kernel)
    + mha_fwd()."""
    _dev(a, w, b, key_valid, qkv, ctx, lse)
    Dh = w.shape[0] // (3 * H)
    _q1_batch_check("qkv_attn_fwd", B, L, H, drop)
    call("ttmi_qkv_attn_fwd", code(a.dtype), B, L, H, Dh, _p(a), _p(w), _p(b), _p(key_valid),
         float(drop[0]), _p(drop[1]), _p(qkv), _p(ctx), _p(lse), _s())
    return ctx


def mha_bwd(qkv: Tensor, key_valid: Tensor, lse: Tensor, dctx: Tensor, B: int, L: int, H: int,
            dqkv: Tensor, drop: Drop = NO_DROP):
    Dh = qkv.shape[1] // (3 * H)
    _q1_batch_check("mha_bwd", B, L, H, drop)
    call("ttmi_mha_bwd", code(qkv.dtype), B, L, H, Dh, _p(qkv), _p(key_valid), _p(lse), _p(dctx),
         float(drop[0]), _p(drop[1]), _p(dqkv), _s())
    return dqkv


def attn_block_fwd(a: Tensor, w_in: Tensor, b_in: Tensor, key_valid: Tensor, B: int, L: int, H: int,
                   qkv: Tensor, ctx: Tensor, lse: Tensor, drop: Drop, wo: Tensor, bo: Tensor,
                   res: Tensor, n2w: Tensor, n2b: Tensor, eps: float, drop1: Drop, x1: Tensor,
                   a2: Tensor, m2: Tensor, r2: Tensor) -> None:
    """The attention sub-block forward in one launch (ttmi_attn_block_fwd, ABI 21): in_proj,
    attention, out_proj + residual + dropout 1, norm2."""
    _dev(a, w_in, b_in, key_valid, qkv, ctx, lse, wo, bo, res, n2w, n2b, x1, a2, m2, r2)
    _q1_batch_check("attn_block_fwd", B, L, H, drop)
    d = _L.AttnBlockDesc()
    d.B, d.L, d.H, d.Dh = B, L, H, a.shape[1] // H
    d.a, d.w_in, d.b_in, d.key_valid = _p(a), _p(w_in), _p(b_in), _p(key_valid)
    d.drop_p, d.drop_seed = float(drop[0]), _p(drop[1])
    d.qkv, d.ctx, d.lse = _p(qkv), _p(ctx), _p(lse)
    d.wo, d.bo, d.res, d.n2w, d.n2b, d.eps = _p(wo), _p(bo), _p(res), _p(n2w), _p(n2b), float(eps)
    d.drop1_p, d.drop1_seed = float(drop1[0]), _p(drop1[1])
    d.x1, d.a2, d.m2, d.r2 = _p(x1), _p(a2), _p(m2), _p(r2)
    call("ttmi_attn_block_fwd", ctypes.byref(d), _s())


_FFN_OK: dict = {}


def ffn_block_supported(dtype: torch.dtype, D: int, F: int, bwd: bool = False) -> bool:
    """Whether ttmi_ffn_block_fwd (``bwd``: ttmi_ffn_block_bwd) serves this (dtype, D, F).  The
    forward serves D = 128 with F in {256, 512} and D = 256 with F = 1024; the backward D = 128."""
    if dtype not in (torch.bfloat16,):
        return False
    key = (code(dtype), D, F, bwd)
    if key not in _FFN_OK:
        fn = _L.load().ttmi_ffn_block_bwd_supported if bwd else _L.load().ttmi_ffn_block_supported
        _FFN_OK[key] = bool(fn(*key[:3]))
    return _FFN_OK[key]


def ffn_block_fwd(a: Tensor, w1: Tensor, b1: Tensor, w2: Tensor, b2: Tensor, res: Tensor,
                  drop_f: Drop, drop2: Drop, h: Tensor, x2: Tensor, lnw: Tensor, lnb: Tensor,
                  eps: float, y: Tensor, mean: Tensor, rstd: Tensor,
                  kv: Optional[Tuple[Tensor, Tensor, Tensor]] = None) -> Tensor:
    """The feed-forward sub-block and the next layer's norm1 in one launch (ttmi_ffn_block_fwd,
    ABI 21): h = drop_f(relu(a·w1ᵀ + b1)), x2 = res + drop2(h·w2ᵀ + b2), y = LN(x2) — as
    linear(act=1) + linear_res_ln, with h never read back.  ``kv = (wkv, bkv, out)`` (ABI 22):
    also out = y·wkvᵀ + bkv (wkv [2D, D] bf16, out a [M, 2D] bf16 view with unit column stride,
    e.g. qkv[:, D:]): the next layer's K / V projection, the row panel's bits."""
    _dev(a, w1, b1, w2, b2, res, h, x2, lnw, lnb, y, mean, rstd)
    M, D = a.shape
    F = w1.shape[0]
    for t, shp in ((a, (M, D)), (w1, (F, D)), (w2, (D, F)), (res, (M, D)), (h, (M, F)), (x2, (M, D)),
                   (y, (M, D))):
        if tuple(t.shape) != shp or not t.is_contiguous():
            raise ValueError(f"ffn_block_fwd: operand of shape {tuple(t.shape)} (contiguous {shp} expected)")
    d = _L.FfnBlockDesc()
    d.M, d.D, d.F = M, D, F
    d.a, d.w1, d.b1, d.w2, d.b2, d.res = _p(a), _p(w1), _p(b1), _p(w2), _p(b2), _p(res)
    d.dropf_p, d.dropf_seed = float(drop_f[0]), _p(drop_f[1])
    d.drop2_p, d.drop2_seed = float(drop2[0]), _p(drop2[1])
    d.h, d.x2, d.lnw, d.lnb, d.eps = _p(h), _p(x2), _p(lnw), _p(lnb), float(eps)
    d.y, d.mean, d.rstd = _p(y), _p(mean), _p(rstd)
    if kv is not None:
        wkv, bkv, out = kv
        if (tuple(wkv.shape) != (2 * D, D) or not wkv.is_contiguous() or wkv.dtype != torch.bfloat16
                or tuple(bkv.shape) != (2 * D,) or tuple(out.shape) != (M, 2 * D) or out.stride(1) != 1
                or out.dtype != torch.bfloat16):
            raise ValueError("ffn_block_fwd: kv needs wkv [2D, D] bf16, bkv [2D], out [M, 2D] bf16 rows")
        _dev(wkv, bkv, out)
        d.wkv, d.bkv, d.kv, d.ld_kv = _p(wkv), _p(bkv.contiguous()), _p(out), out.stride(0)
    if kv is not None and D != 128:
        raise ValueError("ffn_block_fwd: the fused K / V projection serves D = 128")
    call("ttmi_ffn_block_fwd", ctypes.byref(d), _s())
    return x2


def ffn_block_bwd(dy2: Tensor, w2t: Tensor, w1t: Tensor, h: Tensor, gate_scale: float, dz1: Tensor,
                  x1: Tensor, m2: Tensor, r2: Tensor, n2w: Tensor, res: Tensor, dx1: Tensor, dy1: Tensor,
                  drop1: Drop, n2w_grad: Optional[Tensor], n2b_grad: Optional[Tensor]) -> Tensor:
    """The feed-forward sub-block's input-grad half in one launch (ttmi_ffn_block_bwd, ABI 21):
    dz1 = (dy2·W2) ⊙ [h > 0]·gate_scale (linear(dy2, w2t, gate=h)'s bits), then
    linear_ln_bwd(dz1, w1t, ...)'s dx1 / dy1 / norm2 grads (sums folded in workgroup order, with
    the step's weight gradients inside deferred_wgrad)."""
    _dev(dy2, w2t, w1t, h, dz1, x1, m2, r2, n2w, res, dx1, dy1)
    M, D = dy2.shape
    F = w2t.shape[0]
    for t, shp in ((dy2, (M, D)), (w2t, (F, D)), (w1t, (D, F)), (h, (M, F)), (dz1, (M, F)), (x1, (M, D)),
                   (res, (M, D)), (dx1, (M, D)), (dy1, (M, D))):
        if tuple(t.shape) != shp or not t.is_contiguous():
            raise ValueError(f"ffn_block_bwd: operand of shape {tuple(t.shape)} (contiguous {shp} expected)")
    _L.load()
    G = int(_L._lib.ttmi_ffn_block_bwd_sum_blocks(M))
    ws = torch.empty(max(G, 1) * 2 * D, device=dy2.device, dtype=torch.float32)
    d = _L.FfnBlockBwdDesc()
    d.M, d.D, d.F = M, D, F
    d.dy2, d.w2t, d.w1t, d.h, d.gate_scale = _p(dy2), _p(w2t), _p(w1t), _p(h), float(gate_scale)
    d.dz1, d.x1, d.m2, d.r2, d.n2w, d.res = _p(dz1), _p(x1), _p(m2), _p(r2), _p(n2w), _p(res)
    d.dx1, d.dy1 = _p(dx1), _p(dy1)
    d.drop1_p, d.drop1_seed = float(drop1[0]), _p(drop1[1])
    d.sum_ws = _p(ws)
    folds = []
    for j, gr in enumerate((n2w_grad, n2b_grad)):
        if gr is not None and G > 0:
            f = FoldDesc()
            f.part, f.S, f.s_stride, f.M, f.N = ws.data_ptr() + 4 * D * j, G, 2 * D, 1, D
            f.C, f.ldc, f.accumulate, f.fx_shift = _p(gr), D, 1, 0
            folds.append((f, ws, gr))
    call("ttmi_ffn_block_bwd", ctypes.byref(d), _s())
    _run_folds(folds)
    return dx1


def mha_bwd_dy(qkv: Tensor, key_valid: Tensor, lse: Tensor, dy: Tensor, wot: Tensor, B: int, L: int,
               H: int, dqkv: Tensor, drop: Drop = NO_DROP) -> Tensor:
    """mha_bwd with dctx = dy·W_o computed in the launch (ABI 21; wot = the W_oᵀ mirror):
    bit-identical to linear(dy, wot) + mha_bwd where the row panel serves that linear."""
    _dev(qkv, key_valid, lse, dy, wot, dqkv)
    Dh = qkv.shape[1] // (3 * H)
    _q1_batch_check("mha_bwd_dy", B, L, H, drop)
    call("ttmi_mha_bwd_dy", B, L, H, Dh, _p(qkv), _p(key_valid), _p(lse), _p(dy), _p(wot), float(drop[0]),
         _p(drop[1]), _p(dqkv), _s())
    return dqkv


# ----------------------------------------------------------------------------- user head
def user_concat_fwd(x: Tensor, len_src: Optional[Tensor], gender: Tensor, G: Tensor,
                    country: Tensor, C: Tensor, comb: Tensor, rows: Tensor, B: int, L: int):
    D = x.shape[1]
    call("ttmi_user_concat_fwd", code(comb.dtype), B, L, D, _p(x), _p(len_src), _p(gender), _p(G),
         G.shape[1], _p(country), _p(C), C.shape[1], _p(comb), _p(rows), G.shape[0], C.shape[0],
         id_err_ptr(gender), _s())
    return comb


def user_concat_bwd(dcomb: Tensor, rows: Tensor, gender: Tensor, dg: int, country: Tensor,
                    dc: int, dx: Tensor, dG: Optional[Tensor], dC: Optional[Tensor],
                    accumulate: bool = True, n_tables: Tuple[int, int] = (1, 1)):
    """Concat backward: dx rows (one writer each) and the demographic embedding gradients,
    whose rows users share, through int64 fixed-point accumulators folded into dG / dC.
    n_tables = (rows of G, rows of C): the ids are clamped into them as in the forward."""
    B = dcomb.shape[0]
    D = dcomb.shape[1] - dg - dc
    aG = _fx_zero("concat.dG", dG.numel(), dG.device) if dG is not None else None
    aC = _fx_zero("concat.dC", dC.numel(), dC.device) if dC is not None else None
    call("ttmi_user_concat_bwd", B, D, _p(dcomb), _p(rows), _p(gender), dg, _p(country), dc,
         _p(dx), _p(aG), _p(aC), int(accumulate), int(n_tables[0]), int(n_tables[1]), _s())
    fx_folds([(aG, dG), (aC, dC)])


# ----------------------------------------------------------------------------- batchnorm
def batchnorm_fwd(z: Tensor, w: Tensor, b: Tensor, y: Tensor, mean: Tensor, rstd: Tensor,
                  running_mean: Optional[Tensor], running_var: Optional[Tensor],
                  num_batches: Optional[Tensor], *, eps: float = 1e-5, momentum: float = 0.1,
                  relu: bool = True, drop: Drop = NO_DROP, training: bool = True):
    B, C = z.shape
    call("ttmi_batchnorm_fwd", code(y.dtype), B, C, _p(z), _p(w), _p(b), eps, momentum,
         _p(running_mean), _p(running_var), _p(num_batches), int(training), int(relu),
         float(drop[0]),
         _p(drop[1]), _p(y), _p(mean), _p(rstd), _s())
    return y


def item_head_desc(modal: Tensor, W: Dict[str, Tensor], P: Dict[str, Tensor],
                   bufs: Dict[str, Optional[Tensor]], drop: Drop, eps: float, out: Dict[str, Tensor],
                   momentum: float = 0.1) -> ItemHeadDesc:
    """The ttmi_item_head_desc of one training forward of the item late-fusion MLP (the
    caller keeps modal, the weights and ``out`` alive until its launches are issued)."""
    B = modal.shape[0]
    _dev(modal, *out.values())
    d = ItemHeadDesc()
    d.B, d.K, d.N1, d.D = B, modal.shape[1], W["fusion_layer.0.weight"].shape[0], W["fusion_layer.4.weight"].shape[0]
    d.modal, d.w0, d.b0 = _p(modal), _p(W["fusion_layer.0.weight"]), _p(P["fusion_layer.0.bias"])
    d.bn_w, d.bn_b = _p(P["fusion_layer.1.weight"]), _p(P["fusion_layer.1.bias"])
    d.bn_eps, d.momentum = 1e-5, momentum
    d.running_mean = _p(bufs.get("fusion_layer.1.running_mean"))
    d.running_var = _p(bufs.get("fusion_layer.1.running_var"))
    d.num_batches_tracked = _p(bufs.get("fusion_layer.1.num_batches_tracked"))
    d.drop_p, d.drop_seed = float(drop[0]), _p(drop[1])
    d.w4, d.b4 = _p(W["fusion_layer.4.weight"]), _p(P["fusion_layer.4.bias"])
    d.ln_w, d.ln_b, d.ln_eps = _p(P["fusion_layer.5.weight"]), _p(P["fusion_layer.5.bias"]), eps
    d.modal16, d.z, d.bn_mean, d.bn_rstd = _p(out["m16"]), _p(out["z"]), _p(out["bn_mean"]), _p(out["bn_rstd"])
    d.y1, d.y2, d.out, d.m5, d.r5 = _p(out["y1"]), _p(out["y2"]), _p(out["out"]), _p(out["m5"]), _p(out["r5"])
    d.ws = None
    if "out_hat" in out:       # InfoNCE's l2norm of the item embedding, in stage C (ABI 15)
        d.out_hat, d.out_norm = _p(out["out_hat"]), _p(out["out_norm"])
    if B <= 512:               # BatchNorm statistics in stage A, applied in C (no BN launch)
        _L.load()
        part = torch.empty(int(_L._lib.ttmi_item_head_bn_part_floats(B)), device=modal.device)
        out["_bn_part"] = part            # kept alive with the outputs
        d.bn_part = _p(part)
        d.bn_cnt = _p(_zero_ws("ttmi_item_head_bn_counter_bytes", (0,), modal.device))
    return d


def item_head_fwd(modal: Tensor, W: Dict[str, Tensor], P: Dict[str, Tensor],
                  bufs: Dict[str, Optional[Tensor]], drop: Drop, eps: float, out: Dict[str, Tensor],
                  momentum: float = 0.1) -> Dict[str, Tensor]:
    """The item late-fusion MLP forward in training mode in three launches (ttmi_item_head_fwd):
    fills out's m16, z, bn_mean, bn_rstd, y1, y2, out, m5, r5 exactly as cast_bf16 + linear +
    batchnorm_fwd(relu, dropout) + linear + layernorm_fwd write them."""
    d = item_head_desc(modal, W, P, bufs, drop, eps, out, momentum)
    call("ttmi_item_head_fwd", ctypes.byref(d), _s())
    return out


def item_head_fwd_stages(d: ItemHeadDesc, stages: int) -> None:
    """ttmi_item_head_fwd_stages: stage mask 1 = cast + Linear 0, 2 = BatchNorm + ReLU +
    dropout, 4 = Linear 4 + LayerNorm."""
    call("ttmi_item_head_fwd_stages", ctypes.byref(d), stages, _s())


def item_head_bwd_desc(dout: Tensor, y2: Tensor, m5: Tensor, r5: Tensor, ln_w: Tensor, w4t: Tensor,
                       dy2: Tensor, dy1: Tensor, ws: Tensor) -> ItemHeadBwdDesc:
    """ttmi_item_head_bwd_desc: LN(fusion_layer.5) backward + fusion_layer.4 input gradient."""
    _dev(dout, y2, m5, r5, ln_w, w4t, dy2, dy1, ws)
    B, D = dout.shape
    if w4t.dtype != torch.bfloat16 or dy2.dtype != torch.bfloat16 or not all(
            t.is_contiguous() for t in (dout, y2, w4t, dy2, dy1)):
        raise ValueError("item_head_bwd: contiguous operands, bf16 w4t / dy2")
    d = ItemHeadBwdDesc()
    d.B, d.D, d.N1 = B, D, w4t.shape[0]
    d.dout, d.y2, d.m5, d.r5, d.ln_w = _p(dout), _p(y2), _p(m5), _p(r5), _p(ln_w)
    d.w4t, d.dy2, d.dy1, d.ws = _p(w4t), _p(dy2), _p(dy1), _p(ws)
    return d


def item_head_bwd_ws(B: int, device, D: int = 128) -> Tensor:
    """[nblk][2][D] LayerNorm column sums of ttmi_item_head_bwd_c (nblk = ceil(B / 16))."""
    return torch.empty((B + 15) // 16 * 2 * D, device=device)


def item_head_bwd_c(d: ItemHeadBwdDesc) -> None:
    call("ttmi_item_head_bwd_c", ctypes.byref(d), _s())


def ln_sum_folds(ws: Tensor, grads: Sequence[Tensor], rows: int, D: int, S: Optional[int] = None,
                 consume: bool = False) -> None:
    """Fold per-block column sums ws [S][rows][D] (row j -> grads[j], accumulated, in block
    order; S defaults to all of ws) with the deferred weight gradients, or now outside
    ``deferred_wgrad``.  ``consume``: the fold leaves the partials zero."""
    nblk = ws.numel() // (rows * D) if S is None else S
    folds = []
    for j, g in enumerate(grads):
        f = FoldDesc()
        f.part, f.S, f.s_stride, f.M, f.N = ws.data_ptr() + 4 * D * j, nblk, rows * D, 1, D
        f.C, f.ldc, f.accumulate, f.fx_shift = _p(g), D, 3 if consume else 1, 0
        folds.append((f, ws, g))
    _run_folds(folds)


def item_head_fusable(W: Dict[str, Tensor], modal: Tensor, dtype) -> bool:
    """Shapes ttmi_item_head_fwd takes (include/ttmi.h): bf16, 512 -> 512 -> BN -> D, D = 128
    or (ABI 21) the reference's default 256."""
    w0, w4 = W["fusion_layer.0.weight"], W["fusion_layer.4.weight"]
    return (dtype == torch.bfloat16 and modal.dim() == 2 and modal.shape[0] > 1 and
            modal.shape[1] == 512 and modal.dtype == torch.float32 and tuple(w0.shape) == (512, 512) and
            tuple(w4.shape) in ((128, 512), (256, 512)) and w0.dtype == torch.bfloat16 and
            w4.dtype == torch.bfloat16)


def batchnorm_bwd(dy: Tensor, z: Tensor, w: Tensor, mean: Tensor, rstd: Tensor, y: Tensor,
                  dz: Tensor, dw: Tensor, db: Tensor, *, gate_scale: float = 1.0,
                  gated: bool = True, dz16: Optional[Tensor] = None):
    """BatchNorm1d backward; dz16 (bf16, contiguous) optionally receives a copy of dz."""
    B, C = z.shape
    if dz16 is not None and dz16.dtype != torch.bfloat16:
        raise ValueError("batchnorm_bwd: dz16 must be bf16")
    call("ttmi_batchnorm_bwd", code(y.dtype), B, C, _p(dy), _p(z), _p(w), _p(mean), _p(rstd),
         _p(y), gate_scale, int(gated), _p(dz), _p(dw), _p(db), _p(dz16), _s())
    return dz


# ----------------------------------------------------------------------------- InfoNCE
def infonce_workspace(B: int, D: int) -> int:
    _L.load()
    return int(_L._lib.ttmi_infonce_workspace(B, D))


def infonce_fwd(u: Tensor, it: Tensor, user_idx: Optional[Tensor], inv_tau: float, u_hat: Tensor,
                i_hat: Tensor, norms: Tensor, logits: Tensor, lse: Tensor, loss: Tensor,
                ws: Tensor):
    B, D = u.shape
    call("ttmi_infonce_fwd", B, D, _p(u), _p(it), _p(user_idx), inv_tau, _p(u_hat), _p(i_hat),
         _p(norms), _p(logits), _p(lse), _p(loss), _p(ws), _s())


def infonce_fwd_acc(u: Tensor, it: Tensor, user_idx: Optional[Tensor], inv_tau: float, u_hat: Tensor,
                    i_hat: Tensor, norms: Tensor, logits: Tensor, lse: Tensor, loss: Tensor, ws: Tensor,
                    loss_acc: Optional[Tensor]):
    """infonce_fwd with the combine inside the logits launch and ``loss_acc`` += loss
    (ttmi_infonce_fwd_acc: two launches; D % 64 == 0, D <= 256)."""
    B, D = u.shape
    cnt = _zero_ws("ttmi_infonce_counter_bytes", (B,), u.device)
    call("ttmi_infonce_fwd_acc", B, D, _p(u), _p(it), _p(user_idx), inv_tau, _p(u_hat), _p(i_hat),
         _p(norms), _p(logits), _p(lse), _p(loss), _p(ws), _p(cnt), _p(loss_acc), _s())


def infonce_fwd_pre(user_idx: Optional[Tensor], inv_tau: float, u_hat: Tensor, i_hat: Tensor,
                    norms: Tensor, logits: Tensor, lse: Tensor, loss: Tensor, ws: Tensor,
                    fused_combine: bool = True, loss_acc: Optional[Tensor] = None):
    """infonce_fwd on rows already normalised by their producers (ttmi_infonce_fwd_pre); with
    ``fused_combine`` the lse / loss combine runs inside the logits launch (persistent zero
    arrival counters); ``loss_acc`` (fp32 device scalar, needs the fused combine) += loss."""
    B, D = u_hat.shape
    if loss_acc is not None and (not fused_combine or loss_acc.dtype != torch.float32):
        raise ValueError("infonce_fwd_pre: loss_acc needs fused_combine and fp32")
    cnt = _zero_ws("ttmi_infonce_counter_bytes", (B,), u_hat.device) if fused_combine else None
    call("ttmi_infonce_fwd_pre", B, D, _p(user_idx), inv_tau, _p(u_hat), _p(i_hat), _p(norms),
         _p(logits), _p(lse), _p(loss), _p(ws), _p(cnt), _p(loss_acc), _s())


def infonce_bwd(u_hat: Tensor, i_hat: Tensor, norms: Tensor, logits: Tensor, lse: Tensor,
                user_idx: Optional[Tensor], inv_tau: float, dloss: Optional[Tensor], du: Tensor,
                di: Tensor, ws: Tensor, du16: Optional[Tensor] = None, fused_finish: bool = True):
    """du16 (bf16 [B, D], optional): a bf16 copy of du from the same launch.  fused_finish:
    the normalise backward runs inside the logit-gradient launch (ttmi_infonce_bwd_fused)."""
    B, D = u_hat.shape
    if du16 is not None and (du16.dtype != torch.bfloat16 or du16.shape != du.shape):
        raise ValueError("infonce_bwd: du16 must be bf16 shaped like du")
    if fused_finish:      # one launch: the split partials are summed by the last arriver (ABI 18)
        cnt = _zero_ws("ttmi_infonce_bwd_counter_bytes", (B,), u_hat.device)
        call("ttmi_infonce_bwd_fused", B, D, _p(u_hat), _p(i_hat), _p(norms), _p(logits), _p(lse),
             _p(user_idx), inv_tau, _p(dloss), _p(du), _p(di), _p(du16), _p(ws), _p(cnt), _s())
        return
    call("ttmi_infonce_bwd16", B, D, _p(u_hat), _p(i_hat), _p(norms), _p(logits), _p(lse),
         _p(user_idx), inv_tau, _p(dloss), _p(du), _p(di), _p(du16), _p(ws), _s())


# ----------------------------------------------------------------------------- misc
# Parameter writes through raw pointers (AdamW, TrainStep graph replays) do not
# move torch's version counters; writers bump this epoch so caches of derived operands (the
# eval-mode bf16 weight copies, user_tower.inference_operands) see the change.
PARAM_EPOCH = [0]


def bump_param_epoch() -> None:
    PARAM_EPOCH[0] += 1


def adamw_fx_range(p: Tensor, g: Tensor, m: Tensor, v: Tensor, p_bf16: Optional[Tensor], hyper: Tensor,
                   step: Tensor, fx: Tuple[Tensor, Tensor], zero_grad: bool = False,
                   skip_if: Optional[int] = None) -> Tuple[int, int]:
    """AdamW over the flat slot ``fx[1]`` alone, its gradient read from (and cleared in) the
    fixed-point accumulator ``fx[0]`` (ttmi_adamw_fx on the slot's sub-range); returns the slot's
    (offset, length) for adamw(skip=...)."""
    acc, view = fx
    off, cnt = (view.data_ptr() - g.data_ptr()) // g.element_size(), view.numel()
    if off % 4 or cnt % 4 or off < 0 or off + cnt > g.numel():
        raise ValueError("adamw_fx_range: the slot must be float4-aligned inside the flat buffer")
    e = 4 * off
    call("ttmi_adamw_fx", cnt, p.data_ptr() + e, g.data_ptr() + e, m.data_ptr() + e, v.data_ptr() + e,
         (p_bf16.data_ptr() + 2 * off) if p_bf16 is not None else None, _p(hyper), _p(step),
         int(zero_grad), _p(acc), 0, cnt, FX_GRAD_SHIFT, skip_if, _s())
    return off, cnt


def adamw(p: Tensor, g: Tensor, m: Tensor, v: Tensor, p_bf16: Optional[Tensor], hyper: Tensor,
          step: Tensor, zero_grad: bool = False,
          fx: Optional[Tuple[Tensor, Tensor]] = None, fold_plan=None,
          skip: Optional[Tuple[int, int]] = None, skip_if: Optional[int] = None):
    """Fused AdamW over flat buffers.  ``fx`` = (acc, grad_view): the gradient of the slot
    ``grad_view`` (a view into ``g``) is still in the int64 fixed-point accumulator ``acc``
    (fx_grad_sink): read from there and ``acc`` cleared (ttmi_adamw_fx).  ``fold_plan``
    (WgradPending(defer_fold=True).plan): the step's weight-gradient partials are folded and
    applied in the same launch (ttmi_adamw_folded).  ``skip_if`` (id_err_ptr): the update is
    skipped on the device when a lookup of this step met an id outside its table."""
    bump_param_epoch()
    if skip is not None:                   # (offset, length) updated by adamw_fx_range
        if fx is not None:
            raise ValueError("adamw: skip and fx are exclusive")
        call("ttmi_adamw_folded_skip", p.numel(), _p(p), _p(g), _p(m), _p(v), _p(p_bf16), _p(hyper),
             _p(step), int(zero_grad), None, 0, 0, FX_GRAD_SHIFT,
             ctypes.byref(fold_plan) if fold_plan is not None else None, int(skip[0]), int(skip[1]),
             skip_if, _s())
        return
    if fold_plan is not None:
        acc, off, cnt = None, 0, 0
        if fx is not None:
            acc, view = fx
            off, cnt = (view.data_ptr() - g.data_ptr()) // g.element_size(), view.numel()
        call("ttmi_adamw_folded", p.numel(), _p(p), _p(g), _p(m), _p(v), _p(p_bf16), _p(hyper),
             _p(step), int(zero_grad), _p(acc), off, cnt, FX_GRAD_SHIFT, ctypes.byref(fold_plan), skip_if,
             _s())
        return
    if fx is None:
        call("ttmi_adamw", p.numel(), _p(p), _p(g), _p(m), _p(v), _p(p_bf16), _p(hyper), _p(step),
             int(zero_grad), skip_if, _s())
        return
    acc, view = fx
    off = (view.data_ptr() - g.data_ptr()) // g.element_size()
    call("ttmi_adamw_fx", p.numel(), _p(p), _p(g), _p(m), _p(v), _p(p_bf16), _p(hyper), _p(step),
         int(zero_grad), _p(acc), off, view.numel(), FX_GRAD_SHIFT, skip_if, _s())


_FX_SINK: List[list] = []


@contextlib.contextmanager
def fx_grad_sink():
    """Inside the block, ``seq_embed_bwd`` leaves the item-embedding gradient in its int64
    fixed-point accumulator and appends (acc, grad) to the yielded list instead of folding it
    into ``grad``: the caller's AdamW reads it from there (``adamw(fx=...)``).  Only for a
    single-process step whose gradient is not all-reduced."""
    sink: list = []
    _FX_SINK.append(sink)
    try:
        yield sink
    finally:
        _FX_SINK.pop()


def batch_copy(dsts, srcs):
    """One launch copying each srcs[i] into dsts[i] (same byte sizes)."""
    n = len(dsts)
    D = (ctypes.c_void_p * n)(*[t.data_ptr() for t in dsts])
    S = (ctypes.c_void_p * n)(*[t.data_ptr() for t in srcs])
    for d, s_ in zip(dsts, srcs):
        if d.numel() * d.element_size() != s_.numel() * s_.element_size():
            raise ValueError("batch_copy: size mismatch")
    N = (ctypes.c_int64 * n)(*[t.numel() * t.element_size() for t in dsts])
    call("ttmi_batch_copy", n, D, S, N, _s())


def transpose_batch(dsts, srcs, seeds=None):
    """One launch: dsts[i] = srcs[i].t() for 2-D bf16 matrices (dsts[i] is [cols, rows]).
    ``seeds=(base, step, seeds_tensor, inc_step)`` also draws the step's dropout seeds in the
    same launch (``dropout_seeds``'s semantics, one extra workgroup)."""
    n = len(dsts)
    if n == 0 and seeds is None:
        return
    for d, s_ in zip(dsts, srcs):
        if s_.dim() != 2 or d.shape != (s_.shape[1], s_.shape[0]) or not s_.is_contiguous() \
                or not d.is_contiguous() or s_.dtype != torch.bfloat16 or d.dtype != torch.bfloat16:
            raise ValueError("transpose_batch: need contiguous bf16 [R,C] -> [C,R]")
    D = (ctypes.c_void_p * n)(*[t.data_ptr() for t in dsts])
    S = (ctypes.c_void_p * n)(*[t.data_ptr() for t in srcs])
    R = (ctypes.c_int64 * n)(*[t.shape[0] for t in srcs])
    C = (ctypes.c_int64 * n)(*[t.shape[1] for t in srcs])
    if seeds is None:
        call("ttmi_transpose_bf16_batch", n, D, S, R, C, _s())
        return
    base, step, sd, inc = seeds
    if step.dtype != torch.int32 or sd.dtype != torch.int64 or not (0 < sd.numel() <= 256):
        raise ValueError("transpose_batch: seeds need an int32 step and 1..256 int64 seeds")
    call("ttmi_transpose_bf16_batch_seeds", n, D, S, R, C, base & (2**64 - 1), _p(step), _p(sd),
         sd.numel(), int(inc), _s())


def step_prologue(copy_dsts, copy_srcs, tr_dsts, tr_srcs, step: Tensor, seeds=None) -> None:
    """One launch (ttmi_step_prologue): batch_copy(copy_dsts, copy_srcs), the transposes
    tr_dsts[i] = tr_srcs[i].t() (bf16), and ``seeds=(base, seeds_tensor)``: the step's dropout
    seeds with the step count advanced (dropout_seeds(..., inc_step=True)); seeds=None: the step
    count alone advances (step_inc)."""
    nc, nt = len(copy_dsts), len(tr_dsts)
    for d, s_ in zip(copy_dsts, copy_srcs):
        if d.numel() * d.element_size() != s_.numel() * s_.element_size():
            raise ValueError("step_prologue: copy size mismatch")
    for d, s_ in zip(tr_dsts, tr_srcs):
        if s_.dim() != 2 or d.shape != (s_.shape[1], s_.shape[0]) or not s_.is_contiguous() \
                or not d.is_contiguous() or s_.dtype != torch.bfloat16 or d.dtype != torch.bfloat16:
            raise ValueError("step_prologue: transposes need contiguous bf16 [R,C] -> [C,R]")
    if step.dtype != torch.int32:
        raise ValueError("step_prologue: the step count is int32")
    CD = (ctypes.c_void_p * max(nc, 1))(*[t.data_ptr() for t in copy_dsts])
    CS = (ctypes.c_void_p * max(nc, 1))(*[t.data_ptr() for t in copy_srcs])
    NB = (ctypes.c_int64 * max(nc, 1))(*[t.numel() * t.element_size() for t in copy_dsts])
    TD = (ctypes.c_void_p * max(nt, 1))(*[t.data_ptr() for t in tr_dsts])
    TS = (ctypes.c_void_p * max(nt, 1))(*[t.data_ptr() for t in tr_srcs])
    R = (ctypes.c_int64 * max(nt, 1))(*[t.shape[0] for t in tr_srcs])
    C = (ctypes.c_int64 * max(nt, 1))(*[t.shape[1] for t in tr_srcs])
    base, sd = seeds if seeds is not None else (0, None)
    if sd is not None and (sd.dtype != torch.int64 or not (0 < sd.numel() <= 256)):
        raise ValueError("step_prologue: 1..256 int64 seeds")
    call("ttmi_step_prologue", nc, CD, CS, NB, nt, TD, TS, R, C, base & (2**64 - 1), _p(step), _p(sd),
         sd.numel() if sd is not None else 0, 1, _s())


def step_inc(step: Tensor):
    call("ttmi_step_inc", _p(step), _s())


def dropout_seeds(base: int, step: Tensor, seeds: Tensor, inc_step: bool = False):
    """Per-site dropout seeds of the live step (inc_step: increment the step first, in the
    same launch)."""
    call("ttmi_dropout_seeds", base & (2**64 - 1), _p(step), _p(seeds), seeds.numel(),
         int(inc_step), _s())


def cast_bf16(src: Tensor, dst: Tensor) -> Tensor:
    call("ttmi_cast_f32_bf16", src.numel(), _p(src), _p(dst), _s())
    return dst


def dropout_bwd(dx: Tensor, dy: Tensor, colsum: Optional[Tensor], drop: Drop = NO_DROP,
                drop_rows: Optional[Tensor] = None) -> Tensor:
    M, N = dx.shape
    call("ttmi_dropout_bwd", code(dy.dtype), M, N, _p(dx), N, float(drop[0]), _p(drop[1]), N,
         _p(drop_rows), _p(dy), N, _p(colsum), _s())
    return dy


# ----------------------------------------------------------------------------- pruning
def last_rows(len_src: Tensor, rows: Tensor) -> Tensor:
    B, L = len_src.shape
    call("ttmi_last_rows", B, L, _p(len_src), _p(rows), _s())
    return rows


def last_rows_gather(len_src: Tensor, x: Tensor, rows: Tensor, out: Tensor) -> Tensor:
    """rows[b] = the last valid row of sequence b; out[b] = x[rows[b]] (one launch)."""
    B, L = len_src.shape
    D = x.shape[1]
    call("ttmi_last_rows_gather", B, L, D, _p(len_src), _p(x), _p(rows), _p(out), _s())
    return out


def gather_rows(x: Tensor, rows: Tensor, out: Tensor) -> Tensor:
    call("ttmi_gather_rows", rows.numel(), x.shape[1], _p(x), _p(rows), _p(out), _s())
    return out


def scatter_add_rows(src: Tensor, rows: Tensor, dst: Tensor) -> Tensor:
    call("ttmi_scatter_add_rows", rows.numel(), src.shape[1], _p(src), _p(rows), _p(dst), _s())
    return dst


def mha_q1_fwd(qkv: Tensor, key_valid: Tensor, rows: Tensor, B: int, L: int, H: int,
               ctx: Tensor, lse: Tensor, drop: Drop = NO_DROP):
    Dh = qkv.shape[1] // (3 * H)
    call("ttmi_mha_q1_fwd", code(qkv.dtype), B, L, H, Dh, _p(qkv), _p(key_valid), _p(rows),
         float(drop[0]), _p(drop[1]), _p(ctx), _p(lse), _s())
    return ctx


def _q1_batch_check(who: str, B: int, L: int, H: int, drop: Drop) -> None:
    """The attention kernels (full and one-query) index dropout masks in 32 bits: with dropout
    on, B·H·L² < 2^32 (without dropout any batch size runs: eval and inference encoding)."""
    if float(drop[0]) > 0 and B * H * L * L >= 1 << 32:
        raise ValueError(f"{who}: with attention dropout on, batch {B} x {H} heads x L={L} exceeds the "
                         f"32-bit mask index (B*H*L*L < 2^32); split the batch")


def mha_q1_gather_fwd(qkv: Tensor, key_valid: Tensor, x: Tensor, rows: Tensor, x_rows: Tensor,
                      B: int, L: int, H: int, ctx: Tensor, lse: Tensor, drop: Drop = NO_DROP,
                      co_item: Optional[ItemHeadDesc] = None) -> Tensor:
    """last_rows_gather + mha_q1_fwd in one launch: rows[b] = the last valid row of sequence b
    (right padding), x_rows[b] = x[rows[b]], ctx[b] = its one-query attention.  ``co_item``
    (item_head_desc): the item head's stage A runs on the same grid (ABI 18)."""
    _dev(qkv, key_valid, x, rows, x_rows, ctx, lse)
    D = qkv.shape[1] // 3
    if x.dtype != torch.float32 or x.shape[1] != D or x_rows.shape != (B, D) or rows.dtype != torch.int32:
        raise TypeError("mha_q1_gather_fwd: x / x_rows fp32 [*, D], rows int32 [B]")
    _q1_batch_check("mha_q1_gather_fwd", B, L, H, drop)
    args = (code(qkv.dtype), B, L, H, D // H, _p(qkv), _p(key_valid), _p(x), _p(rows), _p(x_rows),
            float(drop[0]), _p(drop[1]), _p(ctx), _p(lse))
    if co_item is None:
        call("ttmi_mha_q1_gather_fwd", *args, _s())
    else:
        call("ttmi_mha_q1_gather_item_fwd", *args, ctypes.byref(co_item), _s())
    return ctx


def mha_q1_proj_gather_fwd(qkv: Tensor, key_valid: Tensor, a_in: Tensor, wq: Tensor, bq: Tensor,
                           x: Tensor, rows: Tensor, x_rows: Tensor, B: int, L: int, H: int, ctx: Tensor,
                           lse: Tensor, drop: Drop = NO_DROP,
                           co_item: Optional[ItemHeadDesc] = None) -> Tensor:
    """mha_q1_gather_fwd whose query rows are projected in the launch (ABI 21): q =
    a_in[row]·wqᵀ + bq for the gathered rows only, written into qkv's Q columns there; the
    caller has filled qkv's K / V columns (the pruned layer's 256-column projection)."""
    _dev(qkv, key_valid, a_in, wq, bq, x, rows, x_rows, ctx, lse)
    D = qkv.shape[1] // 3
    _q1_batch_check("mha_q1_proj_gather_fwd", B, L, H, drop)
    call("ttmi_mha_q1_proj_gather_fwd", B, L, H, D // H, _p(qkv), _p(key_valid), _p(a_in), _p(wq),
         _p(bq), _p(x), _p(rows), _p(x_rows), float(drop[0]), _p(drop[1]), _p(ctx), _p(lse),
         ctypes.byref(co_item) if co_item is not None else None, _s())
    return ctx


def bn_bwd_desc(dy: Tensor, z: Tensor, w: Tensor, mean: Tensor, rstd: Tensor, y: Tensor,
                dz: Tensor, dw: Tensor, db: Tensor, *, gate_scale: float = 1.0, gated: bool = True,
                dz16: Optional[Tensor] = None) -> BnBwdDesc:
    """ttmi_bn_bwd_desc of a batchnorm_bwd call (the caller keeps the tensors alive)."""
    _dev(dy, z, w, mean, rstd, y, dz, dw, db, dz16)
    if dz16 is not None and dz16.dtype != torch.bfloat16:
        raise ValueError("bn_bwd_desc: dz16 must be bf16")
    d = BnBwdDesc()
    d.dtype, (d.B, d.C) = code(y.dtype), z.shape
    d.dy, d.z, d.w, d.mean, d.rstd, d.y = _p(dy), _p(z), _p(w), _p(mean), _p(rstd), _p(y)
    d.gate_scale, d.gated = gate_scale, int(gated)
    d.dz, d.dw, d.db, d.dz16 = _p(dz), _p(dw), _p(db), _p(dz16)
    return d


def bn_bwd_run(d: BnBwdDesc) -> None:
    """ttmi_batchnorm_bwd from a bn_bwd_desc (its own launch)."""
    call("ttmi_batchnorm_bwd", d.dtype, d.B, d.C, d.dy, d.z, d.w, d.mean, d.rstd, d.y, d.gate_scale,
         d.gated, d.dz, d.dw, d.db, d.dz16, _s())


def mha_q1_bwd(qkv: Tensor, key_valid: Tensor, rows: Tensor, lse: Tensor, dctx: Tensor, B: int,
               L: int, H: int, dqkv: Tensor, drop: Drop = NO_DROP, bn: Optional[BnBwdDesc] = None):
    """One-query attention backward; ``bn`` (bn_bwd_desc): the item head's BatchNorm1d backward
    runs on the same grid (ttmi_mha_q1_bnr_bwd, ABI 18)."""
    Dh = qkv.shape[1] // (3 * H)
    _q1_batch_check("mha_q1_bwd", B, L, H, drop)
    call("ttmi_mha_q1_bnr_bwd", code(qkv.dtype), B, L, H, Dh, _p(qkv), _p(key_valid), _p(rows),
         _p(lse), _p(dctx), float(drop[0]), _p(drop[1]), _p(dqkv),
         ctypes.byref(bn) if bn is not None else None, _s())
    return dqkv


def mha_q1_kv_bwd(qkv: Tensor, key_valid: Tensor, rows: Tensor, lse: Tensor, dctx: Tensor, B: int, L: int,
                  H: int, dqkv: Tensor, drop: Drop, wqt: Tensor, a_in: Tensor, dq_rows: Tensor, a_rows: Tensor,
                  dyq: Tensor, bn: Optional[BnBwdDesc] = None) -> None:
    """The pruned layer's one-query backward for a K / V-only in_proj input grad
    (ttmi_mha_q1_kv_bwd, ABI 21): dqkv's K / V columns (its Q columns untouched), the gathered
    rows' dq (bf16) and a_in rows, and dyq = dq·W_q (fp32, wqt = the in_proj transposed mirror)."""
    _dev(qkv, key_valid, rows, lse, dctx, dqkv, wqt, a_in, dq_rows, a_rows, dyq)
    _q1_batch_check("mha_q1_kv_bwd", B, L, H, drop)
    d = _L.Q1KvBwdDesc()
    d.B, d.L, d.H, d.Dh = B, L, H, qkv.shape[1] // (3 * H)
    d.qkv, d.key_valid, d.rows, d.lse, d.dctx = _p(qkv), _p(key_valid), _p(rows), _p(lse), _p(dctx)
    d.drop_p, d.drop_seed = float(drop[0]), _p(drop[1])
    d.dqkv, d.wqt, d.ld_wqt, d.a_in = _p(dqkv), _p(wqt), wqt.stride(0), _p(a_in)
    d.dq_rows, d.a_rows, d.dyq = _p(dq_rows), _p(a_rows), _p(dyq)
    d.bn = ctypes.cast(ctypes.pointer(bn), ctypes.c_void_p) if bn is not None else None
    call("ttmi_mha_q1_kv_bwd", ctypes.byref(d), _s())


def colsum(x: Tensor, out: Tensor) -> Tensor:
    M, N = x.shape
    call("ttmi_colsum", code(x.dtype), M, N, _p(x), N, _p(out), _s())
    return out


# ----------------------------------------------------------------------------- text encoder
def deb_embed_fwd(ids: Tensor, table: Tensor, w: Tensor, b: Tensor, eps: float,
                  mask: Optional[Tensor], y32: Optional[Tensor], y16: Tensor,
                  drop: Drop = NO_DROP) -> Tensor:
    """LN(table[ids]) · mask (· dropout) -> y32 fp32 [M,H] and y16 bf16 (row stride)."""
    M = ids.numel()
    H = table.shape[1]
    if y16.shape[0] < M or y16.stride(0) < H or (y32 is not None and y32.numel() < M * H):
        raise ValueError("deb_embed_fwd: output too small")
    call("ttmi_deb_embed_fwd", M, H, _p(ids), _p(table), _p(w), _p(b), eps, _p(mask),
         float(drop[0]), _p(drop[1]), _p(y32), _p(y16), y16.stride(0), table.shape[0],
         id_err_ptr(ids), _s())
    return y16


def deb_ln_fwd(z: Tensor, w: Tensor, b: Tensor, eps: float, y32: Optional[Tensor],
               y16: Optional[Tensor], mean: Tensor, rstd: Tensor, *,
               yq: Optional[Tensor] = None, yv: Optional[Tensor] = None,
               drop_q: Drop = NO_DROP, drop_v: Drop = NO_DROP) -> None:
    """Post-LayerNorm; yq / yv (bf16 [M, H]) optionally receive bf16(dropout(y)) with the
    next layer's LoRA-dropout masks (drop_q / drop_v share p)."""
    M, H = z.shape
    if float(drop_q[0]) != float(drop_v[0]):
        raise ValueError("deb_ln_fwd: the q and v LoRA dropouts share p")
    call("ttmi_deb_ln_fwd", M, H, _p(z), _p(w), _p(b), eps, _p(y32), _p(y16),
         y16.stride(0) if y16 is not None else 0, _p(mean), _p(rstd), _p(yq), _p(yv),
         float(drop_q[0]), _p(drop_q[1]), _p(drop_v[1]), _s())


def deb_gelu(x: Tensor, y: Tensor) -> Tensor:
    call("ttmi_deb_gelu", x.numel(), _p(x), _p(y), _s())
    return y


def dis_attn(B: int, S: int, nh: int, q: Tensor, k: Tensor, v: Tensor, posq: Tensor,
             posk: Tensor, mask: Tensor, delta: Tensor, inv_scale: float, ctx: Tensor,
             lse: Tensor, drop: Drop = NO_DROP, *, dctx: Optional[Tensor] = None,
             dq: Optional[Tensor] = None, dk: Optional[Tensor] = None,
             dv: Optional[Tensor] = None, lora_u: Optional[Tensor] = None,
             lora_bq: Optional[Tensor] = None, lora_hu: Optional[Tensor] = None,
             lora_pb: Optional[Tensor] = None, order: Optional[Tensor] = None) -> None:
    """Disentangled self-attention forward (dctx None) or backward.  q/k/v/ctx/dq/dk/dv are
    column views (head h at column h·64) sharing a row stride; posq/posk [npos, ·].
    order: dis_attn_order(mask) of this batch (optional; longest sequences first)."""
    H = nh * 64
    for name, t in (("q", q), ("k", k), ("v", v), ("ctx", ctx)):
        if t.shape[0] != B * S or t.shape[1] < H:
            raise ValueError(f"dis_attn: {name} must be [B·S, >= {H}]")
    if posq.shape[0] != posk.shape[0] or posq.shape[1] < H or delta.numel() < 2 * S - 1:
        raise ValueError("dis_attn: bad relative tables")
    if mask.numel() < B * S or lse.numel() < B * nh * S:
        raise ValueError("dis_attn: mask / lse too small")
    d = DisAttnDesc()
    d.B, d.S, d.nh, d.d_head, d.npos = B, S, nh, 64, posq.shape[0]
    d.q, d.k, d.v, d.ldqkv = _p(q), _p(k), _p(v), q.stride(0)
    if k.stride(0) != q.stride(0) or v.stride(0) != q.stride(0):
        raise ValueError("dis_attn: q, k, v must share a row stride")
    d.posq, d.posk, d.ldpos = _p(posq), _p(posk), posq.stride(0)
    if posk.stride(0) != posq.stride(0):
        raise ValueError("dis_attn: posq/posk must share a row stride")
    d.mask, d.delta, d.inv_scale = _p(mask), _p(delta), inv_scale
    d.drop_p, d.drop_seed = float(drop[0]), _p(drop[1])
    d.ctx, d.ldctx, d.lse = _p(ctx), ctx.stride(0), _p(lse)
    if order is not None:
        if order.dtype != torch.int32 or order.numel() < B:
            raise ValueError("dis_attn: order must be int32 [B] (dis_attn_order)")
        d.order = _p(order)
    if dctx is None:
        call("ttmi_dis_attn_fwd", ctypes.byref(d), _s())
        return
    for name, t in (("dq", dq), ("dk", dk), ("dv", dv), ("dctx", dctx)):
        if t is None or t.shape[0] != B * S or t.shape[1] < H:
            raise ValueError(f"dis_attn: {name} must be [B·S, >= {H}]")
    if lora_u is not None:
        if lora_u.numel() < d.npos * 8 or lora_hu.numel() < B * S * nh * 8 or \
                lora_pb.numel() < d.npos * 8 or lora_bq.numel() < H * 8:
            raise ValueError("dis_attn: LoRA buffers too small")
    d.dctx, d.lddctx = _p(dctx), dctx.stride(0)
    d.dq, d.dk, d.dv, d.lddqkv = _p(dq), _p(dk), _p(dv), dq.stride(0)
    d.lora_u, d.lora_bq, d.lora_hu, d.lora_pb = _p(lora_u), _p(lora_bq), _p(lora_hu), _p(lora_pb)
    scratch = torch.empty(B * nh * S, device=q.device)        # D_i = dO_i·O_i
    d.dq_scratch = _p(scratch)
    if lora_u is not None:
        pbx = torch.empty(int(_L.load().ttmi_dis_attn_pbx_floats(B, S, nh)), device=q.device)
        d.lora_pbx = _p(pbx)
    call("ttmi_dis_attn_bwd", ctypes.byref(d), _s())


def user_head_fwd(ctx: Tensor, res: Tensor, drop_rows: Optional[Tensor], W: Dict[str, Tensor],
                  P: Dict[str, Tensor], pre: str, gender: Tensor, country: Tensor, eps: float,
                  drops: Tuple[Drop, Drop, Drop], out: Dict[str, Tensor],
                  co_item: Optional[ItemHeadDesc] = None,
                  normed: Optional[Tuple[Tensor, Tensor]] = None, co_stage: str = "A") -> None:
    """The user tower head in one launch (ttmi_user_head_fwd): the pruned last layer's
    out-proj + residual + norm2 + FFN on the gathered rows, the demographic concat and the
    fusion MLP.  ``pre`` is the last layer's parameter prefix; ``out`` holds x1, a2, m2, r2, h,
    comb, rows, z, az, mz, rz, u (allocated by the caller)."""
    B, D = ctx.shape
    d = UserHeadDesc()
    d.B, d.D = B, D
    d.F = W[pre + "linear1.weight"].shape[0]
    d.dg, d.dc = P["gender_embedding.weight"].shape[1], P["country_embedding.weight"].shape[1]
    d.eps = eps
    d.ctx, d.res, d.drop_rows = _p(ctx), _p(res), _p(drop_rows)
    d.wo, d.bo = _p(W[pre + "self_attn.out_proj.weight"]), _p(P[pre + "self_attn.out_proj.bias"])
    d.n2w, d.n2b = _p(P[pre + "norm2.weight"]), _p(P[pre + "norm2.bias"])
    d.w1, d.b1 = _p(W[pre + "linear1.weight"]), _p(P[pre + "linear1.bias"])
    d.w2, d.b2 = _p(W[pre + "linear2.weight"]), _p(P[pre + "linear2.bias"])
    d.gender, d.G = _p(gender), _p(P["gender_embedding.weight"])
    d.country, d.C = _p(country), _p(P["country_embedding.weight"])
    d.n_genders = P["gender_embedding.weight"].shape[0]
    d.n_countries = P["country_embedding.weight"].shape[0]
    d.id_err = id_err_ptr(gender)
    d.wf0, d.bf0 = _p(W["fusion_layer.0.weight"]), _p(P["fusion_layer.0.bias"])
    d.lnw, d.lnb = _p(P["fusion_layer.1.weight"]), _p(P["fusion_layer.1.bias"])
    d.wf3, d.bf3 = _p(W["fusion_layer.3.weight"]), _p(P["fusion_layer.3.bias"])
    (d.d1_p, d1), (d.dff_p, dff), (d.d2_p, d2) = [(float(p), s) for p, s in drops]
    d.d1_seed, d.dff_seed, d.d2_seed = _p(d1), _p(dff), _p(d2)
    for k in ("x1", "a2", "m2", "r2", "h", "comb", "rows", "z", "az", "mz", "rz", "u"):
        setattr(d, k, _p(out[k]))
    if normed is not None:     # (u_hat [B, D], norms [B]): InfoNCE's l2norm of u, same launch
        d.u_hat, d.u_norm = _p(normed[0]), _p(normed[1])
    # the FFN split over its hidden units (ABI 21): arrival counts (reset by each launch) and
    # exchange slots (overwritten before they are read), one buffer per (device, B, F)
    d.ffn_ws = _p(_zero_ws("ttmi_user_head_ffn_ws_bytes", (B, d.F), ctx.device))
    if co_item is None:
        call("ttmi_user_head_fwd", ctypes.byref(d), _s())
    elif co_stage == "A":      # item head stage A on the CUs the 16-row user blocks leave idle
        call("ttmi_user_item_head_fwd", ctypes.byref(d), ctypes.byref(co_item), _s())
    elif co_stage == "C":      # stage C (stage A ran beside the one-query attention, ABI 18)
        call("ttmi_user_item_head_fwd_c", ctypes.byref(d), ctypes.byref(co_item), _s())
    else:                      # "AC": both item stages, C waiting for A's statistics in-launch
        call("ttmi_user_item_head_fwd_ac", ctypes.byref(d), ctypes.byref(co_item), _s())


def user_head_bwd(du16: Tensor, saved: Dict[str, Tensor], drop_rows: Tensor, W: Dict[str, Tensor],
                  P: Dict[str, Tensor], pre: str, gender: Tensor, country: Tensor, ffn_scale: float,
                  drops: Tuple[Drop, Drop], dG: Tensor, dC: Tensor,
                  ln_grads: Tuple[Tensor, Tensor, Tensor, Tensor],
                  co_item: Optional[ItemHeadBwdDesc] = None) -> Dict[str, Tensor]:
    """Backward of user_head_fwd in one launch (ttmi_user_head_bwd).  ``saved``: az, z, mz, rz,
    h, x1, m2, r2 of the forward; ``drops`` = (drop1, drop2).  Returns dz16, dy2, dz1, dx1, dy1,
    dctx; the four LayerNorm parameter gradients (``ln_grads``: fusion LN weight, bias, norm2
    weight, bias) are folded from per-block sums (deferred with the step's weight gradients
    inside ``deferred_wgrad``)."""
    B, D = du16.shape
    F = W[pre + "linear1.weight"].shape[0]
    dev = du16.device
    bf = torch.bfloat16
    o = dict(dz16=torch.empty(B, D, device=dev, dtype=bf), dy2=torch.empty(B, D, device=dev, dtype=bf),
             dz1=torch.empty(B, F, device=dev, dtype=bf), dx1=torch.empty(B, D, device=dev),
             dy1=torch.empty(B, D, device=dev, dtype=bf), dctx=torch.empty(B, D, device=dev, dtype=bf))
    nblk = (B + 15) // 16
    ws = torch.empty(nblk * 4 * D, device=dev)      # [nblk][4][D] column sums
    d = UserHeadBwdDesc()
    d.B, d.D, d.F = B, D, F
    d.dg, d.dc = P["gender_embedding.weight"].shape[1], P["country_embedding.weight"].shape[1]
    d.ffn_scale = ffn_scale
    d.du = _p(du16)
    for k in ("az", "z", "mz", "rz", "h", "x1", "m2", "r2"):
        setattr(d, k, _p(saved[k]))
    d.drop_rows, d.gender, d.country = _p(drop_rows), _p(gender), _p(country)
    d.n_genders = P["gender_embedding.weight"].shape[0]
    d.n_countries = P["country_embedding.weight"].shape[0]
    T = ".T"
    d.wf3t, d.wf0t = _p(W["fusion_layer.3.weight" + T]), _p(W["fusion_layer.0.weight" + T])
    d.w2t, d.w1t = _p(W[pre + "linear2.weight" + T]), _p(W[pre + "linear1.weight" + T])
    d.wot = _p(W[pre + "self_attn.out_proj.weight" + T])
    d.lnw, d.n2w = _p(P["fusion_layer.1.weight"]), _p(P[pre + "norm2.weight"])
    (d.d1_p, s1), (d.d2_p, s2) = [(float(p), sd) for p, sd in drops]
    d.d1_seed, d.d2_seed = _p(s1), _p(s2)
    aG = _fx_zero("head.dG", dG.numel(), dev)      # int64 fixed point (ABI 16), folded below
    aC = _fx_zero("head.dC", dC.numel(), dev)
    d.dG, d.dC = _p(aG), _p(aC)
    for k in ("dz16", "dy2", "dz1", "dx1", "dy1", "dctx"):
        setattr(d, k, _p(o[k]))
    d.ws = _p(ws)
    d.ffn_ws = _p(_zero_ws("ttmi_user_head_ffn_ws_bytes", (B, F), dev))   # (the forward's buffer)
    if co_item is None:
        call("ttmi_user_head_bwd", ctypes.byref(d), _s())
    else:      # the item head's row-local backward on the idle CUs (ABI 15)
        call("ttmi_user_item_head_bwd", ctypes.byref(d), ctypes.byref(co_item), _s())
    ln_sum_folds(ws, ln_grads, 4, D, S=nblk)
    fx_folds([(aG, dG), (aC, dC)])
    return o


def user_head_bwd_fusable(W: Dict[str, Tensor], pre: str) -> bool:
    """The transposed weight mirrors ttmi_user_head_bwd reads are present."""
    return all(n + ".T" in W for n in ("fusion_layer.3.weight", "fusion_layer.0.weight",
                                       pre + "linear2.weight", pre + "linear1.weight",
                                       pre + "self_attn.out_proj.weight"))


def user_head_fusable(W: Dict[str, Tensor], P: Dict[str, Tensor], pre: str, D: int,
                      dtype) -> bool:
    """Shapes ttmi_user_head_fwd takes (include/ttmi.h): D = 128 with F in {256, 512}, or the
    reference's default width D = 256 with F = 1024 (the FFN-split kernels only, ABI 21)."""
    F = W[pre + "linear1.weight"].shape[0]
    shape_ok = (D == 128 and F % 256 == 0 and F <= 512) or \
        (D == 256 and F == 1024 and not os.environ.get("TTMI_HEAD_NOSPLIT"))
    return (dtype == torch.bfloat16 and shape_ok and
            P["gender_embedding.weight"].shape[1] == 16 and
            P["country_embedding.weight"].shape[1] == 32 and
            all(W[n].dtype == torch.bfloat16 for n in (
                pre + "self_attn.out_proj.weight", pre + "linear1.weight", pre + "linear2.weight",
                "fusion_layer.0.weight", "fusion_layer.3.weight")))


def dis_attn_order(mask: Tensor, B: int, S: int) -> Tensor:
    """[B] int32 batch order for dis_attn: sequences by live 64-row blocks, longest first."""
    if mask.numel() < B * S or mask.dtype != torch.int64:
        raise ValueError("dis_attn_order: mask must be int64 [B, S]")
    order = torch.empty(B, device=mask.device, dtype=torch.int32)
    call("ttmi_dis_attn_order", _p(mask), B, S, _p(order), _s())
    return order


def deb_pool_fwd(x: Tensor, mask: Tensor, out: Tensor) -> Tensor:
    B, H = out.shape
    S = mask.shape[1]
    call("ttmi_deb_pool_fwd", B, S, H, _p(x), _p(mask), _p(out), _s())
    return out


def skinny_wgrad(W: Tensor, S: Tensor, C: Tensor, Mw: int, *, ldc_m: int, ldc_c: int,
                 alpha: float = 1.0, group: int = 0, sgs: int = 8) -> Tensor:
    """C[m, c] += alpha · Σ_r W[r, m] · S[r, (m / group)·sgs + c] (rank-8 LoRA gradients);
    W, S 2-D row-major views over the same R rows (column slices allowed)."""
    _dev(W, S, C)
    if W.dtype != torch.bfloat16 or S.dtype not in (torch.bfloat16, torch.float32) or C.dtype != torch.float32:
        raise TypeError("skinny_wgrad: W bf16, S bf16/fp32, C fp32")
    if W.shape[0] != S.shape[0] or W.shape[1] < Mw:
        raise ValueError("skinny_wgrad: W and S must share R rows; W needs Mw columns")
    # int64 fixed-point scratch in C's layout (left zero by the call): one per stream, since
    # calls on one stream are ordered (the step runs these on a side stream)
    span = (Mw - 1) * ldc_m + 7 * ldc_c + 1
    acc = _fx_zero(f"skinny@{_s()}", span, C.device)
    call("ttmi_skinny_wgrad", W.shape[0], Mw, _p(W), W.stride(0), _p(S), int(S.dtype == torch.float32),
         S.stride(0), group or Mw, sgs, alpha, _p(C), ldc_m, ldc_c, _p(acc), _s())
    return C


def lora_dx(dL: Tensor, aq: Tensor, av: Tensor, scale: float, drop_q: Drop, drop_v: Drop,
            dx: Tensor, ld_drop: int) -> Tensor:
    """dx += scale·(drop_q(dL[:, :8]·Aq) + drop_v(dL[:, 8:16]·Av)); the two dropouts share p."""
    _dev(dL, aq, av, dx)
    M, H = dx.shape
    if float(drop_q[0]) != float(drop_v[0]):
        raise ValueError("lora_dx: q and v LoRA dropout must share p")
    call("ttmi_lora_dx", M, H, _p(dL), dL.stride(0), _p(aq), _p(av), scale, float(drop_q[0]),
         _p(drop_q[1]), _p(drop_v[1]), ld_drop, _p(dx), dx.stride(0), _s())
    return dx


def deb_pool_bwd(dout: Tensor, mask: Tensor, dx: Tensor) -> Tensor:
    B, H = dout.shape
    S = mask.shape[1]
    call("ttmi_deb_pool_bwd", B, S, H, _p(dout), _p(mask), _p(dx), _s())
    return dx


def dropout_to(x: Tensor, y: Tensor, drop: Drop = NO_DROP) -> Tensor:
    """y = dropout(x) (fp32 x [M,N] contiguous -> y of any dtype with its own row stride; the
    mask index is m·N + n, as in every other dropout site)."""
    M, N = x.shape
    call("ttmi_dropout_bwd", code(y.dtype), M, N, _p(x), N, float(drop[0]), _p(drop[1]), N,
         None, _p(y), y.stride(0), None, _s())
    return y


# ----------------------------------------------------------------------------- retrieval
def topk_rows(scores: Tensor, K: int, out_val: Tensor, out_idx: Tensor,
              skip_first: bool = False) -> None:
    """Top-K per row of fp32 scores (descending, ties by lower index); column 0 excluded
    (as -inf) when skip_first."""
    R, V = scores.shape
    if scores.dtype != torch.float32 or scores.stride(1) != 1:
        raise ValueError("topk_rows: scores must be fp32 with unit column stride")
    if out_val.numel() < R * K or out_idx.numel() < R * K or out_idx.dtype != torch.int64:
        raise ValueError("topk_rows: outputs must be [R, K] (int64 indices)")
    call("ttmi_topk_rows", R, V, K, _p(scores), scores.stride(0), int(skip_first), _p(out_val),
         _p(out_idx), _s())


def rank_of(idx: Tensor, target: Tensor, rank: Tensor) -> Tensor:
    B, K = idx.shape
    if target.numel() < B or rank.numel() < B:
        raise ValueError("rank_of: target / rank too small")
    call("ttmi_rank_of", B, K, _p(idx), _p(target), _p(rank), _s())
    return rank


def catalogue_rows(x: Tensor, ids: Tensor, dense: Tensor) -> Tensor:
    """dense[ids[r]] = normalize(nan_to_num(normalize(x[r], 1e-12)), 1e-8) (the indexers'
    per-batch tail, evaluate_metrics.py:58-104)."""
    _dev(x, ids, dense)
    if x.dtype != torch.float32 or dense.dtype != torch.float32 or ids.dtype != torch.int64:
        raise TypeError("catalogue_rows: fp32 rows and index, int64 ids")
    if x.stride(1) != 1 or not dense.is_contiguous() or not ids.is_contiguous():
        raise ValueError("catalogue_rows: rows must be unit-stride, index and ids contiguous")
    n, D = x.shape
    if dense.shape[1] != D or ids.shape[0] != n:
        raise ValueError("catalogue_rows: shape mismatch")
    call("ttmi_catalogue_rows", n, D, _p(x), x.stride(0), _p(ids), dense.shape[0], _p(dense),
         id_err_ptr(ids), _s())
    return dense


def mask_items(scores: Tensor, ids: Tensor) -> Tensor:
    """scores[r, ids[r, j]] = -inf (ids int64 [R, Lh]; out-of-range ids ignored)."""
    R, V = scores.shape
    ids = ids.to(torch.int64).contiguous()
    if ids.shape[0] != R or scores.stride(1) != 1:
        raise ValueError("mask_items: ids must be [R, Lh] and scores row-major")
    call("ttmi_mask_items", R, V, _p(scores), scores.stride(0), _p(ids), ids.shape[1], _s())
    return scores

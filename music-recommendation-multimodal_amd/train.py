"""Training drivers — drop-in for the hot loop of reference src/train.py.

* ``setup_ddp`` / ``cleanup_ddp`` / ``train_one_epoch``: the reference's functions
  (train.py:29-76) with the same signatures; ``train_one_epoch`` runs unchanged against
  ``TwoTowerModel`` + any torch optimizer (the module path goes through autograd).
* ``TrainStep``: the MI355X-native step.  Parameters are re-homed into one flat fp32
  buffer (views keep the module's ``state_dict`` working), gradients land in a flat buffer
  written directly by the kernels, AdamW is one fused kernel that also refreshes the bf16
  GEMM-operand mirror, and the whole forward + backward + update is captured once into a
  HIP graph and replayed per step.  Dropout seeds and the Adam step count live in device
  memory so replays draw fresh masks and correct bias corrections.  Under
  ``torch.distributed`` (one process per GPU, RCCL) the flat gradient is averaged with one
  all-reduce between the backward graph and the update graph (reference DDP semantics:
  per-rank BatchNorm statistics, averaged gradients — train.py:300).
"""
from __future__ import annotations

import contextlib
import logging
import os
from typing import Callable, Dict, List, Optional, Sequence

import torch
import torch.distributed as dist

from . import cnn
from . import comm
from . import functional as F
from . import text as T
from . import ops
from .two_tower import TwoTowerModel
from .user_tower import _gemm_names, add_transposes, encoder_weight_names
from .item_tower import ITEM_GEMMS

Tensor = torch.Tensor
logger = logging.getLogger(__name__)
# the item-embedding rows' AdamW beside the side-stream weight-gradient GEMMs (TrainStep._update)
_ADAM_SPLIT = os.environ.get("TTMI_ADAM_SPLIT", "0") == "1"


# ------------------------------------------------------------------ reference-shaped API
def setup_ddp() -> int:
    """train.py:29-35: torchrun env -> process group (RCCL via the 'nccl' backend)."""
    if "LOCAL_RANK" in os.environ:
        local_rank = int(os.environ["LOCAL_RANK"])
        torch.cuda.set_device(local_rank)
        dist.init_process_group(backend="nccl")
        return local_rank
    return 0


def cleanup_ddp() -> None:
    if dist.is_initialized():
        dist.destroy_process_group()


def train_one_epoch(model, dataloader, optimizer, device, epoch, is_main_process=True,
                    log_interval=50):
    """train.py:41-76 with bf16 compute: no GradScaler is needed (no fp16 overflow range)."""
    model.train()
    total_loss = 0.0
    num_batches = len(dataloader)
    for i, batch in enumerate(dataloader):
        for k, v in batch.items():
            if isinstance(v, torch.Tensor):
                batch[k] = v.to(device)
        optimizer.zero_grad(set_to_none=True)
        loss, _, _, _ = model(batch)
        # nn.Embedding raises inside the forward, before any update: wait for the forward's
        # lookups, and raise for an id outside its table before backward / optimizer.step()
        ops.check_id_errors(sync=True)
        loss.backward()
        optimizer.step()
        loss_val = loss.item()
        total_loss += loss_val
        if is_main_process and (i + 1) % log_interval == 0:
            logger.info(f"Epoch {epoch} [{i + 1}/{num_batches}] | Loss: {loss_val:.4f}")
        del loss, batch
    return total_loss / max(num_batches, 1)


# ------------------------------------------------------------------ flat parameter store
class FlatParams:
    """All parameters of a module in one fp32 buffer (256-byte aligned slots).

    ``param.data`` is re-pointed at its slot, so the module and its state_dict keep
    working; ``grad``, ``exp_avg``, ``exp_avg_sq`` and (optionally) a bf16 ``mirror`` share
    the same layout.  ``tail`` lists name prefixes whose slots go last (in module order): the
    parameters whose gradients the backward finishes last, so the all-reduce of everything
    before ``tail_offset`` can start while they are still being computed.  Device-agnostic
    (also used by the CPU/gloo tests)."""

    ALIGN = 64  # elements (256 B)

    def __init__(self, module: torch.nn.Module, mirror_dtype: Optional[torch.dtype] = None,
                 tail: Sequence[str] = (), grad_extra: int = 0):
        self.names, self.shapes, self.offsets = [], [], []
        # trainable parameters only: frozen ones (the peft-frozen DeBERTa base) get neither
        # gradients nor AdamW updates (torch's AdamW skips params whose grad is None)
        params = [(n, p) for n, p in module.named_parameters() if p.requires_grad]
        is_tail = [any(n.startswith(t) for t in tail) for n, _ in params]
        params = [q for q, t in zip(params, is_tail) if not t] + \
                 [q for q, t in zip(params, is_tail) if t]
        n_head = len(params) - sum(is_tail)
        dev = params[0][1].device
        off = 0
        self.tail_offset = None
        for k, (n, p) in enumerate(params):
            if k == n_head:
                self.tail_offset = off
            self.names.append(n)
            self.shapes.append(tuple(p.shape))
            self.offsets.append(off)
            off += (p.numel() + self.ALIGN - 1) // self.ALIGN * self.ALIGN
        self.numel = off
        if self.tail_offset is None:
            self.tail_offset = off
        self.data = torch.zeros(off, device=dev, dtype=torch.float32)
        for (n, p), o in zip(params, self.offsets):
            self.data[o:o + p.numel()].copy_(p.detach().reshape(-1))
            p.data = self.data[o:o + p.numel()].view(p.shape)
        # grad_extra: fp32 slots after the gradients that ride the same all-reduce (TrainStep
        # carries rank 0's BatchNorm buffers there); AdamW only walks the first `numel`
        self.grad = torch.zeros(off + grad_extra, device=dev, dtype=torch.float32)
        self.grad_extra = self.grad[off:]
        self.exp_avg = torch.zeros_like(self.data)
        self.exp_avg_sq = torch.zeros_like(self.data)
        self.mirror = None
        if mirror_dtype is not None and mirror_dtype != torch.float32:
            self.mirror = torch.zeros(off, device=dev, dtype=mirror_dtype)

    def views(self, buf: Tensor, prefix: str = "") -> Dict[str, Tensor]:
        out = {}
        for n, s, o in zip(self.names, self.shapes, self.offsets):
            if n.startswith(prefix):
                k = 1
                for d in s:
                    k *= d
                out[n[len(prefix):]] = buf[o:o + k].view(s)
        return out


class FlatBuffers:
    """The module's floating-point buffers (BatchNorm running mean / var) re-homed into one
    fp32 buffer, so DDP's ``broadcast_buffers`` (rank 0's buffers overwrite every rank's at
    the start of each forward, reference train.py:300) is one collective.  Integer buffers
    (``num_batches_tracked``) advance identically on every rank and are left in place."""

    def __init__(self, module: torch.nn.Module):
        bufs = [(n, b) for n, b in module.named_buffers() if b.is_floating_point()]
        self.numel = sum(b.numel() for _, b in bufs)
        self.data = None
        if not bufs:
            return
        self.data = torch.empty(self.numel, device=bufs[0][1].device, dtype=torch.float32)
        o = 0
        for n, b in bufs:
            k = b.numel()
            self.data[o:o + k].copy_(b.detach().reshape(-1).float())
            b.data = self.data[o:o + k].view(b.shape)
            o += k


class GradSync:
    """Data-parallel gradient averaging over the flat buffer (reference DDP, train.py:300).

    Each rank pre-scales its loss gradient by 1/world (``loss_scale``) so one SUM
    all-reduce of the flat buffer yields the average.  The buffer is reduced in
    ``bucket_bytes`` slices (RCCL rings run per-link bound on xGMI; 32 MiB buckets keep every
    call well above the latency knee).  ``start`` launches a slice's reduction asynchronously
    (RCCL runs it on its own stream, overlapping the rest of the backward)."""

    def __init__(self, group=None, bucket_bytes: int = 32 << 20):
        self.group = group
        self.world = comm.world_size(group)
        # the collectives run: world > 1, or comm.force_dp at world 1 (the RCCL rehearsal)
        self.active = comm.dp_active(group)
        self.bucket = max(1, bucket_bytes // 4)

    @property
    def loss_scale(self) -> float:
        return 1.0 / self.world

    def start(self, flat_grad: Tensor) -> List:
        if not self.active:
            return []
        n = flat_grad.numel()
        return [comm.all_reduce_sum(flat_grad[s:s + self.bucket], self.group, async_op=True)
                for s in range(0, n, self.bucket)]

    def __call__(self, flat_grad: Tensor) -> None:
        for w in self.start(flat_grad):
            w.wait()


class _Segments:
    """A step recorded as HIP-graph segments separated by host actions (the collectives, which
    run between graph replays on the same stream).  With no cut the step is one graph.  In
    eager mode ``cut`` runs its action at once, so one code path serves both.  ``inline``
    (collectives that can be captured, comm.capturable): ``cut`` records its action into the
    open graph, so the whole step stays one graph."""

    def __init__(self, device, capture: bool, pool=None, inline: bool = False):
        self.device = device
        self.capture = capture
        self.pool = pool
        self.inline = inline
        self.items: List = []           # ("graph", CUDAGraph) | ("host", fn)
        self.cur = None
        self.stream = None

    def begin(self) -> None:
        if self.capture:
            self.stream = torch.cuda.Stream(self.device)
            self.stream.wait_stream(torch.cuda.current_stream(self.device))
            self._ctx = torch.cuda.stream(self.stream)
            self._ctx.__enter__()
            self._open()

    def _open(self) -> None:
        self.cur = torch.cuda.CUDAGraph()
        # collectives in the graph: thread-local capture, so that the process group's watchdog
        # thread may still query the events of earlier (uncaptured) collectives meanwhile (a
        # global-mode capture makes that query fail and the watchdog abort the process)
        self.cur.capture_begin(pool=self.pool,
                               capture_error_mode="thread_local" if self.inline else "global")

    def _close(self) -> None:
        self.cur.capture_end()
        self.items.append(("graph", self.cur))
        self.cur = None

    def cut(self, fn: Callable[[], None]) -> None:
        if not self.capture or self.inline:
            fn()
            return
        self._close()
        self.items.append(("host", fn))
        self._open()

    def end(self) -> None:
        if self.capture:
            self._close()
            self._ctx.__exit__(None, None, None)
            torch.cuda.current_stream(self.device).wait_stream(self.stream)

    def abort(self) -> None:
        """Leave a capture that raised: end it (its graph is discarded) and the capture stream."""
        if not self.capture:
            return
        if self.cur is not None:
            try:
                self.cur.capture_end()
            except Exception:                 # an invalidated capture refuses to end cleanly
                pass
            self.cur = None
        self.items = []
        if getattr(self, "_ctx", None) is not None:
            self._ctx.__exit__(None, None, None)
            self._ctx = None
            torch.cuda.current_stream(self.device).wait_stream(self.stream)

    def replay(self) -> None:
        for kind, x in self.items:
            if kind == "graph":
                x.replay()
            else:
                x()

    @property
    def n_graphs(self) -> int:
        return sum(1 for k, _ in self.items if k == "graph")


def _no_cut(fn: Callable[[], None]) -> None:
    fn()


class _Entry:
    """Per batch-signature state: static inputs, the recorded step and its outputs."""

    def __init__(self, static: Dict[str, Tensor]):
        self.static = static
        self.seg: Optional[_Segments] = None
        self.loss: Optional[Tensor] = None
        self.logits: Optional[Tensor] = None


# ------------------------------------------------------------------ the fused step
class TrainStep:
    """Fused, graph-captured training step for ``TwoTowerModel`` (cfg-2 precomputed item
    inputs, or cfg-3 raw mels / covers / tabular with ``precomputed_modalities=False``).

    ``step(batch)`` stages the batch into static device buffers, replays the captured
    forward+backward(+update) graph and returns the device loss tensor (no host sync).
    A batch of a new shape (the reference DataLoader's ragged last batch, train.py:259-266)
    gets its own static buffers and graph; later batches of a known shape reuse theirs.

    Data-parallel (one process per GPU, RCCL): the gradient average is split in two buckets —
    everything but the user tower's first encoder layer and input block is all-reduced
    asynchronously while those are still being differentiated (DDP's bucketed overlap), the
    rest after the backward; BatchNorm running buffers follow rank 0 at the start of every
    step (DDP ``broadcast_buffers``, carried by the previous step's gradient all-reduce).  With ``model.global_negatives`` (BASELINE cfg 5) the
    loss all-gathers û, î, user_idx between the forward and loss graphs and reduce-scatters
    the key gradients before the tower backward; ``loss`` is then this rank's share (the
    mean over ranks is the loss of the concatenated batch)."""

    INPUT_KEYS = ("history_ids", "history_mask", "user_gender", "user_country", "user_idx",
                  "target_modal", "target_audio", "target_image", "target_tabular",
                  "target_input_ids", "target_attention_mask")
    RAW_ENCODERS = (("audio_encoder.backbone.", 1), ("visual_encoder.backbone.", 3))
    # gradients finished last by the backward (user tower layer 0 + input block): bucket 2
    LATE = ("user_tower.item_embedding.", "user_tower.position_embedding.",
            "user_tower.layer_norm.", "user_tower.transformer_encoder.layers.0.")

    def __init__(self, model: TwoTowerModel, lr: float = 1e-4, betas=(0.9, 0.999),
                 eps: float = 1e-8, weight_decay: float = 0.01, use_graph: bool = True,
                 seed: int = 0, group=None, broadcast_buffers: bool = True,
                 overlap_grad_sync: Optional[bool] = None, grad_sink: bool = True,
                 capture_collectives: Optional[bool] = None):
        self.model = model
        # grad_sink (one process only): the [V, D] item-embedding gradient stays in its int64
        # fixed-point accumulator and AdamW reads it there (a 31 MB conversion pass saved), so
        # its slot of flat.grad reads ZERO between backward and update.  Anything that must see
        # complete gradients there (clipping, norms, hooks) needs grad_sink=False.
        self.grad_sink = grad_sink
        # one process: the weight-gradient fold runs inside the AdamW launch (ABI 19), so the
        # folded slots of flat.grad are never written either (same caveat as grad_sink)
        self.fold_in_update = grad_sink and os.environ.get("TTMI_FOLD_IN_UPDATE", "1") != "0"
        self._fold = None
        self._pend = None
        self._keep = None
        model.train()
        dev = next(model.parameters()).device
        self.device = dev
        self.ucfg = model.user_tower.cfg()
        self.icfg = model.item_tower.cfg()
        self.p_item = model.item_tower.fusion_layer[3].p
        self.dtype = self.ucfg.dtype
        self.group = group if group is not None else getattr(model, "process_group", None)
        self.sync = GradSync(self.group)
        self.world = self.sync.world
        # the data-parallel schedule: world > 1, or comm.force_dp at world 1 (RCCL rehearsal)
        self.dp = self.sync.active
        # the collectives recorded inside the step's HIP graph (RCCL) instead of host cuts
        self.capture_collectives = self.dp and (comm.capturable(self.group)
                                                if capture_collectives is None else capture_collectives)
        self.global_negatives = bool(getattr(model, "global_negatives", False))
        # two-bucket overlap (the head bucket all-reduced while layer 0 and the input block are
        # differentiated) is opt-in: measured at world size 1 on RCCL it costs the rank ~38 us
        # of compute (its GEMMs split from the tail's, cross-stream graph joins), about what it
        # hides of an 8-GPU ring all-reduce of its 2.8 MB; the default computes
        # every weight gradient in the one-process schedule and all-reduces once
        if overlap_grad_sync is None:
            overlap_grad_sync = os.environ.get("TTMI_DP_OVERLAP", "0") == "1"
        self.overlap = overlap_grad_sync and self.dp and self.ucfg.n_layers >= 2
        self.fold_in_update = self.fold_in_update and not self.dp
        # the weight-gradient GEMMs planned (their partials folded later): inside AdamW in one
        # process; data-parallel, by a fold launch before the tail all-reduce — either way the
        # GEMMs can run early on the side stream beside the input block's backward
        self.plan_wgrad = self.fold_in_update or (
            self.dp and os.environ.get("TTMI_DP_PLAN_WGRAD", "1") != "0")
        self._split_cuts = False               # capturing with host cuts (segmented schedule)
        self._extra_filled = False
        self.fbufs = FlatBuffers(model)
        self.broadcast_buffers = broadcast_buffers and self.dp and \
            self.fbufs.data is not None
        # fp32 slots after the gradients that ride the all-reduce: rank 0's BatchNorm buffers
        # (broadcast_buffers) and, data-parallel, every rank's 8 id-range flags (1.0f when
        # raised): summed, they make every rank skip the update of a step in which any rank met
        # an id outside a table, so the replicas never diverge
        self.n_bufx = self.fbufs.numel if self.broadcast_buffers else 0
        self.flag_off = (self.n_bufx + 3) // 4 * 4 if self.dp else None
        self.flat = FlatParams(model, self.dtype, tail=self.LATE if self.overlap else (),
                               grad_extra=self.flag_off + 8 if self.dp else self.n_bufx)
        ops.bump_param_epoch()                 # parameters now live in (and move with) the flat buffer
        if self.dp:                            # DDP's constructor: rank 0's parameters and buffers
            src = comm.group_src(0, self.group)
            comm.broadcast(self.flat.data, src, self.group)
            if self.fbufs.data is not None:
                comm.broadcast(self.fbufs.data, src, self.group)
        if self.broadcast_buffers:
            # broadcast_buffers without a collective of its own: rank 0's buffers after step
            # k's forward are exactly what DDP broadcasts at the start of step k + 1, so they
            # ride step k's gradient all-reduce (rank 0 adds them, the others add zeros) into
            # the gradient's extra slots, which the next step's staging launch copies over every
            # rank's buffers (AdamW and the backward never write those slots)
            self.flat.grad_extra[:self.n_bufx].copy_(self.fbufs.data)
            self.bzero = torch.zeros_like(self.fbufs.data)
            self.is_root = comm.rank(self.group) == 0
        self.hyper = torch.tensor([lr, betas[0], betas[1], eps, weight_decay],
                                  dtype=torch.float64, device=dev)
        self.step_t = torch.zeros(1, dtype=torch.int32, device=dev)
        self.seeds = torch.zeros(F.N_SITES, dtype=torch.int64, device=dev)
        self.base_seed = seed & ((1 << 63) - 1)
        self.dloss = torch.full((1,), self.sync.loss_scale, dtype=torch.float32, device=dev)
        # running sum of the step losses on the device (the reference loop's total_loss,
        # src/train.py:68, without a host sync per step): read / reset via loss_sum
        self.loss_sum = torch.zeros(1, dtype=torch.float32, device=dev)
        self.Pu = self.flat.views(self.flat.data, "user_tower.")
        self.Pi = self.flat.views(self.flat.data, "item_tower.")
        self.Gu = self.flat.views(self.flat.grad, "user_tower.")
        self.Gi = self.flat.views(self.flat.grad, "item_tower.")
        if self.flat.mirror is not None:
            Mu = self.flat.views(self.flat.mirror, "user_tower.")
            Mi = self.flat.views(self.flat.mirror, "item_tower.")
            self.Wu = dict(self.Pu)
            self.Wu.update({n: Mu[n] for n in _gemm_names(list(self.Pu))})
            add_transposes(self.Wu, _gemm_names(list(self.Pu)))   # refreshed every step
            self.Wi = dict(self.Pi)
            self.Wi.update({n: Mi[n] for n in ITEM_GEMMS})
            w4 = self.Wi.get("fusion_layer.4.weight")
            if w4 is not None and w4.dim() == 2:   # W4ᵀ: the item head backward's k-major operand
                self.Wi[F.transposed_name("fusion_layer.4.weight")] = torch.empty(
                    w4.shape[1], w4.shape[0], device=w4.device, dtype=w4.dtype)
        else:
            self.Wu, self.Wi = self.Pu, self.Pi
        self.bufs = {k[len("item_tower."):]: v for k, v in model.named_buffers()
                     if k.startswith("item_tower.")}
        self.raw_items = not model.item_tower.precomputed_modalities     # cfg 3
        if self.raw_items:
            it = model.item_tower
            self.p_tab = it.tabular_encoder.mlp[3].p
            self.text_dim = it.modal_dims[2]

            def sub(d, pre):
                return {k[len(pre):]: v for k, v in d.items() if k.startswith(pre)}
            self.enc = [(sub(self.Pi, pre), sub(self.Gi, pre), sub(self.bufs, pre), c)
                        for pre, c in self.RAW_ENCODERS]
            pre = "tabular_encoder."
            self.tab = (sub(self.Pi, pre), sub(self.Gi, pre), sub(self.bufs, pre))
            self.text = None
            if it.with_text:                                   # cfg 4: LoRA + projection
                pre = "text_encoder."
                self.text = (it.text_encoder, sub(self.Pi, pre), sub(self.Gi, pre))
                self.text_seeds = torch.zeros(T.N_TEXT_SITES, dtype=torch.int64, device=dev)
        # dropout anywhere in the step: the prologue draws the seeds
        self._draw = self.ucfg.p_drop > 0 or self.p_item > 0 or (self.raw_items and self.p_tab > 0)
        self.sync_mirror()
        self.use_graph = use_graph
        self._entries: Dict[tuple, _Entry] = {}
        self._cur: Optional[_Entry] = None
        self._pending: List = []               # in-flight async bucket reductions
        self.loss: Optional[Tensor] = None
        self.logits: Optional[Tensor] = None

    # ---------------------------------------------------------------- pieces
    def sync_mirror(self) -> None:
        """Refresh the bf16 operand mirror from the fp32 masters (call after external
        parameter edits, e.g. load_state_dict)."""
        if self.flat.mirror is not None:
            ops.cast_bf16(self.flat.data, self.flat.mirror)

    def _fwd_bwd(self, b: Dict[str, Tensor], cut: Callable = _no_cut, fx_sink: bool = False) -> None:
        """Forward + backward into the flat gradient.  ``cut(fn)`` marks a point where a
        collective ``fn`` runs between graph segments (see _Segments).  ``fx_sink``: leave the
        item-embedding gradient in its fixed-point accumulator for the update (self._fx)."""
        # the gradient buffer is zero here: it starts zeroed and the fused AdamW clears it.  The
        # step's prologue — Wᵀ mirrors of the just-updated bf16 weights, the dropout seeds, the
        # step count — ran in the staging launch (_stage), ahead of the graph
        seeds = self.seeds if self._draw else None
        # cfg 2: the item head's first stage rides in the user head launch (idle CUs)
        # and both heads also write InfoNCE's l2norm of their rows (no normalise launch)
        normed = None
        if not self.raw_items and not self.global_negatives:
            B, D = b["history_ids"].shape[0], self.ucfg.D
            normed = (torch.empty(B, D, device=self.device), torch.empty(B, D, device=self.device),
                      torch.empty(2 * B, device=self.device))
        co = None if self.raw_items else F.item_fusion_fwd_begin(
            self.Pi, self.Wi, b["target_modal"], self.icfg, seeds, self.bufs, self.p_item,
            normed=(normed[1], normed[2][B:]) if normed is not None else None)
        u, ust = F.user_tower_fwd(self.Pu, self.Wu, b["history_ids"], b["user_gender"],
                                  b["user_country"], b.get("history_mask"), self.ucfg, seeds,
                                  co_item=co, normed=(normed[0], normed[2][:B]) if co is not None and
                                  normed is not None else None)
        self._normed = normed if co is not None and ust.normed else None
        if self.raw_items:
            modal, rst = self._raw_items_fwd(b, seeds)
        else:
            modal = b["target_modal"]
        if co is not None:
            it, ist = F.item_fusion_fwd_end(co)
        else:
            it, ist = F.item_fusion_fwd(self.Pi, self.Wi, modal, self.icfg, seeds,
                                        self.bufs, self.p_item)
        self._fx = None
        # one process: the step's weight-gradient partials are folded inside the AdamW launch
        with ops.deferred_wgrad(defer_fold=self.plan_wgrad) as pend, \
                (ops.fx_grad_sink() if fx_sink else contextlib.nullcontext([])) as sink:
            # one fold launch for the step's weight grads; with the GEMMs on the side stream
            # (ops.wgrad_launch_early) the update joins them (_update)
            pend.hold_join = True
            self._bwd(b, u, it, modal, ust, ist, rst if self.raw_items else None, cut, pend)
        self._fold = (pend.plan, pend.keep) if pend.plan is not None else None
        self._pend = pend
        if sink:
            acc, view = sink[0]
            if view.data_ptr() >= self.flat.grad.data_ptr() and \
                    view.data_ptr() + 4 * view.numel() <= self.flat.grad.data_ptr() + 4 * self.flat.numel:
                self._fx = (acc, view)
            else:                              # not a slot of the flat gradient: fold it now
                ops.fx_folds([(acc, view)])

    def _bwd(self, b, u, it, modal, ust, ist, rst, cut, pend) -> None:
        du = torch.empty_like(u)
        di = torch.empty_like(it)
        du16 = None
        if self.global_negatives:         # cfg 5: negatives from every rank's batch
            gst = F.infonce_global_prep(u, it, b.get("user_idx"), self.model.temperature,
                                        self.group)
            if gst.dp:
                cut(lambda: F.infonce_global_gather(gst, self.group))
            loss = F.infonce_global_loss(gst)
            self.loss_sum.add_(loss.view(1))
            logits = gst.s_u2i
            F.infonce_global_loss_bwd(gst, self.dloss)
            if gst.dp:
                cut(lambda: F.infonce_global_scatter(gst, self.group))
            F.infonce_global_norm_bwd(gst, du, di)
        else:
            loss, logits, _, _, lst = F.infonce_fwd(u, it, b.get("user_idx"),
                                                    self.model.temperature, normed=self._normed,
                                                    loss_acc=self.loss_sum)
            du16 = torch.empty(u.shape, device=u.device, dtype=self.ucfg.dtype) \
                if self.ucfg.dtype == torch.bfloat16 else None
            F.infonce_bwd(lst, self.dloss, du, di, du16)
        # cfg 2: the item head's row-local backward rides in the user head backward launch
        ib = None if self.raw_items else F.item_fusion_bwd_begin(
            self.Pi, self.Wi, ist, di, self.Gi, self.icfg, self.p_item)
        if ib is None:
            dmodal = torch.empty(modal.shape, device=modal.device) if self.raw_items else None
            F.item_fusion_bwd(self.Pi, self.Wi, ist, di, self.Gi, self.icfg, self.p_item, dmodal)
            if self.raw_items:
                self._raw_items_bwd(rst, dmodal)
        hook = None
        if self.overlap:
            def hook(i: int) -> None:
                if i != 1:       # every gradient before the tail slots is final
                    return
                if self._split_cuts:           # host cuts: complete them here, reduce at the cut
                    pend.flush_on(torch.cuda.current_stream(self.device))
                    self._fill_extra()
                    cut(self._sync_head)
                    return
                # their GEMMs + folds and the head bucket's all-reduce run on the side stream
                # (RCCL's own stream after it) while this stream differentiates layer 0 and
                # the input block; the update joins them
                side = ops.wgrad_side_stream(self.device)
                pend.flush_on(side)
                with torch.cuda.stream(side):
                    self._fill_extra()         # BN buffers + id flags: final since the forward
                    self._sync_head()
        F.user_tower_bwd(self.Pu, self.Wu, ust, du, self.Gu, self.ucfg, du16, on_layer_done=hook,
                         co_item=ib)
        self.loss, self.logits = loss, logits

    def _mirror_transposes(self):
        """(dsts, srcs) of every Wᵀ mirror of the bf16 weights (user tower encoder + fusion MLP,
        item W4), refreshed by each step's prologue after the previous step's AdamW."""
        if self.flat.mirror is None:
            return [], []
        T = F.transposed_name
        names = [n for n in encoder_weight_names(_gemm_names(list(self.Pu))) if T(n) in self.Wu]
        dsts = [self.Wu[T(n)] for n in names]
        srcs = [self.Wu[n] for n in names]
        t4 = T("fusion_layer.4.weight")
        if t4 in self.Wi:
            dsts.append(self.Wi[t4])
            srcs.append(self.Wi["fusion_layer.4.weight"])
        return dsts, srcs

    def _fill_extra(self) -> None:
        """The all-reduced slots after the gradients: rank 0's BatchNorm buffers (the others add
        zeros) and this rank's id-range flags; one copy launch."""
        gx = self.flat.grad_extra
        dsts, srcs = [], []
        if self.broadcast_buffers:
            dsts.append(gx[:self.n_bufx])
            srcs.append(self.fbufs.data if self.is_root else self.bzero)
        if self.dp:
            dsts.append(gx[self.flag_off:self.flag_off + 8])
            srcs.append(ops.id_err_flags(self.flat.data))
        if dsts:
            ops.batch_copy(dsts, srcs)
        self._extra_filled = True

    def _sync_head(self) -> None:
        self._pending = self.sync.start(self.flat.grad[:self.flat.tail_offset])

    def _sync_tail(self) -> None:
        g = self.flat.grad[self.flat.tail_offset:] if self.overlap else self.flat.grad
        works = self._pending + self.sync.start(g)
        self._pending = []
        for w in works:
            w.wait()

    def _raw_items_fwd(self, b: Dict[str, Tensor], seeds: Optional[Tensor]):
        """cfg 3 item encoders (item_tower.py:131-147): audio/visual ResNet-18, zero text slot,
        tabular MLP, concatenated in the reference's order."""
        outs, saved = [], []
        for (P, _, bufs, c), key in zip(self.enc, ("target_audio", "target_image")):
            o, st = cnn.resnet18_fwd(P, b[key], c, bufs)
            outs.append(o)
            saved.append(st)
        B = outs[0].shape[0]
        P, _, bufs = self.tab
        t, tst = cnn.tabular_fwd(P, b["target_tabular"], bufs, seeds, self.p_tab)
        xst = ts = None
        if self.text is not None:
            enc, TP, _ = self.text
            ts = None
            if seeds is not None:
                ops.dropout_seeds(self.base_seed ^ 0x7E47, self.step_t, self.text_seeds)
                ts = self.text_seeds
            text, xst = T.text_fwd(enc, TP, b["target_input_ids"], b["target_attention_mask"],
                                   ts, True)
        else:
            text = torch.zeros(B, self.text_dim, device=t.device)
        return torch.cat([outs[0], outs[1], text, t], dim=1), (saved, tst, xst, ts)

    def _raw_items_bwd(self, rst, dmodal: Tensor) -> None:
        saved, tst, xst, ts = rst
        o = 0
        for (P, G, _, c), st in zip(self.enc, saved):
            n = G["fc.bias"].numel()
            cnn.resnet18_bwd(P, st, dmodal[:, o:o + n], G, c)
            o += n
        if xst is not None:
            enc, TP, TG = self.text
            T.text_bwd(enc, TP, xst, dmodal[:, o:o + self.text_dim], TG, ts)
        o += self.text_dim
        P, G, _ = self.tab
        cnn.tabular_bwd(P, tst, dmodal[:, o:], G)

    def _update(self) -> None:
        f = self.flat
        pend, self._pend = self._pend, None
        plan = self._fold[0] if self._fold else None
        # a step whose lookups met an id outside a table (on any rank) updates nothing
        skip_if = f.grad_extra[self.flag_off:].data_ptr() if self.dp else ops.id_err_ptr(f.data)
        if pend is not None and pend.side is not None and self._fx is not None and _ADAM_SPLIT:
            # the item-embedding rows' update (their gradient complete in the fixed-point
            # accumulator) runs while the weight-gradient GEMMs finish on the side stream; the
            # rest of the flat buffer after the join
            skip = ops.adamw_fx_range(f.data, f.grad, f.exp_avg, f.exp_avg_sq, f.mirror, self.hyper,
                                      self.step_t, self._fx, zero_grad=True, skip_if=skip_if)
            pend.join()
            ops.adamw(f.data, f.grad, f.exp_avg, f.exp_avg_sq, f.mirror, self.hyper, self.step_t,
                      zero_grad=True, fold_plan=plan, skip=skip, skip_if=skip_if)
        else:
            if pend is not None:
                pend.join()
            ops.adamw(f.data, f.grad, f.exp_avg, f.exp_avg_sq, f.mirror, self.hyper, self.step_t,
                      zero_grad=True, fx=self._fx, fold_plan=plan, skip_if=skip_if)
        self._fx = None
        self._fold = None

    def _body(self, b: Dict[str, Tensor], cut: Callable = _no_cut) -> None:
        # one process: the item-embedding gradient goes from its fixed-point accumulator
        # straight into AdamW (no fold pass over the [V, D] table); with DDP it is folded
        # into the flat gradient for the all-reduce
        self._extra_filled = False
        self._fwd_bwd(b, cut, fx_sink=not self.dp and self.grad_sink)
        if self.dp:
            # complete the gradient before the tail all-reduce: join the side stream (the head
            # bucket's GEMMs, folds and all-reduce launch; the early weight-gradient GEMMs) and
            # fold the planned partials here instead of inside AdamW
            self._pend.join()
            if self._fold is not None:
                ops.fold_plan_run(self._fold[0])
                self._keep = self._fold[1]
                self._fold = None
            if not self._extra_filled:
                self._fill_extra()
            cut(self._sync_tail)
        self._update()
        self._keep = None

    # ---------------------------------------------------------------- capture
    @staticmethod
    def _signature(batch: Dict[str, Tensor]) -> tuple:
        return tuple((k, tuple(batch[k].shape), batch[k].dtype)
                     for k in TrainStep.INPUT_KEYS if k in batch)

    def check(self) -> None:
        """Wait for the queued steps and raise IndexError if any of them met an embedding id
        outside its table (the reference's nn.Embedding raises, user_tower.py:26,30-31).  The
        device lookups clamp such an id and set a flag; that step's AdamW then updates nothing
        (parameters, moments and the bf16 mirror keep their values; its BatchNorm running
        statistics and ``loss_sum`` do include it, and Adam's step count advances), and
        ``step()`` raises at its start for any earlier step that has finished, with no sync of
        its own.  Call ``check()`` at the end of a loop so the last steps are covered too."""
        ops.check_id_errors(sync=True)

    def _stage(self, batch: Dict[str, Tensor]) -> Dict[str, Tensor]:
        sig = self._signature(batch)
        e = self._entries.get(sig)
        if e is None:
            e = _Entry({k: torch.empty(batch[k].shape, dtype=batch[k].dtype, device=self.device)
                        for k in self.INPUT_KEYS if k in batch})
            self._entries[sig] = e
        self._cur = e
        keys = list(e.static)
        srcs = [batch[k] for k in keys]
        # the step's prologue in one launch (ttmi_step_prologue), ahead of the graph: the batch
        # into the static inputs, the device id-range flags cleared (this step's AdamW skips
        # only for this step's bad ids), data-parallel: rank 0's BatchNorm buffers from the last
        # all-reduce over this rank's (DDP broadcast_buffers); the Wᵀ mirrors of the updated
        # bf16 weights; the dropout seeds and the step count
        fl_dst, fl_src = ops.id_err_step_reset(self.flat.data)
        xd, xs = [fl_dst], [fl_src]
        if self.broadcast_buffers:
            xd.append(self.fbufs.data)
            xs.append(self.flat.grad_extra[:self.n_bufx])
        if all(t.is_cuda and t.is_contiguous() and t.dtype == e.static[k].dtype
               for k, t in zip(keys, srcs)):
            xd, xs = [e.static[k] for k in keys] + xd, srcs + xs
        else:
            for k, t in zip(keys, srcs):
                e.static[k].copy_(t, non_blocking=True)
        td, ts = self._mirror_transposes()
        ops.step_prologue(xd, xs, td, ts, self.step_t,
                          (self.base_seed, self.seeds) if self._draw else None)
        return e.static

    def _state(self):
        return [self.flat.data, self.flat.exp_avg, self.flat.exp_avg_sq, self.step_t, self.loss_sum,
                *self.bufs.values()] + ([self.flat.mirror] if self.flat.mirror is not None else []) + \
            ([self.flat.grad_extra] if self.dp else [])

    def _capture(self, e: _Entry) -> None:
        b = e.static
        snap = [t.clone() for t in self._state()]
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):          # warm-up: load code objects, size the pool
            self._body(b)
        torch.cuda.current_stream(self.device).wait_stream(side)
        for t, s in zip(self._state(), snap):   # undo the warm-up's state changes
            t.copy_(s)
        torch.cuda.synchronize(self.device)
        if self.capture_collectives:
            comm.quiesce_before_capture()       # the watchdog retires the warm-up's collectives
        try:
            seg = self._record(b)
        except Exception as exc:
            if not self.capture_collectives:
                raise
            # Collectives recorded into the graph were refused at this world size (exercised on
            # the GPU at world 1 only: RCCL needs a device per rank).  Fall back to the segmented
            # schedule, collectives between graph replays, rather than fail the run.
            logging.getLogger(__name__).warning(
                "TrainStep: recording the collectives into the step graph failed (%s); "
                "falling back to graph segments with the collectives between them", exc)
            for t, s0 in zip(self._state(), snap):
                t.copy_(s0)
            torch.cuda.synchronize(self.device)
            self.capture_collectives = False
            seg = self._record(b)
        e.seg, e.loss, e.logits = seg, self.loss, self.logits

    def _record(self, b: Dict[str, Tensor]) -> _Segments:
        seg = _Segments(self.device, capture=True, pool=torch.cuda.graph_pool_handle(),
                        inline=self.capture_collectives)
        self._split_cuts = self.dp and not seg.inline
        try:
            seg.begin()
            self._body(b, seg.cut)
            seg.end()
        except BaseException:
            seg.abort()
            raise
        finally:
            self._split_cuts = False
        return seg

    def step(self, batch: Dict[str, Tensor]) -> Tensor:
        ops.check_id_errors()                  # bad ids of earlier (finished) steps: IndexError
        ops.bump_param_epoch()                 # the replay below rewrites the parameters
        b = self._stage(batch)
        e = self._cur
        if not self.use_graph:
            self._body(b)
            return self.loss
        if e.seg is None:
            self._capture(e)
        e.seg.replay()
        self.loss, self.logits = e.loss, e.logits
        return self.loss

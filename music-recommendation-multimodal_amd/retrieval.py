"""Global retrieval evaluation, top-K serving and checkpoint interchange — SURVEY §8(f)
ranks 2-4: drop-ins for reference src/evaluate_metrics.py:107-192 (``calculate_metrics_global``),
the scoring half of src/inference.py's ``recommend`` (:228-323) and the checkpoint loading of
inference.py:97-107 / evaluate_metrics.py:300-305.

Users are scored against the whole catalogue: ``scores = û·Îᵀ`` (fp32 MFMA GEMM, ttmi_gemm),
column 0 (the padding item) excluded, top-K per user by radix select (``ttmi_topk_rows``),
and the rank of each user's target (``ttmi_rank_of``): Recall@k = rank < k, NDCG@k =
1/log2(rank + 2) when rank < k (the reference's gains, evaluate_metrics.py:172-181).
"""
from __future__ import annotations

import math
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as TF

from . import ops

Tensor = torch.Tensor


def dense_item_index(item_ids: Tensor, embeddings: Tensor, vocab_size: int) -> Tensor:
    """compute_all_item_embeddings' tail (evaluate_metrics.py:84-104): nan_to_num, L2-normalise
    (eps 1e-8), scatter rows into a dense [vocab_size, D] table (row 0 = padding = 0)."""
    emb = TF.normalize(torch.nan_to_num(embeddings.float(), nan=0.0), p=2, dim=1, eps=1e-8)
    dense = torch.zeros(vocab_size, emb.shape[1], device=emb.device)
    dense[item_ids.long()] = emb
    return dense


def score_catalogue(user_emb: Tensor, item_emb: Tensor, out: Optional[Tensor] = None) -> Tensor:
    """scores [B, V] = user_emb [B, D] · item_emb [V, D]ᵀ in fp32 (evaluate_metrics.py:150)."""
    u = user_emb.float().contiguous()
    it = item_emb.float().contiguous()
    B, D = u.shape
    V = it.shape[0]
    out = out if out is not None else torch.empty(B, V, device=u.device)
    ops.gemm(u, it, out, B, V, D, lda=D, a_kmajor=True, ldb=D, b_kmajor=True, ldc=V)
    return out


def topk_items(user_emb: Tensor, item_emb: Tensor, k: int,
               skip_padding: bool = True) -> Tuple[Tensor, Tensor]:
    """(scores, indices) [B, k] of the k best catalogue items per user, descending (ties by
    lower index), the padding item 0 excluded (evaluate_metrics.py:153-158)."""
    scores = score_catalogue(user_emb, item_emb)
    B = scores.shape[0]
    val = torch.empty(B, k, device=scores.device)
    idx = torch.empty(B, k, device=scores.device, dtype=torch.int64)
    ops.topk_rows(scores, k, val, idx, skip_first=skip_padding)
    return val, idx


def target_ranks(user_emb: Tensor, item_emb: Tensor, targets: Tensor, max_k: int) -> Tensor:
    """Rank of each target in the user's top-max_k list (max_k when absent), int32 [B]."""
    _, idx = topk_items(user_emb, item_emb, max_k)
    rank = torch.empty(idx.shape[0], device=idx.device, dtype=torch.int32)
    ops.rank_of(idx, targets.long().contiguous(), rank)
    return rank


def metrics_from_ranks(ranks: Tensor, k_list: Sequence[int]) -> Dict[str, Tensor]:
    """Per-user Recall@k and NDCG@k from target ranks (evaluate_metrics.py:163-181)."""
    r = ranks.float()
    out = {}
    for k in k_list:
        hit = r < k
        out[f"Recall@{k}"] = hit.float()
        out[f"NDCG@{k}"] = torch.where(hit, 1.0 / torch.log2(r + 2.0), torch.zeros_like(r))
    return out


class GlobalEvaluator:
    """The per-batch work of calculate_metrics_global (evaluate_metrics.py:139-161): user
    embedding (eval) -> fp32 catalogue scores -> top-max_k -> target ranks, replayed from a HIP
    graph captured once per batch signature (size, present keys, dtypes); the eval loop is then
    one graph launch per batch instead of ~25 host-issued kernels.  Batches are staged into the
    graph's static inputs; ``ranks`` returns the graph's static output (valid until the next
    call).  The user tower's cached bf16 weights are re-checked before every replay, so a
    model trained between evaluations is scored with its current weights."""

    KEYS = ("history_ids", "history_mask", "user_gender", "user_country", "target_id")

    def __init__(self, model, item_embeddings: Tensor, max_k: int, use_graph: bool = True):
        self.model = model
        self.items = item_embeddings.float().contiguous()
        self.max_k = max_k
        # graphs only for this package's model: a foreign model may keep host-side state
        # (or run host syncs) per call, which a replay would not reproduce
        self._tower = getattr(model, "user_tower", None)
        if not hasattr(self._tower, "inference_operands"):
            self._tower = None
        self.use_graph = use_graph and self._tower is not None
        self._graphs: Dict[tuple, tuple] = {}

    def _run(self, b: Dict[str, Tensor]) -> Tensor:
        u = self.model.get_user_embedding(history_ids=b["history_ids"],
                                          history_mask=b.get("history_mask"),
                                          user_gender=b.get("user_gender"),
                                          user_country=b.get("user_country"))
        return target_ranks(u, self.items, b["target_id"], self.max_k)

    def ranks(self, batch: Dict[str, Tensor]) -> Tensor:
        ops.check_id_errors()          # ids outside a table in an earlier (finished) batch
        dev = self.items.device
        b = {k: batch[k].to(dev, non_blocking=True) for k in self.KEYS if batch.get(k) is not None}
        self.model.eval()
        with torch.no_grad():
            opkey = None
            if self._tower is not None:
                P, W = self._tower.inference_operands()      # refresh cached weights (host check)
                # a graph replays the buffers it was captured on: when the cache rebuilt them
                # (new storages, e.g. TrainStep re-homed the parameters), every graph is stale
                opkey = tuple(t.data_ptr() for t in P.values()) + \
                    tuple(t.data_ptr() for t in W.values())
                if opkey != getattr(self, "_opkey", None):
                    self._graphs.clear()
                    self._opkey = opkey
            if not self.use_graph:
                return self._run(b)
            sig = tuple((k, tuple(t.shape), t.dtype) for k, t in sorted(b.items()))
            ent = self._graphs.get(sig)
            if ent is None:
                static = {k: t.clone() for k, t in b.items()}
                side = torch.cuda.Stream(dev)
                side.wait_stream(torch.cuda.current_stream(dev))
                with torch.cuda.stream(side):              # warm-up: code objects, pool sizes
                    self._run(static)
                torch.cuda.current_stream(dev).wait_stream(side)
                torch.cuda.synchronize(dev)
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):
                    out = self._run(static)
                ent = self._graphs[sig] = (static, out, graph)
            static, out, graph = ent
            ops.batch_copy([static[k] for k in static], [b[k].contiguous() for k in static])
            graph.replay()
            return out


class CatalogueIndexer:
    """The catalogue index of compute_all_item_embeddings (evaluate_metrics.py:24-104) and
    index_catalog (inference.py:137-209): every item's tower embedding (model.eval(): BatchNorm
    on running statistics, no dropout), L2-normalised as get_item_embedding does, NaN -> 0,
    normalised again with eps 1e-8, scattered into a dense [vocab_size, D] table whose row i is
    item id i (row 0, padding, and items never seen stay 0).  The table stays on the device
    (it feeds GlobalEvaluator / recommend directly).  Per batch: the item-tower forward and
    the fused normalise-and-scatter kernel (ttmi_catalogue_rows), replayed from one HIP graph
    per batch signature; the batch carries ``target_id`` and the item inputs under the
    reference's keys (``target_image``, ``target_audio``, ``target_input_ids``,
    ``target_attention_mask``, ``target_tabular``) or cfg 2's ``target_modal``."""

    KEYS = ("target_id", "target_modal", "target_image", "target_audio", "target_input_ids",
            "target_attention_mask", "target_tabular")

    def __init__(self, model, vocab_size: int, device=None, use_graph: bool = True):
        self.model = model
        self.vocab_size = vocab_size
        self.device = device if device is not None else next(model.parameters()).device
        self.use_graph = use_graph
        D = model.item_tower.embedding_dim
        self.dense = torch.zeros(vocab_size, D, device=self.device)
        self._graphs: Dict[tuple, tuple] = {}

    def _item(self, b: Dict[str, Tensor]) -> Tensor:
        it = self.model.item_tower
        if "target_modal" in b:
            return it.fuse(b["target_modal"])
        return it(images=b.get("target_image"), audio=b.get("target_audio"),
                  input_ids=b.get("target_input_ids"),
                  attention_mask=b.get("target_attention_mask"), tabular=b["target_tabular"])

    def _run(self, b: Dict[str, Tensor]) -> None:
        emb = self._item(b).float()
        ops.catalogue_rows(emb, b["target_id"].long().contiguous(), self.dense)

    def add(self, batch: Dict[str, Tensor]) -> None:
        """Index one batch of items."""
        ops.check_id_errors()          # target_id / token ids outside their tables, earlier batches
        dev = self.device
        b = {k: batch[k].to(dev, non_blocking=True) for k in self.KEYS if batch.get(k) is not None}
        b["target_id"] = b["target_id"].long()
        self.model.eval()
        with torch.no_grad():
            if not self.use_graph:
                self._run(b)
                return
            # a graph replays the storages it was captured on: when the item tower's parameters
            # or buffers were re-homed (TrainStep's flat buffers, load_state_dict into new
            # tensors), every captured graph is stale
            it = self.model.item_tower
            opkey = tuple(t.data_ptr() for t in it.parameters()) + \
                tuple(t.data_ptr() for t in it.buffers())
            if opkey != getattr(self, "_opkey", None):
                self._graphs.clear()
                self._opkey = opkey
            sig = tuple((k, tuple(t.shape), t.dtype) for k, t in sorted(b.items()))
            ent = self._graphs.get(sig)
            if ent is None:
                static = {k: t.clone() for k, t in b.items()}
                side = torch.cuda.Stream(dev)
                side.wait_stream(torch.cuda.current_stream(dev))
                with torch.cuda.stream(side):              # warm-up: code objects, pool sizes
                    self._run(static)
                torch.cuda.current_stream(dev).wait_stream(side)
                torch.cuda.synchronize(dev)
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):
                    self._run(static)
                ent = self._graphs[sig] = (static, graph)
            static, graph = ent
            ops.batch_copy([static[k] for k in static], [b[k].contiguous() for k in static])
            graph.replay()

    def index(self, loader: Iterable) -> Tensor:
        """Zero the table, index every batch of ``loader``, return the dense [V, D] index."""
        self.dense.zero_()
        for batch in loader:
            self.add(batch)
        ops.check_id_errors(sync=True)     # dense[target_id] = emb raises for a bad id (:102)
        return self.dense


def compute_all_item_embeddings(model, loader: Iterable, vocab_size: int, device=None,
                                use_graph: bool = True) -> Tuple[Tensor, int]:
    """evaluate_metrics.py:24-104's result, (dense [vocab_size, D], vocab_size), from a loader
    over the unique catalogue items (the reference builds that loader from its dataset)."""
    ix = CatalogueIndexer(model, vocab_size, device, use_graph=use_graph)
    return ix.index(loader), vocab_size


def calculate_metrics_global(model, val_loader: Iterable, item_embeddings: Tensor, device,
                             k_list: List[int] = [10, 20], use_graph: bool = True) -> Dict[str, float]:
    """evaluate_metrics.py:107-192 on libttmi kernels: same batch keys, same metrics."""
    model.eval()
    ev = GlobalEvaluator(model, item_embeddings.to(device), max(k_list), use_graph=use_graph)
    per: Dict[str, List[Tensor]] = {f"Recall@{k}": [] for k in k_list}
    per.update({f"NDCG@{k}": [] for k in k_list})
    with torch.no_grad():
        for batch in val_loader:
            ranks = ev.ranks(batch)
            for name, v in metrics_from_ranks(ranks, k_list).items():
                per[name].append(v.cpu())
    ops.check_id_errors(sync=True)
    return {name: torch.cat(v).mean().item() for name, v in per.items()}


def recommend(model, history_ids: Tensor, item_embeddings: Tensor, k: int = 10,
              user_gender: Optional[Tensor] = None, user_country: Optional[Tensor] = None,
              max_len: int = 50) -> Tuple[Tensor, Tensor]:
    """inference.py:254-310 for a batch of users: keep the last ``max_len`` history items,
    user embedding (eval, L2-normalised with eps 1e-8), scores against the catalogue, padding
    item and history items excluded, top-k -> (scores [B, k], item indices [B, k])."""
    model.eval()
    hist = history_ids[:, -max_len:].long()
    with torch.no_grad():
        u = model.get_user_embedding(history_ids=hist, user_gender=user_gender,
                                     user_country=user_country)
        u = TF.normalize(u, p=2, dim=1, eps=1e-8)
        scores = score_catalogue(u, item_embeddings.to(u.device))
        ops.mask_items(scores, hist)
        B = scores.shape[0]
        val = torch.empty(B, k, device=scores.device)
        idx = torch.empty(B, k, device=scores.device, dtype=torch.int64)
        ops.topk_rows(scores, k, val, idx, skip_first=True)
    return val, idx


def reference_state_dict(source) -> Dict[str, Tensor]:
    """A reference checkpoint (path or dict) with DDP's ``module.`` prefix stripped
    (inference.py:97-107).  Files are read with torch.load(weights_only=True): tensors only."""
    sd = torch.load(source, map_location="cpu", weights_only=True) if isinstance(source, str) \
        else dict(source)
    if sd and next(iter(sd)).startswith("module."):
        sd = {k[len("module."):] if k.startswith("module.") else k: v for k, v in sd.items()}
    return sd


def model_from_reference_checkpoint(source, vocab_size: Optional[int] = None,
                                    num_genders: Optional[int] = None, **kw):
    """Build a TwoTowerModel whose dimensions come from the checkpoint (inference.py:109-128:
    countries from user_tower.country_embedding, tabular width from the tabular encoder, the
    embedding width from the item embedding; here also the vocabulary, genders, history length,
    encoder depth and the text encoder's shape) and load it (strict: every key must match).
    Explicit keyword arguments override what the checkpoint implies; the head count is not
    recorded in a state_dict (default 4, as train.py:289-297 builds it)."""
    from .two_tower import TwoTowerModel
    from .text import TextCfg
    sd = reference_state_dict(source)
    ue = sd["user_tower.item_embedding.weight"]
    D = ue.shape[1]
    if vocab_size is None:
        vocab_size = ue.shape[0]
    if num_genders is None:
        num_genders = sd["user_tower.gender_embedding.weight"].shape[0]
    kw.setdefault("num_countries", sd["user_tower.country_embedding.weight"].shape[0])
    kw.setdefault("max_seq_len", sd["user_tower.position_embedding.weight"].shape[0])
    pre = "user_tower.transformer_encoder.layers."
    kw.setdefault("user_num_layers", len({k[len(pre):].split(".")[0] for k in sd if k.startswith(pre)}))
    if "item_tower.tabular_encoder.mlp.0.weight" in sd:
        kw.setdefault("tabular_input_dim", sd["item_tower.tabular_encoder.mlp.0.weight"].shape[1])
        kw.setdefault("precomputed_modalities", False)
        tp = "item_tower.text_encoder.transformer.base_model.model."
        with_text = any(k.startswith("item_tower.text_encoder.") for k in sd)
        kw.setdefault("with_text", with_text)
        if with_text and "text_cfg" not in kw:
            lp = tp + "encoder.layer."
            word = sd[tp + "embeddings.word_embeddings.weight"]
            kw["text_cfg"] = TextCfg(
                vocab_size=word.shape[0], hidden=word.shape[1],
                layers=len({k[len(lp):].split(".")[0] for k in sd if k.startswith(lp)}),
                intermediate=sd[lp + "0.intermediate.dense.weight"].shape[0],
                heads=word.shape[1] // 64,
                position_buckets=sd[tp + "encoder.rel_embeddings.weight"].shape[0] // 2)
    else:
        kw.setdefault("tabular_input_dim", 128)
        kw.setdefault("precomputed_modalities", True)
    model = TwoTowerModel(vocab_size=vocab_size, num_genders=num_genders, user_embedding_dim=D,
                          item_embedding_dim=D, **kw)
    model.load_state_dict(sd)
    return model

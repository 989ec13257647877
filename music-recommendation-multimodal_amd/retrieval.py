"""Global retrieval evaluation and top-K serving — SURVEY §8(f) rank 2, drop-in for reference
src/evaluate_metrics.py:107-192 (``calculate_metrics_global``) and the scoring half of
src/inference.py's ``recommend``.

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


def calculate_metrics_global(model, val_loader: Iterable, item_embeddings: Tensor, device,
                             k_list: List[int] = [10, 20]) -> Dict[str, float]:
    """evaluate_metrics.py:107-192 on libttmi kernels: same batch keys, same metrics."""
    model.eval()
    item_embeddings = item_embeddings.to(device).float()
    per: Dict[str, List[Tensor]] = {f"Recall@{k}": [] for k in k_list}
    per.update({f"NDCG@{k}": [] for k in k_list})
    max_k = max(k_list)
    with torch.no_grad():
        for batch in val_loader:
            user_emb = model.get_user_embedding(
                history_ids=batch["history_ids"].to(device),
                history_mask=batch["history_mask"].to(device),
                user_gender=batch["user_gender"].to(device),
                user_country=batch["user_country"].to(device))
            ranks = target_ranks(user_emb, item_embeddings, batch["target_id"].to(device), max_k)
            for name, v in metrics_from_ranks(ranks, k_list).items():
                per[name].append(v.cpu())
    return {name: torch.cat(v).mean().item() for name, v in per.items()}

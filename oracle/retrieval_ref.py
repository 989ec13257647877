"""ORACLE — test infrastructure only (never imported by the product path).

CPU restatement of reference src/evaluate_metrics.py:143-185 (calculate_metrics_global's
per-batch body): scores = û·Îᵀ, scores[:, 0] = -inf, torch.topk(max_k), Recall@k = any hit in
the first k, NDCG@k = 1/log2(rank + 2) at the hit.  Pinned by tests/golden/retrieval.npz, which
the reference function itself produced (tools/make_golden_retrieval.py)."""
from __future__ import annotations

from typing import Dict, Sequence

import torch

Tensor = torch.Tensor


def retrieval_metrics(user_emb: Tensor, item_emb: Tensor, targets: Tensor,
                      k_list: Sequence[int] = (10, 20)) -> Dict[str, Tensor]:
    scores = user_emb.float() @ item_emb.float().t()
    scores[:, 0] = -float("inf")
    max_k = max(k_list)
    _, topk = torch.topk(scores, k=max_k, dim=1)
    t = targets.long().unsqueeze(1)
    out = {}
    for k in k_list:
        preds = topk[:, :k]
        hits = (preds == t).any(dim=1)
        out[f"Recall@{k}"] = hits.float()
        ndcg = torch.zeros(hits.shape[0])
        pos = (preds == t).nonzero(as_tuple=False)
        if pos.shape[0] > 0:
            ndcg[pos[:, 0]] = 1.0 / torch.log2(pos[:, 1].float() + 2.0)
        out[f"NDCG@{k}"] = ndcg
    return out

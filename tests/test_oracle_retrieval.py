"""Retrieval oracle (oracle/retrieval_ref.py) against the metrics the reference's own
calculate_metrics_global produced (tests/golden/retrieval.npz, tools/make_golden_retrieval.py)."""
import numpy as np
import torch

from conftest import load_golden
from oracle import retrieval_ref as rr


def test_retrieval_oracle_vs_reference_fixture():
    z = load_golden("retrieval.npz")
    m = rr.retrieval_metrics(torch.tensor(z["users"]), torch.tensor(z["items"]),
                             torch.tensor(z["targets"]), (10, 20))
    for k in ("Recall@10", "Recall@20", "NDCG@10", "NDCG@20"):
        assert abs(m[k].mean().item() - float(z["metric/" + k])) < 1e-6, k

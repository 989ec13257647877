"""Generate tests/golden/retrieval.npz by running the REFERENCE calculate_metrics_global
(src/evaluate_metrics.py:107-192) on synthetic embeddings.  Build container only: the
reference's own imports need transformers (present) and src.data.dataset (absent in the
reference tree), for which an empty stand-in module is registered, as SURVEY §8(c) records.
A stub model returns the given user embeddings; targets are planted at known ranks so both
hits and misses occur."""
import os
import sys
import types

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"


def main():
    import transformers  # noqa: F401  (probes torchvision; must import before the stubs)
    stub = types.ModuleType("src.data.dataset")
    stub.MultimodalDataset = object
    sys.modules.setdefault("src.data", types.ModuleType("src.data"))
    sys.modules["src.data.dataset"] = stub
    tv = types.ModuleType("torchvision")
    tv.models = types.ModuleType("torchvision.models")
    sys.modules.setdefault("torchvision", tv)
    sys.modules.setdefault("torchvision.models", tv.models)
    peft = types.ModuleType("peft")
    peft.get_peft_model = lambda *a, **k: None
    peft.LoraConfig = object
    peft.TaskType = types.SimpleNamespace(FEATURE_EXTRACTION="FEATURE_EXTRACTION")
    sys.modules.setdefault("peft", peft)
    sys.path.insert(0, REF)
    from src import evaluate_metrics as em

    g = torch.Generator().manual_seed(0)
    V, D, B, nb = 3001, 64, 48, 3
    items = torch.nn.functional.normalize(torch.randn(V, D, generator=g), dim=1)
    items[0] = 0.0
    users = torch.nn.functional.normalize(torch.randn(B * nb, D, generator=g), dim=1)
    scores = users @ items.t()
    scores[:, 0] = -float("inf")
    order = torch.argsort(scores, dim=1, descending=True)
    plant = torch.tensor([0, 1, 5, 9, 10, 15, 19, 20, 50, 2999] * (B * nb // 10 + 1))[:B * nb]
    targets = order[torch.arange(B * nb), plant.clamp(max=V - 2)]

    class Stub:
        def __init__(self):
            self.i = 0

        def eval(self):
            return self

        def get_user_embedding(self, history_ids, history_mask, user_gender, user_country):
            out = users[self.i:self.i + history_ids.shape[0]]
            self.i += history_ids.shape[0]
            return out

    loader = []
    for b in range(nb):
        sl = slice(b * B, (b + 1) * B)
        loader.append({"history_ids": torch.ones(B, 5, dtype=torch.long),
                       "history_mask": torch.ones(B, 5, dtype=torch.long),
                       "user_gender": torch.zeros(B, dtype=torch.long),
                       "user_country": torch.zeros(B, dtype=torch.long),
                       "target_id": targets[sl]})
    res = em.calculate_metrics_global(Stub(), loader, items, "cpu", k_list=[10, 20])
    z = {"users": users.numpy(), "items": items.numpy(), "targets": targets.numpy()}
    for k, v in res.items():
        z["metric/" + k] = np.array(v)
    path = os.path.join(ROOT, "tests", "golden", "retrieval.npz")
    np.savez_compressed(path, **z)
    print(path, res)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Generate tests/golden/serving.npz by RUNNING THE REFERENCE inference functions
(src/inference.py ``index_catalog`` :137-209 and ``recommend_for_user`` :213-300) in the build
container (the GPU box never sees the reference; only the arrays travel).

Recipe: tools/make_golden.py's import stand-ins (torchvision / peft / src.data.dataset), the
reference's own TwoTowerModel with identity modality encoders (the late-fusion head on
precomputed 128-d modality embeddings, as BASELINE cfg 2), in eval mode with non-trivial
BatchNorm running statistics.  ``MultimodalDataset`` — absent from the reference snapshot — is a
minimal stand-in that serves those embeddings and the interaction frame.  ``index_catalog``
writes the dense index with torch.save (read back here with weights_only=True);
``recommend_for_user`` prints its top-10, which is parsed (artist names encode the item id;
scores are printed to 4 decimals, the ids are the pinned quantity).

Usage: python tools/make_golden_serving.py   (writes tests/golden/serving.npz)
"""
from __future__ import annotations

import contextlib
import io
import os
import re
import sys
import tempfile
import types

import numpy as np
import pandas as pd
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import make_golden as mg  # noqa: E402

V, D, L_HIST, USER = 97, 32, 63, "u7"
N_ITEMS = V - 1          # the reference sizes the index len(item_id_mapper) + 1


class _CatalogueDataset(torch.utils.data.Dataset):
    """Stand-in for the reference's MultimodalDataset as index_catalog builds it
    (inference.py:148-155): one row per unique track, the item keys its loader reads."""

    modal = None          # [n_tracks, 512] precomputed modality embeddings, set by main()

    def __init__(self, interactions_df, item_id_mapper, img_dir=None, text_data=None,
                 tokenizer=None, encoders=None, **kw):
        self.df = interactions_df.reset_index(drop=True)
        self.mapper = item_id_mapper

    def __len__(self):
        return len(self.df)

    def __getitem__(self, i):
        tid = self.df["track_id"][i]
        m = self.modal[int(tid[1:])]
        return {"target_id": self.mapper[tid], "target_audio": m[0:128], "target_image": m[128:256],
                "target_input_ids": m[256:384], "target_attention_mask": torch.ones(1, dtype=torch.long),
                "target_tabular": m[384:512]}


def main():
    ut, it, tt, tr = mg._import_reference()
    from src import inference as inf
    inf.MultimodalDataset = _CatalogueDataset
    mg._stub_item_encoders(it)
    torch.manual_seed(3)
    model = tt.TwoTowerModel(vocab_size=V, tabular_input_dim=128, num_genders=3, num_countries=5,
                             max_seq_len=50, user_embedding_dim=D, item_embedding_dim=D,
                             user_num_heads=4, user_num_layers=2, user_dropout=0.1, use_lora=False)
    g = torch.Generator().manual_seed(4)
    with torch.no_grad():
        bn = model.item_tower.fusion_layer[1]
        bn.running_mean.copy_(torch.randn(512, generator=g) * 0.2)
        bn.running_var.copy_(0.5 + torch.rand(512, generator=g))
    model.eval()
    # catalogue: tracks t1..t{N_ITEMS} mapped to a permutation of the ids 1..V-1
    ids = (torch.randperm(V - 1, generator=g) + 1).tolist()
    mapper = {f"t{j + 1}": ids[j] for j in range(N_ITEMS)}
    modal = torch.randn(N_ITEMS + 1, 512, generator=g)
    _CatalogueDataset.modal = modal
    # one user's history (chronological order scrambled in the frame), longer than 50
    hist_tracks = [f"t{int(j) + 1}" for j in torch.randint(0, N_ITEMS, (L_HIST,), generator=g)]
    times = torch.randperm(L_HIST, generator=g).tolist()
    rows = [{"user_id": USER, "track_id": t, "timestamp": f"2021-01-01 00:{s // 60:02d}:{s % 60:02d}",
             "gender_idx": 2, "country_idx": 4} for t, s in zip(hist_tracks, times)]
    other = [{"user_id": "u9", "track_id": f"t{j + 1}", "timestamp": "2020-01-01 00:00:00",
              "gender_idx": 0, "country_idx": 1} for j in range(N_ITEMS)]
    df = pd.DataFrame(rows + other)
    df["artist_name"] = [f"A{mapper[t]}" for t in df["track_id"]]
    df["track_name"] = "T"
    df["album_name"] = "X"
    ref_dataset = types.SimpleNamespace(item_id_mapper=mapper, img_dir=None, text_data=None,
                                        tokenizer=None, encoders=None, interactions_df=df)
    with tempfile.TemporaryDirectory() as tmp:
        idx_path = os.path.join(tmp, "index", "items.pt")
        args = types.SimpleNamespace(batch_size=16, index_path=idx_path, user_id=USER)
        inf.index_catalog(args, model, ref_dataset, df, "cpu")
        dense = torch.load(idx_path, map_location="cpu", weights_only=True)
        out = io.StringIO()
        with contextlib.redirect_stdout(out):
            inf.recommend_for_user(args, model, ref_dataset, "cpu")
    text = out.getvalue()
    sect = text.split("Top 10 Recommendations:")[1]
    top = re.findall(r"^\s+\d+\. A(\d+) - T \(Score: ([-0-9.]+)\)", sect, re.M)
    assert len(top) == 10, text
    chron = df[df.user_id == USER].sort_values("timestamp")["track_id"].tolist()
    hist_ids = [mapper[t] for t in chron]
    arrays = {"modal": mg._np(modal[1:]), "catalogue_ids": np.array(ids, dtype=np.int64),
              "dense": mg._np(dense), "history": np.array(hist_ids, dtype=np.int64),
              "gender": np.array([2]), "country": np.array([4]),
              "top_ids": np.array([int(a) for a, _ in top], dtype=np.int64),
              "top_scores": np.array([float(b) for _, b in top], dtype=np.float32),
              "cfg": np.array([V, D, 50, 3, 5])}
    for k, v in model.state_dict().items():
        arrays["p/" + k] = mg._np(v)
    mg._save("serving.npz", **arrays)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ by RUNNING THE REFERENCE MODULES.

Runs only in the survey/build container, where /root/reference exists (the GPU box never
sees the reference).  The fixtures hold data only — inputs, the reference's own
parameter initialisation, and the reference's outputs/gradients — as .npz files.

Import recipe: ``import transformers`` first, then empty stand-ins for the
absent ``torchvision``, ``torchvision.models`` and ``peft`` modules, then
``src.models.*`` from /root/reference.  The multimodal item tower's modality encoders
(ResNet-18 x2, mDeBERTa) are replaced by identity stand-ins so that the reference's own
``MultimodalItemEncoder`` concat + fusion head runs on precomputed 128-d modality
embeddings — exactly BASELINE cfg 2.  ``src.data.dataset`` (missing from the snapshot) is
a stand-in too so ``src/train.py`` imports and its ``train_one_epoch`` runs unchanged.

Usage: python tools/make_golden.py   (writes tests/golden/*.npz)
"""
from __future__ import annotations

import os
import sys
import types
import warnings

import numpy as np
import torch
import torch.nn as nn

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")


def _import_reference():
    import transformers  # noqa: F401  (probes torchvision.__spec__ on import)
    tv = types.ModuleType("torchvision")
    tvm = types.ModuleType("torchvision.models")
    tv.models = tvm
    sys.modules.setdefault("torchvision", tv)
    sys.modules.setdefault("torchvision.models", tvm)
    peft = types.ModuleType("peft")

    class _TaskType:
        FEATURE_EXTRACTION = "FEATURE_EXTRACTION"
    peft.TaskType = _TaskType
    peft.LoraConfig = object
    peft.get_peft_model = lambda m, c: m
    sys.modules.setdefault("peft", peft)
    data_pkg = types.ModuleType("src.data")
    ds = types.ModuleType("src.data.dataset")
    ds.MultimodalDataset = object
    sys.modules.setdefault("src.data", data_pkg)
    sys.modules.setdefault("src.data.dataset", ds)
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import src.models.item_tower as it
    import src.models.two_tower as tt
    import src.models.user_tower as ut
    import src.train as tr
    global REAL_TABULAR
    REAL_TABULAR = it.TabularEncoder      # kept before _stub_item_encoders replaces it
    return ut, it, tt, tr


REAL_TABULAR = None


class _Identity(nn.Module):
    """Stand-in modality encoder: returns its (precomputed embedding) input."""

    def __init__(self, *a, **k):
        super().__init__()

    def forward(self, x, *rest):
        return x


def _np(t):
    return t.detach().cpu().numpy()


def _save(name, **arrays):
    os.makedirs(OUT, exist_ok=True)
    path = os.path.join(OUT, name)
    np.savez_compressed(path, **arrays)
    print("wrote", path, sum(a.nbytes for a in arrays.values()) // 1024, "KiB")


def user_tower_case(ut, name, V, D, L, B, H, n_g, n_c, lengths, left_pad=(), use_mask=True,
                    seed=0):
    torch.manual_seed(seed)
    m = ut.SequentialUserEncoder(V, n_g, n_c, D, L, H, 2, 0.0)
    m.train()
    g = torch.Generator().manual_seed(seed + 1)
    ids = torch.randint(1, V, (B, L), generator=g)
    mask = torch.zeros(B, L, dtype=torch.long)
    for b, n in enumerate(lengths):
        if b in left_pad:
            mask[b, L - n:] = 1
        else:
            mask[b, :n] = 1
    ids = ids * mask
    gender = torch.randint(0, n_g, (B,), generator=g)
    country = torch.randint(0, n_c, (B,), generator=g)
    out = m(ids, gender, country, mask if use_mask else None)
    G = torch.randn(out.shape, generator=g)
    (out * G).sum().backward()
    arrays = {"cfg": np.array([V, D, L, B, H, n_g, n_c, int(use_mask)], dtype=np.int64),
              "history_ids": _np(ids), "history_mask": _np(mask),
              "user_gender": _np(gender), "user_country": _np(country),
              "out": _np(out), "upstream": _np(G)}
    for k, v in m.state_dict().items():
        arrays["p/" + k] = _np(v)
    for k, v in m.named_parameters():
        arrays["g/" + k] = _np(v.grad)
    _save(name, **arrays)


def infonce_case(tt, name, B, D, n_users, seed):
    g = torch.Generator().manual_seed(seed)
    u = torch.randn(B, D, generator=g, requires_grad=True)
    i = torch.randn(B, D, generator=g, requires_grad=True)
    uid = torch.randint(0, n_users, (B,), generator=g)
    fake = types.SimpleNamespace(temperature=0.07, user_tower=lambda **k: u,
                                 item_tower=lambda **k: i)
    arrays = {"u": _np(u), "i": _np(i), "user_idx": _np(uid)}
    for tag, batch in (("nomask", {}), ("mask", {"user_idx": uid})):
        batch = dict(batch, history_ids=None, user_gender=None, user_country=None,
                     history_mask=None, target_image=None, target_audio=None,
                     target_input_ids=None, target_attention_mask=None, target_tabular=None)
        u.grad = None
        i.grad = None
        loss, logits, un, inn = tt.TwoTowerModel.forward(fake, batch)
        loss.backward()
        arrays.update({f"{tag}/loss": _np(loss), f"{tag}/logits": _np(logits),
                       f"{tag}/u_hat": _np(un), f"{tag}/i_hat": _np(inn),
                       f"{tag}/du": _np(u.grad), f"{tag}/di": _np(i.grad)})
    _save(name, **arrays)


def _stub_item_encoders(it):
    it.AudioEncoder = _Identity
    it.VisualEncoder = _Identity
    it.TextEncoder = _Identity
    it.TabularEncoder = _Identity


def _modal_batch(modal):
    return {"target_audio": modal[:, 0:128], "target_image": modal[:, 128:256],
            "target_input_ids": modal[:, 256:384], "target_attention_mask": None,
            "target_tabular": modal[:, 384:512]}


def item_fusion_case(it, name, B, D, seed):
    _stub_item_encoders(it)
    torch.manual_seed(seed)
    m = it.MultimodalItemEncoder(tabular_input_dim=128, embedding_dim=D)
    m.fusion_layer[3].p = 0.0       # parity run: dropout off (SURVEY §7 "Dropout RNG")
    m.train()
    g = torch.Generator().manual_seed(seed + 1)
    modal = torch.randn(B, 512, generator=g)
    mb = _modal_batch(modal)
    sd0 = {k: v.clone() for k, v in m.state_dict().items()}
    out = m(images=mb["target_image"], audio=mb["target_audio"],
            input_ids=mb["target_input_ids"], attention_mask=None, tabular=mb["target_tabular"])
    G = torch.randn(out.shape, generator=g)
    (out * G).sum().backward()
    arrays = {"modal": _np(modal), "out": _np(out), "upstream": _np(G)}
    for k, v in sd0.items():
        arrays["p/" + k] = _np(v)
    for k, v in m.state_dict().items():
        arrays["after/" + k] = _np(v)
    for k, v in m.named_parameters():
        arrays["g/" + k] = _np(v.grad)
    _save(name, **arrays)


def tabular_case(name, T, B, seed):
    """The reference's own TabularEncoder (item_tower.py:85-98: Linear -> BatchNorm1d -> ReLU ->
    Dropout -> Linear) in train mode with dropout off: output, parameter gradients under a
    random upstream, and the BatchNorm running statistics after the step."""
    torch.manual_seed(seed)
    m = REAL_TABULAR(input_dim=T, embedding_dim=128)
    m.mlp[3].p = 0.0
    m.train()
    g = torch.Generator().manual_seed(seed + 1)
    x = torch.randn(B, T, generator=g)
    sd0 = {k: v.clone() for k, v in m.state_dict().items()}
    out = m(x)
    G = torch.randn(out.shape, generator=g)
    (out * G).sum().backward()
    arrays = {"x": _np(x), "out": _np(out), "upstream": _np(G),
              "cfg": np.array([T, B], dtype=np.int64)}
    for k, v in sd0.items():
        arrays["p/" + k] = _np(v)
    for k, v in m.state_dict().items():
        arrays["after/" + k] = _np(v)
    for k, v in m.named_parameters():
        arrays["g/" + k] = _np(v.grad)
    _save(name, **arrays)


def train_step_case(it, tt, tr, name, V, D, L, B, n_g, n_c, n_steps, seed):
    _stub_item_encoders(it)
    torch.manual_seed(seed)
    model = tt.TwoTowerModel(vocab_size=V, tabular_input_dim=128, num_genders=n_g,
                             num_countries=n_c, max_seq_len=L, user_embedding_dim=D,
                             user_num_heads=4, user_num_layers=2, user_dropout=0.0,
                             item_embedding_dim=D, use_lora=False)
    model.item_tower.fusion_layer[3].p = 0.0
    sd0 = {k: v.clone() for k, v in model.state_dict().items()}
    g = torch.Generator().manual_seed(seed + 1)
    batches, arrays = [], {}
    for s in range(n_steps):
        lengths = torch.randint(1, L + 1, (B,), generator=g)
        mask = (torch.arange(L)[None] < lengths[:, None]).long()
        ids = torch.randint(1, V, (B, L), generator=g) * mask
        modal = torch.randn(B, 512, generator=g)
        b = {"history_ids": ids, "history_mask": mask,
             "user_gender": torch.randint(0, n_g, (B,), generator=g),
             "user_country": torch.randint(0, n_c, (B,), generator=g),
             "user_idx": torch.randint(0, 4, (B,), generator=g)}
        for k, v in b.items():
            arrays[f"batch{s}/{k}"] = _np(v)
        arrays[f"batch{s}/target_modal"] = _np(modal)
        b.update(_modal_batch(modal))
        b = {k: v for k, v in b.items() if v is not None}
        b["target_attention_mask"] = torch.ones(B, 1, dtype=torch.long)
        batches.append(b)
    losses = []
    orig_forward = model.forward

    def rec_forward(batch):
        out = orig_forward(batch)
        losses.append(float(out[0]))
        return out
    model.forward = rec_forward
    opt = torch.optim.AdamW(model.parameters(), lr=1e-4)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        mean_loss = tr.train_one_epoch(model, batches, opt, torch.device("cpu"), 1,
                                       is_main_process=False)
    arrays["cfg"] = np.array([V, D, L, B, n_g, n_c, n_steps], dtype=np.int64)
    arrays["losses"] = np.array(losses, dtype=np.float32)
    arrays["mean_loss"] = np.array(mean_loss, dtype=np.float32)
    for k, v in sd0.items():
        arrays["p0/" + k] = _np(v)
    for k, v in model.state_dict().items():
        arrays["p1/" + k] = _np(v)
    _save(name, **arrays)


def main():
    ut, it, tt, tr = _import_reference()
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        user_tower_case(ut, "user_tower_small.npz", V=101, D=32, L=8, B=6, H=4, n_g=3, n_c=5,
                        lengths=[8, 3, 1, 0, 8, 5], seed=0)
        user_tower_case(ut, "user_tower_nomask.npz", V=101, D=32, L=8, B=6, H=4, n_g=3,
                        n_c=5, lengths=[8, 3, 1, 0, 8, 5], use_mask=False, seed=10)
        user_tower_case(ut, "user_tower_leftpad.npz", V=101, D=32, L=8, B=4, H=4, n_g=2,
                        n_c=4, lengths=[8, 3, 5, 1], left_pad=(1, 2), seed=20)
        user_tower_case(ut, "user_tower_d128.npz", V=257, D=128, L=50, B=8, H=4, n_g=3,
                        n_c=64, lengths=[50, 17, 1, 33, 0, 49, 2, 25], seed=30)
        infonce_case(tt, "infonce_b8.npz", B=8, D=32, n_users=4, seed=40)
        infonce_case(tt, "infonce_b64.npz", B=64, D=128, n_users=24, seed=41)
        tabular_case("tabular_t128.npz", T=128, B=16, seed=70)
        tabular_case("tabular_t37.npz", T=37, B=16, seed=71)
        item_fusion_case(it, "item_fusion.npz", B=8, D=32, seed=50)
        train_step_case(it, tt, tr, "train_step.npz", V=101, D=32, L=8, B=8, n_g=3, n_c=5,
                        n_steps=2, seed=60)


if __name__ == "__main__":
    if sys.argv[1:] == ["tabular"]:     # only the TabularEncoder fixtures
        _import_reference()
        tabular_case("tabular_t128.npz", T=128, B=16, seed=70)
        tabular_case("tabular_t37.npz", T=37, B=16, seed=71)
    else:
        main()

"""Generate tests/golden/deberta_tiny.npz from transformers' own DebertaV2Model (the reference's
dependency, item_tower.py:47; pinned 4.57.3, 5.15.0 here) with a tiny mdeberta-like config.

Runs only in the build container (transformers is not needed on the GPU box).  The model gets
random weights; the peft LoRA deltas (scale alpha/r = 4) are merged into query_proj/value_proj,
which is exactly peft's forward with the LoRA dropout off.  Saved: inputs, the peft-named
parameters (base weights + lora_A/lora_B), last_hidden_state, the TextEncoder output
(mean-pool + projection), and gradients of sum(out * upstream) w.r.t. the merged query/value
weights and biases, key_proj weight and the rel_embeddings table."""
import math
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from transformers import DebertaV2Config, DebertaV2Model  # noqa: E402

H, NH, NL, I, V, R, ALPHA = 128, 2, 2, 256, 500, 8, 32
B, S, OUT = 3, 160, 32


def main():
    torch.manual_seed(0)
    cfg = DebertaV2Config(vocab_size=V, hidden_size=H, num_hidden_layers=NL, num_attention_heads=NH,
                          intermediate_size=I, hidden_act="gelu", hidden_dropout_prob=0.0,
                          attention_probs_dropout_prob=0.0, max_position_embeddings=512,
                          type_vocab_size=0, relative_attention=True, max_relative_positions=-1,
                          position_buckets=256, norm_rel_ebd="layer_norm", share_att_key=True,
                          pos_att_type=["p2c", "c2p"], layer_norm_eps=1e-7,
                          position_biased_input=False, pad_token_id=0, initializer_range=0.02)
    model = DebertaV2Model(cfg).float()
    model.train()
    g = torch.Generator().manual_seed(1)
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    # randomise LN affine params too, so the fixture exercises them
    for k in sd:
        if "LayerNorm" in k:
            sd[k] = (1.0 if k.endswith("weight") else 0.0) + 0.1 * torch.randn(sd[k].shape, generator=g)
        elif k.endswith(".bias"):
            sd[k] = 0.02 * torch.randn(sd[k].shape, generator=g)
    lora = {}
    for i in range(NL):
        for proj in ("query_proj", "value_proj"):
            base = f"encoder.layer.{i}.attention.self.{proj}"
            A = (torch.rand(R, H, generator=g) * 2 - 1) / math.sqrt(H)
            Bm = torch.randn(H, R, generator=g) * 0.05
            lora[base] = (A, Bm)
            sd[base + ".weight"] = sd[base + ".weight"] + (ALPHA / R) * Bm @ A
    model.load_state_dict(sd)
    lengths = torch.tensor([S, 150, 40])                 # full, long (log buckets), short
    mask = (torch.arange(S)[None] < lengths[:, None]).long()
    ids = torch.randint(1, V, (B, S), generator=g) * mask
    proj = {"projection.0.weight": torch.randn(512, H, generator=g) / math.sqrt(H),
            "projection.0.bias": 0.02 * torch.randn(512, generator=g),
            "projection.3.weight": torch.randn(OUT, 512, generator=g) / math.sqrt(512),
            "projection.3.bias": 0.02 * torch.randn(OUT, generator=g)}
    up = torch.randn(B, OUT, generator=g)
    hs = model(input_ids=ids, attention_mask=mask).last_hidden_state
    m = mask.unsqueeze(-1).expand(hs.size()).float()
    pooled = (hs * m).sum(1) / torch.clamp(m.sum(1), min=1e-9)
    out = F.linear(torch.relu(F.linear(pooled, proj["projection.0.weight"], proj["projection.0.bias"])),
                   proj["projection.3.weight"], proj["projection.3.bias"])
    (out * up).sum().backward()
    pd = dict(model.named_parameters())
    z = {"cfg": np.array([H, NH, NL, I, V, R, ALPHA, B, S, OUT]), "input_ids": ids.numpy(),
         "attention_mask": mask.numpy(), "upstream": up.numpy(),
         "last_hidden": hs.detach().numpy(), "out": out.detach().numpy()}
    pre = "transformer.base_model.model."
    for k, v in sd.items():
        if k.endswith("position_ids"):
            continue
        base = k.rsplit(".", 1)[0]
        if base in lora:
            A, Bm = lora[base]
            leaf = k.rsplit(".", 1)[1]
            w = v if leaf == "bias" else v - (ALPHA / R) * Bm @ A      # un-merged base weight
            z[f"p/{pre}{base}.base_layer.{leaf}"] = w.numpy()
            if leaf == "weight":
                z[f"p/{pre}{base}.lora_A.default.weight"] = A.numpy()
                z[f"p/{pre}{base}.lora_B.default.weight"] = Bm.numpy()
        else:
            z[f"p/{pre}{k}"] = v.numpy()
    for k, v in proj.items():
        z[f"p/{k}"] = v.numpy()
    for i in range(NL):
        for proj_name in ("query_proj", "value_proj", "key_proj"):
            base = f"encoder.layer.{i}.attention.self.{proj_name}"
            z[f"g/{base}.weight"] = pd[base + ".weight"].grad.numpy()   # merged-weight grad
            z[f"g/{base}.bias"] = pd[base + ".bias"].grad.numpy()
    z["g/encoder.rel_embeddings.weight"] = pd["encoder.rel_embeddings.weight"].grad.numpy()
    out_path = os.path.join(ROOT, "tests", "golden", "deberta_tiny.npz")
    np.savez_compressed(out_path, **z)
    print("wrote", out_path, "out", out.shape, "keys", len(z))


if __name__ == "__main__":
    main()

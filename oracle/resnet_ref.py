"""ORACLE — test infrastructure only (never imported by the product path).

CPU fp32 restatement of the cfg-3 item encoders of reference src/models/item_tower.py:
* AudioEncoder (item_tower.py:9-25) and VisualEncoder (:27-39): torchvision resnet18 with
  conv1 replaced by Conv2d(in_ch, 64, 7, 2, 3, bias=False) for audio, fc replaced by
  Linear(512, embedding_dim).  BatchNorm2d runs in train mode on batch statistics.
* TabularEncoder (:85-98): Linear(T, 256) → BatchNorm1d → ReLU → Dropout → Linear(256, 128).
* MultimodalItemEncoder.forward (:131-152) for cfg 3 (zero text slot).

torchvision (pinned 0.24.1 in the reference's uv.lock) is not installed here, so the
ResNet-18 topology is restated from its published definition (BasicBlock [2, 2, 2, 2];
conv1 7x7/2 pad 3 → BN → ReLU → maxpool 3/2 pad 1; a 1x1/2 conv + BN downsample on the first
block of layers 2-4; adaptive average pool; fc) with torchvision's parameter names and
initialisation (kaiming_normal_ fan_out/relu convs, BN weight 1 / bias 0, default Linear).
The reference has no tests for these modules, so parity against the reference is unpinned
(SURVEY §8c); the restatement is pinned to torch's own F.conv2d / F.batch_norm /
F.max_pool2d semantics.
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch
import torch.nn.functional as F

from oracle import two_tower_ref as ttr

Tensor = torch.Tensor

# (layer name, in channels, out channels, stride of its first block)
LAYERS = (("layer1", 64, 64, 1), ("layer2", 64, 128, 2), ("layer3", 128, 256, 2),
          ("layer4", 256, 512, 2))


def conv_names(prefix: str = ""):
    """(name, Cin, Cout, kernel, stride, pad) of every conv in torchvision resnet18 order."""
    out = []
    for lname, cin, cout, s in LAYERS:
        for bi in range(2):
            ci = cin if bi == 0 else cout
            st = s if bi == 0 else 1
            base = f"{prefix}{lname}.{bi}."
            out.append((base + "conv1.weight", ci, cout, 3, st, 1))
            out.append((base + "conv2.weight", cout, cout, 3, 1, 1))
            if bi == 0 and (st != 1 or ci != cout):
                out.append((base + "downsample.0.weight", ci, cout, 1, st, 0))
    return out


def init_resnet18(in_ch: int, out_dim: int, generator: torch.Generator,
                  prefix: str = "") -> Dict[str, Tensor]:
    p: Dict[str, Tensor] = {}

    def conv(name, cin, cout, k):
        std = math.sqrt(2.0 / (cout * k * k))              # kaiming_normal_(fan_out, relu)
        p[prefix + name] = torch.randn(cout, cin, k, k, generator=generator) * std

    def bn(name, c):
        p[prefix + name + ".weight"] = torch.ones(c)
        p[prefix + name + ".bias"] = torch.zeros(c)
        p[prefix + name + ".running_mean"] = torch.zeros(c)
        p[prefix + name + ".running_var"] = torch.ones(c)

    conv("conv1.weight", in_ch, 64, 7)
    bn("bn1", 64)
    for name, cin, cout, k, _, _ in conv_names():
        conv(name, cin, cout, k)
        bn(name.replace("conv", "bn").replace("downsample.0.weight", "downsample.1")
           .replace(".weight", ""), cout)
    bound = 1.0 / math.sqrt(512)
    p[prefix + "fc.weight"] = (torch.rand(out_dim, 512, generator=generator) * 2 - 1) * bound
    p[prefix + "fc.bias"] = (torch.rand(out_dim, generator=generator) * 2 - 1) * bound
    return p


def _bn(x: Tensor, p: Dict[str, Tensor], name: str, update) -> Tensor:
    """Train-mode BatchNorm (batch statistics; running buffers updated when ``update``), or
    eval mode (``update == "eval"``: the running statistics)."""
    rm, rv = p.get(name + ".running_mean"), p.get(name + ".running_var")
    if update == "eval":
        return F.batch_norm(x, rm, rv, p[name + ".weight"], p[name + ".bias"], training=False,
                            eps=1e-5)
    if not update:
        rm = rv = None
    return F.batch_norm(x, rm, rv, p[name + ".weight"], p[name + ".bias"], training=True,
                        momentum=0.1, eps=1e-5)


def resnet18_forward(p: Dict[str, Tensor], x: Tensor, prefix: str = "",
                     update_running: bool = False) -> Tensor:
    """torchvision resnet18.forward (train-mode BN) with the replaced conv1/fc."""
    y = F.conv2d(x, p[prefix + "conv1.weight"], stride=2, padding=3)
    y = F.relu(_bn(y, p, prefix + "bn1", update_running))
    y = F.max_pool2d(y, 3, 2, 1)
    for lname, cin, cout, s in LAYERS:
        for bi in range(2):
            base = f"{prefix}{lname}.{bi}."
            st = s if bi == 0 else 1
            idn = y
            h = F.conv2d(y, p[base + "conv1.weight"], stride=st, padding=1)
            h = F.relu(_bn(h, p, base + "bn1", update_running))
            h = F.conv2d(h, p[base + "conv2.weight"], stride=1, padding=1)
            h = _bn(h, p, base + "bn2", update_running)
            if base + "downsample.0.weight" in p:
                idn = F.conv2d(y, p[base + "downsample.0.weight"], stride=st)
                idn = _bn(idn, p, base + "downsample.1", update_running)
            y = F.relu(h + idn)
    y = F.adaptive_avg_pool2d(y, 1).flatten(1)
    return F.linear(y, p[prefix + "fc.weight"], p[prefix + "fc.bias"])


def tabular_forward(p: Dict[str, Tensor], x: Tensor, prefix: str = "mlp.", p_drop: float = 0.0,
                    drop=None, update_running: bool = False) -> Tensor:
    """TabularEncoder (item_tower.py:85-98) in train mode; dropout at site SITE_TAB."""
    z = F.linear(x, p[prefix + "0.weight"], p[prefix + "0.bias"])
    z = _bn(z, p, prefix + "1", update_running)
    z = F.relu(z)
    if p_drop > 0 and drop is not None:
        z = drop(ttr.SITE_TAB, z, p_drop)
    return F.linear(z, p[prefix + "4.weight"], p[prefix + "4.bias"])


def item_tower_raw_forward(p: Dict[str, Tensor], batch: Dict[str, Tensor], p_drop: float = 0.0,
                           drop=None, running: Optional[Dict[str, Tensor]] = None,
                           text_dim: int = 128, update_running: bool = False,
                           text_cfg=None, eval_mode: bool = False) -> Tensor:
    """MultimodalItemEncoder.forward (item_tower.py:131-152) for cfg 3: audio ResNet-18 on
    ``target_audio``, visual ResNet-18 on ``target_image``, a zero text slot (or, with
    ``text_cfg``, the cfg-4 mDeBERTa-LoRA TextEncoder of deberta_ref), the tabular MLP on ``target_tabular``; concatenated in the reference's
    fixed order (:147) into the fusion head.  ``p`` holds item-tower names without the
    ``item_tower.`` prefix.  eval_mode: every BatchNorm on its running statistics (``p`` holds
    them, ``running`` the fusion head's), dropout off — the indexers' model.eval()."""
    if eval_mode:
        update_running, p_drop = "eval", 0.0
    audio = resnet18_forward(p, batch["target_audio"], "audio_encoder.backbone.", update_running)
    visual = resnet18_forward(p, batch["target_image"], "visual_encoder.backbone.",
                              update_running)
    if text_cfg is not None:        # cfg 4: the mDeBERTa-LoRA branch (deberta_ref, dropout off)
        from oracle import deberta_ref
        text = deberta_ref.text_encoder_forward(
            p, batch["target_input_ids"], batch["target_attention_mask"], text_cfg,
            prefix="text_encoder.transformer.base_model.model.", proj_prefix="text_encoder.projection.")
    else:
        text = torch.zeros(audio.shape[0], text_dim)
    tab = tabular_forward(p, batch["target_tabular"], "tabular_encoder.mlp.", p_drop, drop,
                          update_running)
    modal = torch.cat([audio, visual, text, tab], dim=1)
    return ttr.item_fusion_forward(p, modal, p_drop, drop, running, eval_mode=eval_mode)


def synthetic_items(B: int, tabular_dim: int, mel=(128, 256), cover=(224, 224),
                    generator: Optional[torch.Generator] = None) -> Dict[str, Tensor]:
    """cfg-3 item inputs (BASELINE configs[2]): N(0,1) mel-spectrograms [B,1,128,256],
    ImageNet-normalised-like covers N(0,1) [B,3,224,224], tabular features N(0,1) [B,T]."""
    g = generator
    return {"target_audio": torch.randn(B, 1, *mel, generator=g),
            "target_image": torch.randn(B, 3, *cover, generator=g),
            "target_tabular": torch.randn(B, tabular_dim, generator=g)}

"""MultimodalItemEncoder — drop-in for reference src/models/item_tower.py:100-152.

The late-fusion head (item_tower.py:122-129: Linear(512,512) -> BatchNorm1d -> ReLU ->
Dropout(0.1) -> Linear(512,D) -> LayerNorm(D)) runs on libttmi kernels with the reference's
parameter/buffer names (``fusion_layer.{0,1,4,5}.*``, BatchNorm running stats included).

BASELINE cfg 2 feeds the head *precomputed* 128-d modality embeddings; this module accepts
them either concatenated (``fuse(modal[B, 512])``, order audio|visual|text|tabular as in
item_tower.py:147) or through the reference ``forward(images, audio, input_ids,
attention_mask, tabular)`` signature with each argument already a [B, 128] embedding.
The raw-input encoders (ResNet-18 on mels/covers, mDeBERTa+LoRA) are the next rows of the
build plan and are not constructed here yet.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn

from . import functional as F
from .user_tower import make_operands, new_dropout_seeds

Tensor = torch.Tensor
ITEM_GEMMS = ("fusion_layer.0.weight", "fusion_layer.4.weight")
_BUF = ("fusion_layer.1.running_mean", "fusion_layer.1.running_var",
        "fusion_layer.1.num_batches_tracked")


class _ItemFusionFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cfg, names, seeds, p_drop, bufs, modal, *params):
        P = dict(zip(names, params))
        W = make_operands(P, cfg.dtype, ITEM_GEMMS)
        out, st = F.item_fusion_fwd(P, W, modal, cfg, seeds, bufs, p_drop)
        ctx.saved = (cfg, names, P, W, st, p_drop, modal.requires_grad)
        return out

    @staticmethod
    def backward(ctx, dout):
        cfg, names, P, W, st, p_drop, need_dmodal = ctx.saved
        del ctx.saved
        grads = {n: torch.zeros_like(P[n]) for n in names}
        dmodal = None
        if need_dmodal:
            dmodal = torch.empty(st.modal.shape, device=dout.device, dtype=torch.float32)
        F.item_fusion_bwd(P, W, st, dout.contiguous().float(), grads, cfg, p_drop, dmodal)
        return (None,) * 5 + (dmodal,) + tuple(grads[n] for n in names)


class MultimodalItemEncoder(nn.Module):
    def __init__(self, tabular_input_dim: int, embedding_dim: int = 256, audio_dim: int = 128,
                 visual_dim: int = 128, text_model_name: str = "microsoft/mdeberta-v3-base",
                 text_dim: int = 128, tabular_dim: int = 128, use_lora: bool = True, *,
                 precomputed_modalities: bool = True,
                 compute_dtype: torch.dtype = torch.bfloat16):
        super().__init__()
        if not precomputed_modalities:
            raise NotImplementedError(
                "raw-input modality encoders (ResNet-18 audio/visual, mDeBERTa+LoRA text, tabular "
                "MLP) are not built yet (SURVEY §7 steps 6-7); pass precomputed modality "
                "embeddings (BASELINE cfg 2)")
        self.embedding_dim = embedding_dim
        self.modal_dims = (audio_dim, visual_dim, text_dim, tabular_dim)
        self.compute_dtype = compute_dtype
        self.tabular_input_dim = tabular_input_dim
        fusion_input_dim = sum(self.modal_dims)
        self.fusion_layer = nn.Sequential(
            nn.Linear(fusion_input_dim, 512),
            nn.BatchNorm1d(512),
            nn.ReLU(),
            nn.Dropout(0.1),
            nn.Linear(512, embedding_dim),
            nn.LayerNorm(embedding_dim),
        )

    def cfg(self) -> F.TowerCfg:
        return F.TowerCfg(D=self.embedding_dim, dtype=self.compute_dtype)

    def fuse(self, modal: Tensor, seeds: Optional[Tensor] = None) -> Tensor:
        """Fusion head on concatenated modality embeddings [B, sum(modal_dims)]."""
        cfg = self.cfg()
        p_drop = self.fusion_layer[3].p if self.training else 0.0
        if p_drop > 0 and seeds is None:
            seeds = new_dropout_seeds(modal.device)
        names, params = zip(*self.named_parameters())
        bufs = dict(self.named_buffers())
        modal = modal.contiguous().float()
        if not self.training:
            P = dict(zip(names, [p.detach() for p in params]))
            W = make_operands(P, cfg.dtype, ITEM_GEMMS)
            out, _ = F.item_fusion_fwd(P, W, modal, cfg, None, bufs, 0.0, training=False)
            return out
        if torch.is_grad_enabled() and (any(p.requires_grad for p in params) or modal.requires_grad):
            return _ItemFusionFn.apply(cfg, list(names), seeds, p_drop, bufs, modal, *params)
        P = dict(zip(names, [p.detach() for p in params]))
        W = make_operands(P, cfg.dtype, ITEM_GEMMS)
        out, _ = F.item_fusion_fwd(P, W, modal, cfg, seeds, bufs, p_drop)
        return out

    def forward(self, images: Tensor, audio: Tensor, input_ids: Tensor,
                attention_mask: Optional[Tensor], tabular: Tensor) -> Tensor:
        """Reference signature (item_tower.py:131-152) with precomputed [B, 128] embeddings."""
        return self.fuse(torch.cat([audio, images, input_ids, tabular], dim=1))

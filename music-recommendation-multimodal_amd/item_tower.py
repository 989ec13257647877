"""MultimodalItemEncoder — drop-in for reference src/models/item_tower.py:100-152.

The late-fusion head (item_tower.py:122-129: Linear(512,512) -> BatchNorm1d -> ReLU ->
Dropout(0.1) -> Linear(512,D) -> LayerNorm(D)) runs on libttmi kernels with the reference's
parameter/buffer names (``fusion_layer.{0,1,4,5}.*``, BatchNorm running stats included).

Two input modes:
* ``precomputed_modalities=True`` (BASELINE cfg 2): the head takes precomputed 128-d modality
  embeddings, either concatenated (``fuse(modal[B, 512])``, order audio|visual|text|tabular as
  in item_tower.py:147) or through ``forward(images, audio, input_ids, attention_mask,
  tabular)`` with each argument already a [B, 128] embedding.
* ``precomputed_modalities=False`` (cfg 3): the raw-input encoders are built with the
  reference's names — ``audio_encoder`` (ResNet-18 on [B,1,H,W] mels, item_tower.py:9-25),
  ``visual_encoder`` (ResNet-18 on [B,3,224,224] covers, :27-39; random init, ImageNet
  weights are a download), ``tabular_encoder`` (:85-98) — all on the libttmi conv/BN/pool
  kernels (cnn.py).  With ``with_text=True`` (cfg 4) it also builds ``text_encoder``, the
  mDeBERTa-v3 + LoRA lyrics encoder (:41-83, text.py) fed ``input_ids``/``attention_mask``;
  without it (cfg 3, no text branch) the text slot is a zero 128-d vector, or ``input_ids``
  itself when it is a floating-point [B, text_dim] precomputed text embedding.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn

from . import cnn
from . import functional as F
from .text import TextCfg, TextEncoder
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
                 precomputed_modalities: bool = False, with_text: bool = True,
                 text_cfg: Optional[TextCfg] = None,
                 compute_dtype: torch.dtype = torch.bfloat16):
        super().__init__()
        self.precomputed_modalities = precomputed_modalities
        self.with_text = with_text and not precomputed_modalities
        if not precomputed_modalities:
            self.audio_encoder = cnn.AudioEncoder(embedding_dim=audio_dim)
            self.visual_encoder = cnn.VisualEncoder(embedding_dim=visual_dim)
            if self.with_text:                                  # cfg 4
                self.text_encoder = TextEncoder(model_name=text_model_name,
                                                embedding_dim=text_dim, use_lora=use_lora,
                                                cfg=text_cfg)
            self.tabular_encoder = cnn.TabularEncoder(input_dim=tabular_input_dim,
                                                      embedding_dim=tabular_dim)
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
        names, params = zip(*self.fusion_layer.named_parameters(prefix="fusion_layer"))
        bufs = dict(self.fusion_layer.named_buffers(prefix="fusion_layer"))
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

    def text_slot(self, input_ids: Optional[Tensor], B: int, device) -> Tensor:
        """cfg 3 text slot: a precomputed float [B, text_dim] embedding, else zeros."""
        td = self.modal_dims[2]
        if input_ids is not None and input_ids.is_floating_point() \
                and tuple(input_ids.shape) == (B, td):
            return input_ids.float()
        return torch.zeros(B, td, device=device)

    def forward(self, images: Tensor, audio: Tensor, input_ids: Optional[Tensor],
                attention_mask: Optional[Tensor], tabular: Tensor,
                seeds: Optional[Tensor] = None) -> Tensor:
        """Reference signature (item_tower.py:131-152).  Precomputed mode: every argument is a
        [B, 128] embedding.  Raw mode: audio [B,1,H,W], images [B,3,H,W], tabular [B,T]."""
        if self.precomputed_modalities:
            return self.fuse(torch.cat([audio, images, input_ids, tabular], dim=1), seeds)
        if self.training and seeds is None:
            seeds = new_dropout_seeds(audio.device)
        audio_emb = self.audio_encoder(audio)
        visual_emb = self.visual_encoder(images)
        if self.with_text:
            text_emb = self.text_encoder(input_ids, attention_mask)
        else:
            text_emb = self.text_slot(input_ids, audio.shape[0], audio.device)
        tabular_emb = self.tabular_encoder(tabular, seeds)
        combined = torch.cat([audio_emb, visual_emb, text_emb, tabular_emb], dim=1)
        return self.fuse(combined, seeds)

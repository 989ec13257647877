"""TwoTowerModel — drop-in for reference src/models/two_tower.py:8-168.

``forward(batch)`` returns ``(loss, logits, user_emb, item_emb)`` exactly like the
reference: symmetric in-batch InfoNCE over L2-normalised embeddings with τ = 0.07 and the
same-user collision mask (-1e4) when ``batch['user_idx']`` is present.  The loss, logits
and normalisation run in fp32 on libttmi kernels (``ttmi_infonce_fwd/bwd``).

Item inputs: cfg 2 — ``batch['target_modal']`` [B, 512] precomputed modality embeddings
(audio|visual|text|tabular), or the reference's item keys each carrying a precomputed [B, 128]
embedding; cfg 3 (``precomputed_modalities=False``) — the reference's raw item keys
``target_audio`` [B,1,128,256], ``target_image`` [B,3,224,224], ``target_tabular`` [B,T]
(two_tower.py:90-96).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch
import torch.nn as nn
import torch.nn.functional as TF

from . import functional as F
from .item_tower import MultimodalItemEncoder
from .user_tower import SequentialUserEncoder

Tensor = torch.Tensor


class _InfoNCEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, temperature, user_idx, u, it):
        loss, logits, u_hat, i_hat, st = F.infonce_fwd(u, it, user_idx, temperature)
        ctx.st = st
        ctx.mark_non_differentiable(logits, u_hat, i_hat)
        return loss, logits, u_hat, i_hat

    @staticmethod
    def backward(ctx, dloss, _dlogits, _du_hat, _di_hat):
        st = ctx.st
        del ctx.st
        du = torch.empty_like(st.u_hat)
        di = torch.empty_like(st.i_hat)
        F.infonce_bwd(st, dloss.reshape(1).float().contiguous(), du, di)
        return None, None, du, di


def infonce(user_emb: Tensor, item_emb: Tensor, user_idx: Optional[Tensor],
            temperature: float = 0.07):
    """Symmetric InfoNCE of two_tower.py:98-140 on libttmi kernels."""
    u = user_emb.float().contiguous()
    i = item_emb.float().contiguous()
    if torch.is_grad_enabled() and (u.requires_grad or i.requires_grad):
        return _InfoNCEFn.apply(temperature, user_idx, u, i)
    loss, logits, uh, ih, _ = F.infonce_fwd(u, i, user_idx, temperature)
    return loss, logits, uh, ih


class _GlobalInfoNCEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, temperature, user_idx, group, u, it):
        loss, logits, u_hat, i_hat, st = F.infonce_global_fwd(u, it, user_idx, temperature, group)
        ctx.st, ctx.group = st, group
        ctx.mark_non_differentiable(logits, u_hat, i_hat)
        return loss, logits, u_hat, i_hat

    @staticmethod
    def backward(ctx, dloss, _dlogits, _du_hat, _di_hat):
        st, group = ctx.st, ctx.group
        del ctx.st
        du = torch.empty_like(st.u_hat)
        di = torch.empty_like(st.i_hat)
        F.infonce_global_bwd(st, dloss.reshape(1).float().contiguous(), du, di, group)
        return None, None, None, du, di


def infonce_global(user_emb: Tensor, item_emb: Tensor, user_idx: Optional[Tensor],
                   temperature: float = 0.07, group=None):
    """Global in-batch negatives (BASELINE cfg 5): this rank's share of the reference InfoNCE
    over every rank's batch (RCCL all-gather of û, î, user_idx; reduce-scatter of the key
    grads).  logits are this rank's u2i rows [B, world·B].  Averaging the per-rank losses (or
    DDP's gradient average) gives the loss of the concatenated batch."""
    u = user_emb.float().contiguous()
    i = item_emb.float().contiguous()
    if torch.is_grad_enabled() and (u.requires_grad or i.requires_grad):
        return _GlobalInfoNCEFn.apply(temperature, user_idx, group, u, i)
    loss, logits, uh, ih, _ = F.infonce_global_fwd(u, i, user_idx, temperature, group)
    return loss, logits, uh, ih


class TwoTowerModel(nn.Module):
    def __init__(self, vocab_size: int, tabular_input_dim: int, num_genders: int = 1,
                 num_countries: int = 1, max_seq_len: int = 50, user_embedding_dim: int = 256,
                 user_num_heads: int = 4, user_num_layers: int = 2, user_dropout: float = 0.1,
                 item_embedding_dim: int = 256, audio_dim: int = 128, visual_dim: int = 128,
                 text_model_name: str = "microsoft/mdeberta-v3-base", text_dim: int = 128,
                 tabular_dim: int = 128, use_lora: bool = True, temperature: float = 0.07, *,
                 compute_dtype: torch.dtype = torch.bfloat16,
                 precomputed_modalities: bool = False, with_text: bool = True,
                 text_cfg=None, global_negatives: bool = False, process_group=None):
        super().__init__()
        self.global_negatives = global_negatives   # cfg 5: negatives from every rank's batch
        self.process_group = process_group
        assert user_embedding_dim == item_embedding_dim, \
            f"User dim ({user_embedding_dim}) must match Item dim ({item_embedding_dim})"
        self.temperature = temperature
        self.user_tower = SequentialUserEncoder(
            vocab_size=vocab_size, num_genders=num_genders, num_countries=num_countries,
            embedding_dim=user_embedding_dim, max_seq_len=max_seq_len, num_heads=user_num_heads,
            num_layers=user_num_layers, dropout=user_dropout, compute_dtype=compute_dtype)
        self.item_tower = MultimodalItemEncoder(
            tabular_input_dim=tabular_input_dim, embedding_dim=item_embedding_dim,
            audio_dim=audio_dim, visual_dim=visual_dim, text_model_name=text_model_name,
            text_dim=text_dim, tabular_dim=tabular_dim, use_lora=use_lora,
            precomputed_modalities=precomputed_modalities, with_text=with_text,
            text_cfg=text_cfg, compute_dtype=compute_dtype)

    def _item(self, batch: Dict[str, Tensor], seeds: Optional[Tensor] = None) -> Tensor:
        if "target_modal" in batch:
            return self.item_tower.fuse(batch["target_modal"], seeds)
        if not self.item_tower.precomputed_modalities:        # cfg 3: raw mels/covers/tabular
            return self.item_tower(images=batch["target_image"], audio=batch["target_audio"],
                                   input_ids=batch.get("target_input_ids"),
                                   attention_mask=batch.get("target_attention_mask"),
                                   tabular=batch["target_tabular"], seeds=seeds)
        modal = torch.cat([batch["target_audio"], batch["target_image"],
                           batch["target_input_ids"], batch["target_tabular"]], dim=1)
        return self.item_tower.fuse(modal, seeds)

    def forward(self, batch: Dict[str, Tensor], seeds: Optional[Tensor] = None):
        user_emb = self.user_tower(history_ids=batch["history_ids"],
                                   user_gender=batch["user_gender"],
                                   user_country=batch["user_country"],
                                   history_mask=batch.get("history_mask"), seeds=seeds)
        item_emb = self._item(batch, seeds)
        if self.global_negatives:
            return infonce_global(user_emb, item_emb, batch.get("user_idx"), self.temperature,
                                  self.process_group)
        return infonce(user_emb, item_emb, batch.get("user_idx"), self.temperature)

    def get_user_embedding(self, history_ids, history_mask=None, user_gender=None,
                           user_country=None):
        if user_gender is None:
            user_gender = torch.zeros_like(history_ids[:, 0])
        if user_country is None:
            user_country = torch.zeros_like(history_ids[:, 0])
        emb = self.user_tower(history_ids=history_ids, history_mask=history_mask,
                              user_gender=user_gender, user_country=user_country)
        return TF.normalize(emb, p=2, dim=1)

    def get_item_embedding(self, images, audio, input_ids, attention_mask, tabular):
        emb = self.item_tower(images=images, audio=audio, input_ids=input_ids,
                              attention_mask=attention_mask, tabular=tabular)
        return TF.normalize(emb, p=2, dim=1)

"""SequentialUserEncoder — drop-in for reference src/models/user_tower.py:4-144.

Same constructor arguments, same ``forward(history_ids, user_gender, user_country,
history_mask=None)`` contract and the same ``state_dict`` keys (nn.TransformerEncoder layout:
``transformer_encoder.layers.{i}.self_attn.in_proj_weight`` ...), so reference checkpoints
load unchanged.  The parameters are plain fp32 ``nn.Parameter``s held in container modules;
the computation is the libttmi kernel schedule of ``functional.user_tower_fwd/bwd``.

Semantics kept from the reference: ``padding_idx=0`` rows get no gradient but
are looked up and initialised non-zero; key padding from ``history_mask`` (or
``history_ids != 0`` when the mask is None); causal attention; a query row whose keys are all
masked yields 0 (torch's train-mode SDPA; the reference's eval fast path gives NaN there,
this module gives 0 in both modes); the last-valid gather assumes right padding exactly as
the reference does.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.nn as nn

from . import functional as F
from . import ops
from .ops import ATTN_LMAX

Tensor = torch.Tensor

GEMM_WEIGHTS = ("self_attn.in_proj_weight", "self_attn.out_proj.weight", "linear1.weight",
                "linear2.weight")


class _SelfAttentionParams(nn.Module):
    """Parameter container with nn.MultiheadAttention's names (packed in_proj)."""

    def __init__(self, d_model: int):
        super().__init__()
        self.in_proj_weight = nn.Parameter(torch.empty(3 * d_model, d_model))
        self.in_proj_bias = nn.Parameter(torch.empty(3 * d_model))
        self.out_proj = nn.Linear(d_model, d_model)


class _EncoderLayerParams(nn.Module):
    """Parameter container with nn.TransformerEncoderLayer's names."""

    def __init__(self, d_model: int, dim_ff: int):
        super().__init__()
        self.self_attn = _SelfAttentionParams(d_model)
        self.linear1 = nn.Linear(d_model, dim_ff)
        self.linear2 = nn.Linear(dim_ff, d_model)
        self.norm1 = nn.LayerNorm(d_model)
        self.norm2 = nn.LayerNorm(d_model)


class _EncoderParams(nn.Module):
    def __init__(self, d_model: int, dim_ff: int, num_layers: int):
        super().__init__()
        self.layers = nn.ModuleList([_EncoderLayerParams(d_model, dim_ff) for _ in range(num_layers)])


def make_operands(P: dict, dtype: torch.dtype, gemm_names) -> dict:
    """GEMM operand view of the fp32 masters: bf16 copies (libttmi cast kernel) plus the
    transposed mirrors of the encoder weights, or P itself in fp32."""
    if dtype == torch.float32:
        return P
    W = dict(P)
    for n in gemm_names:
        src = P[n].contiguous()
        W[n] = ops.cast_bf16(src, torch.empty(src.shape, device=src.device, dtype=dtype))
    add_transposes(W, gemm_names)
    refresh_transposes(W, gemm_names)
    return W


def cfg_dtype_bf16(dtype: torch.dtype) -> bool:
    return dtype == torch.bfloat16


def encoder_weight_names(names) -> List[str]:
    """Weights with a transposed mirror: every encoder-layer GEMM weight and the fusion MLP's
    two (the fused head backward, ttmi_user_head_bwd, reads all of them k-major)."""
    return [n for n in names if n.endswith(GEMM_WEIGHTS) or n.endswith(("fusion_layer.0.weight",
                                                                        "fusion_layer.3.weight"))]


def add_transposes(W: dict, gemm_names) -> None:
    """Allocate W[name + '.T'] ([in, out] bf16) for every weight encoder_weight_names lists."""
    for n in encoder_weight_names(gemm_names):
        w = W[n]
        W[F.transposed_name(n)] = torch.empty(w.shape[1], w.shape[0], device=w.device,
                                              dtype=w.dtype)


def refresh_transposes(W: dict, gemm_names, seeds=None) -> None:
    """W[name + '.T'] = W[name]ᵀ for all encoder-layer weights in one launch (plus the step's
    dropout seeds when ``seeds`` = (base, step, table, inc_step) is given)."""
    names = [n for n in encoder_weight_names(gemm_names) if F.transposed_name(n) in W]
    ops.transpose_batch([W[F.transposed_name(n)] for n in names], [W[n] for n in names], seeds)


def _gemm_names(names: List[str]):
    return [n for n in names if n.endswith(GEMM_WEIGHTS) or n in ("fusion_layer.0.weight",
                                                                   "fusion_layer.3.weight")]


class _UserTowerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cfg, names, seeds, ids, gender, country, mask, *params):
        P = dict(zip(names, params))
        W = make_operands(P, cfg.dtype, _gemm_names(names))
        u, st = F.user_tower_fwd(P, W, ids, gender, country, mask, cfg, seeds)
        ctx.saved = (cfg, names, P, W, st)
        return u

    @staticmethod
    def backward(ctx, du):
        cfg, names, P, W, st = ctx.saved
        del ctx.saved
        grads = {n: torch.zeros_like(P[n]) for n in names}
        F.user_tower_bwd(P, W, st, du.contiguous().float(), grads, cfg)
        return (None,) * 7 + tuple(grads[n] for n in names)


def new_dropout_seeds(device) -> Tensor:
    """Fresh per-call seed table for eager (non-graph) training forwards."""
    base = int(torch.randint(0, 2 ** 62, (), dtype=torch.int64).item())   # torch CPU generator
    return F.seed_table(F.site_seeds(base, 0), device)


class SequentialUserEncoder(nn.Module):
    def __init__(self, vocab_size: int, num_genders: int = 1, num_countries: int = 1,
                 embedding_dim: int = 256, max_seq_len: int = 50, num_heads: int = 4,
                 num_layers: int = 2, dropout: float = 0.1, *,
                 compute_dtype: torch.dtype = torch.bfloat16, prune_last: bool = True):
        super().__init__()
        if embedding_dim % num_heads:
            raise ValueError("embedding_dim must be divisible by num_heads")
        # the tuned attention kernels (ttmi_attn.hip) keep a whole sequence's K/V head slice in
        # one workgroup's LDS up to 64 positions and tile longer ones over 64-key blocks
        # (ttmi_attn_long.hip) up to TTMI_ATTN_LMAX, for head widths that are multiples of 8 up
        # to 64.  Other shapes (the reference accepts any) run the generic attention kernels
        # (ttmi_attn_generic.hip, ABI 22) on an unpruned last layer: correct, not fast.
        d_h = embedding_dim // num_heads
        if max_seq_len <= 0:
            raise ValueError(f"max_seq_len must be positive (got {max_seq_len})")
        if d_h > 512:
            raise ValueError(f"head width embedding_dim / num_heads must be <= 512 (got {d_h})")
        if not (max_seq_len <= ATTN_LMAX and d_h <= 64 and d_h % 8 == 0):
            prune_last = False          # the one-query kernels serve the tuned shapes only
        self.embedding_dim = embedding_dim
        self.max_seq_len = max_seq_len
        self.num_heads = num_heads
        self.num_layers = num_layers
        self.compute_dtype = compute_dtype
        self.prune_last = prune_last
        self.item_embedding = nn.Embedding(vocab_size, embedding_dim, padding_idx=0)
        self.gender_embedding = nn.Embedding(num_genders, 16)
        self.country_embedding = nn.Embedding(num_countries, 32)
        self.position_embedding = nn.Embedding(max_seq_len, embedding_dim)
        self.transformer_encoder = _EncoderParams(embedding_dim, 4 * embedding_dim, num_layers)
        self.layer_norm = nn.LayerNorm(embedding_dim)
        self.dropout = nn.Dropout(dropout)
        self.fusion_layer = nn.Sequential(
            nn.Linear(embedding_dim + 16 + 32, embedding_dim),
            nn.LayerNorm(embedding_dim),
            nn.ReLU(),
            nn.Linear(embedding_dim, embedding_dim),
        )
        self.reset_parameters()

    def reset_parameters(self) -> None:
        """Reference init (user_tower.py:62-71 over nn.MultiheadAttention defaults)."""
        for layer in self.transformer_encoder.layers:
            nn.init.xavier_uniform_(layer.self_attn.in_proj_weight)
            nn.init.zeros_(layer.self_attn.in_proj_bias)
        for m in self.modules():
            if isinstance(m, nn.Embedding):
                nn.init.xavier_normal_(m.weight)
            elif isinstance(m, nn.Linear):
                nn.init.xavier_normal_(m.weight)
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0)
            elif isinstance(m, nn.LayerNorm):
                nn.init.constant_(m.bias, 0)
                nn.init.constant_(m.weight, 1.0)

    def cfg(self) -> F.TowerCfg:
        return F.TowerCfg(D=self.embedding_dim, H=self.num_heads, n_layers=self.num_layers,
                          p_drop=self.dropout.p if self.training else 0.0,
                          dtype=self.compute_dtype, prune_last=self.prune_last)

    def forward(self, history_ids: Tensor, user_gender: Tensor, user_country: Tensor,
                history_mask: Optional[Tensor] = None, seeds: Optional[Tensor] = None) -> Tensor:
        # an id outside an embedding table met by an earlier (finished) launch raises here, as
        # nn.Embedding raises (user_tower.py:26,30-31); the device lookups clamp and flag it
        ops.check_id_errors()
        cfg = self.cfg()
        if cfg.p_drop > 0 and seeds is None:
            seeds = new_dropout_seeds(history_ids.device)
        names, params = zip(*self.named_parameters())
        ids = history_ids.contiguous()
        mask = None if history_mask is None else history_mask.contiguous()
        if torch.is_grad_enabled() and any(p.requires_grad for p in params):
            return _UserTowerFn.apply(cfg, list(names), seeds, ids, user_gender.contiguous(),
                                      user_country.contiguous(), mask, *params)
        P, W = self.inference_operands()
        u, _ = F.user_tower_fwd(P, W, ids, user_gender.contiguous(), user_country.contiguous(),
                                mask, cfg, seeds)
        return u

    def inference_operands(self):
        """(P, W) for no-grad forwards.  The bf16 GEMM copies and transposed mirrors are cached
        and rebuilt only when a parameter changed (storage or in-place version): an eval loop
        over a fixed model casts its weights once, not once per batch.  A changed parameter at
        the same storage is re-cast into the same buffers, so a captured graph that reads them
        stays valid (GlobalEvaluator in retrieval.py re-checks before every replay).  Raw-pointer
        parameter writers (TrainStep, ops.adamw) bump ops.PARAM_EPOCH, which is part of the key."""
        names, params = zip(*self.named_parameters())
        key = tuple((p.data_ptr(), p._version) for p in params) + (ops.PARAM_EPOCH[0], self.compute_dtype)
        c = getattr(self, "_inf_cache", None)
        if c is not None and c[0] == key:
            return c[1], c[2]
        P = dict(zip(names, [p.detach() for p in params]))
        gn = _gemm_names(list(names))
        if (c is not None and c[0][-1] == key[-1] and cfg_dtype_bf16(self.compute_dtype)
                and all(a[0] == b[0] for a, b in zip(c[0][:-2], key[:-2]))):
            W = c[2]                                    # same storages: refresh in place
            for n in gn:
                ops.cast_bf16(P[n].contiguous(), W[n])
            refresh_transposes(W, gn)
            for n in P:
                if n not in gn:
                    W[n] = P[n]
        else:
            W = make_operands(P, self.compute_dtype, gn)
        self._inf_cache = (key, P, W)
        return P, W

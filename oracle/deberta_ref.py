"""ORACLE — test infrastructure only (never imported by the product path).

CPU fp32 restatement of the cfg-4 text encoder, reference src/models/item_tower.py:41-83:
``TextEncoder`` = ``AutoModel.from_pretrained("microsoft/mdeberta-v3-base")`` (a DebertaV2Model)
wrapped by peft LoRA (r=8, alpha=32, dropout 0.1, target_modules query_proj/value_proj,
:51-59), masked mean-pool (:73-80) and Linear(768,512) -> ReLU -> Dropout(0.1) -> Linear(512,D)
(:63-68, :83).

Third-party arithmetic restated here:
* transformers 4.57.3 (reference uv.lock:4924) ``DebertaV2Model``; the container has 5.15.0,
  whose modeling_deberta_v2.py is followed line by line:
  - embeddings (DebertaV2Embeddings.forward): word embedding, LayerNorm(eps), times the 2-D
    attention mask, dropout (position_biased_input = False and type_vocab_size = 0 for
    mdeberta-v3-base, so no position / token-type terms);
  - encoder (DebertaV2Encoder.forward): pairwise mask m_i·m_j; relative positions
    build_relative_position(S, S, bucket_size=position_buckets, max_position=512) with
    make_log_bucket_position; rel_embeddings = LayerNorm(rel_embeddings.weight) once per
    forward (norm_rel_ebd = "layer_norm");
  - DisentangledSelfAttention.forward / disentangled_attention_bias with share_att_key and
    pos_att_type = c2p|p2c: scale = sqrt(d_head·3);
      score[i,j] = (Q_i·K_j + Q_i·posK[c2p(i,j)] + K_j·posQ[p2c(i,j)]) / scale
    where posQ = query_proj(rel), posK = key_proj(rel) (the *shared* projections, so the
    query_proj LoRA delta applies to posQ too), c2p(i,j) = clamp(rel(i,j) + span, 0, 2·span-1),
    p2c(i,j) = clamp(-rel(j,i) + span, ...), span = position_buckets; masked entries =
    finfo(fp32).min, softmax, dropout, ·V;
  - DebertaV2SelfOutput / Intermediate (GELU, erf form) / Output: post-LayerNorm residuals.
  The golden fixture tests/golden/deberta_tiny.npz was produced by transformers' own
  DebertaV2Model (tools/make_golden_deberta.py) and pins this restatement.
* peft 0.18.0 (uv.lock:2996) is absent: LoRA is restated as
  y = W x + b + (alpha/r)·B(A(Dropout(x))), A kaiming-uniform(a=sqrt(5)), B = 0 at init.  With
  the LoRA dropout off this equals a merged weight W + (alpha/r)·B·A, which is how the fixture
  pins it (parity of the peft wrapper itself is unpinned: no reference test covers it).

Parameter names follow the peft-wrapped reference: ``transformer.base_model.model.<DebertaV2
key>`` with ``query_proj/value_proj`` split into ``base_layer.{weight,bias}`` and
``lora_A.default.weight`` [r, H] / ``lora_B.default.weight`` [H, r]; ``projection.{0,3}.*``.
Functions here take the DebertaV2Model-level names (``encoder.layer.0.attention.self.
query_proj.base_layer.weight`` ...) via ``prefix``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, Optional

import torch
import torch.nn.functional as F

Tensor = torch.Tensor


@dataclass(frozen=True)
class DebertaCfg:
    """mdeberta-v3-base values (public config)."""
    vocab_size: int = 251000
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    intermediate: int = 3072
    position_buckets: int = 256
    max_position: int = 512           # max_relative_positions = -1 -> max_position_embeddings
    eps: float = 1e-7
    lora_r: int = 8
    lora_alpha: int = 32

    @property
    def d_head(self) -> int:
        return self.hidden // self.heads

    @property
    def lora_scale(self) -> float:
        return self.lora_alpha / self.lora_r


def log_bucket_position(rel: Tensor, bucket_size: int, max_position: int) -> Tensor:
    """make_log_bucket_position (modeling_deberta_v2.py:57-69)."""
    sign = torch.sign(rel)
    mid = bucket_size // 2
    abs_pos = torch.where((rel < mid) & (rel > -mid), torch.tensor(mid - 1).type_as(rel),
                          torch.abs(rel))
    log_pos = torch.ceil(torch.log(abs_pos / mid) /
                         torch.log(torch.tensor((max_position - 1) / mid)) * (mid - 1)) + mid
    return torch.where(abs_pos <= mid, rel.type_as(log_pos), log_pos * sign)


def relative_position(S: int, cfg: DebertaCfg) -> Tensor:
    """build_relative_position (modeling_deberta_v2.py:72-102): bucket(i - j), [S, S] int64."""
    q = torch.arange(S)
    rel = q[:, None] - q[None, :]
    return log_bucket_position(rel, cfg.position_buckets, cfg.max_position).to(torch.long)


def rel_index(S: int, cfg: DebertaCfg) -> Tensor:
    """delta(i, j) = clamp(bucket(i - j) + span, 0, 2·span - 1): the posK row of c2p(i, j) and
    (bucket being odd) the posQ row of p2c(i, j), i.e. score[i, j] uses Q_i·posK[delta(i, j)]
    and K_j·posQ[delta(i, j)]."""
    span = cfg.position_buckets
    return torch.clamp(relative_position(S, cfg) + span, 0, 2 * span - 1)


def lora_linear(x: Tensor, p: Dict[str, Tensor], name: str, scale: float,
                lora_drop=None) -> Tensor:
    """peft lora.Linear: base_layer(x) + scale·lora_B(lora_A(dropout(x)))."""
    y = F.linear(x, p[name + ".base_layer.weight"], p[name + ".base_layer.bias"])
    xd = lora_drop(x) if lora_drop is not None else x
    return y + scale * F.linear(F.linear(xd, p[name + ".lora_A.default.weight"]),
                                p[name + ".lora_B.default.weight"])


def _proj(x: Tensor, p: Dict[str, Tensor], name: str, cfg: DebertaCfg, lora_drop=None) -> Tensor:
    if name + ".lora_A.default.weight" in p:
        return lora_linear(x, p, name, cfg.lora_scale, lora_drop)
    if name + ".base_layer.weight" in p:
        return F.linear(x, p[name + ".base_layer.weight"], p[name + ".base_layer.bias"])
    return F.linear(x, p[name + ".weight"], p[name + ".bias"])


def disentangled_attention(h: Tensor, rel: Tensor, mask2: Tensor, p: Dict[str, Tensor], pre: str,
                           cfg: DebertaCfg, delta: Tensor) -> Tensor:
    """DisentangledSelfAttention.forward (modeling_deberta_v2.py:191-274, :276-346) with
    share_att_key and c2p|p2c; dropout off."""
    B, S, Hd = h.shape
    nh, dh = cfg.heads, cfg.d_head

    def heads(t):                       # [B, S, H] -> [B, nh, S, dh]
        return t.view(t.shape[0], t.shape[1], nh, dh).permute(0, 2, 1, 3)

    q = heads(_proj(h, p, pre + "query_proj", cfg))
    k = heads(_proj(h, p, pre + "key_proj", cfg))
    v = heads(_proj(h, p, pre + "value_proj", cfg))
    pos_q = heads(_proj(rel[None], p, pre + "query_proj", cfg))[0]    # [nh, 2span, dh]
    pos_k = heads(_proj(rel[None], p, pre + "key_proj", cfg))[0]
    scale = math.sqrt(dh * 3)
    c2c = q @ k.transpose(-1, -2)
    c2p_all = q @ pos_k.transpose(-1, -2)                               # [B, nh, S, 2span]
    c2p = torch.gather(c2p_all, -1, delta.expand(B, nh, S, S))
    p2c_all = k @ pos_q.transpose(-1, -2)                               # [B, nh, S(k), 2span]
    # p2c rows are keys r: index clamp(-bucket(r - c) + span) = delta[c][r] (bucket is odd)
    p2c = torch.gather(p2c_all, -1, delta.t().expand(B, nh, S, S)).transpose(-1, -2)
    scores = (c2c + c2p + p2c) / scale
    scores = scores.masked_fill(~mask2[:, None].bool(), torch.finfo(torch.float32).min)
    probs = torch.softmax(scores, dim=-1)
    ctx = probs @ v                                                     # [B, nh, S, dh]
    return ctx.permute(0, 2, 1, 3).reshape(B, S, Hd)


def deberta_forward(p: Dict[str, Tensor], input_ids: Tensor, attention_mask: Tensor,
                    cfg: DebertaCfg, prefix: str = "") -> Tensor:
    """DebertaV2Model.forward (modeling_deberta_v2.py:720-800) -> last_hidden_state [B,S,H]."""
    S = input_ids.shape[1]
    m = attention_mask.to(torch.float32)
    x = F.embedding(input_ids, p[prefix + "embeddings.word_embeddings.weight"])
    x = F.layer_norm(x, (cfg.hidden,), p[prefix + "embeddings.LayerNorm.weight"],
                     p[prefix + "embeddings.LayerNorm.bias"], cfg.eps)
    x = x * m[:, :, None]
    mask2 = m[:, None, :] * m[:, :, None]                               # [B, S, S]
    rel = F.layer_norm(p[prefix + "encoder.rel_embeddings.weight"], (cfg.hidden,),
                       p[prefix + "encoder.LayerNorm.weight"], p[prefix + "encoder.LayerNorm.bias"],
                       cfg.eps)
    delta = rel_index(S, cfg)
    for i in range(cfg.layers):
        L = f"{prefix}encoder.layer.{i}."
        ctx = disentangled_attention(x, rel, mask2, p, L + "attention.self.", cfg, delta)
        a = F.layer_norm(F.linear(ctx, p[L + "attention.output.dense.weight"],
                                  p[L + "attention.output.dense.bias"]) + x, (cfg.hidden,),
                         p[L + "attention.output.LayerNorm.weight"],
                         p[L + "attention.output.LayerNorm.bias"], cfg.eps)
        hmid = F.gelu(F.linear(a, p[L + "intermediate.dense.weight"],
                               p[L + "intermediate.dense.bias"]))
        x = F.layer_norm(F.linear(hmid, p[L + "output.dense.weight"], p[L + "output.dense.bias"])
                         + a, (cfg.hidden,), p[L + "output.LayerNorm.weight"],
                         p[L + "output.LayerNorm.bias"], cfg.eps)
    return x


def text_encoder_forward(p: Dict[str, Tensor], input_ids: Tensor, attention_mask: Tensor,
                         cfg: DebertaCfg, prefix: str = "transformer.base_model.model.",
                         proj_prefix: str = "projection.") -> Tensor:
    """TextEncoder.forward (item_tower.py:70-83): mean-pool over the mask (clamp 1e-9) and the
    projection MLP (dropout off)."""
    tok = deberta_forward(p, input_ids, attention_mask, cfg, prefix)
    m = attention_mask.unsqueeze(-1).expand(tok.size()).float()
    pooled = (tok * m).sum(1) / torch.clamp(m.sum(1), min=1e-9)
    z = torch.relu(F.linear(pooled, p[proj_prefix + "0.weight"], p[proj_prefix + "0.bias"]))
    return F.linear(z, p[proj_prefix + "3.weight"], p[proj_prefix + "3.bias"])


def init_text_params(cfg: DebertaCfg, out_dim: int, generator: torch.Generator,
                     prefix: str = "transformer.base_model.model.", lora: bool = True,
                     std: float = 0.02, lora_b_std: float = 0.0) -> Dict[str, Tensor]:
    """DebertaV2 _init_weights (normal(0, initializer_range=0.02) Linear/Embedding, zero bias,
    LN 1/0) + peft LoRA init (A kaiming-uniform a=sqrt(5), B zeros unless lora_b_std > 0 for
    tests) + nn.Linear defaults for the projection."""
    g = generator
    H, I = cfg.hidden, cfg.intermediate
    p: Dict[str, Tensor] = {}

    def lin(name, o, i, wrap=False):
        w = torch.randn(o, i, generator=g) * std
        b = torch.zeros(o)
        if wrap and lora:
            p[name + ".base_layer.weight"], p[name + ".base_layer.bias"] = w, b
            bound = 1.0 / math.sqrt(i)                 # kaiming_uniform_(a=sqrt(5)) on [r, i]
            p[name + ".lora_A.default.weight"] = (torch.rand(cfg.lora_r, i, generator=g) * 2 - 1) * bound
            p[name + ".lora_B.default.weight"] = torch.randn(o, cfg.lora_r, generator=g) * lora_b_std
        else:
            p[name + ".weight"], p[name + ".bias"] = w, b

    def ln(name):
        p[name + ".weight"], p[name + ".bias"] = torch.ones(H), torch.zeros(H)

    pre = prefix
    p[pre + "embeddings.word_embeddings.weight"] = torch.randn(cfg.vocab_size, H, generator=g) * std
    p[pre + "embeddings.word_embeddings.weight"][0] = 0.0          # padding_idx row
    ln(pre + "embeddings.LayerNorm")
    p[pre + "encoder.rel_embeddings.weight"] = torch.randn(2 * cfg.position_buckets, H, generator=g) * std
    ln(pre + "encoder.LayerNorm")
    for i in range(cfg.layers):
        L = f"{pre}encoder.layer.{i}."
        lin(L + "attention.self.query_proj", H, H, wrap=True)
        lin(L + "attention.self.key_proj", H, H)
        lin(L + "attention.self.value_proj", H, H, wrap=True)
        lin(L + "attention.output.dense", H, H)
        ln(L + "attention.output.LayerNorm")
        lin(L + "intermediate.dense", I, H)
        lin(L + "output.dense", H, I)
        ln(L + "output.LayerNorm")
    for name, o, i in (("projection.0", 512, H), ("projection.3", out_dim, 512)):
        bound = 1.0 / math.sqrt(i)
        p[name + ".weight"] = (torch.rand(o, i, generator=g) * 2 - 1) * bound
        p[name + ".bias"] = (torch.rand(o, generator=g) * 2 - 1) * bound
    return p


def synthetic_text(B: int, S: int, vocab: int, generator: Optional[torch.Generator] = None,
                   min_len: int = 16):
    """tokens ~U[1, vocab), lengths ~U[min_len, S], prefix mask."""
    g = generator
    lengths = torch.randint(min(min_len, S), S + 1, (B,), generator=g)
    mask = (torch.arange(S)[None] < lengths[:, None]).long()
    ids = torch.randint(1, vocab, (B, S), generator=g) * mask
    return ids, mask

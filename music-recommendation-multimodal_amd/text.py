"""TextEncoder — the cfg-4 lyrics branch, drop-in for reference src/models/item_tower.py:41-83.

``AutoModel.from_pretrained("microsoft/mdeberta-v3-base")`` (a transformers DebertaV2Model) wrapped
by peft LoRA (r=8, alpha=32, dropout 0.1 on ``query_proj`` / ``value_proj``), masked mean-pool
and Linear(768,512) -> ReLU -> Dropout(0.1) -> Linear(512, D), on libttmi kernels:

* embeddings: ``ttmi_deb_embed_fwd`` (gather + LayerNorm + mask + dropout);
* every Linear: ``ttmi_gemm`` (bias / dropout / residual / GELU epilogues).  LoRA on the x path
  rides inside the QKV GEMM: its operand is ``[X | s·drop(X)·Aᵀ | 0]`` (H + 64 columns) and its
  weight ``[W_qkv | B_q, B_v | 0]``, so one launch computes ``W x + b + s·B(A(drop(x)))``;
* relative positions: ``posQ|posK = [rel | s·drop(rel)·A_qᵀ | 0] · W_aug[q,k]ᵀ`` per layer
  (share_att_key: query_proj's LoRA applies to posQ too);
* attention: ``ttmi_dis_attn_fwd/bwd`` (fused c2c + c2p + p2c, online softmax);
* post-LayerNorms: ``ttmi_deb_ln_fwd`` / ``ttmi_layernorm_bwd``; GELU: the intermediate GEMM's epilogue (``pre_out``) and the
  GEMM's GELU' epilogue; mean-pool: ``ttmi_deb_pool_fwd/bwd``.

Parameter names are the peft-wrapped reference's (``transformer.base_model.model.encoder.
layer.{i}.attention.self.query_proj.base_layer.weight``, ``...lora_A.default.weight``,
``projection.{0,3}.*``).  As with peft, the base model is frozen: only the LoRA matrices and the
projection train, so the backward runs input-gradient GEMMs only.  The pretrained checkpoint
is a download (unavailable offline): weights are random-initialised with DebertaV2's
initialiser unless loaded with ``load_state_dict``.  ``use_lora=False`` (full fine-tuning)
is not built.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch
import torch.nn as nn

from . import ops

Tensor = torch.Tensor

PREFIX = "transformer.base_model.model."
PAD = 64                      # augmented-operand columns (LoRA t_q | t_v | zeros)

# text-encoder dropout sites (own seed table of N_TEXT_SITES)
N_TEXT_SITES = 128
TSITE_EMB, TSITE_PROJ = 0, 127


def tsite(layer: int, k: int) -> int:
    """k: 0 attention probs, 1 attention output, 2 FFN output, 3 LoRA-q(x), 4 LoRA-v(x),
    5 pos_dropout(rel), 6 LoRA-q(rel)."""
    return 1 + 8 * layer + k


@dataclass(frozen=True)
class TextCfg:
    vocab_size: int = 251000
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    intermediate: int = 3072
    position_buckets: int = 256
    max_position: int = 512
    eps: float = 1e-7
    lora_r: int = 8
    lora_alpha: int = 32
    lora_dropout: float = 0.1
    hidden_dropout: float = 0.1
    attn_dropout: float = 0.1

    @property
    def npos(self) -> int:
        return 2 * self.position_buckets

    @property
    def scale(self) -> float:
        return self.lora_alpha / self.lora_r


# ---------------------------------------------------------------------------- module tree
class _LoraLinear(nn.Module):
    """peft lora.Linear container: base_layer + lora_A/lora_B['default'] (+ lora_dropout)."""

    def __init__(self, i: int, o: int, r: int, p: float):
        super().__init__()
        self.base_layer = nn.Linear(i, o)
        self.lora_dropout = nn.ModuleDict({"default": nn.Dropout(p)})
        self.lora_A = nn.ModuleDict({"default": nn.Linear(i, r, bias=False)})
        self.lora_B = nn.ModuleDict({"default": nn.Linear(r, o, bias=False)})
        nn.init.zeros_(self.lora_B["default"].weight)        # peft init: B = 0


class _SelfAttn(nn.Module):
    def __init__(self, c: TextCfg):
        super().__init__()
        H = c.hidden
        self.query_proj = _LoraLinear(H, H, c.lora_r, c.lora_dropout)
        self.key_proj = nn.Linear(H, H)
        self.value_proj = _LoraLinear(H, H, c.lora_r, c.lora_dropout)


class _Out(nn.Module):
    def __init__(self, i: int, o: int, eps: float):
        super().__init__()
        self.dense = nn.Linear(i, o)
        self.LayerNorm = nn.LayerNorm(o, eps=eps)


class _Attention(nn.Module):
    def __init__(self, c: TextCfg):
        super().__init__()
        self.self = _SelfAttn(c)
        self.output = _Out(c.hidden, c.hidden, c.eps)


class _Intermediate(nn.Module):
    def __init__(self, c: TextCfg):
        super().__init__()
        self.dense = nn.Linear(c.hidden, c.intermediate)


class _Layer(nn.Module):
    def __init__(self, c: TextCfg):
        super().__init__()
        self.attention = _Attention(c)
        self.intermediate = _Intermediate(c)
        self.output = _Out(c.intermediate, c.hidden, c.eps)


class _Embeddings(nn.Module):
    def __init__(self, c: TextCfg):
        super().__init__()
        self.word_embeddings = nn.Embedding(c.vocab_size, c.hidden, padding_idx=0)
        self.LayerNorm = nn.LayerNorm(c.hidden, eps=c.eps)


class _Encoder(nn.Module):
    def __init__(self, c: TextCfg):
        super().__init__()
        self.layer = nn.ModuleList([_Layer(c) for _ in range(c.layers)])
        self.rel_embeddings = nn.Embedding(c.npos, c.hidden)
        self.LayerNorm = nn.LayerNorm(c.hidden, eps=c.eps)


class _DebertaV2(nn.Module):
    def __init__(self, c: TextCfg):
        super().__init__()
        self.embeddings = _Embeddings(c)
        self.encoder = _Encoder(c)


# ---------------------------------------------------------------------------- frozen cache
class _Frozen:
    """bf16 GEMM mirrors of the frozen base weights (built once, rebuilt if any base
    parameter's version or storage changes, e.g. after load_state_dict)."""

    def __init__(self):
        self.key = None
        self.deltas: Dict[int, Tensor] = {}        # S -> delta table (weight-independent)

    def refresh(self, enc: "TextEncoder") -> None:
        c = enc.cfg
        base = dict(enc.transformer.base_model.model.named_parameters())
        key = tuple((p.data_ptr(), p._version) for p in base.values())
        if key == self.key:
            return
        dev = next(iter(base.values())).device
        H, I = c.hidden, c.intermediate

        def bf(t):
            return ops.cast_bf16(t.detach().contiguous(), torch.empty(t.shape, device=dev,
                                                                      dtype=torch.bfloat16))
        self.table = bf(base["embeddings.word_embeddings.weight"])
        self.layers = []
        for i in range(c.layers):
            L = f"encoder.layer.{i}."
            A = L + "attention.self."
            waug = torch.zeros(3 * H, H + PAD, device=dev, dtype=torch.bfloat16)
            for r, name in enumerate(("query_proj.base_layer", "key_proj", "value_proj.base_layer")):
                ops.dropout_to(base[A + name + ".weight"].detach(), waug[r * H:(r + 1) * H, :H])
            bqkv = torch.cat([base[A + "query_proj.base_layer.bias"].detach(),
                              base[A + "key_proj.bias"].detach(),
                              base[A + "value_proj.base_layer.bias"].detach()]).contiguous()
            wo = bf(base[L + "attention.output.dense.weight"])
            w1 = bf(base[L + "intermediate.dense.weight"])
            w2 = bf(base[L + "output.dense.weight"])
            # k-major mirrors of the input-grad operands (dX = dY·W reads Wᵀ rows), so the
            # backward token GEMMs take the 256x256 LDS-DMA tile kernel
            wqkv = waug[:, :H].contiguous()
            t = [torch.empty(m.shape[1], m.shape[0], device=dev, dtype=torch.bfloat16)
                 for m in (wo, w1, w2, wqkv)]
            ops.transpose_batch(t, [wo, w1, w2, wqkv])
            self.layers.append(dict(waug=waug, bqkv=bqkv, wo=wo, w1=w1, w2=w2,
                                    woT=t[0], w1T=t[1], w2T=t[2], wqkvT=t[3]))
        self.rel = torch.empty(c.npos, H, device=dev)
        m = torch.empty(c.npos, device=dev)
        ops.deb_ln_fwd(base["encoder.rel_embeddings.weight"].detach().contiguous(),
                       base["encoder.LayerNorm.weight"].detach(),
                       base["encoder.LayerNorm.bias"].detach(), c.eps, self.rel, None, m,
                       torch.empty_like(m))
        self.base = {k: v.detach() for k, v in base.items()}
        self.key = key

    def delta(self, S: int, c: TextCfg, dev) -> Tensor:
        """delta(rel) for rel = -(S-1)..S-1: clamp(log-bucket(rel) + span, 0, npos-1) with
        make_log_bucket_position's float32 arithmetic (modeling_deberta_v2.py:57-69)."""
        key = (S, str(dev))
        if key not in self.deltas:
            rel = torch.arange(-(S - 1), S, dtype=torch.long)
            mid = c.position_buckets // 2
            sign = torch.sign(rel)
            abs_pos = torch.where((rel < mid) & (rel > -mid), torch.tensor(mid - 1), rel.abs())
            log_pos = torch.ceil(torch.log(abs_pos / mid) /
                                 torch.log(torch.tensor((c.max_position - 1) / mid)) * (mid - 1)) + mid
            bucket = torch.where(abs_pos <= mid, rel.to(log_pos.dtype), log_pos * sign).long()
            d = torch.clamp(bucket + c.position_buckets, 0, c.npos - 1).to(torch.int16)
            self.deltas[key] = d.to(dev)
        return self.deltas[key]


# ---------------------------------------------------------------------------- functional
@dataclass
class _LayerSaved:
    xaug: Tensor
    xq: Tensor
    xv: Tensor
    qkv: Tensor
    posqk: Tensor
    relq: Tensor
    u: Optional[Tensor]
    ctx: Tensor
    lse: Tensor
    z1: Tensor
    m1: Tensor
    r1: Tensor
    pre: Tensor
    z2: Tensor
    m2: Tensor
    r2: Tensor


@dataclass
class TextSaved:
    B: int
    S: int
    mask: Tensor
    delta: Tensor
    layers: List[_LayerSaved] = field(default_factory=list)
    pooled16: Optional[Tensor] = None
    y1: Optional[Tensor] = None
    aq16: List[Tensor] = field(default_factory=list)
    av16: List[Tensor] = field(default_factory=list)
    training: bool = True
    order: Optional[Tensor] = None     # ops.dis_attn_order(mask): per-sequence kernel order


def _drop(p: float, seeds: Optional[Tensor], site: int):
    if p > 0 and seeds is not None:
        return (p, seeds[site:site + 1])
    return ops.NO_DROP


_SIDE: Dict[str, "torch.cuda.Stream"] = {}


def _side_stream(dev) -> "torch.cuda.Stream":
    """One side stream per device for the backward's LoRA-gradient streams (created on first
    use, i.e. in an eager step before any graph capture)."""
    key = str(dev)
    if key not in _SIDE:
        _SIDE[key] = torch.cuda.Stream(dev)
    return _SIDE[key]


def _mm(A, B, C, M, N, K, *, lda, ldb, ldc, a_k=True, b_k=True, **kw):
    return ops.gemm(A, B, C, M, N, K, lda=lda, a_kmajor=a_k, ldb=ldb, b_kmajor=b_k, ldc=ldc, **kw)


def text_fwd(enc: "TextEncoder", P: Dict[str, Tensor], ids: Tensor, mask: Tensor,
             seeds: Optional[Tensor], training: bool):
    """Forward of TextEncoder (item_tower.py:70-83) -> ([B, D] fp32, TextSaved).  P holds the
    trainable tensors (LoRA A/B per layer, projection) by TextEncoder parameter name."""
    c = enc.cfg
    Fz = enc.frozen
    Fz.refresh(enc)
    dev = ids.device
    B, S = ids.shape
    M, H, I, nh, Ha = B * S, c.hidden, c.intermediate, c.heads, c.hidden + PAD
    s = c.scale
    mask = mask.to(torch.int64).contiguous()
    ids = ids.to(torch.int64).contiguous()
    delta = Fz.delta(S, c, dev)
    st = TextSaved(B, S, mask, delta, training=training)
    st.order = ops.dis_attn_order(mask, B, S)         # shared by every layer's fwd and bwd
    pd = c.hidden_dropout if training else 0.0
    pa = c.attn_dropout if training else 0.0
    pl = c.lora_dropout if training else 0.0
    bf = torch.bfloat16
    x32 = torch.empty(M, H, device=dev)
    xaug = torch.zeros(M, Ha, device=dev, dtype=bf)
    ops.deb_embed_fwd(ids, Fz.table, Fz.base["embeddings.LayerNorm.weight"],
                      Fz.base["embeddings.LayerNorm.bias"], c.eps, mask, x32, xaug,
                      drop=_drop(pd, seeds, TSITE_EMB))
    nxt_qv = None
    for l in range(c.layers):
        W = Fz.layers[l]
        lp = f"{PREFIX}encoder.layer.{l}.attention.self."
        Aq, Bq = P[lp + "query_proj.lora_A.default.weight"], P[lp + "query_proj.lora_B.default.weight"]
        Av, Bv = P[lp + "value_proj.lora_A.default.weight"], P[lp + "value_proj.lora_B.default.weight"]
        r = Aq.shape[0]
        waug = W["waug"]
        ops.dropout_to(Bq.detach().contiguous(), waug[0:H, H:H + r])          # LoRA columns
        ops.dropout_to(Bv.detach().contiguous(), waug[2 * H:3 * H, H + r:H + 2 * r])
        aq16 = ops.cast_bf16(Aq.detach().contiguous(), torch.empty(Aq.shape, device=dev, dtype=bf))
        av16 = ops.cast_bf16(Av.detach().contiguous(), torch.empty(Av.shape, device=dev, dtype=bf))
        st.aq16.append(aq16)
        st.av16.append(av16)
        # x path: t_q = s·drop(x)·Aqᵀ, t_v = s·drop(x)·Avᵀ into the augmented columns
        if pl > 0 and nxt_qv is not None:       # made by the previous layer's post-LN kernel
            xq, xv = nxt_qv
        elif pl > 0:
            xq = ops.dropout_to(x32, torch.empty(M, H, device=dev, dtype=bf), _drop(pl, seeds, tsite(l, 3)))
            xv = ops.dropout_to(x32, torch.empty(M, H, device=dev, dtype=bf), _drop(pl, seeds, tsite(l, 4)))
        else:
            xq = xv = xaug[:, :H]
        nxt_qv = None
        _mm(xq, aq16, xaug[:, H:H + r], M, r, H, lda=xq.stride(0), ldb=H, ldc=Ha, alpha=s)
        _mm(xv, av16, xaug[:, H + r:H + 2 * r], M, r, H, lda=xv.stride(0), ldb=H, ldc=Ha, alpha=s)
        qkv = torch.empty(M, 3 * H, device=dev, dtype=bf)
        _mm(xaug, waug, qkv, M, 3 * H, Ha, lda=Ha, ldb=Ha, ldc=3 * H, bias=W["bqkv"])
        # relative path: posQ|posK = [drop(rel) | s·drop(drop(rel))·Aqᵀ | 0]·W_aug[q,k]ᵀ
        reld = ops.dropout_to(Fz.rel, torch.empty(c.npos, H, device=dev), _drop(pd, seeds, tsite(l, 5))) \
            if pd > 0 else Fz.rel
        relq = ops.dropout_to(reld, torch.empty(c.npos, H, device=dev), _drop(pl, seeds, tsite(l, 6))) \
            if pl > 0 else reld
        relaug = torch.zeros(c.npos, Ha, device=dev, dtype=bf)
        ops.dropout_to(reld, relaug[:, :H])
        aq32 = Aq.detach().contiguous()
        u = torch.empty(c.npos, r, device=dev)
        _mm(relq, aq32, u, c.npos, r, H, lda=H, ldb=H, ldc=r)                 # fp32 GEMM
        _mm(relq, aq32, relaug[:, H:H + r], c.npos, r, H, lda=H, ldb=H, ldc=Ha, alpha=s)
        posqk = torch.empty(c.npos, 2 * H, device=dev, dtype=bf)
        _mm(relaug, waug, posqk, c.npos, 2 * H, Ha, lda=Ha, ldb=Ha, ldc=2 * H, bias=W["bqkv"])
        # attention
        ctx = torch.empty(M, H, device=dev, dtype=bf)
        lse = torch.empty(B * nh * S, device=dev)
        ops.dis_attn(B, S, nh, qkv[:, :H], qkv[:, H:2 * H], qkv[:, 2 * H:], posqk[:, :H],
                     posqk[:, H:], mask, delta, 1.0 / math.sqrt(64 * 3), ctx, lse,
                     _drop(pa, seeds, tsite(l, 0)), order=st.order)
        # output projection + residual + LN, FFN + residual + LN
        L = f"encoder.layer.{l}."
        z1 = torch.empty(M, H, device=dev)
        _mm(ctx, W["wo"], z1, M, H, H, lda=H, ldb=H, ldc=H,
            bias=Fz.base[L + "attention.output.dense.bias"], drop=_drop(pd, seeds, tsite(l, 1)),
            ld_drop=H, residual=x32, ld_res=H)
        a32 = torch.empty(M, H, device=dev)
        a16 = torch.empty(M, H, device=dev, dtype=bf)
        m1, r1 = torch.empty(M, device=dev), torch.empty(M, device=dev)
        ops.deb_ln_fwd(z1, Fz.base[L + "attention.output.LayerNorm.weight"],
                       Fz.base[L + "attention.output.LayerNorm.bias"], c.eps, a32, a16, m1, r1)
        # intermediate.dense + GELU in one epilogue: hh = GELU(pre), pre kept for GELU'
        pre = torch.empty(M, I, device=dev, dtype=bf)
        hh = torch.empty(M, I, device=dev, dtype=bf)
        _mm(a16, W["w1"], hh, M, I, H, lda=H, ldb=H, ldc=I, bias=Fz.base[L + "intermediate.dense.bias"],
            act=2, pre_out=pre)
        z2 = torch.empty(M, H, device=dev)
        _mm(hh, W["w2"], z2, M, H, I, lda=I, ldb=I, ldc=H, bias=Fz.base[L + "output.dense.bias"],
            drop=_drop(pd, seeds, tsite(l, 2)), ld_drop=H, residual=a32, ld_res=H)
        del hh
        x32n = torch.empty(M, H, device=dev)
        xaugn = torch.zeros(M, Ha, device=dev, dtype=bf)
        m2, r2 = torch.empty(M, device=dev), torch.empty(M, device=dev)
        if pl > 0 and l + 1 < c.layers and H % 256 == 0:   # next layer's LoRA inputs, fused
            nxt_qv = (torch.empty(M, H, device=dev, dtype=bf), torch.empty(M, H, device=dev, dtype=bf))
            ops.deb_ln_fwd(z2, Fz.base[L + "output.LayerNorm.weight"],
                           Fz.base[L + "output.LayerNorm.bias"], c.eps, x32n, xaugn, m2, r2,
                           yq=nxt_qv[0], yv=nxt_qv[1], drop_q=_drop(pl, seeds, tsite(l + 1, 3)),
                           drop_v=_drop(pl, seeds, tsite(l + 1, 4)))
        else:
            ops.deb_ln_fwd(z2, Fz.base[L + "output.LayerNorm.weight"],
                           Fz.base[L + "output.LayerNorm.bias"], c.eps, x32n, xaugn, m2, r2)
        st.layers.append(_LayerSaved(xaug, xq, xv, qkv, posqk, relq, u, ctx, lse, z1, m1, r1, pre,
                                     z2, m2, r2))
        x32, xaug = x32n, xaugn
    # masked mean-pool + projection head
    pooled = ops.deb_pool_fwd(x32, mask, torch.empty(B, H, device=dev))
    p16 = ops.cast_bf16(pooled, torch.empty(B, H, device=dev, dtype=bf))
    w0 = ops.cast_bf16(P["projection.0.weight"].detach().contiguous(),
                       torch.empty(P["projection.0.weight"].shape, device=dev, dtype=bf))
    w3 = ops.cast_bf16(P["projection.3.weight"].detach().contiguous(),
                       torch.empty(P["projection.3.weight"].shape, device=dev, dtype=bf))
    y1 = torch.empty(B, w0.shape[0], device=dev, dtype=bf)
    pp = enc.projection[2].p if training else 0.0
    ops.linear(p16, w0, P["projection.0.bias"].detach(), y1, act=1, drop=_drop(pp, seeds, TSITE_PROJ))
    out = torch.empty(B, w3.shape[0], device=dev)
    ops.linear(y1, w3, P["projection.3.bias"].detach(), out)
    st.pooled16, st.y1 = p16, y1
    st.w0, st.w3, st.pp, st.x32_last = w0, w3, pp, None
    return out, st


def text_bwd(enc: "TextEncoder", P: Dict[str, Tensor], st: TextSaved, dout: Tensor,
             G: Dict[str, Tensor], seeds: Optional[Tensor]) -> None:
    """Backward of text_fwd: accumulates the LoRA and projection gradients into G."""
    c = enc.cfg
    Fz = enc.frozen
    dev = dout.device
    B, S = st.B, st.S
    M, H, I, nh, Ha = B * S, c.hidden, c.intermediate, c.heads, c.hidden + PAD
    s = c.scale
    bf = torch.bfloat16
    pd = c.hidden_dropout if st.training else 0.0
    pa = c.attn_dropout if st.training else 0.0
    pl = c.lora_dropout if st.training else 0.0
    # projection head
    dc = ops.dropout_to(dout.contiguous().float(), torch.empty(dout.shape, device=dev, dtype=bf))
    ops.linear_dw(dc, st.y1, G["projection.3.weight"], G["projection.3.bias"])
    dy1 = torch.empty(st.y1.shape, device=dev, dtype=bf)
    scale_p = 1.0 / (1.0 - st.pp) if st.pp > 0 else 1.0
    ops.linear_dx(dc, st.w3, dy1, gate=st.y1, gate_scale=scale_p)
    ops.linear_dw(dy1, st.pooled16, G["projection.0.weight"], G["projection.0.bias"])
    dpooled = torch.empty(B, H, device=dev)
    ops.linear_dx(dy1, st.w0, dpooled)
    dx = ops.deb_pool_bwd(dpooled, st.mask, torch.empty(M, H, device=dev))
    main = torch.cuda.current_stream(dev)
    side = _side_stream(dev)
    keep = []
    for l in reversed(range(c.layers)):
        sv = st.layers[l]
        W = Fz.layers[l]
        L = f"encoder.layer.{l}."
        lp = f"{PREFIX}encoder.layer.{l}.attention.self."
        r = st.aq16[l].shape[0]
        if r != 8:
            raise NotImplementedError("text backward kernels are built for LoRA rank 8 (the reference's r)")
        dz2 = torch.empty(M, H, device=dev)
        g2 = torch.empty(M, H, device=dev, dtype=bf)        # bf16(dropout'(dz2)), same kernel
        ops.layernorm_bwd(dx, sv.z2, sv.m2, sv.r2, Fz.base[L + "output.LayerNorm.weight"], dz2, None,
                          None, dx16=g2, drop=_drop(pd, seeds, tsite(l, 2)))
        dpre = torch.empty(M, I, device=dev, dtype=bf)
        _mm(g2, W["w2T"], dpre, M, I, H, lda=H, ldb=H, ldc=I, act=3, gate=sv.pre, ld_gate=I)
        da = torch.empty(M, H, device=dev)
        _mm(dpre, W["w1T"], da, M, H, I, lda=I, ldb=I, ldc=H, residual=dz2, ld_res=H)
        dz1 = torch.empty(M, H, device=dev)
        g1 = torch.empty(M, H, device=dev, dtype=bf)
        ops.layernorm_bwd(da, sv.z1, sv.m1, sv.r1, Fz.base[L + "attention.output.LayerNorm.weight"],
                          dz1, None, None, dx16=g1, drop=_drop(pd, seeds, tsite(l, 1)))
        dctx = torch.empty(M, H, device=dev, dtype=bf)
        _mm(g1, W["woT"], dctx, M, H, H, lda=H, ldb=H, ldc=H)
        dqkv = torch.empty(M, 3 * H, device=dev, dtype=bf)
        bq32 = P[lp + "query_proj.lora_B.default.weight"].detach().contiguous()
        hu = torch.empty(M * nh * 8, device=dev)
        pb = torch.empty(c.npos * 8, device=dev)                  # Σ over batch and heads
        ops.dis_attn(B, S, nh, sv.qkv[:, :H], sv.qkv[:, H:2 * H], sv.qkv[:, 2 * H:],
                     sv.posqk[:, :H], sv.posqk[:, H:], st.mask, st.delta, 1.0 / math.sqrt(64 * 3),
                     sv.ctx, sv.lse, _drop(pa, seeds, tsite(l, 0)), dctx=dctx, dq=dqkv[:, :H],
                     dk=dqkv[:, H:2 * H], dv=dqkv[:, 2 * H:], lora_u=sv.u, lora_bq=bq32,
                     lora_hu=hu, lora_pb=pb, order=st.order)
        # input gradient through the QKV GEMM (+ residual) and the LoRA branch.  The rank-8
        # LoRA weight gradients are HBM streams that no later op of this backward reads: they
        # run on a side stream under the (MFMA-bound) dgrad GEMM.  dL goes first so the side
        # stream can start on it; its inputs stay referenced in `keep` until the streams join.
        gAq, gBq = G[lp + "query_proj.lora_A.default.weight"], G[lp + "query_proj.lora_B.default.weight"]
        gAv, gBv = G[lp + "value_proj.lora_A.default.weight"], G[lp + "value_proj.lora_B.default.weight"]
        dL = torch.empty(M, 2 * r, device=dev, dtype=bf)
        _mm(dqkv, W["waug"][:, H:], dL, M, 2 * r, 3 * H, lda=3 * H, ldb=Ha, ldc=2 * r, b_k=False)
        side.wait_stream(main)
        keep.append((dqkv, dL, hu, pb))
        with torch.cuda.stream(side):
            # dB = dYᵀ·t (t = s·u lives in the augmented operand columns)
            ops.skinny_wgrad(dqkv[:, :H], sv.xaug[:, H:H + r], gBq, H, ldc_m=r, ldc_c=1)
            ops.skinny_wgrad(dqkv[:, 2 * H:], sv.xaug[:, H + r:H + 2 * r], gBv, H, ldc_m=r, ldc_c=1)
            # dA = s·dLᵀ·drop(x)
            ops.skinny_wgrad(sv.xq, dL[:, :r], gAq, H, ldc_m=1, ldc_c=H, alpha=s)
            ops.skinny_wgrad(sv.xv, dL[:, r:], gAv, H, ldc_m=1, ldc_c=H, alpha=s)
            # relative path: posQ = query_proj(rel) carries the q LoRA too:
            # dBq[h·64 + d, c] += s·Σ_m K[m, h·64 + d]·HU[m, h, c]  (per-head slices of HU)
            ops.skinny_wgrad(sv.qkv[:, H:2 * H], hu.view(M, nh * 8), gBq, H, ldc_m=r, ldc_c=1,
                             alpha=s, group=64, sgs=8)
            du = pb
            _mm(du, sv.relq, gAq, r, H, c.npos, lda=r, ldb=H, ldc=H, a_k=False, b_k=False, alpha=s,
                accumulate=True)
        dxn = torch.empty(M, H, device=dev)
        _mm(dqkv, W["wqkvT"], dxn, M, H, 3 * H, lda=3 * H, ldb=3 * H, ldc=H, residual=dz1, ld_res=H)
        # dx += s·drop'(dL·A) for q and v in one pass over dx
        ops.lora_dx(dL, st.aq16[l], st.av16[l], s, _drop(pl, seeds, tsite(l, 3)),
                    _drop(pl, seeds, tsite(l, 4)), dxn, H)
        dx = dxn
    main.wait_stream(side)
    del keep
    # the embeddings are frozen: the gradient stops here


class _TextFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, enc, names, seeds, ids, mask, *params):
        P = dict(zip(names, params))
        out, st = text_fwd(enc, P, ids, mask, seeds, True)
        ctx.saved = (enc, names, P, st, seeds)
        return out

    @staticmethod
    def backward(ctx, dout):
        enc, names, P, st, seeds = ctx.saved
        del ctx.saved
        G = {n: torch.zeros_like(P[n]) for n in names}
        text_bwd(enc, P, st, dout, G, seeds)
        return (None,) * 5 + tuple(G[n] for n in names)


class TextEncoder(nn.Module):
    """item_tower.py:41-83 with libttmi kernels (see the module docstring)."""

    def __init__(self, model_name: str = "microsoft/mdeberta-v3-base", embedding_dim: int = 128,
                 use_lora: bool = True, cfg: Optional[TextCfg] = None):
        super().__init__()
        if not use_lora:
            raise NotImplementedError("TextEncoder(use_lora=False) (full DeBERTa fine-tuning) "
                                      "is not built; the reference default is use_lora=True")
        self.model_name = model_name
        self.cfg = cfg or TextCfg()
        c = self.cfg
        self.transformer = nn.Module()
        self.transformer.base_model = nn.Module()
        self.transformer.base_model.model = _DebertaV2(c)
        self.projection = nn.Sequential(nn.Linear(c.hidden, 512), nn.ReLU(), nn.Dropout(0.1),
                                        nn.Linear(512, embedding_dim))
        self._init_base()
        for n, p in self.transformer.named_parameters():      # peft: only LoRA trains
            p.requires_grad_("lora_" in n)
        self.frozen = _Frozen()

    @torch.no_grad()
    def _init_base(self):
        """DebertaV2PreTrainedModel._init_weights: normal(0, 0.02) Linear / Embedding weights,
        zero biases and padding row, LayerNorm 1/0 (LoRA A keeps nn.Linear's kaiming-uniform,
        B is zero, as peft initialises them)."""
        for name, m in self.transformer.named_modules():
            if "lora_" in name:
                continue
            if isinstance(m, nn.Linear):
                m.weight.normal_(0.0, 0.02)
                if m.bias is not None:
                    m.bias.zero_()
            elif isinstance(m, nn.Embedding):
                m.weight.normal_(0.0, 0.02)
                if m.padding_idx is not None:
                    m.weight[m.padding_idx].zero_()
            elif isinstance(m, nn.LayerNorm):
                m.weight.fill_(1.0)
                m.bias.zero_()

    def trainable(self):
        return [(n, p) for n, p in self.named_parameters() if p.requires_grad]

    def forward(self, input_ids: Tensor, attention_mask: Tensor,
                seeds: Optional[Tensor] = None) -> Tensor:
        ops.check_id_errors()          # token ids outside the word table met by earlier launches
        names, params = zip(*self.trainable())
        if self.training and seeds is None:
            seeds = torch.randint(-(2 ** 62), 2 ** 62, (N_TEXT_SITES,), device=input_ids.device,
                                  dtype=torch.int64)
        if self.training and torch.is_grad_enabled():
            return _TextFn.apply(self, list(names), seeds, input_ids, attention_mask, *params)
        out, _ = text_fwd(self, dict(zip(names, [p.detach() for p in params])), input_ids,
                          attention_mask, seeds, self.training)
        return out

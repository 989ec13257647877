"""Explicit forward/backward schedules of the two-tower step on libttmi kernels.

This is the functional core shared by the drop-in nn.Modules (``user_tower.py``,
``item_tower.py``, ``two_tower.py`` wrap it in autograd Functions) and the graph-captured
``train.TrainStep``.  Each ``*_fwd`` returns its output and a state object holding what the
matching ``*_bwd`` needs; each ``*_bwd`` ACCUMULATES parameter gradients into the fp32
tensors of a ``grads`` dict (so a flat gradient buffer can be zeroed once per step).

Parameter dicts use the reference ``state_dict`` names (without the tower prefix):
``P`` holds the fp32 master tensors, ``W`` the GEMM operands in the compute dtype (the bf16
mirror, or ``P`` itself in fp32 mode).
"""
from __future__ import annotations

import os

from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Tuple

import torch

from . import comm, ops

Tensor = torch.Tensor

# Dropout site ids (restated by oracle/two_tower_ref.py: SITE_*).
SITE_EMB = 0
SITE_TAB = 62       # tabular encoder dropout (item_tower.py:94)
SITE_ITEM = 63


def site_attn(i: int) -> int:
    return 1 + 4 * i


def site_drop1(i: int) -> int:
    return 2 + 4 * i


def site_ffn(i: int) -> int:
    return 3 + 4 * i


def site_drop2(i: int) -> int:
    return 4 + 4 * i


def _splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return x ^ (x >> 31)


N_SITES = 64


def site_seeds(base: int, step: int) -> Dict[int, int]:
    """Per-site dropout seeds of one step; restates ttmi_dropout_seeds (device) exactly:
    seeds[s] = splitmix64(splitmix64(base) ^ (step*64 + s))."""
    return {s: _splitmix64(_splitmix64(base) ^ ((step * 64 + s) & 0xFFFFFFFFFFFFFFFF))
            for s in range(N_SITES)}


def seed_table(seeds: Dict[int, int], device) -> Tensor:
    """Upload a site->seed dict as the int64 [N_SITES] device table the kernels read."""
    vals = [0] * N_SITES
    for k, v in seeds.items():
        vals[k] = v - (1 << 64) if v >= (1 << 63) else v
    return torch.tensor(vals, dtype=torch.int64, device=device)


@dataclass
class TowerCfg:
    D: int
    H: int = 4
    n_layers: int = 2
    p_drop: float = 0.0
    dtype: torch.dtype = torch.bfloat16
    eps: float = 1e-5
    # Run the last encoder layer only for the gathered last-valid row of each sequence
    # (K/V still from every token).  Output- and gradient-identical (ttmi.h, "Last-layer
    # pruning"); False runs the full layer.
    prune_last: bool = True


def _drop(cfg: TowerCfg, seeds: Optional[Tensor], site: int, p: Optional[float] = None):
    """(p, device seed view) for one dropout site; ``seeds`` is the [N_SITES] table."""
    p = cfg.p_drop if p is None else p
    if p <= 0.0 or seeds is None:
        return ops.NO_DROP
    return (p, seeds[site:site + 1])


def _scale(p: float) -> float:
    return 1.0 / (1.0 - p) if p > 0 else 1.0


# ===================================================================================== user
@dataclass
class LayerSaved:
    x: Tensor          # layer input (fp32 residual)
    a1: Tensor         # LN1(x)        (compute dtype)
    m1: Tensor
    r1: Tensor
    qkv: Tensor        # (compute dtype)
    ctx: Tensor        # attention output (compute dtype)
    lse: Tensor
    x1: Tensor         # after attention residual (fp32)
    a2: Tensor         # LN2(x1)
    m2: Tensor
    r2: Tensor
    h: Tensor          # dropout(relu(linear1)) (compute dtype)
    rows: Optional[Tensor] = None   # pruned layer: int32 [B] gathered rows (x1/a2/h/ctx are [B,*])


@dataclass
class UserSaved:
    ids: Tensor
    key_valid: Tensor
    gender: Tensor
    country: Tensor
    m0: Tensor
    r0: Tensor
    layers: List[LayerSaved] = field(default_factory=list)
    comb: Optional[Tensor] = None
    rows: Optional[Tensor] = None
    z: Optional[Tensor] = None
    mz: Optional[Tensor] = None
    rz: Optional[Tensor] = None
    az: Optional[Tensor] = None
    seeds: Optional[Tensor] = None
    normed: bool = False          # the fused head also wrote InfoNCE's l2norm of u


def transposed_name(name: str) -> str:
    """Key of the transposed bf16 weight mirror (k-major operand of the input-grad GEMM)."""
    return name + ".T"


def _dx(dy: Tensor, W: Dict[str, Tensor], name: str, out: Tensor, gate: Optional[Tensor] = None,
        gate_scale: float = 1.0) -> Tensor:
    """Input grad of an nn.Linear: dY · W.  Uses the transposed mirror when present (both
    operands k-major: the row-panel kernel), else reads W in its natural layout."""
    wt = W.get(transposed_name(name))
    if wt is not None:
        return ops.linear(dy, wt, None, out, gate=gate, gate_scale=gate_scale)
    return ops.linear_dx(dy, W[name], out, gate=gate, gate_scale=gate_scale)


def _ln_k_ok(D: int, K: int, M: int = 0) -> bool:
    """K a fused LayerNorm-epilogue GEMM takes at LayerNorm width D (ttmi_linear_ln_bwd /
    ttmi_linear_res_ln): D = 128 with W resident in LDS, D = 256 with W streamed (ABI 19), whose
    DMA offsets are 32-bit: its [M, K] bf16 operand must stay under 4 GB (else the unfused
    path runs)."""
    if D == 128:
        return K % 128 == 0 and 0 < K <= 512
    return D == 256 and K % 256 == 0 and 0 < K <= 1024 and M * K * 2 < (1 << 32)


def _ln_fusable(W: Dict[str, Tensor], pre: str, D: int, M: int) -> bool:
    """The layer's input-grad GEMMs can carry the LayerNorm backward in their epilogue:
    bf16 with the transposed weight mirrors present and the LayerNorm width 128 or 256."""
    wt1 = W.get(transposed_name(pre + "linear1.weight"))
    wti = W.get(transposed_name(pre + "self_attn.in_proj_weight"))
    return (wt1 is not None and wti is not None and _ln_k_ok(D, wt1.shape[1], M)
            and _ln_k_ok(D, wti.shape[1], M))


# The item head's stages A and C both inside the fused user head launch (C polling A's
# BatchNorm statistics in-launch, ttmi_user_item_head_fwd_ac) measured 104 us against 18 + 17 us
# for A beside the one-query attention and C beside the user head: off until that wait is fixed
_HEAD_AC = os.environ.get("TTMI_HEAD_AC", "0") == "1"


# the fused in_proj + attention launch (ttmi_qkv_attn_fwd); TTMI_NO_QA=1 restores the
# ttmi_linear + ttmi_mha_fwd pair (A/B measurements)
_QA = os.environ.get("TTMI_NO_QA", "0") != "1"


def _qa_ok(w_in: Tensor, a1: Tensor, L: int, H: int) -> bool:
    D = a1.shape[1]
    return (_QA and a1.dtype == torch.bfloat16 and w_in.dtype == torch.bfloat16
            and tuple(w_in.shape) == (3 * D, D) and w_in.is_contiguous() and a1.is_contiguous()
            and ops.qkv_attn_supported(a1.dtype, L, H, D // H))


# the attention sub-block in one launch (ttmi_attn_block_fwd); TTMI_NO_BLOCK=1 runs the
# out-projection + residual + norm2 as its own launch (A/B measurements)
_BLOCK = os.environ.get("TTMI_NO_BLOCK", "0") != "1"

# the pruned layer's query projected inside the one-query attention (ttmi_mha_q1_proj_gather_fwd);
# TTMI_NO_Q1PROJ=1 restores the full 384-column projection (A/B measurements)
_Q1PROJ = os.environ.get("TTMI_NO_Q1PROJ", "0") != "1"


def _q1_proj_ok(w_in: Tensor, a1: Tensor, L: int, H: int) -> bool:
    D = a1.shape[1]
    return (_Q1PROJ and a1.dtype == torch.bfloat16 and w_in.dtype == torch.bfloat16 and D == 128
            and H * 32 == D and L <= 64 and tuple(w_in.shape) == (3 * D, D) and w_in.is_contiguous()
            and a1.is_contiguous())


# the attention backward computes dctx from dy1 itself (ttmi_mha_bwd_dy); TTMI_NO_DYATT=1
# restores the out-projection input-grad launch (A/B measurements)
_DYATT = os.environ.get("TTMI_NO_DYATT", "0") != "1"


# the pruned layer's K / V-only in_proj input grad (ttmi_mha_q1_kv_bwd + dy_add); TTMI_NO_KVB=1
# restores the full-dqkv form (A/B measurements)
_KVB = os.environ.get("TTMI_NO_KVB", "0") != "1"

# the feed-forward sub-block in one launch (ttmi_ffn_block_fwd); TTMI_NO_FFN=1 runs the FFN1
# row panel + ttmi_linear_res_ln pair (A/B measurements)
_FFN = os.environ.get("TTMI_NO_FFN", "0") != "1"

# the pruned layer's K / V projection inside the previous layer's FFN block (ABI 22);
# TTMI_NO_FFN_KV=1 runs it as its own row-panel launch (A/B measurements)
_FFN_KV = os.environ.get("TTMI_NO_FFN_KV", "0") != "1"


def _lp(i: int) -> str:
    return f"transformer_encoder.layers.{i}."


def _resln_ok(W: Dict[str, Tensor], name: str, D: int, M: int) -> bool:
    """The Linear `name` can end its residual sub-block with the following LayerNorm fused
    (ttmi_linear_res_ln): bf16 weight [D, K], D = 128 (K % 128 == 0, K <= 512) or D = 256
    (K in {256, 512, 768, 1024}) over M rows."""
    w = W[name]
    return w.dtype == torch.bfloat16 and w.shape[0] == D and _ln_k_ok(D, w.shape[1], M)


def user_tower_fwd(P: Dict[str, Tensor], W: Dict[str, Tensor], ids: Tensor, gender: Tensor,
                   country: Tensor, mask: Optional[Tensor], cfg: TowerCfg,
                   seeds: Optional[Tensor] = None, co_item: Optional["ItemHeadPending"] = None,
                   normed: Optional[Tuple[Tensor, Tensor]] = None):
    """SequentialUserEncoder.forward (reference user_tower.py:73-144), train mode.  ``co_item``
    (item_fusion_fwd_begin): the item head's first stage rides in the fused user head launch
    when that path runs (``co_item.a_done`` tells item_fusion_fwd_end).  ``normed`` = (u_hat,
    norms[:B]): that launch also writes InfoNCE's l2norm of u (``st.normed`` says so)."""
    dev = ids.device
    B, L = ids.shape
    D, H, dt = cfg.D, cfg.H, cfg.dtype
    M = B * L
    key_valid = ids if mask is None else mask
    if key_valid.dtype != torch.int64:
        key_valid = key_valid.to(torch.int64)
    f32 = dict(device=dev, dtype=torch.float32)
    x = torch.empty(M, D, **f32)
    m0 = torch.empty(M, **f32)
    r0 = torch.empty(M, **f32)

    def ln_out(R: int):
        return (torch.empty(R, D, device=dev, dtype=dt), torch.empty(R, **f32),
                torch.empty(R, **f32))

    # nxt: the next layer's norm1 output (a1, m1, r1) when a fused kernel already produced it;
    # nxt_qkv: the next (pruned) layer's qkv buffer whose K / V columns it also produced
    nxt = None
    nxt_qkv = None
    norm1 = None
    if cfg.n_layers > 0 and dt == torch.bfloat16:
        nxt = ln_out(M)
        norm1 = (P[_lp(0) + "norm1.weight"], P[_lp(0) + "norm1.bias"], cfg.eps) + nxt
    ops.seq_embed_fwd(ids, P["item_embedding.weight"], P["position_embedding.weight"],
                      P["layer_norm.weight"], P["layer_norm.bias"], x, m0, r0, eps=cfg.eps,
                      drop=_drop(cfg, seeds, SITE_EMB), norm1=norm1)
    st = UserSaved(ids=ids, key_valid=key_valid, gender=gender, country=country, m0=m0, r0=r0,
                   seeds=seeds)
    for i in range(cfg.n_layers):
        pre = _lp(i)
        pruned = cfg.prune_last and i == cfg.n_layers - 1
        if nxt is not None:
            (a1, m1, r1), nxt = nxt, None
        else:
            a1, m1, r1 = ln_out(M)
            ops.layernorm_fwd(x, P[pre + "norm1.weight"], P[pre + "norm1.bias"], a1, m1, r1, eps=cfg.eps)
        w_in, b_in = W[pre + "self_attn.in_proj_weight"], P[pre + "self_attn.in_proj_bias"]
        fused_qa = not pruned and _qa_ok(w_in, a1, L, H)
        # the pruned layer reads Q at the gathered rows only: K / V over every row (a 256-column
        # projection: inside the previous layer's FFN block launch when that ran, ABI 22), Q
        # inside the one-query attention launch (ABI 21)
        proj_q1 = pruned and _q1_proj_ok(w_in, a1, L, H)
        if nxt_qkv is not None:
            qkv, nxt_qkv = nxt_qkv, None
        else:
            qkv = torch.empty(M, 3 * D, device=dev, dtype=dt)
            if proj_q1:
                ops.gemm(a1, w_in[D:], qkv[:, D:], M, 2 * D, D, lda=D, a_kmajor=True, ldb=D, b_kmajor=True,
                         ldc=3 * D, bias=b_in[D:])
            elif not fused_qa:
                ops.linear(a1, w_in, b_in, qkv)
        F_ = W[pre + "linear1.weight"].shape[0]
        if pruned:
            rows = torch.empty(B, device=dev, dtype=torch.int32)
            R, res_in, drows = B, torch.empty(B, D, **f32), rows
            ctx = torch.empty(B, D, device=dev, dtype=dt)
            lse = torch.empty(B * H, **f32)
            # the last-valid rows, their residual rows and the one-query attention: one launch
            # (with the item head's stage A on the same grid when its BatchNorm statistics are
            # merged in-launch: stage C then rides in the user head launch, ABI 18)
            # (the item head's two stages ride in the fused user head launch, stage C waiting
            # in-launch for stage A's BatchNorm statistics, ABI 18; without the fused head, stage
            # A rides on this grid instead)
            head_fused = ops.user_head_fusable(W, P, pre, D, dt)
            co_ac = co_item is not None and co_item.bn_fused and head_fused and _HEAD_AC
            co_a = co_item is not None and co_item.bn_fused and L <= 64 and not co_ac
            if proj_q1:
                ops.mha_q1_proj_gather_fwd(qkv, key_valid, a1, w_in[:D], b_in[:D], x, rows, res_in, B, L,
                                           H, ctx, lse, _drop(cfg, seeds, site_attn(i)),
                                           co_item=co_item.desc if co_a else None)
            else:
                ops.mha_q1_gather_fwd(qkv, key_valid, x, rows, res_in, B, L, H, ctx, lse,
                                      _drop(cfg, seeds, site_attn(i)),
                                      co_item=co_item.desc if co_a else None)
            if co_a:
                co_item.a_done = True
            if head_fused:      # the rest of the tower: one launch
                F_ = W[pre + "linear1.weight"].shape[0]
                Wc = D + P["gender_embedding.weight"].shape[1] + P["country_embedding.weight"].shape[1]
                o = dict(x1=torch.empty(B, D, **f32), a2=torch.empty(B, D, device=dev, dtype=dt),
                         m2=torch.empty(B, **f32), r2=torch.empty(B, **f32),
                         h=torch.empty(B, F_, device=dev, dtype=dt),
                         comb=torch.empty(B, Wc, device=dev, dtype=dt),
                         rows=torch.empty(B, device=dev, dtype=torch.int32),
                         z=torch.empty(B, D, **f32), az=torch.empty(B, D, device=dev, dtype=dt),
                         mz=torch.empty(B, **f32), rz=torch.empty(B, **f32), u=torch.empty(B, D, **f32))
                ops.user_head_fwd(ctx, res_in, drows, W, P, pre, gender, country, cfg.eps,
                                  (_drop(cfg, seeds, site_drop1(i)), _drop(cfg, seeds, site_ffn(i)),
                                   _drop(cfg, seeds, site_drop2(i))), o,
                                  co_item=co_item.desc if co_item is not None else None,
                                  normed=normed,
                                  co_stage="AC" if co_ac else ("C" if co_a else "A"))
                if co_item is not None:
                    co_item.c_done = co_ac or co_a
                    co_item.a_done = True
                st.normed = normed is not None
                st.layers.append(LayerSaved(x, a1, m1, r1, qkv, ctx, lse, o["x1"], o["a2"], o["m2"],
                                            o["r2"], o["h"], rows))
                st.comb, st.rows, st.z = o["comb"], o["rows"], o["z"]
                st.mz, st.rz, st.az = o["mz"], o["rz"], o["az"]
                return o["u"], st
        else:
            rows, R, res_in, drows = None, M, x, None
            ctx = torch.empty(M, D, device=dev, dtype=dt)
            lse = torch.empty(B * H * L, **f32)
        x1 = torch.empty(R, D, **f32)
        a2, m2, r2 = ln_out(R)
        name = pre + "self_attn.out_proj.weight"
        block = (not pruned and fused_qa and _BLOCK and 38 <= L <= 64 and W[name].dtype == torch.bfloat16
                 and tuple(W[name].shape) == (D, D))
        if not pruned:
            if block:        # in_proj + attention + out_proj + residual + norm2, one launch
                ops.attn_block_fwd(a1, w_in, b_in, key_valid, B, L, H, qkv, ctx, lse,
                                   _drop(cfg, seeds, site_attn(i)), W[name], P[pre + "self_attn.out_proj.bias"],
                                   res_in, P[pre + "norm2.weight"], P[pre + "norm2.bias"], cfg.eps,
                                   _drop(cfg, seeds, site_drop1(i)), x1, a2, m2, r2)
            elif fused_qa:   # in_proj + attention, one launch (bit-identical to the pair at M >= 2048)
                ops.qkv_attn_fwd(a1, w_in, b_in, key_valid, B, L, H, qkv, ctx, lse,
                                 _drop(cfg, seeds, site_attn(i)))
            elif ops.mha_tuned_supported(L, D // H):
                ops.mha_fwd(qkv, key_valid, B, L, H, ctx, lse, _drop(cfg, seeds, site_attn(i)))
            else:            # head widths / lengths the tuned kernels refuse (the constructor unprunes)
                ops.mha_generic_fwd(qkv, key_valid, B, L, H, ctx, lse, _drop(cfg, seeds, site_attn(i)))
        if block:
            pass
        elif not pruned and _resln_ok(W, name, D, R):    # out_proj + residual + norm2, one kernel
            ops.linear_res_ln(ctx, W[name], P[pre + "self_attn.out_proj.bias"], res_in, x1,
                              P[pre + "norm2.weight"], P[pre + "norm2.bias"], a2, m2, r2,
                              eps=cfg.eps, drop=_drop(cfg, seeds, site_drop1(i)))
        else:
            ops.linear(ctx, W[name], P[pre + "self_attn.out_proj.bias"], x1,
                       drop=_drop(cfg, seeds, site_drop1(i)), residual=res_in, drop_rows=drows)
            ops.layernorm_fwd(x1, P[pre + "norm2.weight"], P[pre + "norm2.bias"], a2, m2, r2, eps=cfg.eps)
        h = torch.empty(R, F_, device=dev, dtype=dt)
        x2 = torch.empty(R, D, **f32)
        name = pre + "linear2.weight"
        w1 = W[pre + "linear1.weight"]
        if (not pruned and i + 1 < cfg.n_layers and _FFN and w1.dtype == torch.bfloat16
                and W[name].dtype == torch.bfloat16 and R * F_ * 2 < (1 << 30)
                and ops.ffn_block_supported(dt, D, F_)):
            # FFN1 + ReLU / dropout + FFN2 + residual + the next layer's norm1, one launch; when the
            # next layer is the pruned one, its K / V projection too
            nxt = ln_out(M)
            nx = _lp(i + 1)
            kv = None
            w_nx = W[nx + "self_attn.in_proj_weight"]
            if (_FFN_KV and cfg.prune_last and i + 1 == cfg.n_layers - 1
                    and _q1_proj_ok(w_nx, nxt[0], L, H)):
                nxt_qkv = torch.empty(M, 3 * D, device=dev, dtype=dt)
                kv = (w_nx[D:], P[nx + "self_attn.in_proj_bias"][D:], nxt_qkv[:, D:])
            ops.ffn_block_fwd(a2, w1, P[pre + "linear1.bias"], W[name], P[pre + "linear2.bias"], x1,
                              _drop(cfg, seeds, site_ffn(i)), _drop(cfg, seeds, site_drop2(i)), h, x2,
                              P[nx + "norm1.weight"], P[nx + "norm1.bias"], cfg.eps, *nxt, kv=kv)
            st.layers.append(LayerSaved(x, a1, m1, r1, qkv, ctx, lse, x1, a2, m2, r2, h, rows))
            x = x2
            continue
        ops.linear(a2, w1, P[pre + "linear1.bias"], h, act=1,
                   drop=_drop(cfg, seeds, site_ffn(i)), drop_rows=drows)
        if not pruned and i + 1 < cfg.n_layers and _resln_ok(W, name, D, R):
            # linear2 + residual + the next layer's norm1, one kernel
            nxt = ln_out(M)
            nx = _lp(i + 1)
            ops.linear_res_ln(h, W[name], P[pre + "linear2.bias"], x1, x2, P[nx + "norm1.weight"],
                              P[nx + "norm1.bias"], *nxt, eps=cfg.eps,
                              drop=_drop(cfg, seeds, site_drop2(i)))
        else:
            ops.linear(h, W[name], P[pre + "linear2.bias"], x2,
                       drop=_drop(cfg, seeds, site_drop2(i)), residual=x1, drop_rows=drows)
        st.layers.append(LayerSaved(x, a1, m1, r1, qkv, ctx, lse, x1, a2, m2, r2, h, rows))
        x = x2
    gathered = cfg.prune_last and cfg.n_layers > 0
    G = P["gender_embedding.weight"]
    C = P["country_embedding.weight"]
    comb = torch.empty(B, D + G.shape[1] + C.shape[1], device=dev, dtype=dt)
    rows = torch.empty(B, device=dev, dtype=torch.int32)
    if gathered:   # x is already [B, D] (the pruned last layer's gathered rows)
        ops.user_concat_fwd(x, None, gender, G, country, C, comb, rows, B, 1)
    else:
        ops.user_concat_fwd(x, key_valid, gender, G, country, C, comb, rows, B, L)
    z = torch.empty(B, D, **f32)
    ops.linear(comb, W["fusion_layer.0.weight"], P["fusion_layer.0.bias"], z)
    az = torch.empty(B, D, device=dev, dtype=dt)
    mz = torch.empty(B, **f32)
    rz = torch.empty(B, **f32)
    ops.layernorm_fwd(z, P["fusion_layer.1.weight"], P["fusion_layer.1.bias"], az, mz, rz,
                      eps=cfg.eps, relu=True)
    u = torch.empty(B, D, **f32)
    ops.linear(az, W["fusion_layer.3.weight"], P["fusion_layer.3.bias"], u)
    st.comb, st.rows, st.z, st.mz, st.rz, st.az = comb, rows, z, mz, rz, az
    return u, st


def user_tower_bwd(P: Dict[str, Tensor], W: Dict[str, Tensor], st: UserSaved, du: Tensor,
                   grads: Dict[str, Tensor], cfg: TowerCfg, du16: Optional[Tensor] = None,
                   on_layer_done: Optional[Callable[[int], None]] = None,
                   co_item: Optional["ItemBwdPending"] = None) -> None:
    """Backward of user_tower_fwd; accumulates into ``grads`` (fp32, reference names).  du16:
    du already in the compute dtype (InfoNCE backward's bf16 copy), saving the cast launch.
    ``on_layer_done(i)`` is called once encoder layer i's parameter gradients are final (the
    data-parallel step starts a bucket's all-reduce there).  ``co_item``
    (item_fusion_bwd_begin): the item head's row-local backward rides in the fused user head
    launch when that path runs; item_fusion_bwd_end(co_item) runs right after the head, before
    any encoder layer, so the item gradients are final by the first ``on_layer_done``."""
    dev = du.device
    B, L = st.ids.shape
    D, H, dt = cfg.D, cfg.H, cfg.dtype
    M = B * L
    seeds = st.seeds
    f32 = dict(device=dev, dtype=torch.float32)
    gathered = cfg.prune_last and cfg.n_layers > 0
    G = P["gender_embedding.weight"]
    C = P["country_embedding.weight"]
    head = None
    last = _lp(cfg.n_layers - 1) if cfg.n_layers > 0 else ""
    if gathered and du16 is not None and du16.dtype == torch.bfloat16 and \
            ops.user_head_fusable(W, P, last, D, dt) and ops.user_head_bwd_fusable(W, last):
        # the head's backward (fusion MLP, concat, the pruned layer's FFN / LN2 / out_proj input
        # grads) in one launch; its weight gradients are the same deferred GEMMs
        i = cfg.n_layers - 1
        s = st.layers[i]
        saved = dict(az=st.az, z=st.z, mz=st.mz, rz=st.rz, h=s.h, x1=s.x1, m2=s.m2, r2=s.r2)
        head = ops.user_head_bwd(
            du16, saved, s.rows, W, P, last, st.gender, st.country, _scale(cfg.p_drop),
            (_drop(cfg, seeds, site_drop1(i)), _drop(cfg, seeds, site_drop2(i))),
            grads["gender_embedding.weight"], grads["country_embedding.weight"],
            (grads["fusion_layer.1.weight"], grads["fusion_layer.1.bias"],
             grads[last + "norm2.weight"], grads[last + "norm2.bias"]),
            co_item=co_item.desc if co_item is not None else None)
        if co_item is not None:
            co_item.done = True
        ops.linear_dw(du16, st.az, grads["fusion_layer.3.weight"], grads["fusion_layer.3.bias"])
        ops.linear_dw(head["dz16"], st.comb, grads["fusion_layer.0.weight"], grads["fusion_layer.0.bias"])
        ops.linear_dw(head["dy2"], s.h, grads[last + "linear2.weight"], grads[last + "linear2.bias"])
        ops.linear_dw(head["dz1"], s.a2, grads[last + "linear1.weight"], grads[last + "linear1.bias"])
        ops.linear_dw(head["dy1"], s.ctx, grads[last + "self_attn.out_proj.weight"],
                      grads[last + "self_attn.out_proj.bias"])
        dx = None
    else:
        dx = _head_bwd_unfused(P, W, st, du, grads, cfg, du16, gathered)
    bn_co = None       # the item BatchNorm backward, on the pruned layer's one-query grid
    if co_item is not None:
        bn_co = item_fusion_bwd_end(co_item, defer_bn=gathered and L <= 64)
    # ---- encoder layers, reversed (user_tower.py:37-45)
    p = cfg.p_drop
    dy2_next = None        # layer i's dy2, emitted by layer i+1's fused LN1 backward
    for i in reversed(range(cfg.n_layers)):
        pre = _lp(i)
        s = st.layers[i]
        R = s.x1.shape[0]                 # B for the pruned layer, M otherwise
        drows = s.rows
        F_ = W[pre + "linear1.weight"].shape[0]
        fuse = _ln_fusable(W, pre, D, R)
        # the attention backward computes dctx = dy1·W_o itself (ttmi_mha_bwd_dy, ABI 21)
        wot = W.get(transposed_name(pre + "self_attn.out_proj.weight"))
        dy_attn = (_DYATT and drows is None and dt == torch.bfloat16 and D == 128 and H == 4 and L <= 64
                   and wot is not None and not (head is not None and i == cfg.n_layers - 1))
        if head is not None and i == cfg.n_layers - 1:
            dctx, dx1 = head["dctx"], head["dx1"]
        else:
            dx1, dctx, dy2_next = _layer_tail_bwd(P, W, s, dx, dy2_next, grads, cfg, seeds, i, pre,
                                                  R, drows, F_, fuse, D, dt, p, want_dctx=not dy_attn)
        dqkv = torch.empty(M, 3 * D, device=dev, dtype=dt)
        wti = W.get(transposed_name(pre + "self_attn.in_proj_weight"))
        # the pruned layer's dQ lives on its B gathered rows only: its in_proj input grad runs
        # on the K / V columns (K = 256) with dq·W_q added to those rows' dY in the LN1 backward,
        # and the Q rows' weight gradient is a B-row GEMM (ABI 21)
        kv_only = (drows is not None and fuse and _KVB and dt == torch.bfloat16 and D == 128 and H == 4
                   and L <= 64 and wti is not None and wti.dtype == torch.bfloat16)
        if kv_only:
            dq_g = torch.empty(B, D, device=dev, dtype=dt)
            a_g = torch.empty(B, D, device=dev, dtype=dt)
            dyq = torch.empty(B, D, **f32)
            ops.mha_q1_kv_bwd(s.qkv, st.key_valid, drows, s.lse, dctx, B, L, H, dqkv,
                              _drop(cfg, seeds, site_attn(i)), wti, s.a1, dq_g, a_g, dyq,
                              bn=bn_co.desc if bn_co else None)
            if bn_co is not None:
                bn_co.finish()
                bn_co = None
        elif drows is not None:
            ops.mha_q1_bwd(s.qkv, st.key_valid, drows, s.lse, dctx, B, L, H, dqkv,
                           _drop(cfg, seeds, site_attn(i)), bn=bn_co.desc if bn_co else None)
            if bn_co is not None:
                bn_co.finish()
                bn_co = None
        elif dy_attn:      # (dctx holds dy1 here)
            ops.mha_bwd_dy(s.qkv, st.key_valid, s.lse, dctx, wot, B, L, H, dqkv,
                           _drop(cfg, seeds, site_attn(i)))
        elif ops.mha_tuned_supported(L, D // H):
            ops.mha_bwd(s.qkv, st.key_valid, s.lse, dctx, B, L, H, dqkv,
                        _drop(cfg, seeds, site_attn(i)))
        else:
            ops.mha_generic_bwd(s.qkv, st.key_valid, s.lse, s.ctx, dctx, B, L, H, dqkv,
                                _drop(cfg, seeds, site_attn(i)))
        gw_in, gb_in = grads[pre + "self_attn.in_proj_weight"], grads[pre + "self_attn.in_proj_bias"]
        if kv_only:
            ops.linear_dw(dqkv[:, D:], s.a1, gw_in[D:], gb_in[D:])
            ops.linear_dw(dq_g, a_g, gw_in[:D], gb_in[:D])
        else:
            ops.linear_dw(dqkv, s.a1, gw_in, gb_in)
        dxn = torch.empty(M, D, **f32)
        if fuse:     # in_proj input grad + LN1 backward (+ the layer below's dropout2 backward);
            # the pruned layer's residual grad dx1 [B, D] lands on its gathered rows in-kernel
            emit = i > 0
            nxt = torch.empty(M, D, device=dev, dtype=dt) if emit else None
            ops.linear_ln_bwd(dqkv[:, D:] if kv_only else dqkv, wti[:, D:] if kv_only else wti, s.x,
                              s.m1, s.r1, P[pre + "norm1.weight"], dxn,
                              grads[pre + "norm1.weight"], grads[pre + "norm1.bias"],
                              res=dx1, res_rows=drows, res_L=L if drows is not None else 0,
                              next_=nxt,
                              drop=_drop(cfg, seeds, site_drop2(i - 1)) if emit else ops.NO_DROP,
                              dy_add=dyq if kv_only else None)
            dy2_next = nxt
        else:
            da1 = torch.empty(M, D, **f32)
            _dx(dqkv, W, pre + "self_attn.in_proj_weight", da1)
            if drows is not None:
                ops.layernorm_bwd(da1, s.x, s.m1, s.r1, P[pre + "norm1.weight"], dxn,
                                  grads[pre + "norm1.weight"], grads[pre + "norm1.bias"])
                ops.scatter_add_rows(dx1, drows, dxn)      # residual path of the gathered rows
            else:
                ops.layernorm_bwd(da1, s.x, s.m1, s.r1, P[pre + "norm1.weight"], dxn,
                                  grads[pre + "norm1.weight"], grads[pre + "norm1.bias"], res=dx1)
        dx = dxn
        if bn_co is not None:         # no one-query launch carried it
            ops.bn_bwd_run(bn_co.desc)
            bn_co.finish()
            bn_co = None
        if on_layer_done is not None:
            on_layer_done(i)
    # ---- input block (user_tower.py:83-93)
    # every weight gradient is recorded: the grouped GEMMs run on a side stream beside the
    # input block's backward (its 4-wave, 2 KB-LDS workgroups fit beside theirs on a CU)
    ops.wgrad_launch_early()
    ops.seq_embed_bwd(st.ids, P["item_embedding.weight"], P["position_embedding.weight"],
                      P["layer_norm.weight"], st.m0, st.r0, dx, grads["item_embedding.weight"],
                      grads["position_embedding.weight"], grads["layer_norm.weight"],
                      grads["layer_norm.bias"], drop=_drop(cfg, seeds, SITE_EMB), padding_idx=0)


def _head_bwd_unfused(P, W, st, du, grads, cfg, du16, gathered):
    """The user fusion MLP and concat backward as separate launches; returns dx (the grad of
    the last encoder layer's output rows)."""
    dev = du.device
    B, L = st.ids.shape
    D, dt = cfg.D, cfg.dtype
    M = B * L
    f32 = dict(device=dev, dtype=torch.float32)
    # ---- user fusion MLP (user_tower.py:51-57, :142)
    if du16 is not None and du16.dtype == dt:
        du_c = du16
    else:
        du_c = torch.empty(B, D, device=dev, dtype=dt)
        ops.dropout_bwd(du, du_c, None)
    ops.linear_dw(du_c, st.az, grads["fusion_layer.3.weight"], grads["fusion_layer.3.bias"])
    daz = torch.empty(B, D, **f32)
    ops.linear_dx(du_c, W["fusion_layer.3.weight"], daz)
    dz = torch.empty(B, D, **f32)
    dz_c = torch.empty(B, D, device=dev, dtype=dt)
    ops.layernorm_bwd(daz, st.z, st.mz, st.rz, P["fusion_layer.1.weight"], dz,
                      grads["fusion_layer.1.weight"], grads["fusion_layer.1.bias"], gate=st.az,
                      dx16=dz_c if dt == torch.bfloat16 else None)
    if dt != torch.bfloat16:
        ops.dropout_bwd(dz, dz_c, None)
    ops.linear_dw(dz_c, st.comb, grads["fusion_layer.0.weight"], grads["fusion_layer.0.bias"])
    dcomb = torch.empty(B, st.comb.shape[1], **f32)
    ops.linear_dx(dz_c, W["fusion_layer.0.weight"], dcomb)
    gathered = cfg.prune_last and cfg.n_layers > 0
    # gathered: every row of dx [B, D] is written once (no zero fill); else only B of M rows
    dx = torch.empty(B, D, **f32) if gathered else torch.zeros(M, D, **f32)
    G = P["gender_embedding.weight"]
    C = P["country_embedding.weight"]
    ops.user_concat_bwd(dcomb, st.rows, st.gender, G.shape[1], st.country, C.shape[1], dx,
                        grads["gender_embedding.weight"], grads["country_embedding.weight"],
                        accumulate=not gathered, n_tables=(G.shape[0], C.shape[0]))
    return dx


def _layer_tail_bwd(P, W, s, dx, dy2_next, grads, cfg, seeds, i, pre, R, drows, F_, fuse, D, dt, p,
                    want_dctx=True):
    """One encoder layer's backward from its output grad dx down to dctx (FFN, LN2, residual,
    out_proj input grad).  Returns dx1 (the grad of the attention residual), dctx and the
    pending dy2 (None).  ``want_dctx`` False: dctx is left to the attention backward
    (ttmi_mha_bwd_dy) and dy1, the out-projection's output grad, is returned in its place."""
    dev = dx.device
    f32 = dict(device=dev, dtype=torch.float32)
    if dy2_next is not None:
        dy2 = dy2_next
    else:
        dy2 = torch.empty(R, D, device=dev, dtype=dt)
        ops.dropout_bwd(dx, dy2, None, _drop(cfg, seeds, site_drop2(i)), drop_rows=drows)
    ops.linear_dw(dy2, s.h, grads[pre + "linear2.weight"], grads[pre + "linear2.bias"])
    dz1 = torch.empty(R, F_, device=dev, dtype=dt)
    w2t = W.get(transposed_name(pre + "linear2.weight"))
    w1t = W.get(transposed_name(pre + "linear1.weight"))
    if (fuse and drows is None and _FFN and dt == torch.bfloat16 and w2t is not None and w1t is not None
            and w2t.dtype == torch.bfloat16 and w1t.dtype == torch.bfloat16 and R * F_ * 2 < (1 << 30)
            and D == 128 and ops.ffn_block_supported(dt, D, F_, bwd=True)):
        # (D = 256: the fused backward is served but measured slower than the pair)
        # FFN2 input grad + ReLU / dropout gate + FFN1 input grad + norm2 backward, one launch
        dx1 = torch.empty(R, D, **f32)
        dy1 = torch.empty(R, D, device=dev, dtype=dt)
        ops.ffn_block_bwd(dy2, w2t, w1t, s.h, _scale(p), dz1, s.x1, s.m2, s.r2, P[pre + "norm2.weight"], dx,
                          dx1, dy1, _drop(cfg, seeds, site_drop1(i)), grads[pre + "norm2.weight"],
                          grads[pre + "norm2.bias"])
        ops.linear_dw(dz1, s.a2, grads[pre + "linear1.weight"], grads[pre + "linear1.bias"])
        ops.linear_dw(dy1, s.ctx, grads[pre + "self_attn.out_proj.weight"],
                      grads[pre + "self_attn.out_proj.bias"])
        if not want_dctx:
            return dx1, dy1, None
        dctx = torch.empty(R, D, device=dev, dtype=dt)
        _dx(dy1, W, pre + "self_attn.out_proj.weight", dctx)
        return dx1, dctx, None
    _dx(dy2, W, pre + "linear2.weight", dz1, gate=s.h, gate_scale=_scale(p))
    ops.linear_dw(dz1, s.a2, grads[pre + "linear1.weight"], grads[pre + "linear1.bias"])
    dx1 = torch.empty(R, D, **f32)
    dy1 = torch.empty(R, D, device=dev, dtype=dt)
    if fuse:     # linear1 input grad + LN2 backward + dropout1 backward, one kernel
        ops.linear_ln_bwd(dz1, W[transposed_name(pre + "linear1.weight")], s.x1, s.m2, s.r2,
                          P[pre + "norm2.weight"], dx1, grads[pre + "norm2.weight"],
                          grads[pre + "norm2.bias"], res=dx, next_=dy1,
                          drop=_drop(cfg, seeds, site_drop1(i)), drop_rows=drows)
    else:
        da2 = torch.empty(R, D, **f32)
        _dx(dz1, W, pre + "linear1.weight", da2)
        ops.layernorm_bwd(da2, s.x1, s.m2, s.r2, P[pre + "norm2.weight"], dx1,
                          grads[pre + "norm2.weight"], grads[pre + "norm2.bias"], res=dx)
        ops.dropout_bwd(dx1, dy1, None, _drop(cfg, seeds, site_drop1(i)), drop_rows=drows)
    ops.linear_dw(dy1, s.ctx, grads[pre + "self_attn.out_proj.weight"],
                  grads[pre + "self_attn.out_proj.bias"])
    if not want_dctx:
        return dx1, dy1, None
    dctx = torch.empty(R, D, device=dev, dtype=dt)
    _dx(dy1, W, pre + "self_attn.out_proj.weight", dctx)
    return dx1, dctx, None


# ===================================================================================== item
@dataclass
class ItemSaved:
    modal: Tensor      # fusion input in compute dtype
    z: Tensor
    bn_mean: Tensor
    bn_rstd: Tensor
    y1: Tensor
    y2: Tensor
    m5: Tensor
    r5: Tensor
    seeds: Optional[Tensor] = None


def item_fusion_fwd(P: Dict[str, Tensor], W: Dict[str, Tensor], modal: Tensor, cfg: TowerCfg,
                    seeds: Optional[Tensor] = None,
                    buffers: Optional[Dict[str, Tensor]] = None, p_drop: float = 0.1,
                    training: bool = True):
    """MultimodalItemEncoder fusion head (reference item_tower.py:122-129, :147-150) on the
    concatenated [audio, visual, text, tabular] embeddings ``modal`` [B, 512] (fp32)."""
    dev = modal.device
    B = modal.shape[0]
    dt = cfg.dtype
    f32 = dict(device=dev, dtype=torch.float32)
    bufs = buffers or {}
    if training and ops.item_head_fusable(W, modal, dt):
        # the whole MLP in three launches (cast + Linear; BatchNorm + ReLU + dropout; Linear +
        # LayerNorm), saving what the unfused ops below save
        H1, D = W["fusion_layer.0.weight"].shape[0], W["fusion_layer.4.weight"].shape[0]
        o = dict(m16=torch.empty(modal.shape, device=dev, dtype=dt), z=torch.empty(B, H1, **f32),
                 bn_mean=torch.empty(H1, **f32), bn_rstd=torch.empty(H1, **f32),
                 y1=torch.empty(B, H1, device=dev, dtype=dt), y2=torch.empty(B, D, **f32),
                 out=torch.empty(B, D, **f32), m5=torch.empty(B, **f32), r5=torch.empty(B, **f32))
        ops.item_head_fwd(modal.contiguous(), W, P, bufs, _drop(cfg, seeds, SITE_ITEM, p_drop), cfg.eps, o)
        return o["out"], ItemSaved(o["m16"], o["z"], o["bn_mean"], o["bn_rstd"], o["y1"], o["y2"],
                                   o["m5"], o["r5"], seeds)
    if dt == torch.float32:
        m_c = modal.contiguous()
    else:
        m_c = ops.cast_bf16(modal.contiguous(), torch.empty(modal.shape, device=dev, dtype=dt))
    H1 = W["fusion_layer.0.weight"].shape[0]
    z = torch.empty(B, H1, **f32)
    ops.linear(m_c, W["fusion_layer.0.weight"], P["fusion_layer.0.bias"], z)
    y1 = torch.empty(B, H1, device=dev, dtype=dt)
    bn_mean = torch.empty(H1, **f32)
    bn_rstd = torch.empty(H1, **f32)
    ops.batchnorm_fwd(z, P["fusion_layer.1.weight"], P["fusion_layer.1.bias"], y1, bn_mean, bn_rstd,
                      bufs.get("fusion_layer.1.running_mean"), bufs.get("fusion_layer.1.running_var"),
                      bufs.get("fusion_layer.1.num_batches_tracked"), relu=True,
                      drop=_drop(cfg, seeds, SITE_ITEM, p_drop), training=training)
    D = W["fusion_layer.4.weight"].shape[0]
    y2 = torch.empty(B, D, **f32)
    ops.linear(y1, W["fusion_layer.4.weight"], P["fusion_layer.4.bias"], y2)
    out = torch.empty(B, D, **f32)
    m5 = torch.empty(B, **f32)
    r5 = torch.empty(B, **f32)
    ops.layernorm_fwd(y2, P["fusion_layer.5.weight"], P["fusion_layer.5.bias"], out, m5, r5,
                      eps=cfg.eps)
    return out, ItemSaved(m_c, z, bn_mean, bn_rstd, y1, y2, m5, r5, seeds)


@dataclass
class ItemHeadPending:
    """A training forward of the item fusion head split around the user head launch (ABI 15):
    item_fusion_fwd_begin builds the descriptor, user_tower_fwd(co_item=...) issues stage A
    inside the fused user head launch, item_fusion_fwd_end issues the rest."""
    desc: object
    o: Dict[str, Tensor]
    modal: Tensor
    seeds: Optional[Tensor]
    a_done: bool = False
    c_done: bool = False
    bn_fused: bool = False      # BatchNorm statistics merged in stage A (B <= 512)


def item_fusion_fwd_begin(P: Dict[str, Tensor], W: Dict[str, Tensor], modal: Tensor, cfg: TowerCfg,
                          seeds: Optional[Tensor] = None,
                          buffers: Optional[Dict[str, Tensor]] = None,
                          p_drop: float = 0.1,
                          normed: Optional[Tuple[Tensor, Tensor]] = None) -> Optional[ItemHeadPending]:
    """item_fusion_fwd (training) as a pending co-launch, or None when the fused head does not
    take these shapes (then call item_fusion_fwd).  ``normed`` = (i_hat, norms[B:]): stage C
    also writes InfoNCE's l2norm of the item embedding."""
    if not ops.item_head_fusable(W, modal, cfg.dtype):
        return None
    dev = modal.device
    B = modal.shape[0]
    f32 = dict(device=dev, dtype=torch.float32)
    H1, D = W["fusion_layer.0.weight"].shape[0], W["fusion_layer.4.weight"].shape[0]
    o = dict(m16=torch.empty(modal.shape, device=dev, dtype=cfg.dtype), z=torch.empty(B, H1, **f32),
             bn_mean=torch.empty(H1, **f32), bn_rstd=torch.empty(H1, **f32),
             y1=torch.empty(B, H1, device=dev, dtype=cfg.dtype), y2=torch.empty(B, D, **f32),
             out=torch.empty(B, D, **f32), m5=torch.empty(B, **f32), r5=torch.empty(B, **f32))
    if normed is not None:
        o["out_hat"], o["out_norm"] = normed
    m = modal.contiguous()
    d = ops.item_head_desc(m, W, P, buffers or {}, _drop(cfg, seeds, SITE_ITEM, p_drop), cfg.eps, o)
    return ItemHeadPending(d, o, m, seeds, bn_fused=bool(d.bn_part))


def item_fusion_fwd_end(pend: ItemHeadPending):
    """The pending forward's remaining stages; returns (out, ItemSaved) as item_fusion_fwd."""
    stages = (0 if pend.a_done else 1) | (0 if pend.c_done else 6)
    if stages:
        ops.item_head_fwd_stages(pend.desc, stages)
    o = pend.o
    return o["out"], ItemSaved(o["m16"], o["z"], o["bn_mean"], o["bn_rstd"], o["y1"], o["y2"],
                               o["m5"], o["r5"], pend.seeds)


@dataclass
class ItemBwdPending:
    """item_fusion_bwd split around the user head backward launch (ABI 15)."""
    desc: object
    keep: tuple
    dy2: Tensor
    dy1: Tensor
    ws: Tensor
    args: tuple
    done: bool = False


def item_fusion_bwd_begin(P: Dict[str, Tensor], W: Dict[str, Tensor], st: ItemSaved, dout: Tensor,
                          grads: Dict[str, Tensor], cfg: TowerCfg, p_drop: float = 0.1,
                          dmodal: Optional[Tensor] = None) -> Optional[ItemBwdPending]:
    """item_fusion_bwd as a pending co-launch (its LayerNorm backward and Linear-4 input grad
    in the user head backward launch), or None when the shapes or the W4ᵀ mirror are missing."""
    w4t = W.get(transposed_name("fusion_layer.4.weight"))
    B, D = dout.shape
    if cfg.dtype != torch.bfloat16 or w4t is None or D not in (128, 256) or tuple(w4t.shape) != (512, D) \
            or st.y2.dtype != torch.float32:
        return None
    dev = dout.device
    dy2 = torch.empty(B, D, device=dev, dtype=cfg.dtype)
    dy1 = torch.empty(B, w4t.shape[0], device=dev, dtype=torch.float32)
    ws = ops.item_head_bwd_ws(B, dev, D)
    dc = dout.contiguous()
    d = ops.item_head_bwd_desc(dc, st.y2, st.m5, st.r5, P["fusion_layer.5.weight"], w4t, dy2, dy1, ws)
    return ItemBwdPending(d, (dc, w4t), dy2, dy1, ws, (P, W, st, grads, cfg, p_drop, dmodal))


@dataclass
class ItemBnPending:
    """The item head's BatchNorm1d backward held back to ride on another launch's grid
    (ttmi_mha_q1_bnr_bwd, ABI 18): ``desc`` goes to ops.mha_q1_bwd(bn=...), then ``finish()``
    records what depends on it (fusion_layer.0's weight gradient, dmodal)."""
    desc: object
    keep: tuple
    finish: Callable[[], None]


def item_fusion_bwd_end(pend: ItemBwdPending, defer_bn: bool = False) -> Optional[ItemBnPending]:
    """The rest of item_fusion_bwd: the row-local launch if the user head did not carry it,
    the LayerNorm parameter sums, the weight gradients and the BatchNorm backward.  With
    ``defer_bn`` the BatchNorm backward (when its bf16 register path applies) is returned as an
    ItemBnPending for the caller to co-launch; otherwise None."""
    P, W, st, grads, cfg, p_drop, dmodal = pend.args
    if not pend.done:
        ops.item_head_bwd_c(pend.desc)
        pend.done = True
    D = pend.dy2.shape[1]
    ops.ln_sum_folds(pend.ws, (grads["fusion_layer.5.weight"], grads["fusion_layer.5.bias"]), 2, D)
    ops.linear_dw(pend.dy2, st.y1, grads["fusion_layer.4.weight"], grads["fusion_layer.4.bias"])
    if defer_bn and cfg.dtype == torch.bfloat16 and pend.dy1.shape[0] <= 512:
        return _item_bn_pending(P, W, st, pend.dy1, grads, cfg, p_drop, dmodal)
    _item_bwd_tail(P, W, st, pend.dy1, grads, cfg, p_drop, dmodal)
    return None


def _item_bn_pending(P, W, st: ItemSaved, dy1: Tensor, grads, cfg: TowerCfg, p_drop: float,
                     dmodal: Optional[Tensor]) -> ItemBnPending:
    """_item_bwd_tail split at its BatchNorm backward (bf16 register path, B <= 512)."""
    dev = dy1.device
    B, H1 = dy1.shape
    pd = p_drop if st.seeds is not None else 0.0
    dz = torch.empty(B, H1, device=dev, dtype=torch.float32)
    dz_c = torch.empty(B, H1, device=dev, dtype=cfg.dtype)
    d = ops.bn_bwd_desc(dy1, st.z, P["fusion_layer.1.weight"], st.bn_mean, st.bn_rstd, st.y1, dz,
                        grads["fusion_layer.1.weight"], grads["fusion_layer.1.bias"],
                        gate_scale=_scale(pd), gated=True, dz16=dz_c)

    def finish() -> None:
        ops.linear_dw(dz_c, st.modal, grads["fusion_layer.0.weight"], grads["fusion_layer.0.bias"])
        if dmodal is not None:
            ops.linear_dx(dz_c, W["fusion_layer.0.weight"], dmodal)
    return ItemBnPending(d, (dy1, dz, dz_c), finish)


def item_fusion_bwd(P: Dict[str, Tensor], W: Dict[str, Tensor], st: ItemSaved, dout: Tensor,
                    grads: Dict[str, Tensor], cfg: TowerCfg, p_drop: float = 0.1,
                    dmodal: Optional[Tensor] = None) -> None:
    dev = dout.device
    B, D = dout.shape
    dt = cfg.dtype
    f32 = dict(device=dev, dtype=torch.float32)
    dy2 = torch.empty(B, D, **f32)
    dy2_c = torch.empty(B, D, device=dev, dtype=dt)
    ops.layernorm_bwd(dout, st.y2, st.m5, st.r5, P["fusion_layer.5.weight"], dy2,
                      grads["fusion_layer.5.weight"], grads["fusion_layer.5.bias"],
                      dx16=dy2_c if dt == torch.bfloat16 else None)
    if dt != torch.bfloat16:
        ops.dropout_bwd(dy2, dy2_c, None)
    ops.linear_dw(dy2_c, st.y1, grads["fusion_layer.4.weight"], grads["fusion_layer.4.bias"])
    H1 = st.z.shape[1]
    dy1 = torch.empty(B, H1, **f32)
    ops.linear_dx(dy2_c, W["fusion_layer.4.weight"], dy1)
    _item_bwd_tail(P, W, st, dy1, grads, cfg, p_drop, dmodal)


def _item_bwd_tail(P, W, st: ItemSaved, dy1: Tensor, grads, cfg: TowerCfg, p_drop: float,
                   dmodal: Optional[Tensor]) -> None:
    """BatchNorm1d + ReLU + dropout backward and Linear 0 of the item fusion head."""
    dev = dy1.device
    B, H1 = dy1.shape
    dt = cfg.dtype
    f32 = dict(device=dev, dtype=torch.float32)
    pd = p_drop if st.seeds is not None else 0.0
    dz = torch.empty(B, H1, **f32)
    dz_c = torch.empty(B, H1, device=dev, dtype=dt)
    fused16 = dt == torch.bfloat16 and B <= 512
    ops.batchnorm_bwd(dy1, st.z, P["fusion_layer.1.weight"], st.bn_mean, st.bn_rstd, st.y1, dz,
                      grads["fusion_layer.1.weight"], grads["fusion_layer.1.bias"],
                      gate_scale=_scale(pd), gated=True, dz16=dz_c if fused16 else None)
    if not fused16:
        ops.dropout_bwd(dz, dz_c, None)
    ops.linear_dw(dz_c, st.modal, grads["fusion_layer.0.weight"], grads["fusion_layer.0.bias"])
    if dmodal is not None:
        ops.linear_dx(dz_c, W["fusion_layer.0.weight"], dmodal)


# ===================================================================================== loss
@dataclass
class LossSaved:
    u_hat: Tensor
    i_hat: Tensor
    norms: Tensor
    logits: Tensor
    lse: Tensor
    user_idx: Optional[Tensor]
    ws: Tensor
    inv_tau: float


def infonce_fwd(u: Tensor, it: Tensor, user_idx: Optional[Tensor], temperature: float = 0.07,
                normed: Optional[Tuple[Tensor, Tensor, Tensor]] = None,
                loss_acc: Optional[Tensor] = None):
    """TwoTowerModel.forward loss part (reference two_tower.py:98-140): fused kernels — one
    normalise launch, one f32-MFMA logits + masked row/column softmax-statistics launch, one
    combine launch (ttmi_infonce_fwd).  ``normed`` = (u_hat, i_hat, norms) already written by
    the fused heads: the normalise launch is skipped (ttmi_infonce_fwd_pre).  ``loss_acc``
    (fp32 device scalar): += loss (inside the logits launch on the pre-normalised path)."""
    dev = u.device
    B, D = u.shape
    f32 = dict(device=dev, dtype=torch.float32)
    if normed is not None:
        u_hat, i_hat, norms = normed
    else:
        u_hat = torch.empty(B, D, **f32)
        i_hat = torch.empty(B, D, **f32)
        norms = torch.empty(2 * B, **f32)
    logits = torch.empty(B, B, **f32)
    lse = torch.empty(2 * B, **f32)
    loss = torch.empty((), **f32)
    ws = torch.empty(ops.infonce_workspace(B, D), device=dev, dtype=torch.uint8)
    if user_idx is not None and user_idx.dtype != torch.int64:
        user_idx = user_idx.to(torch.int64)
    inv_tau = 1.0 / temperature
    if normed is not None:
        ops.infonce_fwd_pre(user_idx, inv_tau, u_hat, i_hat, norms, logits, lse, loss, ws,
                            loss_acc=loss_acc)
    elif loss_acc is not None and D % 64 == 0 and D <= 256 and loss_acc.dtype == torch.float32:
        # normalise launch + logits launch with the combine and the accumulator (ABI 19)
        ops.infonce_fwd_acc(u.contiguous(), it.contiguous(), user_idx, inv_tau, u_hat, i_hat, norms,
                            logits, lse, loss, ws, loss_acc)
    else:
        ops.infonce_fwd(u.contiguous(), it.contiguous(), user_idx, inv_tau, u_hat, i_hat, norms,
                        logits, lse, loss, ws)
        if loss_acc is not None:
            loss_acc.add_(loss.view(loss_acc.shape))
    return loss, logits, u_hat, i_hat, LossSaved(u_hat, i_hat, norms, logits, lse, user_idx, ws,
                                                 inv_tau)


def infonce_bwd(st: LossSaved, dloss: Optional[Tensor], du: Tensor, di: Tensor,
                du16: Optional[Tensor] = None) -> None:
    ops.infonce_bwd(st.u_hat, st.i_hat, st.norms, st.logits, st.lse, st.user_idx, st.inv_tau,
                    dloss, du, di, st.ws, du16)


def count_flops_user(B: int, L: int, D: int, n_layers: int, ffn: int, extra: int = 48) -> float:
    """Dense GEMM + attention FLOPs of one fwd+bwd of the user tower (for the roofline)."""
    M = B * L
    per_layer = 2 * M * D * (3 * D + D + 2 * ffn) + 4 * B * L * L * D
    fwd = n_layers * per_layer + 2 * B * (D + extra) * D + 2 * B * D * D
    return 3.0 * fwd



# ============================================================ global negatives (cfg 5)
@dataclass
class GlobalLossSaved:
    u_hat: Tensor
    i_hat: Tensor
    nu: Tensor
    ni: Tensor
    U: Tensor            # gathered û of every rank [W·B, D]
    I: Tensor            # gathered î
    uid: Optional[Tensor]
    UID: Optional[Tensor]
    row0: int
    world: int
    inv_tau: float
    s_u2i: Optional[Tensor] = None
    lse_u2i: Optional[Tensor] = None
    s_i2u: Optional[Tensor] = None
    lse_i2u: Optional[Tensor] = None
    duh: Optional[Tensor] = None      # local-row grads [B, D]
    dih: Optional[Tensor] = None
    dU: Optional[Tensor] = None       # key grads for every rank's rows [W·B, D]
    dI: Optional[Tensor] = None
    rs_u: Optional[Tensor] = None     # this rank's share of the key grads (reduce-scattered)
    rs_i: Optional[Tensor] = None
    dp: bool = False                  # the collectives run (world > 1, or comm.force_dp)


def _world_rank(group, local: bool):
    import torch.distributed as dist
    if local or not dist.is_initialized():
        return 1, 0
    return dist.get_world_size(group), dist.get_rank(group)


def infonce_global_prep(u: Tensor, it: Tensor, user_idx: Optional[Tensor], temperature: float,
                        group=None, local: bool = False) -> GlobalLossSaved:
    """Phase 1 of the cfg-5 loss: L2-normalise this rank's rows and size the gathered buffers
    (no collective; TrainStep captures it in the forward graph)."""
    world, rank = _world_rank(group, local)
    dp = not local and comm.dp_active(group)
    B, D = u.shape
    dev = u.device
    f32 = dict(device=dev, dtype=torch.float32)
    u_hat, i_hat = torch.empty(B, D, **f32), torch.empty(B, D, **f32)
    nu, ni = torch.empty(B, **f32), torch.empty(B, **f32)
    ops.l2norm_fwd(u.contiguous().float(), u_hat, nu)
    ops.l2norm_fwd(it.contiguous().float(), i_hat, ni)
    uid = None
    if user_idx is not None:
        uid = user_idx if user_idx.dtype == torch.int64 else user_idx.to(torch.int64)
        uid = uid.contiguous()
    if dp:
        U, I = torch.empty(world * B, D, **f32), torch.empty(world * B, D, **f32)
        UID = torch.empty(world * B, device=dev, dtype=torch.int64) if uid is not None else None
    else:
        U, I, UID = u_hat, i_hat, uid
    return GlobalLossSaved(u_hat, i_hat, nu, ni, U, I, uid, UID, rank * B, world,
                           1.0 / temperature, dp=dp)


def infonce_global_gather(st: GlobalLossSaved, group=None) -> None:
    """Phase 2 (collective): all-gather û, î and user_idx over the group (RCCL)."""
    if not st.dp:
        return
    comm.all_gather_into(st.U, st.u_hat, group)
    comm.all_gather_into(st.I, st.i_hat, group)
    if st.UID is not None:
        comm.all_gather_into(st.UID, st.uid, group)


def infonce_global_loss(st: GlobalLossSaved) -> Tensor:
    """Phase 3: this rank's u2i and i2u rows against every rank's keys; loss_r."""
    B, D = st.u_hat.shape
    C = st.world * B
    f32 = dict(device=st.u_hat.device, dtype=torch.float32)
    st.s_u2i, st.s_i2u = torch.empty(B, C, **f32), torch.empty(B, C, **f32)
    st.lse_u2i, st.lse_i2u = torch.empty(B, **f32), torch.empty(B, **f32)
    ce = torch.empty(2 * B, **f32)
    ops.rowce_fwd(st.u_hat, st.I, st.uid, st.UID, st.row0, st.inv_tau, st.s_u2i, st.lse_u2i, ce[:B])
    ops.rowce_fwd(st.i_hat, st.U, st.uid, st.UID, st.row0, st.inv_tau, st.s_i2u, st.lse_i2u, ce[B:])
    loss = torch.empty(1, **f32)
    ops.sum_scaled(ce, 0.5 / B, loss)
    return loss.view(())


def infonce_global_loss_bwd(st: GlobalLossSaved, dloss: Optional[Tensor]) -> None:
    """Phase 4: local-row grads and key grads for every rank's rows."""
    B, D = st.u_hat.shape
    f32 = dict(device=st.u_hat.device, dtype=torch.float32)
    scale = 0.5 / B
    st.duh, st.dih = torch.empty(B, D, **f32), torch.empty(B, D, **f32)
    st.dI, st.dU = torch.empty(st.world * B, D, **f32), torch.empty(st.world * B, D, **f32)
    ops.rowce_bwd(st.u_hat, st.I, st.s_u2i, st.lse_u2i, st.uid, st.UID, st.row0, st.inv_tau,
                  dloss, scale, st.duh, st.dI)
    ops.rowce_bwd(st.i_hat, st.U, st.s_i2u, st.lse_i2u, st.uid, st.UID, st.row0, st.inv_tau,
                  dloss, scale, st.dih, st.dU)
    if st.dp:
        st.rs_u, st.rs_i = torch.empty(B, D, **f32), torch.empty(B, D, **f32)
    else:
        st.rs_u, st.rs_i = st.dU, st.dI


def infonce_global_scatter(st: GlobalLossSaved, group=None) -> None:
    """Phase 5 (collective): reduce-scatter (SUM) of the key grads back to their owners."""
    if not st.dp:
        return
    comm.reduce_scatter_sum(st.rs_u, st.dU, group)
    comm.reduce_scatter_sum(st.rs_i, st.dI, group)


def infonce_global_norm_bwd(st: GlobalLossSaved, du: Tensor, di: Tensor) -> None:
    """Phase 6: normalize backward of (local-row grad + owned key grad)."""
    ops.l2norm_bwd(st.u_hat, st.nu, st.duh, du, dy2=st.rs_u)
    ops.l2norm_bwd(st.i_hat, st.ni, st.dih, di, dy2=st.rs_i)


def infonce_global_fwd(u: Tensor, it: Tensor, user_idx: Optional[Tensor], temperature: float,
                       group=None, local: bool = False):
    """InfoNCE over the concatenation of every rank's batch (BASELINE cfg 5; the reference
    two_tower.py:98-140 applied to world·B rows).  Returns (loss_r, logits_u2i [B, W·B],
    û_r, î_r, saved); the global loss is the mean of loss_r over ranks, which DDP's 1/world
    gradient scaling realises.  All-gathers û, î and user_idx over `group` (RCCL)."""
    st = infonce_global_prep(u, it, user_idx, temperature, group, local)
    infonce_global_gather(st, group)
    loss = infonce_global_loss(st)
    return loss, st.s_u2i, st.u_hat, st.i_hat, st


def infonce_global_bwd(st: GlobalLossSaved, dloss: Optional[Tensor], du: Tensor, di: Tensor,
                       group=None, local: bool = False) -> None:
    """Backward of infonce_global_fwd for this rank's loss_r: local-row grads, key grads for
    every rank's rows reduce-scattered (SUM) back to their owners, then normalize backward."""
    infonce_global_loss_bwd(st, dloss)
    infonce_global_scatter(st, group)
    infonce_global_norm_bwd(st, du, di)

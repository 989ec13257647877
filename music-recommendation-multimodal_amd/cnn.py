"""cfg-3 item encoders on libttmi kernels: ResNet-18 audio/visual backbones and the tabular
MLP (reference src/models/item_tower.py:9-39, :85-98).

ResNet-18 follows torchvision's resnet18 exactly (BasicBlock [2, 2, 2, 2], conv1 7x7/2 →
BN → ReLU → maxpool 3/2/1, 1x1/2 conv + BN downsample at the first block of layers 2-4,
global average pool, fc), with the reference's replacements (audio conv1 takes 1 channel;
fc → Linear(512, embedding_dim)) and torchvision's parameter names, so checkpoints map
one-to-one.  BatchNorm2d runs in train mode on batch statistics, as in the reference.

Data layout: NHWC bf16 activations; the 1/3-channel image goes to a space-to-depth layout
(ttmi_stem_s2d: [N][H/2][W/2][8 or 16]) so the 7x7/2 stem runs as a 4x4/1 conv (K = 128 / 256
instead of 392 padded taps); conv weights are used through bf16 mirrors (ttmi_conv_weight_prep);
every conv's forward epilogue accumulates the BatchNorm column sums (int64 fixed point, so the
statistics are bit-reproducible), so a conv + BN + ReLU (+ residual) is two launches; the stem's
bn1 + ReLU + maxpool is one (ttmi_stem_pool_fwd, the 112x112 BN output never stored).  All
parameters and grads stay fp32 (torch layouts).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn

from . import functional as F
from . import ops

Tensor = torch.Tensor

LAYERS = (("layer1", 64, 64, 1), ("layer2", 64, 128, 2), ("layer3", 128, 256, 2),
          ("layer4", 256, 512, 2))
STEM_CP = 8          # odd-sized images: the 1- or 3-channel stem input padded to 8 channels
STEM_S2D = True      # even-sized images: the 7x7/2 stem on the space-to-depth input


def stem_s2d_cp(cin: int) -> int:
    """Channels of the space-to-depth stem input (4·cin rounded up to 8: 8 / 16 for 1 / 3)."""
    return (4 * cin + 7) // 8 * 8


def _is_stem(sp: "ConvSpec") -> bool:
    return sp.cin < 8 and sp.k == 7 and sp.stride == 2 and sp.pad == 3


@dataclass(frozen=True)
class ConvSpec:
    name: str          # parameter name of the weight ("conv1.weight", "layer2.0.downsample.0.weight")
    bn: str            # its BatchNorm prefix ("bn1", "layer2.0.downsample.1")
    cin: int
    cout: int
    k: int
    stride: int
    pad: int


def resnet18_convs(in_ch: int) -> List[ConvSpec]:
    specs = [ConvSpec("conv1.weight", "bn1", in_ch, 64, 7, 2, 3)]
    for lname, cin, cout, s in LAYERS:
        for bi in range(2):
            ci = cin if bi == 0 else cout
            st = s if bi == 0 else 1
            b = f"{lname}.{bi}."
            specs.append(ConvSpec(b + "conv1.weight", b + "bn1", ci, cout, 3, st, 1))
            specs.append(ConvSpec(b + "conv2.weight", b + "bn2", cout, cout, 3, 1, 1))
            if bi == 0 and (st != 1 or ci != cout):
                specs.append(ConvSpec(b + "downsample.0.weight", b + "downsample.1", ci, cout, 1,
                                      st, 0))
    return specs


# ---------------------------------------------------------------------------- state
@dataclass
class ConvAct:
    x: Tensor              # conv input (bf16 NHWC)
    H: int
    W: int
    y: Tensor              # conv output, pre-BN (bf16 NHWC)
    mean: Tensor
    rstd: Tensor
    a: Optional[Tensor]    # BN output (after residual/ReLU when fused); None for the stem


@dataclass
class ResNetSaved:
    N: int
    acts: Dict[str, ConvAct] = field(default_factory=dict)
    pool_idx: Optional[Tensor] = None
    feat: Optional[Tensor] = None          # pooled features bf16 [N, 512]
    last: Optional[Tensor] = None          # last block output (avgpool input)
    mirrors: Optional[Dict[str, Tuple[Tensor, Optional[Tensor]]]] = None
    fc_w: Optional[Tensor] = None


def weight_mirrors(P: Dict[str, Tensor], specs: List[ConvSpec], s2d: bool = True):
    """bf16 GEMM mirrors (Wf for FWD, Wd for DGRAD) of every conv weight; the stem's as the
    4x4 kernel over the space-to-depth input when ``s2d`` (ttmi_stem_weight_prep)."""
    out, items = {}, []
    for sp in specs:
        w = P[sp.name].contiguous()
        dev = w.device
        if s2d and _is_stem(sp):
            cp = stem_s2d_cp(sp.cin)
            wf = torch.empty(sp.cout, 4, 4, cp, device=dev, dtype=torch.bfloat16)
            items.append((w, cp, wf, None, True))
            out[sp.name] = (wf, None)
            continue
        cp = STEM_CP if sp.cin < 8 else sp.cin
        wf = torch.empty(sp.cout, sp.k, sp.k, cp, device=dev, dtype=torch.bfloat16)
        wd = None
        if sp.cin >= 8:
            wd = torch.empty(sp.cin, sp.k, sp.k, sp.cout, device=dev, dtype=torch.bfloat16)
        items.append((w, cp, wf, wd, False))
        out[sp.name] = (wf, wd)
    ops.conv_weight_prep_batch(items)          # one launch for the whole network
    return out


def _conv_bn(P, bufs, sp: ConvSpec, x: Tensor, N: int, H: int, W: int, mirrors, stats: Tensor,
             off: int, residual: Optional[Tensor], relu: bool, training: bool,
             mode: int = ops.FWD) -> ConvAct:
    dev = x.device
    C = x.shape[-1]
    Ho, Wo = ops.conv_out_hw(H, W, sp.k, sp.stride, sp.pad)
    y = torch.empty(N, Ho, Wo, sp.cout, device=dev, dtype=torch.bfloat16)
    cs = cq = None                       # eval: BN normalises with the running statistics
    if training:
        n = ops.CONV_STAT_REPS * sp.cout
        cs, cq = stats[off:off + n], stats[off + n:off + 2 * n]
    ops.conv2d(mode, N, H, W, C, sp.cin, sp.cout, sp.k, sp.stride, sp.pad, x=x,
               w=mirrors[sp.name][0], out=y, colsum=cs, colsumsq=cq)
    a = torch.empty_like(y)
    mean = torch.empty(sp.cout, device=dev)
    rstd = torch.empty(sp.cout, device=dev)
    ops.bn2d_fwd(y, cs, cq, P[sp.bn + ".weight"], P[sp.bn + ".bias"], a, mean, rstd,
                 running_mean=bufs.get(sp.bn + ".running_mean"),
                 running_var=bufs.get(sp.bn + ".running_var"),
                 num_batches=bufs.get(sp.bn + ".num_batches_tracked") if training else None,
                 residual=residual, relu=relu)
    return ConvAct(x, H, W, y, mean, rstd, a)


def resnet18_fwd(P: Dict[str, Tensor], x: Tensor, in_ch: int, bufs: Dict[str, Tensor],
                 training: bool = True, fc_dtype: torch.dtype = torch.bfloat16):
    """torchvision resnet18.forward on x [N, in_ch, H, W] fp32 → [N, out] fp32.  training:
    BN on batch statistics (running stats updated when ``bufs`` holds them); otherwise BN on
    ``bufs``' running statistics."""
    dev = x.device
    N, _, H, W = x.shape
    specs = resnet18_convs(in_ch)
    s2d = STEM_S2D and H % 2 == 0 and W % 2 == 0   # the 7x7/2 stem as a 4x4/1 conv (ttmi_stem_s2d)
    mirrors = weight_mirrors(P, specs, s2d)
    # BatchNorm Σy, Σy² replica rows: int64 fixed point (order-independent, include/ttmi.h)
    stats = torch.zeros(2 * ops.CONV_STAT_REPS * sum(sp.cout for sp in specs), device=dev,
                        dtype=torch.int64) if training else None
    st = ResNetSaved(N, mirrors=mirrors)
    sp = specs[0]
    if s2d:
        x0 = torch.empty(N, H // 2, W // 2, stem_s2d_cp(in_ch), device=dev, dtype=torch.bfloat16)
        ops.stem_s2d(x.contiguous().float(), x0.shape[-1], x0)
    else:
        x0 = torch.empty(N, H, W, STEM_CP, device=dev, dtype=torch.bfloat16)
        ops.nchw_to_nhwc(x.contiguous().float(), STEM_CP, x0)
    # stem: conv1 (+ BN column sums) -> fused bn1 + ReLU + maxpool (ttmi_stem_pool_fwd: the
    # full-resolution BN output is never stored; the backward re-derives its ReLU gate)
    Hc, Wc = ops.conv_out_hw(H, W, sp.k, sp.stride, sp.pad)
    yc = torch.empty(N, Hc, Wc, sp.cout, device=dev, dtype=torch.bfloat16)
    cs = cq = None
    if training:
        n = ops.CONV_STAT_REPS * sp.cout
        cs, cq = stats[:n], stats[n:2 * n]
    ops.conv2d(ops.STEM_FWD if s2d else ops.FWD, N, H, W, x0.shape[-1], sp.cin, sp.cout, sp.k,
               sp.stride, sp.pad, x=x0, w=mirrors[sp.name][0], out=yc, colsum=cs, colsumsq=cq)
    mean = torch.empty(sp.cout, device=dev)
    rstd = torch.empty(sp.cout, device=dev)
    Hp, Wp = ops.conv_out_hw(Hc, Wc, 3, 2, 1)
    y = torch.empty(N, Hp, Wp, sp.cout, device=dev, dtype=torch.bfloat16)
    st.pool_idx = torch.empty(N, Hp, Wp, sp.cout, device=dev, dtype=torch.uint8)
    ops.stem_pool_fwd(yc, cs, cq, P[sp.bn + ".weight"], P[sp.bn + ".bias"], y, st.pool_idx, mean, rstd,
                      running_mean=bufs.get(sp.bn + ".running_mean"),
                      running_var=bufs.get(sp.bn + ".running_var"),
                      num_batches=bufs.get(sp.bn + ".num_batches_tracked") if training else None)
    st.acts[sp.name] = ConvAct(x0, H, W, yc, mean, rstd, None)
    off = 2 * ops.CONV_STAT_REPS * sp.cout
    H, W = Hp, Wp
    byname = {s.name: s for s in specs}
    for lname, _, _, _ in LAYERS:
        for bi in range(2):
            b = f"{lname}.{bi}."
            c1, c2 = byname[b + "conv1.weight"], byname[b + "conv2.weight"]
            ds = byname.get(b + "downsample.0.weight")
            idn = y
            if ds is not None:
                ad = _conv_bn(P, bufs, ds, y, N, H, W, mirrors, stats, off, None, False, training)
                off += 2 * ops.CONV_STAT_REPS * ds.cout
                st.acts[ds.name] = ad
                idn = ad.a
            a1 = _conv_bn(P, bufs, c1, y, N, H, W, mirrors, stats, off, None, True, training)
            off += 2 * ops.CONV_STAT_REPS * c1.cout
            st.acts[c1.name] = a1
            H1, W1 = a1.y.shape[1], a1.y.shape[2]
            a2 = _conv_bn(P, bufs, c2, a1.a, N, H1, W1, mirrors, stats, off, idn, True, training)
            off += 2 * ops.CONV_STAT_REPS * c2.cout
            st.acts[c2.name] = a2
            y, H, W = a2.a, H1, W1
    st.last = y
    feat = torch.empty(N, 512, device=dev, dtype=torch.bfloat16)
    ops.avgpool_fwd(y, feat)
    st.feat = feat
    fc_w = P["fc.weight"]
    st.fc_w = ops.cast_bf16(fc_w.contiguous(), torch.empty(fc_w.shape, device=dev, dtype=fc_dtype))
    out = torch.empty(N, fc_w.shape[0], device=dev)
    ops.linear(feat, st.fc_w, P["fc.bias"], out)
    return out, st


def resnet18_bwd(P: Dict[str, Tensor], st: ResNetSaved, dout: Tensor, grads: Dict[str, Tensor],
                 in_ch: int) -> None:
    """Backward of resnet18_fwd: accumulates every parameter grad (torch layouts)."""
    dev = dout.device
    N = st.N
    specs = resnet18_convs(in_ch)
    byname = {s.name: s for s in specs}
    R = ops.CONV_STAT_REPS
    sums = torch.zeros(2 * R * sum(sp.cout for sp in specs), device=dev, dtype=torch.int64)
    sl, o = {}, 0                       # each BatchNorm's [R][2C] fixed-point sums
    for sp in specs:
        sl[sp.name] = sums[o:o + 2 * R * sp.cout]
        o += 2 * R * sp.cout

    def bn_bwd(sp: ConvSpec, act: ConvAct, dy: Tensor, gate: Optional[Tensor],
               g_out: Optional[Tensor] = None) -> Tensor:
        dyc = torch.empty_like(act.y)
        ops.bn2d_bwd(dy, act.y, act.mean, act.rstd, P[sp.bn + ".weight"], sl[sp.name], dyc,
                     grads[sp.bn + ".weight"], grads[sp.bn + ".bias"], gate=gate, g_out=g_out)
        return dyc

    def bn_apply(sp: ConvSpec, act: ConvAct, g: Tensor) -> Tensor:
        """BN backward whose reduction a DGRAD epilogue already did (g gated, sums filled)."""
        dyc = torch.empty_like(act.y)
        ops.bn2d_bwd_apply(g, act.y, act.mean, act.rstd, P[sp.bn + ".weight"], sl[sp.name], dyc,
                           grads[sp.bn + ".weight"], grads[sp.bn + ".bias"])
        return dyc

    def conv_bwd(sp: ConvSpec, act: ConvAct, dyc: Tensor, need_dx: bool,
                 addend: Optional[Tensor] = None, bn_of: Optional[Tuple[ConvSpec, ConvAct]] = None):
        """WGRAD (+ DGRAD).  bn_of = (spec, act) of the BatchNorm+ReLU that produced this conv's
        input: its backward reduction rides in the DGRAD epilogue, which then returns g."""
        C = act.x.shape[-1]
        s2d = _is_stem(sp) and act.x.shape[1] * 2 == act.H     # space-to-depth stem input
        ops.conv2d(ops.STEM_WGRAD if s2d else ops.WGRAD, N, act.H, act.W, C, sp.cin, sp.cout,
                   sp.k, sp.stride, sp.pad, x=act.x, dy=dyc, out=grads[sp.name])
        if not need_dx:
            return None
        dx = torch.empty_like(act.x)
        bn = None
        if bn_of is not None:
            bsp, bact = bn_of
            bn = (bact.a, bact.y, bact.mean, bact.rstd, sl[bsp.name])
        ops.conv2d(ops.DGRAD, N, act.H, act.W, C, sp.cin, sp.cout, sp.k, sp.stride, sp.pad,
                   dy=dyc, w=st.mirrors[sp.name][1], out=dx, addend=addend, bn=bn)
        return dx

    # fc + global average pool
    dc = torch.empty(dout.shape, device=dev, dtype=st.feat.dtype)
    ops.dropout_bwd(dout.contiguous().float(), dc, None)        # cast to the operand dtype
    ops.linear_dw(dc, st.feat, grads["fc.weight"], grads["fc.bias"])
    dfeat = torch.empty(N, 512, device=dev)
    ops.linear_dx(dc, st.fc_w, dfeat)
    dy = torch.empty_like(st.last)
    ops.avgpool_bwd(dfeat, dy)
    # residual stages, reversed.  Every BatchNorm whose input gradient comes out of a DGRAD
    # (bn1 from conv2's, the previous block's bn2 from conv1's) has its backward reduction
    # fused into that DGRAD's epilogue (ttmi_conv_desc.bn_sums) and only its apply pass here.
    fwd_blocks = [f"{lname}.{bi}." for lname, _, _, _ in LAYERS for bi in range(2)]
    gated = False                        # dy is already the gated g of this block's bn2
    for j in reversed(range(len(fwd_blocks))):
        b = fwd_blocks[j]
        c1, c2 = byname[b + "conv1.weight"], byname[b + "conv2.weight"]
        ds = byname.get(b + "downsample.0.weight")
        a1, a2 = st.acts[c1.name], st.acts[c2.name]
        if gated:
            g = dy                                    # dy ⊙ ReLU gate: the identity branch's grad
            d2 = bn_apply(c2, a2, g)
        else:
            g = torch.empty_like(a2.a)
            d2 = bn_bwd(c2, a2, dy, a2.a, g_out=g)
        g1 = conv_bwd(c2, a2, d2, True, bn_of=(c1, a1))
        d1 = bn_apply(c1, a1, g1)
        if ds is not None:
            ad = st.acts[ds.name]
            dd = bn_bwd(ds, ad, g, None)
            idn_dx = conv_bwd(ds, ad, dd, True)
        else:
            idn_dx = g
        prev = None
        if j > 0:                                     # the previous block's bn2 + ReLU output
            pc2 = byname[fwd_blocks[j - 1] + "conv2.weight"]
            prev = (pc2, st.acts[pc2.name])
        dy = conv_bwd(c1, a1, d1, True, addend=idn_dx, bn_of=prev)
        gated = prev is not None
    # max-pool and stem (no input grad: the encoder input is data)
    stem = specs[0]
    act = st.acts[stem.name]
    d0 = torch.empty_like(act.y)
    ops.stem_pool_bwd(dy, st.pool_idx, act.y, act.mean, act.rstd, P[stem.bn + ".weight"],
                      P[stem.bn + ".bias"], sl[stem.name], d0, grads[stem.bn + ".weight"],
                      grads[stem.bn + ".bias"])
    conv_bwd(stem, act, d0, False)


# ---------------------------------------------------------------------------- tabular
@dataclass
class TabSaved:
    x: Tensor
    z: Tensor
    mean: Tensor
    rstd: Tensor
    y1: Tensor
    w0: Tensor
    w4: Tensor
    p_drop: float


def tabular_fwd(P: Dict[str, Tensor], x: Tensor, bufs: Dict[str, Tensor], seeds: Optional[Tensor],
                p_drop: float, site: int = F.SITE_TAB, training: bool = True,
                dtype=torch.bfloat16):
    """TabularEncoder (item_tower.py:85-98): Linear → BN1d → ReLU → Dropout → Linear."""
    dev = x.device
    B, T = x.shape
    if T % 8:
        # the reference's T (14 numerics + one-hot genres) is arbitrary: the GEMM operands
        # are zero-padded to a 16-byte row (the padding columns contribute nothing)
        Tp = (T + 7) // 8 * 8
        xc = ops.dropout_to(x.contiguous().float(), torch.zeros(B, Tp, device=dev, dtype=dtype)[:, :T])
        xc = xc.as_strided((B, Tp), (Tp, 1))
        w0 = ops.dropout_to(P["mlp.0.weight"].contiguous(),
                            torch.zeros(P["mlp.0.weight"].shape[0], Tp, device=dev, dtype=dtype)[:, :T])
        w0 = w0.as_strided((w0.shape[0], Tp), (Tp, 1))
    else:
        xc = ops.cast_bf16(x.contiguous().float(), torch.empty(x.shape, device=dev, dtype=dtype))
        w0 = ops.cast_bf16(P["mlp.0.weight"].contiguous(),
                           torch.empty(P["mlp.0.weight"].shape, device=dev, dtype=dtype))
    w4 = ops.cast_bf16(P["mlp.4.weight"].contiguous(),
                       torch.empty(P["mlp.4.weight"].shape, device=dev, dtype=dtype))
    H1 = w0.shape[0]
    z = torch.empty(B, H1, device=dev)
    ops.linear(xc, w0, P["mlp.0.bias"], z)
    y1 = torch.empty(B, H1, device=dev, dtype=dtype)
    mean, rstd = torch.empty(H1, device=dev), torch.empty(H1, device=dev)
    drop = (p_drop, seeds[site:site + 1]) if (p_drop > 0 and seeds is not None) else ops.NO_DROP
    ops.batchnorm_fwd(z, P["mlp.1.weight"], P["mlp.1.bias"], y1, mean, rstd,
                      bufs.get("mlp.1.running_mean"), bufs.get("mlp.1.running_var"),
                      bufs.get("mlp.1.num_batches_tracked"), relu=True, drop=drop,
                      training=training)
    out = torch.empty(B, w4.shape[0], device=dev)
    ops.linear(y1, w4, P["mlp.4.bias"], out)
    return out, TabSaved(xc, z, mean, rstd, y1, w0, w4, drop[0])


def tabular_bwd(P: Dict[str, Tensor], st: TabSaved, dout: Tensor, grads: Dict[str, Tensor]) -> None:
    dev = dout.device
    dc = torch.empty(dout.shape, device=dev, dtype=st.y1.dtype)
    ops.dropout_bwd(dout.contiguous().float(), dc, None)
    ops.linear_dw(dc, st.y1, grads["mlp.4.weight"], grads["mlp.4.bias"])
    dy1 = torch.empty(st.z.shape, device=dev)
    ops.linear_dx(dc, st.w4, dy1)
    dz = torch.empty_like(dy1)
    scale = 1.0 / (1.0 - st.p_drop) if st.p_drop > 0 else 1.0
    dzc = torch.empty(dz.shape, device=dev, dtype=st.y1.dtype)
    fused16 = dzc.dtype == torch.bfloat16 and dz.shape[0] <= 512   # bf16 copy from the BN kernel
    ops.batchnorm_bwd(dy1, st.z, P["mlp.1.weight"], st.mean, st.rstd, st.y1, dz,
                      grads["mlp.1.weight"], grads["mlp.1.bias"], gate_scale=scale, gated=True,
                      dz16=dzc if fused16 else None)
    if not fused16:
        ops.dropout_bwd(dz, dzc, None)
    gw = grads["mlp.0.weight"]
    if st.x.shape[1] != gw.shape[1]:                  # zero-padded T (see tabular_fwd)
        pad = torch.zeros(gw.shape[0], st.x.shape[1], device=dev)
        ops.linear_dw(dzc, st.x, pad, grads["mlp.0.bias"], defer=False)   # read just below
        gw.add_(pad[:, :gw.shape[1]])
    else:
        ops.linear_dw(dzc, st.x, gw, grads["mlp.0.bias"])


# ---------------------------------------------------------------------------- modules
class BasicBlock(nn.Module):
    """Parameter container with torchvision BasicBlock names (conv1, bn1, conv2, bn2,
    downsample.{0,1}); the computation is resnet18_fwd/bwd."""

    def __init__(self, cin: int, cout: int, stride: int):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(cout)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)
        self.downsample = None
        if stride != 1 or cin != cout:
            self.downsample = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False),
                                            nn.BatchNorm2d(cout))


class _ResNetFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, in_ch, names, bufs, x, *params):
        P = dict(zip(names, params))
        out, st = resnet18_fwd(P, x, in_ch, bufs, training=True)
        ctx.saved = (in_ch, names, P, st)
        return out

    @staticmethod
    def backward(ctx, dout):
        in_ch, names, P, st = ctx.saved
        del ctx.saved
        grads = {n: torch.zeros_like(P[n]) for n in names}
        resnet18_bwd(P, st, dout, grads, in_ch)
        return (None, None, None, None) + tuple(grads[n] for n in names)


class ResNet18(nn.Module):
    """torchvision resnet18 with conv1 → Conv2d(in_ch, 64, 7, 2, 3) and fc → Linear(512, out_dim)
    (AudioEncoder/VisualEncoder backbones, item_tower.py:15-22, :33-36)."""

    def __init__(self, in_ch: int = 3, out_dim: int = 128):
        super().__init__()
        self.in_ch = in_ch
        self.conv1 = nn.Conv2d(in_ch, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        for lname, cin, cout, s in LAYERS:
            setattr(self, lname, nn.Sequential(BasicBlock(cin, cout, s), BasicBlock(cout, cout, 1)))
        self.fc = nn.Linear(512, out_dim)
        for m in self.modules():             # torchvision resnet init
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    def forward(self, x: Tensor) -> Tensor:
        names, params = zip(*self.named_parameters())
        bufs = dict(self.named_buffers())
        if self.training and torch.is_grad_enabled() and any(p.requires_grad for p in params):
            return _ResNetFn.apply(self.in_ch, list(names), bufs, x, *params)
        out, _ = resnet18_fwd(dict(zip(names, [p.detach() for p in params])), x, self.in_ch,
                              bufs, training=self.training)
        return out


class AudioEncoder(nn.Module):
    """item_tower.py:9-25: ResNet-18 on 1-channel mel spectrograms, fc → embedding_dim."""

    def __init__(self, embedding_dim: int = 128):
        super().__init__()
        self.backbone = ResNet18(1, embedding_dim)

    def forward(self, x: Tensor) -> Tensor:
        return self.backbone(x)


class VisualEncoder(nn.Module):
    """item_tower.py:27-39: ResNet-18 on 3-channel covers (ImageNet weights are a download and
    are not available offline: random init), fc → embedding_dim."""

    def __init__(self, embedding_dim: int = 128, pretrained: bool = False):
        super().__init__()
        self.backbone = ResNet18(3, embedding_dim)

    def forward(self, x: Tensor) -> Tensor:
        return self.backbone(x)


class _TabularFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, names, bufs, p_drop, seeds, x, *params):
        P = dict(zip(names, params))
        out, st = tabular_fwd(P, x, bufs, seeds, p_drop)
        ctx.saved = (names, P, st)
        return out

    @staticmethod
    def backward(ctx, dout):
        names, P, st = ctx.saved
        del ctx.saved
        grads = {n: torch.zeros_like(P[n]) for n in names}
        tabular_bwd(P, st, dout, grads)
        return (None, None, None, None, None) + tuple(grads[n] for n in names)


class TabularEncoder(nn.Module):
    """item_tower.py:85-98."""

    def __init__(self, input_dim: int, embedding_dim: int = 128):
        super().__init__()
        self.mlp = nn.Sequential(nn.Linear(input_dim, 256), nn.BatchNorm1d(256), nn.ReLU(),
                                 nn.Dropout(0.1), nn.Linear(256, embedding_dim))

    def forward(self, x: Tensor, seeds: Optional[Tensor] = None) -> Tensor:
        names, params = zip(*self.named_parameters())
        bufs = dict(self.named_buffers())
        p_drop = self.mlp[3].p if self.training else 0.0
        if p_drop > 0 and seeds is None:
            seeds = torch.randint(-(2 ** 62), 2 ** 62, (F.N_SITES,), device=x.device,
                                  dtype=torch.int64)
        if self.training and torch.is_grad_enabled() and any(p.requires_grad for p in params):
            return _TabularFn.apply(list(names), bufs, p_drop, seeds, x, *params)
        out, _ = tabular_fwd(dict(zip(names, [p.detach() for p in params])), x, bufs, seeds,
                             p_drop, training=self.training)
        return out

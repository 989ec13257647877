"""cfg-3 item encoders (ResNet-18 audio/visual backbones, tabular MLP) on the GPU vs the CPU
oracle restatement (oracle/resnet_ref.py) with identical parameters.

bf16 operands through 20 convolutions: the embedding is compared at 5e-2 relative to its
max-abs (bf16 rounding compounds layer over layer, BatchNorm re-normalises it); gradients by
direction against the bf16-emulation yardstick (test_resnet18_vs_oracle's docstring); BN
running stats at 1e-2.  Parity against the reference itself is unpinned (torchvision is
absent).  The cfg-3 model tests run the whole two-tower forward/backward and
the graph-captured TrainStep on raw mels / covers / tabular inputs."""
import numpy as np
import pytest
import torch
import torch.nn.functional as TF

from oracle import resnet_ref as rref
from oracle import two_tower_ref as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-30)


def check_grad(name, g, gref):
    g = g.detach().double().cpu().flatten()
    gref = gref.detach().double().cpu().flatten()
    nr = gref.norm().item()
    if nr < 1e-8:
        assert g.norm().item() < 1e-3, name
        return
    cos = torch.dot(g, gref).item() / (g.norm().item() * nr + 1e-30)
    assert cos > 0.98, (name, cos)
    assert abs(g.norm().item() / nr - 1) < 0.1, (name, g.norm().item() / nr)


class _RB(torch.autograd.Function):
    """bf16 rounding in forward and of the gradient in backward: the GPU path stores both
    the activation and its gradient in bf16 at these points."""

    @staticmethod
    def forward(ctx, x):
        return x.to(torch.bfloat16).float()

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).float()


def rb(x):
    return _RB.apply(x)


class _BnKernel(torch.autograd.Function):
    """Train-mode BatchNorm2d exactly as ttmi_bn2d_fwd / ttmi_bn2d_bwd compute it: batch
    statistics of the UNROUNDED conv output y32 (the conv epilogue's column sums), applied to
    the bf16-stored y; backward from the (bf16) gated gradient g:
    dy32 = bf16(w·rstd·(g − Σg/M − x̂·Σg x̂/M)) with x̂ from the bf16 y (the value the kernel
    reads back), dw = Σg x̂, db = Σg."""

    @staticmethod
    def forward(ctx, y32, w, b):
        mean = y32.mean((0, 2, 3), keepdim=True)
        var = y32.var((0, 2, 3), unbiased=False, keepdim=True)
        rstd = 1.0 / torch.sqrt(var + 1e-5)
        xh = (y32.to(torch.bfloat16).float() - mean) * rstd
        ctx.save_for_backward(xh, rstd, w)
        return xh * w[None, :, None, None] + b[None, :, None, None]

    @staticmethod
    def backward(ctx, g):
        xh, rstd, w = ctx.saved_tensors
        M = g.numel() // g.shape[1]
        s1 = g.sum((0, 2, 3), keepdim=True)
        s2 = (g * xh).sum((0, 2, 3), keepdim=True)
        dx = w[None, :, None, None] * rstd * (g - s1 / M - xh * s2 / M)
        return dx.to(torch.bfloat16).float(), s2.flatten(), s1.flatten()


class _GradRound(torch.autograd.Function):
    """Identity forward; rounds the gradient to bf16 (a branch whose input grad the kernels
    store in bf16 before it is added to another branch's: the downsample conv's DGRAD)."""

    @staticmethod
    def forward(ctx, x):
        return x.clone()

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).float()


# fp32 accumulation orders of the emulated convolutions.  Every one is an equally valid
# "bf16 storage, fp32 accumulation" implementation; they differ only in the order the K
# products are summed, which moves individual bf16 roundings of the stored activations and
# gradients, and the train-mode BatchNorm backward amplifies that (tools/diag_resnet_margin.py
# measures the spread).  "kernel" is the conv kernels' own order (_KConv below): the GPU is
# judged against it; the others show how far equally valid orders spread.
EMU_ORDERS = ("kernel", "torch", "f64", "half", "evenodd", "quarter", "quarters")


def _conv_order(x, w, stride, pad, order):
    if order == "torch":
        return TF.conv2d(x, w, stride=stride, padding=pad)
    if order == "f64" or x.shape[1] < 2:
        return TF.conv2d(x.double(), w.double(), stride=stride, padding=pad).float()
    C = x.shape[1]
    if order == "quarters" and C >= 4:
        q = C // 4
        parts = [TF.conv2d(x[:, i * q:(i + 1) * q if i < 3 else C], w[:, i * q:(i + 1) * q if i < 3 else C],
                           stride=stride, padding=pad) for i in range(4)]
        return ((parts[0] + parts[1]) + parts[2]) + parts[3]
    if order == "evenodd":
        return (TF.conv2d(x[:, 0::2], w[:, 0::2], stride=stride, padding=pad) +
                TF.conv2d(x[:, 1::2], w[:, 1::2], stride=stride, padding=pad))
    h = C // 2 if order == "half" else max(1, C // 4)
    return (TF.conv2d(x[:, h:], w[:, h:], stride=stride, padding=pad) +
            TF.conv2d(x[:, :h], w[:, :h], stride=stride, padding=pad))


# ---- the conv kernels' own accumulation order (ttmi_conv.hip), order "kernel" -------------
# MFMA chunks of 32 products (v_mfma_f32_16x16x32_bf16) are modelled as one exact dot product
# rounded into the fp32 accumulator (acc = fl32(acc + Σ32)); the chunks are added in the
# kernels' k order:
#   FWD    k = (tap, channel), 64-wide k-steps of 2 chunks (conv_dma_kernel; the space-to-depth
#          stem: k = (4x4 tap (a, b), s2d channel (ph·2 + pw)·Cin + ci padded to Cp), i.e. the
#          7x7 tap (2a + ph − 1, 2b + pw − 1));
#   DGRAD  each input pixel sums its stride-lattice taps in (kh, kw) order, 32 output channels a
#          chunk (one tap per 64-channel k-step);
#   WGRAD  the output pixels (n, ho, wo) are split in k_split ranges (conv_plan: per = max(min(8,
#          ksteps), ceil(ksteps / ceil(1024 / tiles))) 64-pixel k-steps), each range summed 32
#          pixels a chunk, the splits then summed in order in chunks of 16 (wgrad_reduce_kernel).
_KCHUNK = 32


def _stem_cols(Cin):
    """Column of the 7x7 unfold (ci·49 + kh·7 + kw) for each k of the s2d stem's K, -1 = zero."""
    cp = 8 if Cin == 1 else 16
    cols = []
    for a in range(4):
        for b in range(4):
            for sc in range(cp):
                q, ci = divmod(sc, Cin)
                kh, kw = 2 * a + (q >> 1) - 1, 2 * b + (q & 1) - 1
                ok = sc < 4 * Cin and 0 <= kh < 7 and 0 <= kw < 7
                cols.append(ci * 49 + kh * 7 + kw if ok else -1)
    return torch.tensor(cols)


def _kernel_cols(x, KH, KW, stride, pad, stem):
    """im2col in the FWD kernel's k order: [N, K, L] float64 (zero columns where the kernel's
    K has padding)."""
    N, C = x.shape[:2]
    u = TF.unfold(x.double(), (KH, KW), padding=pad, stride=stride)       # [N, C·T, L], c-major
    T = KH * KW
    if stem:
        idx = _stem_cols(C)
        u = torch.cat([u, torch.zeros_like(u[:, :1])], 1)
        return u[:, torch.where(idx < 0, torch.full_like(idx, C * T), idx)]
    return u.view(N, C, T, -1).transpose(1, 2).reshape(N, T * C, -1)


def _kernel_w(w, stem):
    Co, C, KH, KW = w.shape
    if stem:
        idx = _stem_cols(C)
        wf = torch.cat([w.double().reshape(Co, -1), torch.zeros(Co, 1, dtype=torch.float64)], 1)
        return wf[:, torch.where(idx < 0, torch.full_like(idx, C * KH * KW), idx)]
    return w.double().permute(0, 2, 3, 1).reshape(Co, KH * KW * C)


class _KConv(torch.autograd.Function):
    """conv2d (no bias) with the FWD / DGRAD / WGRAD accumulation orders of ttmi_conv.hip."""

    @staticmethod
    def forward(ctx, x, w, stride, pad, stem):
        N, C, H, W = x.shape
        Co, _, KH, KW = w.shape
        Ho, Wo = (H + 2 * pad - KH) // stride + 1, (W + 2 * pad - KW) // stride + 1
        cols = _kernel_cols(x, KH, KW, stride, pad, stem)                  # [N, K, L]
        wk = _kernel_w(w, stem)                                              # [Co, K]
        acc = torch.zeros(N, Co, Ho * Wo)
        for k0 in range(0, wk.shape[1], _KCHUNK):
            acc += torch.einsum("ok,nkl->nol", wk[:, k0:k0 + _KCHUNK], cols[:, k0:k0 + _KCHUNK]).float()
        ctx.save_for_backward(x, w)
        ctx.geo = (stride, pad, stem)
        return acc.view(N, Co, Ho, Wo)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        stride, pad, stem = ctx.geo
        N, C, H, W = x.shape
        Co, _, KH, KW = w.shape
        Ho, Wo = gy.shape[2:]
        gd = gy.double()
        dx = None
        if ctx.needs_input_grad[0] and not stem:     # DGRAD (the stem's input grad is never needed)
            s = stride
            buf = torch.zeros(N, C, H + 2 * pad + s * KH, W + 2 * pad + s * KW)
            for kh in range(KH):
                for kw in range(KW):
                    sl = buf[:, :, kh:kh + s * Ho:s, kw:kw + s * Wo:s]
                    for c0 in range(0, Co, _KCHUNK):
                        sl += torch.einsum("nohw,oc->nchw", gd[:, c0:c0 + _KCHUNK],
                                           w[c0:c0 + _KCHUNK, :, kh, kw].double()).float()
            dx = buf[:, :, pad:pad + H, pad:pad + W].contiguous()
        # WGRAD: pixels m = (n, ho, wo); splits as conv_plan; 32-pixel chunks; split order
        cols = _kernel_cols(x, KH, KW, stride, pad, stem)                   # [N, K, L]
        K = cols.shape[1]
        cm = cols.permute(0, 2, 1).reshape(N * Ho * Wo, K)                  # [M, K]
        dm = gd.permute(0, 2, 3, 1).reshape(N * Ho * Wo, Co)                 # [M, Co]
        M = cm.shape[0]
        bm = 128 if Co % 128 == 0 else 64
        tiles = -(-Co // bm) * -(-K // 128)
        ksteps = -(-M // 64)
        want = max(1, -(-1024 // tiles))
        per = max(min(8, ksteps), -(-ksteps // want))
        ksplit = per * 64
        parts = []
        for s0 in range(0, M, ksplit):
            acc = torch.zeros(Co, K)
            for p0 in range(s0, min(M, s0 + ksplit), _KCHUNK):
                acc += (dm[p0:p0 + _KCHUNK].t() @ cm[p0:p0 + _KCHUNK]).float()
            parts.append(acc)
        if len(parts) > 16:                       # chunk totals in place, then the chunk slabs
            parts = [_seq_sum(parts[i:i + 16]) for i in range(0, len(parts), 16)]
        dwk = _seq_sum(parts)
        if stem:
            idx = _stem_cols(C)
            dw = torch.zeros(Co, C * KH * KW)
            dw[:, idx[idx >= 0]] = dwk[:, idx >= 0]
            dw = dw.view(Co, C, KH, KW)
        else:
            dw = dwk.view(Co, KH, KW, C).permute(0, 3, 1, 2).contiguous()
        return dx, dw, None, None, None


def _seq_sum(ts):
    s = torch.zeros_like(ts[0])
    for t in ts:
        s += t
    return s


_ORDER = ["torch"]


def _emu_conv_bn(p, x, wname, bn, stride, pad, residual=None, relu=True, stem=False):
    """conv (bf16 operands, fp32 accumulate in the order _ORDER[0]) -> BN as the kernels
    compute it (_BnKernel) -> residual -> ReLU -> bf16."""
    w = p[wname]
    wq = w.detach().to(torch.bfloat16).float() + (w - w.detach())
    if _ORDER[0] == "kernel":
        y32 = _KConv.apply(x, wq, stride, pad, stem)
    else:
        y32 = _conv_order(x, wq, stride, pad, _ORDER[0])
    out = _BnKernel.apply(y32, p[bn + ".weight"], p[bn + ".bias"])
    if residual is not None:
        out = out + residual
    if relu:
        out = torch.relu(out)
    return rb(out)


def resnet18_bf16_emulation(p, x, prefix="", update_running=False, order="torch"):
    _ORDER[0] = order
    try:
        return _resnet18_bf16_emulation(p, x, prefix)
    finally:
        _ORDER[0] = "torch"


def _resnet18_bf16_emulation(p, x, prefix=""):
    if prefix:
        p = {k[len(prefix):]: v for k, v in p.items() if k.startswith(prefix)}
    y = _emu_conv_bn(p, rb(x), "conv1.weight", "bn1", 2, 3, stem=x.shape[2] % 2 == 0 and x.shape[3] % 2 == 0)
    y = rb(TF.max_pool2d(y, 3, 2, 1))
    for lname, cin, cout, s in rref.LAYERS:
        for bi in range(2):
            b = f"{lname}.{bi}."
            st = s if bi == 0 else 1
            idn = y
            if b + "downsample.0.weight" in p:
                idn = _emu_conv_bn(p, _GradRound.apply(y), b + "downsample.0.weight",
                                   b + "downsample.1", st, 0, relu=False)
            h = _emu_conv_bn(p, y, b + "conv1.weight", b + "bn1", st, 1)
            y = _emu_conv_bn(p, h, b + "conv2.weight", b + "bn2", 1, 1, residual=rb(idn))
    feat = rb(TF.adaptive_avg_pool2d(y, 1).flatten(1))
    w = p["fc.weight"]
    # the kernels take the fc's upstream gradient as a bf16 GEMM operand
    return _GradRound.apply(TF.linear(feat, w.detach().to(torch.bfloat16).float() + (w - w.detach()),
                                      p["fc.bias"]))


def _cos(a, b):
    a = a.detach().double().cpu().flatten()
    b = b.detach().double().cpu().flatten()
    return torch.dot(a, b).item() / (a.norm().item() * b.norm().item() + 1e-30)


@pytest.mark.parametrize("in_ch,H,W,N", [(1, 64, 96, 8), (3, 64, 64, 8),
                                          (1, 128, 256, 4), (3, 224, 224, 4)])
def test_resnet18_vs_oracle(gpu_pkg, in_ch, H, W, N):
    """GPU ResNet-18 vs the fp32 oracle (oracle/resnet_ref.py), with the bf16-emulating
    restatement above as the yardstick for how close any bf16-storage implementation can get.

    Measured on CPU: emulation vs fp32 gives gradient cosines of 0.93 at the stem rising to
    0.98 at layer4 and 1.0 at fc — the train-mode BN backward over 20 layers amplifies bf16
    storage noise.  Which bf16 roundings happen depends on the fp32 accumulation order of the
    convolutions, and at N = 4 that alone moves a BatchNorm parameter's cosine by up to 0.024
    (1x128x256) / 0.036 (3x224²) between the EMU_ORDERS (tools/diag_resnet_margin.py).  The
    conv kernels' own order (_KConv: their k-step / MFMA-chunk / split-K sums) is one of them,
    and it does not narrow the band: at 3x224² its BatchNorm-parameter cosines fall anywhere
    inside the other orders' range (the MFMA's internal summation order, which no emulation
    here knows, already moves individual bf16 roundings).  So per parameter the GPU gradient
    must be as close to fp32 as the worst of those orders within 0.03 in cosine, with a norm
    ratio within 0.05 of the farthest (every parameter, every size); the output must agree to
    5e-2 (fp32) / 2e-2 (the kernel-order emulation)."""
    cnn = gpu_pkg.cnn
    torch.manual_seed(in_ch)
    net = cnn.ResNet18(in_ch, 128).to(DEV)
    g = torch.Generator().manual_seed(11)
    x = torch.randn(N, in_ch, H, W, generator=g)
    up = torch.randn(N, 128, generator=g)
    sd0 = {k: v.detach().cpu().clone() for k, v in net.state_dict().items()}

    def leaf():
        return {k: (v.clone().requires_grad_(True) if v.is_floating_point() and "running" not in k
                    else v.clone()) for k, v in sd0.items()}

    Pr = leaf()
    out_ref = rref.resnet18_forward(Pr, x, update_running=True)
    (out_ref * up).sum().backward()
    emus = []
    for order in EMU_ORDERS:
        Pe = leaf()
        o = resnet18_bf16_emulation(Pe, x, order=order)
        (o * up).sum().backward()
        emus.append((o.detach(), Pe))
    out_emu = emus[0][0]
    out = net(x.to(DEV))
    (out * up.to(DEV)).sum().backward()
    torch.cuda.synchronize()
    assert rel(out, out_emu) < 2e-2, rel(out, out_emu)
    assert rel(out, out_ref) < 5e-2, rel(out, out_ref)
    bad = []
    for name, p in net.named_parameters():
        gr = Pr[name].grad
        cr = _cos(p.grad, gr)
        nr = p.grad.norm().item() / gr.norm().item()
        ce = [_cos(Pe[name].grad, gr) for _, Pe in emus]
        ne = [Pe[name].grad.norm().item() / gr.norm().item() for _, Pe in emus]
        print("GRAD", name, f"gpu~fp32 {cr:.4f} emu~fp32 min {min(ce):.4f} max {max(ce):.4f} "
              f"norm gpu {nr:.4f} emu {min(ne):.4f}..{max(ne):.4f}")
        print("GRAD", name, f"kernel-order emu~fp32 {ce[0]:.4f} norm {ne[0]:.4f}")
        if not (cr > min(ce) - 0.03 and abs(nr - 1) < max(abs(v - 1) for v in ne) + 0.05):
            bad.append((name, cr, min(ce), nr, ne))
    assert not bad, bad
    sd = net.state_dict()
    for k in sd:
        if "running_mean" in k:
            # mean error relative to the batch std (momentum 0.1 applied to both): channel
            # means sit near zero next to their spread, so a plain relative norm is ill-posed
            rv = Pr[k.replace("mean", "var")]
            scale = 0.1 * ((rv - 0.9) / 0.1).clamp_min(0).sqrt()
            assert (sd[k].cpu() - Pr[k]).norm() < 2e-2 * scale.norm(), k
        if "running_var" in k:
            assert rel(sd[k], Pr[k]) < 1e-2, k
        if "num_batches_tracked" in k:
            assert int(sd[k]) == 1, k


def test_tabular_encoder_vs_oracle(gpu_pkg):
    cnn = gpu_pkg.cnn
    torch.manual_seed(0)
    enc = cnn.TabularEncoder(128, 128).to(DEV)
    enc.mlp[3].p = 0.0
    g = torch.Generator().manual_seed(3)
    x = torch.randn(64, 128, generator=g)
    up = torch.randn(64, 128, generator=g)
    Pr = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in enc.named_parameters()}
    out_ref = rref.tabular_forward(Pr, x)
    (out_ref * up).sum().backward()
    out = enc(x.to(DEV))
    (out * up.to(DEV)).sum().backward()
    torch.cuda.synchronize()
    assert rel(out, out_ref) < 3e-2
    for name, p in enc.named_parameters():
        if name == "mlp.0.bias":       # exactly zero in math (BatchNorm follows)
            assert p.grad.abs().max().item() < 3e-2 * max(1.0, Pr[name].grad.abs().max().item())
            continue
        check_grad(name, p.grad, Pr[name].grad)


@pytest.mark.parametrize("name", ["tabular_t128.npz", "tabular_t37.npz"])
def test_tabular_encoder_vs_reference_fixture(gpu_pkg, name):
    """TabularEncoder (the reference's own class ran to make the fixture: item_tower.py:85-98,
    train mode, dropout off; T = 37 exercises the zero-padded operand path) vs the fixture:
    bf16 output within 3e-2, gradients by direction / norm, BN running stats to 1e-2 (the
    running mean is 0.1 x the batch mean of a bf16-operand Linear's output: ~2e-3 of its
    near-zero values)."""
    from conftest import load_golden, sub
    cnn = gpu_pkg.cnn
    z = load_golden(name)
    T, B = z["cfg"].tolist()
    enc = cnn.TabularEncoder(T, 128).to(DEV)
    enc.mlp[3].p = 0.0
    enc.load_state_dict({k: torch.tensor(v) for k, v in sub(z, "p/").items()})
    out = enc(torch.tensor(z["x"]).to(DEV))
    (out * torch.tensor(z["upstream"]).to(DEV)).sum().backward()
    torch.cuda.synchronize()
    assert rel(out, torch.tensor(z["out"])) < 3e-2
    ref_g = sub(z, "g/")
    for name_, p in enc.named_parameters():
        if name_ == "mlp.0.bias":       # exactly zero in math (BatchNorm follows)
            assert p.grad.abs().max().item() < 3e-2 * max(1.0, np.abs(ref_g[name_]).max())
            continue
        check_grad(name_, p.grad, torch.tensor(ref_g[name_]))
    sd = enc.state_dict()
    for k, v in sub(z, "after/").items():
        if "running" in k:
            assert rel(sd[k], torch.tensor(v)) < 1e-2, k
        if "num_batches_tracked" in k:
            assert int(sd[k]) == int(v), k


def test_resnet18_eval_mode_uses_running_stats(gpu_pkg):
    """eval(): BatchNorm2d normalises with the running statistics (nn.BatchNorm2d.eval())."""
    cnn = gpu_pkg.cnn
    torch.manual_seed(4)
    net = cnn.ResNet18(3, 128).to(DEV)
    g = torch.Generator().manual_seed(5)
    with torch.no_grad():
        for _ in range(3):                     # populate the running statistics
            net(torch.randn(8, 3, 64, 64, generator=g).to(DEV))
    net.eval()
    x = torch.randn(4, 3, 64, 64, generator=g)
    with torch.no_grad():
        out = net(x.to(DEV))
    sd = {k: v.detach().cpu() for k, v in net.state_dict().items()}
    assert int(sd["bn1.num_batches_tracked"]) == 3
    y = TF.conv2d(x, sd["conv1.weight"], stride=2, padding=3)

    def bn(t, n):
        return TF.batch_norm(t, sd[n + ".running_mean"], sd[n + ".running_var"],
                             sd[n + ".weight"], sd[n + ".bias"], training=False)
    y = TF.max_pool2d(torch.relu(bn(y, "bn1")), 3, 2, 1)
    for lname, _, _, s in rref.LAYERS:
        for bi in range(2):
            b = f"{lname}.{bi}."
            st = s if bi == 0 else 1
            h = torch.relu(bn(TF.conv2d(y, sd[b + "conv1.weight"], stride=st, padding=1), b + "bn1"))
            h = bn(TF.conv2d(h, sd[b + "conv2.weight"], padding=1), b + "bn2")
            idn = y
            if b + "downsample.0.weight" in sd:
                idn = bn(TF.conv2d(y, sd[b + "downsample.0.weight"], stride=st), b + "downsample.1")
            y = torch.relu(h + idn)
    ref_out = TF.linear(TF.adaptive_avg_pool2d(y, 1).flatten(1), sd["fc.weight"], sd["fc.bias"])
    assert rel(out, ref_out) < 5e-2, rel(out, ref_out)
    assert int(net.state_dict()["bn1.num_batches_tracked"]) == 3     # eval updates nothing


def _cfg3(pkg, B=8, L=12, V=211, T=32, mel=(64, 96), cover=(64, 64), seed=0, p=0.0):
    torch.manual_seed(seed)
    m = pkg.TwoTowerModel(with_text=False, vocab_size=V, tabular_input_dim=T, num_genders=3, num_countries=8,
                          max_seq_len=L, user_embedding_dim=128, item_embedding_dim=128,
                          user_dropout=p, precomputed_modalities=False).to(DEV)
    m.item_tower.fusion_layer[3].p = p
    m.item_tower.tabular_encoder.mlp[3].p = p
    g = torch.Generator().manual_seed(seed + 1)
    batch = ref.synthetic_batch(B, L, V, num_countries=8, generator=g)
    del batch["target_modal"]
    batch.update(rref.synthetic_items(B, T, mel, cover, generator=g))
    return m, batch


@pytest.mark.parametrize("B,mel,cover", [(8, (64, 96), (64, 64)), (4, (128, 256), (224, 224))])
def test_cfg3_two_tower_vs_oracle(gpu_pkg, B, mel, cover):
    """cfg 3 (raw mels / covers / tabular, zero text slot): loss and logits vs the fp32
    oracle, item-tower gradients by direction and norm against the same emulation yardstick in
    three accumulation orders, the conv kernels' own among them (cosine within 0.03 of the
    worst, norm ratio within 0.05 of the farthest; every reduction is fixed-order or int64 fixed
    point, so the GPU value is the same on every run).  bf16 storage through two ResNet-18s moves the
    item embedding ~2 %, which τ = 0.07 amplifies in the logits; the loss bound is 2x the
    deviation of the bf16-emulating oracle (same rounding points as the kernels) + 2e-2: the
    summation order alone moves the full-size loss by that much (tools/diag_cfg3_loss.py: the
    four equivalent kernel paths — register / LDS-DMA tiles x padded / space-to-depth stem —
    give 2.1058 … 2.1185 at B = 4, 224², against 2.0915 fp32 and 2.1018 emulated).
    (The 1e-3 north-star bar is cfg 2's, whose item inputs are precomputed.)  Run at a small
    size and at BASELINE configs[2]'s stated inputs (1x128x256 mels, 3x224x224 covers)."""
    m, batch = _cfg3(gpu_pkg, B=B, mel=mel, cover=cover)
    params = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in m.named_parameters()}
    lref, logits_ref, _, _ = ref.two_tower_loss(params, batch, running=None)
    lref.backward()
    orig = rref.resnet18_forward
    emus = []
    for order in ("kernel", "torch", "f64"):     # bf16-storage yardsticks (see test_resnet18_vs_oracle)
        rref.resnet18_forward = lambda p, x, prefix="", update_running=False, o=order: \
            resnet18_bf16_emulation(p, x, prefix, order=o)
        try:
            pe = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in m.named_parameters()}
            le, le_logits = ref.two_tower_loss(pe, batch, running=None)[:2]
            le.backward()
            emus.append((pe, float(le), le_logits))
        finally:
            rref.resnet18_forward = orig
    pe, lemu, logits_emu = emus[0]
    bd = {k: v.to(DEV) for k, v in batch.items()}
    loss, logits, _, _ = m(bd)
    loss.backward()
    torch.cuda.synchronize()
    bound = 2.0 * abs(lemu - float(lref)) + 2e-2
    assert abs(float(loss) - float(lref)) < bound, (float(loss), float(lref), lemu)
    # same yardstick as the loss: 2x the bf16-emulation's own logit deviation + 1e-2
    assert rel(logits, logits_ref) < 2.0 * rel(logits_emu, logits_ref) + 1e-2, \
        (rel(logits, logits_ref), rel(logits_emu, logits_ref))
    mine = dict(m.named_parameters())
    # identically-zero true gradients (a bias feeding straight into a train-mode BatchNorm:
    # fusion_layer.0.bias, the tabular mlp.0.bias; and every encoder's last bias, whose output
    # enters fusion_layer.0 -> BatchNorm1d, so Σ_batch dmodal = W0ᵀ·Σ dz = 0): noise vs noise
    zero = ("fusion_layer.0.bias", "mlp.0.bias", "backbone.fc.bias", "mlp.4.bias")
    for k in mine:
        if k.startswith("item_tower.") and k.endswith(zero):
            assert mine[k].grad.abs().max().item() < 3e-2 * max(
                1.0, params[k].grad.abs().max().item()), k
    names = [k for k in mine if k.startswith("item_tower.") and not k.endswith(zero)]
    assert any("audio_encoder" in k for k in names) and any("visual_encoder" in k for k in names)
    bad = []
    for k in names:       # as close to fp32 as the bf16 emulations get (see above)
        g, gr = mine[k].grad, params[k].grad
        cos = _cos(g, gr)
        nr = g.norm().item() / gr.norm().item()
        cos_e = min(_cos(e[0][k].grad, gr) for e in emus)
        ne = max(abs(e[0][k].grad.norm().item() / gr.norm().item() - 1) for e in emus)
        print("GRAD", k, f"gpu~fp32 {cos:.4f} emu~fp32 min {cos_e:.4f} norm gpu {nr:.4f} emu dev {ne:.4f}")
        if not (cos > cos_e - 0.03 and abs(nr - 1) < ne + 0.05):
            bad.append((k, cos, cos_e, nr, ne))
    assert not bad, bad


def test_cfg3_train_step_graph_equals_eager_bitexact_and_learns(gpu_pkg):
    """cfg-3 TrainStep (two ResNet-18s + tabular + heads, dropout on): the HIP-graph replay and
    the eager schedule are bit-identical for 3 steps — losses, parameters, BatchNorm running
    buffers, AdamW moments (the conv BatchNorm statistics, the BN backward sums and the split
    conv weight gradients are int64 fixed point or fixed-order) — and the loss decreases."""
    m1, batch = _cfg3(gpu_pkg, B=16, seed=7, p=0.1)
    m2, _ = _cfg3(gpu_pkg, B=16, seed=7, p=0.1)
    bd = {k: v.to(DEV) for k, v in batch.items()}
    s1 = gpu_pkg.TrainStep(m1, lr=1e-3, use_graph=True, seed=11)
    s2 = gpu_pkg.TrainStep(m2, lr=1e-3, use_graph=False, seed=11)
    l1 = []
    for i in range(3):
        a, b = float(s1.step(bd)), float(s2.step(bd))
        assert a == b, (i, a, b)
        l1.append(a)
    torch.cuda.synchronize()
    sa = {k: v.detach().clone() for k, v in m1.state_dict().items()}
    sb = {k: v.detach().clone() for k, v in m2.state_dict().items()}
    sa["__m"], sb["__m"] = s1.flat.exp_avg.clone(), s2.flat.exp_avg.clone()
    sa["__v"], sb["__v"] = s1.flat.exp_avg_sq.clone(), s2.flat.exp_avg_sq.clone()
    bad = [k for k in sa if not torch.equal(sa[k], sb[k])]
    assert not bad, bad[:8]
    l1 += [float(s1.step(bd)) for _ in range(9)]
    assert l1[-1] < l1[0] - 0.2, l1
    bufs = dict(m1.named_buffers())
    assert int(bufs["item_tower.audio_encoder.backbone.bn1.num_batches_tracked"]) == 12
    assert int(bufs["item_tower.tabular_encoder.mlp.1.num_batches_tracked"]) == 12

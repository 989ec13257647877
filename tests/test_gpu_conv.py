"""ResNet-18 building blocks (cfg 3) vs fp32 PyTorch on the same bf16-rounded operands.

Convolutions: FWD output and BatchNorm column statistics, DGRAD (input grad, with the
residual-branch addend) and WGRAD (weight grad in torch layout) against F.conv2d and its
autograd, over the torchvision resnet18 conv shapes (7x7/2 stem with 1 and 3 channels padded
to 8, 3x3/1, 3x3/2, 1x1/2 downsample).  bf16 outputs are compared at bf16 rounding (8e-3),
fp32 reductions at 2e-5 relative (x sqrt(K/256) for long reductions)."""
import math

import pytest
import torch
import torch.nn.functional as TF

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-30)


def nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def nchw(t):
    return t.permute(0, 3, 1, 2).contiguous()


SHAPES = [  # N, Cin, H, W, Co, k, stride, pad
    (2, 1, 30, 40, 64, 7, 2, 3),
    (2, 3, 33, 29, 64, 7, 2, 3),
    (2, 64, 14, 14, 64, 3, 1, 1),
    (3, 64, 15, 13, 128, 3, 2, 1),
    (3, 64, 15, 13, 128, 1, 2, 0),
    (2, 128, 7, 9, 256, 3, 2, 1),
    (2, 256, 5, 4, 512, 3, 1, 1),
    (4, 128, 20, 18, 128, 3, 1, 1),
    (2, 128, 9, 11, 256, 1, 2, 0),
    # full-size cfg-3 shapes (BASELINE configs[2]): the 224² cover stem (M = 25,088 output
    # rows at N = 2), the 1x128x256 mel stem, and visual layer 1/2 at 56²
    (2, 3, 224, 224, 64, 7, 2, 3),
    (2, 1, 128, 256, 64, 7, 2, 3),
    (2, 64, 56, 56, 64, 3, 1, 1),
    (2, 64, 56, 56, 128, 3, 2, 1),
    (2, 64, 56, 56, 128, 1, 2, 0),
]


@pytest.mark.parametrize("bm", ["64", "128", "dma"])
@pytest.mark.parametrize("N,Cin,H,W,Co,k,s,p", SHAPES)
def test_conv_fwd_dgrad_wgrad(gpu_pkg, monkeypatch, bm, N, Cin, H, W, Co, k, s, p):
    """Every FWD/DGRAD kernel on every shape: the register-staged tile at both heights
    (TTMI_CONV_BM, TTMI_CONV_DMA=0) and the 256-row LDS-DMA tile (TTMI_CONV_DMA=1, forced even
    where the grid is small): partial tiles, stride-2 DGRAD parity classes (incl. the empty
    classes of a 1x1/2 conv: dx = addend), the 8-channel padded stems (per-lane taps, k past
    K zero-filled), and WGRAD split-K with the fixed-order partial reduction."""
    if bm == "dma":
        monkeypatch.setenv("TTMI_CONV_DMA", "1")
    else:
        monkeypatch.setenv("TTMI_CONV_DMA", "0")
        monkeypatch.setenv("TTMI_CONV_BM", bm)
    ops = gpu_pkg.ops
    g = torch.Generator().manual_seed(N * 1000 + Cin + Co + k)
    Cp = (Cin + 7) // 8 * 8
    x = torch.randn(N, Cin, H, W, generator=g).to(torch.bfloat16).float()
    w = (torch.randn(Co, Cin, k, k, generator=g) / math.sqrt(Cin * k * k)).to(torch.bfloat16).float()
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    y_ref = TF.conv2d(xr, wr, stride=s, padding=p)
    Ho, Wo = ops.conv_out_hw(H, W, k, s, p)
    assert y_ref.shape[2:] == (Ho, Wo)
    dy = torch.randn(y_ref.shape, generator=g).to(torch.bfloat16).float()
    y_ref.backward(dy)
    # device operands
    xd = torch.empty(N, H, W, Cp, device=DEV, dtype=torch.bfloat16)
    ops.nchw_to_nhwc(x.to(DEV), Cp, xd)
    assert torch.equal(xd[..., :Cin].float().cpu(), nhwc(x))
    wf = torch.empty(Co, k, k, Cp, device=DEV, dtype=torch.bfloat16)
    wd = torch.empty(Cin, k, k, Co, device=DEV, dtype=torch.bfloat16)
    ops.conv_weight_prep(w.to(DEV), Cp, wf, wd)
    y = torch.empty(N, Ho, Wo, Co, device=DEV, dtype=torch.bfloat16)
    R = ops.CONV_STAT_REPS
    csr = torch.zeros(R, Co, device=DEV, dtype=torch.int64)     # int64 fixed point, 2^-24
    cqr = torch.zeros(R, Co, device=DEV, dtype=torch.int64)
    ops.conv2d(ops.FWD, N, H, W, Cp, Cin, Co, k, s, p, x=xd, w=wf, out=y, colsum=csr,
               colsumsq=cqr)
    cs, cq = csr.sum(0).double() * 2.0 ** -24, cqr.sum(0).double() * 2.0 ** -24
    torch.cuda.synchronize()
    yr = y_ref.detach()
    assert rel(nchw(y.float()), yr) < 8e-3
    Kred = Cin * k * k
    tol = 2e-5 * max(1.0, math.sqrt(Kred / 256))
    assert rel(cs, yr.sum((0, 2, 3))) < 5e-3            # stats of the fp32 (pre-round) output
    assert rel(cq, (yr ** 2).sum((0, 2, 3))) < 5e-3
    dyd = nhwc(dy).to(torch.bfloat16).to(DEV)
    dw = torch.full((Co, Cin, k, k), 0.25, device=DEV)
    ops.conv2d(ops.WGRAD, N, H, W, Cp, Cin, Co, k, s, p, x=xd, dy=dyd, out=dw)
    torch.cuda.synchronize()
    Mred = N * Ho * Wo
    assert rel(dw, 0.25 + wr.grad) < 2e-5 * max(1.0, math.sqrt(Mred / 256)) * 4
    if Cp == Cin:
        add = torch.randn(N, H, W, Cin, generator=g).to(torch.bfloat16)
        dx = torch.empty(N, H, W, Cin, device=DEV, dtype=torch.bfloat16)
        ops.conv2d(ops.DGRAD, N, H, W, Cin, Cin, Co, k, s, p, dy=dyd, w=wd, out=dx,
                   addend=add.to(DEV))
        torch.cuda.synchronize()
        assert rel(nchw(dx.float()), xr.grad + nchw(add.float())) < 8e-3


@pytest.mark.parametrize("variant", ["reg", "dma"])
@pytest.mark.parametrize("N,Cin,H,W", [(2, 3, 224, 224), (2, 1, 128, 256), (3, 3, 30, 34),
                                       (2, 1, 16, 18)])
def test_stem_s2d(gpu_pkg, monkeypatch, variant, N, Cin, H, W):
    """The 7x7/2/3 stem as a 4x4/1 conv over the space-to-depth input (ttmi_stem_s2d, conv
    modes 3 / 4): FWD output + BatchNorm column sums and WGRAD in torch's [Co][Cin][7][7]
    layout against F.conv2d and its autograd, on both kernel families."""
    monkeypatch.setenv("TTMI_CONV_DMA", "1" if variant == "dma" else "0")
    ops = gpu_pkg.ops
    g = torch.Generator().manual_seed(N * 100 + Cin + H)
    Co = 64
    x = torch.randn(N, Cin, H, W, generator=g).to(torch.bfloat16).float()
    w = (torch.randn(Co, Cin, 7, 7, generator=g) / math.sqrt(Cin * 49)).to(torch.bfloat16).float()
    wr = w.clone().requires_grad_(True)
    y_ref = TF.conv2d(x, wr, stride=2, padding=3)
    dy = torch.randn(y_ref.shape, generator=g).to(torch.bfloat16).float()
    y_ref.backward(dy)
    Cp = gpu_pkg.cnn.stem_s2d_cp(Cin)
    xd = torch.empty(N, H // 2, W // 2, Cp, device=DEV, dtype=torch.bfloat16)
    ops.stem_s2d(x.to(DEV), Cp, xd)
    xs = x.reshape(N, Cin, H // 2, 2, W // 2, 2).permute(0, 2, 4, 3, 5, 1).reshape(N, H // 2, W // 2, 4 * Cin)
    assert torch.equal(xd[..., :4 * Cin].float().cpu(), xs)
    assert not xd[..., 4 * Cin:].any()
    wf = torch.empty(Co, 4, 4, Cp, device=DEV, dtype=torch.bfloat16)
    ops.stem_weight_prep(w.to(DEV), Cp, wf)
    Ho, Wo = H // 2, W // 2
    y = torch.empty(N, Ho, Wo, Co, device=DEV, dtype=torch.bfloat16)
    R = ops.CONV_STAT_REPS
    csr = torch.zeros(R, Co, device=DEV, dtype=torch.int64)
    cqr = torch.zeros(R, Co, device=DEV, dtype=torch.int64)
    ops.conv2d(ops.STEM_FWD, N, H, W, Cp, Cin, Co, 7, 2, 3, x=xd, w=wf, out=y, colsum=csr, colsumsq=cqr)
    torch.cuda.synchronize()
    yr = y_ref.detach()
    assert rel(nchw(y.float()), yr) < 8e-3
    cs, cq = csr.sum(0).double() * 2.0 ** -24, cqr.sum(0).double() * 2.0 ** -24
    assert rel(cs, yr.sum((0, 2, 3))) < 5e-3
    assert rel(cq, (yr ** 2).sum((0, 2, 3))) < 5e-3
    dyd = nhwc(dy).to(torch.bfloat16).to(DEV)
    dw = torch.full((Co, Cin, 7, 7), 0.25, device=DEV)
    ops.conv2d(ops.STEM_WGRAD, N, H, W, Cp, Cin, Co, 7, 2, 3, x=xd, dy=dyd, out=dw)
    torch.cuda.synchronize()
    assert rel(dw, 0.25 + wr.grad) < 2e-5 * max(1.0, math.sqrt(N * Ho * Wo / 256)) * 4


@pytest.mark.parametrize("N,H,W", [(2, 112, 112), (3, 13, 10)])
def test_stem_pool_fused(gpu_pkg, N, H, W):
    """ttmi_stem_pool_fwd / _bwd (bn1 + ReLU + maxpool with the BN output never stored) against
    the unfused bn2d_fwd + maxpool_fwd and maxpool_bwd + bn2d_bwd: forward bit-identical
    (pooled map, taps, saved stats, running stats), backward dx / dw / db to fp32 reduction
    order (the fused reduce walks other row slabs), eval mode bit-identical."""
    ops = gpu_pkg.ops
    C = 64
    g = torch.Generator().manual_seed(H * 10 + N)
    x = (torch.randn(N, H, W, C, generator=g) * 2 + 0.3).to(torch.bfloat16).to(DEV)
    R = ops.CONV_STAT_REPS
    xf = x.float()
    cs = torch.zeros(R, C, dtype=torch.int64, device=DEV)
    cq = torch.zeros(R, C, dtype=torch.int64, device=DEV)
    cs[0] = torch.round(xf.sum((0, 1, 2)).double() * 2 ** 24).long()
    cq[0] = torch.round((xf ** 2).sum((0, 1, 2)).double() * 2 ** 24).long()
    w = (torch.rand(C, generator=g) + 0.5).to(DEV)
    w[::7] *= -1                                      # negative scales flip the window order
    b = (torch.randn(C, generator=g) * 0.5).to(DEV)
    Ho, Wo = ops.conv_out_hw(H, W, 3, 2, 1)
    rm1, rv1 = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    rm2, rv2 = rm1.clone(), rv1.clone()
    nb1 = torch.zeros(1, dtype=torch.int64, device=DEV)
    nb2 = nb1.clone()
    # unfused reference
    a = torch.empty_like(x)
    m1, r1 = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
    ops.bn2d_fwd(x, cs, cq, w, b, a, m1, r1, running_mean=rm1, running_var=rv1, num_batches=nb1, relu=True)
    y1 = torch.empty(N, Ho, Wo, C, device=DEV, dtype=torch.bfloat16)
    i1 = torch.empty(N, Ho, Wo, C, device=DEV, dtype=torch.uint8)
    ops.maxpool_fwd(a, 3, 2, 1, y1, i1)
    # fused
    y2, i2 = torch.empty_like(y1), torch.empty_like(i1)
    m2, r2 = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
    ops.stem_pool_fwd(x, cs, cq, w, b, y2, i2, m2, r2, running_mean=rm2, running_var=rv2, num_batches=nb2)
    torch.cuda.synchronize()
    assert torch.equal(y1, y2) and torch.equal(i1, i2)
    assert torch.equal(m1, m2) and torch.equal(r1, r2) and torch.equal(rm1, rm2) and torch.equal(rv1, rv2)
    assert nb2.item() == 1
    # eval mode (running statistics)
    y3, i3 = torch.empty_like(y1), torch.empty_like(i1)
    ops.bn2d_fwd(x, None, None, w, b, a, m1, r1, running_mean=rm1, running_var=rv1, relu=True)
    ops.maxpool_fwd(a, 3, 2, 1, y1, i1)
    ops.stem_pool_fwd(x, None, None, w, b, y3, i3, m2, r2, running_mean=rm2, running_var=rv2)
    torch.cuda.synchronize()
    assert torch.equal(y1, y3) and torch.equal(i1, i3)
    # backward
    ops.bn2d_fwd(x, cs, cq, w, b, a, m1, r1, relu=True)
    dy = torch.randn(N, Ho, Wo, C, generator=g).to(torch.bfloat16).to(DEV)
    dpool = torch.empty_like(x)
    ops.maxpool_bwd(dy, i2, 3, 2, 1, dpool)
    sums1 = torch.zeros(2 * R * C, dtype=torch.int64, device=DEV)
    dx1 = torch.empty_like(x)
    dw1, db1 = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    ops.bn2d_bwd(dpool, x, m1, r1, w, sums1, dx1, dw1, db1, gate=a)
    sums2 = torch.zeros_like(sums1)
    dx2 = torch.empty_like(x)
    dw2, db2 = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    ops.stem_pool_bwd(dy, i2, x, m1, r1, w, b, sums2, dx2, dw2, db2)
    torch.cuda.synchronize()
    assert rel(dw2, dw1) < 1e-5 and rel(db2, db1) < 1e-5
    assert rel(dx2.float(), dx1.float()) < 8e-3


@pytest.mark.parametrize("variant", ["reg", "dma"])
@pytest.mark.parametrize("N,C,H,W,Co,s,gate,add", [(2, 64, 14, 14, 64, 1, True, False),
                                                  (3, 64, 15, 13, 128, 2, True, True),
                                                  (2, 128, 9, 11, 128, 1, False, True)])
def test_dgrad_fused_bn_reduce(gpu_pkg, monkeypatch, variant, N, C, H, W, Co, s, gate, add):
    """DGRAD with the producing BatchNorm's backward reduction in its epilogue
    (ttmi_conv_desc.bn_sums) against DGRAD + ttmi_bn2d_bwd_reduce: the gated g bit-identical,
    the fixed-point sums to fp32 partial-sum order; then bn2d_bwd_apply(g) = bn2d_bwd."""
    monkeypatch.setenv("TTMI_CONV_DMA", "1" if variant == "dma" else "0")
    ops = gpu_pkg.ops
    g = torch.Generator().manual_seed(N * 7 + C + Co)
    R = ops.CONV_STAT_REPS
    Ho, Wo = ops.conv_out_hw(H, W, 3, s, 1)
    dy = torch.randn(N, Ho, Wo, Co, generator=g).to(torch.bfloat16).to(DEV)
    w = (torch.randn(C, 3, 3, Co, generator=g) / math.sqrt(9 * Co)).to(torch.bfloat16).to(DEV)
    bx = torch.randn(N, H, W, C, generator=g).to(torch.bfloat16).to(DEV)
    bgate = torch.randn(N, H, W, C, generator=g).to(torch.bfloat16).to(DEV) if gate else None
    addend = torch.randn(N, H, W, C, generator=g).to(torch.bfloat16).to(DEV) if add else None
    mean = torch.randn(C, generator=g).to(DEV) * 0.1
    rstd = (torch.rand(C, generator=g) + 0.5).to(DEV)
    # unfused
    dx = torch.empty(N, H, W, C, device=DEV, dtype=torch.bfloat16)
    ops.conv2d(ops.DGRAD, N, H, W, C, C, Co, 3, s, 1, dy=dy, w=w, out=dx, addend=addend)
    s1 = torch.zeros(2 * R * C, dtype=torch.int64, device=DEV)
    g1 = torch.empty_like(dx)
    wbn = (torch.rand(C, generator=g) + 0.5).to(DEV)
    dxa = torch.empty_like(dx)
    dw1, db1 = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    ops.bn2d_bwd(dx, bx, mean, rstd, wbn, s1, dxa, dw1, db1, gate=bgate, g_out=g1)
    # fused
    g2 = torch.empty_like(dx)
    s2 = torch.zeros_like(s1)
    ops.conv2d(ops.DGRAD, N, H, W, C, C, Co, 3, s, 1, dy=dy, w=w, out=g2, addend=addend,
               bn=(bgate, bx, mean, rstd, s2))
    dxb = torch.empty_like(dx)
    dw2, db2 = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    ops.bn2d_bwd_apply(g2, bx, mean, rstd, wbn, s2, dxb, dw2, db2)
    torch.cuda.synchronize()
    assert torch.equal(g1, g2)
    t1 = s1.view(R, 2 * C).sum(0).double()
    t2 = s2.view(R, 2 * C).sum(0).double()
    assert rel(t2, t1) < 1e-5
    assert rel(dw2, dw1) < 1e-5 and rel(db2, db1) < 1e-5
    assert rel(dxb.float(), dxa.float()) < 8e-3


def test_conv_weight_prep_batch(gpu_pkg):
    """ttmi_conv_weight_prep_batch (one launch for every mirror of a network, split into
    launches of TTMI_WPREP_MAX items) = the per-conv conv_weight_prep / stem_weight_prep."""
    ops = gpu_pkg.ops
    g = torch.Generator().manual_seed(3)
    shapes = [(64, 3, 7, 16, True), (64, 1, 7, 8, False)] + [(64 * (1 + i % 3), 64 * (1 + i % 2), 3 if i % 4 else 1,
                                                              64 * (1 + i % 2), False) for i in range(27)]
    items, ref = [], []
    for Co, Cin, k, Cp, s2d in shapes:
        w = torch.randn(Co, Cin, k, k, generator=g).to(DEV)
        kk = 4 if s2d else k
        wf = torch.full((Co, kk, kk, Cp), 7.0, device=DEV, dtype=torch.bfloat16)
        wd = None if (s2d or Cin < 8) else torch.full((Cin, k, k, Co), 7.0, device=DEV, dtype=torch.bfloat16)
        items.append((w, Cp, wf, wd, s2d))
        rf = torch.empty_like(wf)
        rd = None if wd is None else torch.empty_like(wd)
        if s2d:
            ops.stem_weight_prep(w, Cp, rf)
        else:
            ops.conv_weight_prep(w, Cp, rf, rd)
        ref.append((rf, rd))
    ops.conv_weight_prep_batch(items)
    torch.cuda.synchronize()
    for (w, Cp, wf, wd, s2d), (rf, rd) in zip(items, ref):
        assert torch.equal(wf, rf)
        assert (wd is None) or torch.equal(wd, rd)


@pytest.mark.parametrize("C,relu,res", [(64, True, False), (128, True, True), (512, False, False)])
def test_bn2d_fwd_bwd(gpu_pkg, C, relu, res):
    """BatchNorm2d (train) with stats from the conv epilogue's column sums, residual + ReLU,
    running stats; backward through the ReLU gate with g written for the residual branch."""
    ops = gpu_pkg.ops
    N, H, W = 3, 9, 7
    g = torch.Generator().manual_seed(C)
    x = (torch.randn(N, C, H, W, generator=g) * 2 + 0.3).to(torch.bfloat16).float()
    w = torch.randn(C, generator=g)
    b = torch.randn(C, generator=g)
    r = torch.randn(N, C, H, W, generator=g).to(torch.bfloat16).float()
    rm, rv = torch.randn(C, generator=g), torch.rand(C, generator=g) + 0.5
    xt, wt, bt = x.clone().requires_grad_(True), w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    rm_ref, rv_ref = rm.clone(), rv.clone()
    y_ref = TF.batch_norm(xt, rm_ref, rv_ref, wt, bt, training=True, momentum=0.1, eps=1e-5)
    if res:
        y_ref = y_ref + r
    if relu:
        y_ref = torch.relu(y_ref)
    dy = torch.randn(y_ref.shape, generator=g).to(torch.bfloat16).float()
    y_ref.backward(dy)
    xd = nhwc(x).to(torch.bfloat16).to(DEV)
    R = ops.CONV_STAT_REPS                    # replica rows: spread the sums over them
    cs = torch.zeros(R, C, dtype=torch.float64)
    cq = torch.zeros(R, C, dtype=torch.float64)
    cs[0] = nhwc(x)[:1].double().sum((0, 1, 2))
    cs[R - 1] = nhwc(x)[1:].double().sum((0, 1, 2))
    cq[0] = (nhwc(x)[:1].double() ** 2).sum((0, 1, 2))
    cq[R - 1] = (nhwc(x)[1:].double() ** 2).sum((0, 1, 2))
    # int64 fixed point, scale 2^24 (TTMI_FX_STAT_SHIFT), as the conv epilogue writes them
    cs = torch.round(cs * 2.0 ** 24).to(torch.int64).to(DEV)
    cq = torch.round(cq * 2.0 ** 24).to(torch.int64).to(DEV)
    y = torch.empty_like(xd)
    mean, rstd = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
    rmd, rvd, nb = rm.to(DEV), rv.to(DEV), torch.zeros(1, device=DEV, dtype=torch.int64)
    ops.bn2d_fwd(xd, cs, cq, w.to(DEV), b.to(DEV), y, mean, rstd, running_mean=rmd, running_var=rvd,
                 num_batches=nb, residual=nhwc(r).to(torch.bfloat16).to(DEV) if res else None, relu=relu)
    torch.cuda.synchronize()
    assert rel(nchw(y.float()), y_ref.detach()) < 8e-3
    assert rel(rmd, rm_ref) < 1e-5 and rel(rvd, rv_ref) < 1e-4 and int(nb) == 1
    sums = torch.zeros(ops.CONV_STAT_REPS * 2 * C, device=DEV, dtype=torch.int64)
    dx = torch.empty_like(xd)
    dw, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    gout = torch.empty_like(xd)
    ops.bn2d_bwd(nhwc(dy).to(torch.bfloat16).to(DEV), xd, mean, rstd, w.to(DEV), sums, dx, dw, db,
                 gate=y if relu else None, g_out=gout)
    torch.cuda.synchronize()
    assert rel(nchw(dx.float()), xt.grad) < 1e-2
    assert rel(dw, wt.grad) < 1e-3 and rel(db, bt.grad) < 1e-3
    gexp = dy * (y_ref.detach() > 0).float() if relu else dy
    assert rel(nchw(gout.float()), gexp) < 8e-3


def test_pools(gpu_pkg):
    ops = gpu_pkg.ops
    N, C, H, W = 2, 64, 17, 12
    g = torch.Generator().manual_seed(2)
    x = torch.randn(N, C, H, W, generator=g).to(torch.bfloat16).float()
    xt = x.clone().requires_grad_(True)
    y_ref = TF.max_pool2d(xt, 3, 2, 1)
    dy = torch.randn(y_ref.shape, generator=g).to(torch.bfloat16).float()
    y_ref.backward(dy)
    xd = nhwc(x).to(torch.bfloat16).to(DEV)
    Ho, Wo = y_ref.shape[2:]
    y = torch.empty(N, Ho, Wo, C, device=DEV, dtype=torch.bfloat16)
    idx = torch.empty(N, Ho, Wo, C, device=DEV, dtype=torch.uint8)
    ops.maxpool_fwd(xd, 3, 2, 1, y, idx)
    dx = torch.empty_like(xd)
    ops.maxpool_bwd(nhwc(dy).to(torch.bfloat16).to(DEV), idx, 3, 2, 1, dx)
    torch.cuda.synchronize()
    assert torch.equal(nchw(y.float()).cpu(), y_ref.detach())
    assert rel(nchw(dx.float()), xt.grad) < 8e-3
    # global average pool + its backward (gated by a ReLU output)
    a = torch.empty(N, C, device=DEV, dtype=torch.bfloat16)
    ops.avgpool_fwd(xd, a)
    gy = torch.randn(N, C, generator=g)
    da = torch.empty_like(xd)
    ops.avgpool_bwd(gy.to(DEV), da, gate=xd)
    torch.cuda.synchronize()
    assert rel(a.float(), x.mean((2, 3))) < 8e-3
    exp = (gy[:, :, None, None] / (H * W)).expand(N, C, H, W) * (x > 0).float()
    assert rel(nchw(da.float()), exp) < 8e-3

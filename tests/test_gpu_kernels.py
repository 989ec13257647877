"""Kernel-level parity of libttmi against fp32 PyTorch / the oracle (GPU only).

Tolerances: fp32 paths 2e-5 relative to the tensor's max-abs (the f32 MFMA is an exact fma
chain; only summation order differs); bf16 GEMMs are checked against an fp32 matmul of the
SAME bf16-rounded operands, which they match to fp32 accumulation error.  Dropout masks are
checked element-for-element against the oracle's restatement of the kernels' hash."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as TF

from oracle import two_tower_ref as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-30)


def seed_dev(val):
    v = val - (1 << 64) if val >= (1 << 63) else val
    return torch.tensor([v], dtype=torch.int64, device=DEV)


def keep_mask(seed, shape, p):
    return torch.from_numpy(ref.hash_keep(seed, int(np.prod(shape)), p).reshape(shape))


# ------------------------------------------------------------------------------ GEMM
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("ak,bk", [(1, 1), (1, 0), (0, 1), (0, 0)])
@pytest.mark.parametrize("M,N,K", [(256, 384, 128), (104, 72, 176), (520, 136, 200),
                                   (64, 64, 4096), (25600, 128, 128)])
def test_gemm_layouts(gpu_pkg, dtype, ak, bk, M, N, K):
    ops = gpu_pkg.ops
    g = torch.Generator().manual_seed(M * 7 + N * 3 + K)
    A = torch.randn(M, K, generator=g).to(dtype)
    B = torch.randn(N, K, generator=g).to(dtype)
    expect = A.float() @ B.float().t()
    As = (A if ak else A.t().contiguous()).to(DEV)
    Bs = (B if bk else B.t().contiguous()).to(DEV)
    C = torch.empty(M, N, device=DEV)
    ops.gemm(As, Bs, C, M, N, K, lda=K if ak else M, a_kmajor=ak, ldb=K if bk else N,
             b_kmajor=bk, ldc=N)
    assert rel(C, expect) < 2e-5 * max(1.0, math.sqrt(K / 256))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_epilogue(gpu_pkg, dtype):
    ops = gpu_pkg.ops
    M, N, K = 300, 192, 96
    g = torch.Generator().manual_seed(1)
    A = torch.randn(M, K, generator=g).to(dtype)
    W = torch.randn(N, K, generator=g).to(dtype)
    bias = torch.randn(N, generator=g)
    res = torch.randn(M, N, generator=g)
    gate = torch.randn(M, N, generator=g).to(dtype)
    p, seed = 0.25, 0xDEADBEEF12345
    keep = keep_mask(seed, (M, N), p).float()
    v = torch.relu(A.float() @ W.float().t() * 0.5 + bias) * keep / (1 - p)
    v = torch.where(gate.float() > 0, v * 3.0, torch.zeros_like(v))
    expect_cs = v.sum(0)
    expect = v + res
    C = torch.empty(M, N, device=DEV, dtype=torch.float32)
    cs = torch.zeros(N, device=DEV)
    ops.gemm(A.to(DEV), W.to(DEV), C, M, N, K, lda=K, a_kmajor=True, ldb=K, b_kmajor=True,
             ldc=N, alpha=0.5, bias=bias.to(DEV), act=1, drop=(p, seed_dev(seed)), ld_drop=N,
             gate=gate.to(DEV), ld_gate=N, gate_scale=3.0, residual=res.to(DEV), ld_res=N,
             colsum=cs)
    assert rel(C, expect) < 2e-5
    assert rel(cs, expect_cs) < 2e-5
    # bf16 output rounding
    Cb = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    ops.gemm(A.to(DEV), W.to(DEV), Cb, M, N, K, lda=K, a_kmajor=True, ldb=K, b_kmajor=True,
             ldc=N, bias=bias.to(DEV))
    assert rel(Cb.float(), A.float() @ W.float().t() + bias) < 8e-3


@pytest.mark.parametrize("M,N,K", [(3000, 384, 128), (4100, 512, 128), (2100, 128, 512),
                                   (2048, 128, 384), (2500, 256, 256), (2048, 128, 128),
                                   (3000, 768, 256), (25600, 1024, 256), (2100, 512, 256)])
@pytest.mark.parametrize("epi", ["res", "gate_bf16", "gate_f32", "none"])
def test_gemm_row_panel(gpu_pkg, M, N, K, epi):
    """Skinny-K row-panel kernel (persistent, W-stationary): each epilogue family, fp32 and
    bf16 out, rows not a multiple of the tile; shapes without a panel instantiation take the
    generic kernel and must agree just the same.  N = 512 / 768 / 1,024 at K = 256 (the D = 256
    encoder): column-sliced panels, 256 columns per workgroup (ABI 19)."""
    ops = gpu_pkg.ops
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g).to(torch.bfloat16)
    W = torch.randn(N, K, generator=g).to(torch.bfloat16)
    bias = torch.randn(N, generator=g)
    res = torch.randn(M, N, generator=g)
    gate = torch.randn(M, N, generator=g)
    if epi == "gate_bf16":
        gate = gate.to(torch.bfloat16)
    p, seed = 0.2, 0x1234ABCD5678
    keep = keep_mask(seed, (M, N), p).float()
    base = A.float() @ W.float().t()
    v = torch.relu(base * 0.5 + bias) * keep / (1 - p)
    kw = {}
    if epi == "res":
        v = v + res
        kw = dict(residual=res.to(DEV), ld_res=N)
    elif epi.startswith("gate"):
        v = torch.where(gate.float() > 0, v * 2.0, torch.zeros_like(v))
        kw = dict(gate=gate.to(DEV), ld_gate=N, gate_scale=2.0)
    C = torch.empty(M, N, device=DEV)
    ops.gemm(A.to(DEV), W.to(DEV), C, M, N, K, lda=K, a_kmajor=True, ldb=K, b_kmajor=True,
             ldc=N, alpha=0.5, bias=bias.to(DEV), act=1, drop=(p, seed_dev(seed)), ld_drop=N, **kw)
    assert rel(C, v) < 2e-5 * max(1.0, math.sqrt(K / 256))
    Cb = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    ops.linear(A.to(DEV), W.to(DEV), bias.to(DEV), Cb)
    assert rel(Cb.float(), base + bias) < 8e-3


@pytest.mark.parametrize("M,N,K", [(16384, 1024, 128), (16300, 1000, 192), (65536, 256, 64),
                                   (8192, 2304, 832)])
@pytest.mark.parametrize("epi", ["plain", "res_drop", "gelu_grad", "relu_gate", "acc"])
def test_gemm_big_tile(gpu_pkg, M, N, K, epi):
    """256x256 LDS-DMA tile kernel (the mDeBERTa token GEMMs): every epilogue family it
    takes, rows/columns not a multiple of the tile, and against the generic kernel."""
    ops = gpu_pkg.ops
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g).to(torch.bfloat16).to(DEV)
    W = torch.randn(N, K, generator=g).to(torch.bfloat16).to(DEV)
    bias = torch.randn(N, generator=g).to(DEV)
    base = A.float() @ W.float().t()
    kw, out_dt = {}, torch.float32
    if epi == "plain":
        v, out_dt = base + bias, torch.bfloat16
        kw = dict(bias=bias)
    elif epi == "res_drop":
        res = torch.randn(M, N, generator=g).to(DEV)
        p, seed = 0.1, 0x5EED1234ABCD
        keep = keep_mask(seed, (M, N), p).float().to(DEV)
        v = (base * 0.5 + bias) * keep / (1 - p) + res
        kw = dict(alpha=0.5, bias=bias, drop=(p, seed_dev(seed)), ld_drop=N, residual=res, ld_res=N)
    elif epi == "gelu_grad":
        pre = torch.randn(M, N, generator=g).to(torch.bfloat16).to(DEV)
        x = pre.float()
        gg = 0.5 * (1 + torch.erf(x / math.sqrt(2))) + x * torch.exp(-0.5 * x * x) / math.sqrt(2 * math.pi)
        v, out_dt = base * gg, torch.bfloat16
        kw = dict(act=3, gate=pre, ld_gate=N)
    elif epi == "relu_gate":
        gate = torch.randn(M, N, generator=g).to(torch.bfloat16).to(DEV)
        v = torch.where(gate.float() > 0, torch.relu(base + bias) * 2.0, torch.zeros_like(base))
        kw = dict(bias=bias, act=1, gate=gate, ld_gate=N, gate_scale=2.0)
    else:
        C0 = torch.randn(M, N, generator=g).to(DEV)
        v = C0 + base
        kw = dict(accumulate=True)
    C = C0.clone() if epi == "acc" else torch.empty(M, N, device=DEV, dtype=out_dt)
    ops.gemm(A, W, C, M, N, K, lda=K, a_kmajor=True, ldb=K, b_kmajor=True, ldc=N, **kw)
    tol = (2e-5 * max(1.0, math.sqrt(K / 256))) if out_dt == torch.float32 else 8e-3
    assert rel(C.float(), v) < tol, epi
    assert torch.isfinite(C.float()).all()


@pytest.mark.parametrize("M,N,K", [(16384, 3072, 768), (8192, 1000, 192), (300, 200, 64)])
def test_gemm_gelu_pre_out(gpu_pkg, M, N, K):
    """act 2 with pre_out (DebertaV2Intermediate: dense + GELU, the pre-activation kept for the
    backward): C = GELU(pre) and pre_out = pre, on the 256x256 tile kernel (first two shapes)
    and the generic one (last); bf16 outputs against fp32 torch."""
    ops = gpu_pkg.ops
    g = torch.Generator().manual_seed(M + N)
    A = torch.randn(M, K, generator=g).to(torch.bfloat16).to(DEV)
    W = (torch.randn(N, K, generator=g) / math.sqrt(K)).to(torch.bfloat16).to(DEV)
    bias = torch.randn(N, generator=g).to(DEV)
    pre_ref = A.float() @ W.float().t() + bias
    act_ref = torch.nn.functional.gelu(pre_ref)
    C = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    pre = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    ops.gemm(A, W, C, M, N, K, lda=K, a_kmajor=True, ldb=K, b_kmajor=True, ldc=N, bias=bias, act=2,
             pre_out=pre)
    assert rel(pre.float(), pre_ref) < 8e-3
    assert rel(C.float(), act_ref) < 8e-3
    # the stored pre-activation is what the epilogue activated
    assert rel(C.float(), torch.nn.functional.gelu(pre.float())) < 8e-3
    with pytest.raises(RuntimeError):
        ops.gemm(A, W, C, M, N, K, lda=K, a_kmajor=True, ldb=K, b_kmajor=True, ldc=N, bias=bias,
                 act=0, pre_out=pre)


@pytest.mark.parametrize("s_dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("R,Mw,group,trans", [(65536, 768, 768, False), (3000, 768, 64, False),
                                              (4099, 256, 256, True), (777, 64, 64, True)])
def test_skinny_wgrad(gpu_pkg, s_dt, R, Mw, group, trans):
    """Rank-8 LoRA gradient stream: C += alpha·Wᵀ·S with per-group S slices, both C layouts."""
    ops = gpu_pkg.ops
    g = torch.Generator().manual_seed(R + Mw)
    ngr = Mw // group
    W = torch.randn(R, Mw + 8, generator=g).to(torch.bfloat16).to(DEV)[:, :Mw]
    S = torch.randn(R, ngr * 8 + 8, generator=g).to(s_dt).to(DEV)[:, :ngr * 8]
    C0 = torch.randn(8, Mw, generator=g) if trans else torch.randn(Mw, 8, generator=g)
    C = C0.clone().to(DEV)
    ops.skinny_wgrad(W, S, C, Mw, ldc_m=1 if trans else 8, ldc_c=Mw if trans else 1, alpha=0.5,
                     group=group, sgs=8)
    Wf, Sf = W.float().cpu(), S.float().cpu()
    full = torch.einsum("rm,rgc->mgc", Wf, Sf.view(R, ngr, 8))        # [Mw, ngr, 8]
    sel = full[torch.arange(Mw), torch.arange(Mw) // group]            # [Mw, 8]
    expect = C0 + 0.5 * (sel.t() if trans else sel)
    assert rel(C, expect) < 1e-5


@pytest.mark.parametrize("p", [0.0, 0.1])
@pytest.mark.parametrize("M", [5000, 5003])          # rows per thread: 4 (and a ragged tail)
def test_lora_dx(gpu_pkg, p, M):
    ops = gpu_pkg.ops
    H = 768
    g = torch.Generator().manual_seed(3)
    dL = torch.randn(M, 16, generator=g).to(torch.bfloat16)
    aq = torch.randn(8, H, generator=g).to(torch.bfloat16)
    av = torch.randn(8, H, generator=g).to(torch.bfloat16)
    dx0 = torch.randn(M, H, generator=g)
    sq, sv = 0x1111222233334444, 0x5555666677778888
    yq = 4.0 * dL[:, :8].float() @ aq.float()
    yv = 4.0 * dL[:, 8:].float() @ av.float()
    if p > 0:
        yq = yq * keep_mask(sq, (M, H), p).float() / (1 - p)
        yv = yv * keep_mask(sv, (M, H), p).float() / (1 - p)
    dx = dx0.clone().to(DEV)
    ops.lora_dx(dL.to(DEV), aq.to(DEV), av.to(DEV), 4.0, (p, seed_dev(sq)), (p, seed_dev(sv)), dx, H)
    assert rel(dx, dx0 + yq + yv) < 1e-5


def test_gemm_drop_rows(gpu_pkg):
    """Dropout through a row map (the pruned last layer's gathered rows)."""
    ops = gpu_pkg.ops
    M, N, K = 512, 128, 128
    g = torch.Generator().manual_seed(3)
    A = torch.randn(M, K, generator=g).to(torch.bfloat16)
    W = torch.randn(N, K, generator=g).to(torch.bfloat16)
    p, seed = 0.2, 0x55AA
    rows = torch.randperm(50 * M, generator=g)[:M].to(torch.int32)
    keep = keep_mask(seed, (50 * M, N), p).float()[rows.long()]
    C = torch.empty(M, N, device=DEV)
    ops.linear(A.to(DEV), W.to(DEV), None, C, drop=(p, seed_dev(seed)), drop_rows=rows.to(DEV))
    assert rel(C, (A.float() @ W.float().t()) * keep / (1 - p)) < 2e-5


@pytest.mark.parametrize("split", [0, 1, 7])
def test_gemm_accumulate_split_k(gpu_pkg, split):
    ops = gpu_pkg.ops
    M, N, K = 384, 128, 25600                      # weight-gradient shape (dWin)
    g = torch.Generator().manual_seed(5)
    dy = torch.randn(K, M, generator=g).to(torch.bfloat16)   # [tokens, out]
    x = torch.randn(K, N, generator=g).to(torch.bfloat16)    # [tokens, in]
    gw = torch.ones(M, N, device=DEV)
    gb = torch.full((M,), 2.0, device=DEV)
    ops.linear_dw(dy.to(DEV), x.to(DEV), gw, gb, split_k=split)
    expect = 1.0 + dy.float().t() @ x.float()
    assert rel(gw, expect) < 5e-5
    assert rel(gb, 2.0 + dy.float().sum(0)) < 5e-5       # bias grad from the A row-sums


@pytest.mark.parametrize("M,N,R,split,pad", [
    (384, 128, 25600, 0, 0), (128, 512, 25600, 0, 0), (128, 128, 25600, 0, 64),
    (176, 128, 512, 0, 0), (72, 200, 1000, 0, 8), (512, 512, 512, 0, 0),
    (64, 64, 100, 3, 0), (128, 64, 4096, 8, 0), (136, 72, 777, 16, 32), (8, 8, 1, 0, 0)])
def test_gemm_weight_grad(gpu_pkg, M, N, R, split, pad):
    """Weight-gradient GEMM (LDS-DMA ring kernel): gw[M,N] += alpha dyᵀ x over R rows, bias
    row sums; partial tiles, row tails, strided operands, explicit splits."""
    ops = gpu_pkg.ops
    g = torch.Generator().manual_seed(M * 7 + N + R)
    dy_full = torch.randn(R, M + 2 * pad, generator=g).to(torch.bfloat16).to(DEV)
    x_full = torch.randn(R, N + pad, generator=g).to(torch.bfloat16).to(DEV)
    dy = dy_full[:, pad:pad + M]
    x = x_full[:, :N]
    gw = torch.full((M, N), 0.5, device=DEV)
    gb = torch.full((M,), -1.0, device=DEV)
    ops.gemm(dy, x, gw, M, N, R, lda=M + 2 * pad, a_kmajor=False, ldb=N + pad, b_kmajor=False,
             ldc=N, accumulate=True, alpha=0.75, split_k=split, rowsum_a=gb)
    torch.cuda.synchronize()
    expect = 0.5 + 0.75 * (dy.float().t() @ x.float())
    assert rel(gw, expect) < 5e-5, rel(gw, expect)
    assert rel(gb, -1.0 + dy.float().sum(0)) < 5e-5


# ------------------------------------------------------------------------------ LayerNorm
@pytest.mark.parametrize("D", [32, 128, 176, 512])
@pytest.mark.parametrize("ydt", [torch.float32, torch.bfloat16])
def test_layernorm_fwd_bwd(gpu_pkg, D, ydt):
    ops = gpu_pkg.ops
    M = 333
    g = torch.Generator().manual_seed(D)
    x = torch.randn(M, D, generator=g) * 3 + 1
    w = torch.randn(D, generator=g)
    b = torch.randn(D, generator=g)
    p, seed = 0.1, 42
    keep = keep_mask(seed, (M, D), p).float()
    xt = x.clone().requires_grad_(True)
    wt = w.clone().requires_grad_(True)
    bt = b.clone().requires_grad_(True)
    y_ref = torch.relu(TF.layer_norm(xt, (D,), wt, bt, 1e-5)) * keep / (1 - p)
    y = torch.empty(M, D, device=DEV, dtype=ydt)
    mean = torch.empty(M, device=DEV)
    rstd = torch.empty(M, device=DEV)
    xd = x.to(DEV)
    ops.layernorm_fwd(xd, w.to(DEV), b.to(DEV), y, mean, rstd, relu=True, drop=(p, seed_dev(seed)))
    assert rel(y.float(), y_ref) < (2e-5 if ydt == torch.float32 else 8e-3)
    dy = torch.randn(M, D, generator=g)
    res = torch.randn(M, D, generator=g)
    y_ref.backward(dy)
    dx = torch.empty(M, D, device=DEV)
    dw = torch.zeros(D, device=DEV)
    db = torch.zeros(D, device=DEV)
    # gate with the fp32 output so the mask is exact in both dtypes
    yg = torch.empty(M, D, device=DEV)
    ops.layernorm_fwd(xd, w.to(DEV), b.to(DEV), yg, mean, rstd, relu=True, drop=(p, seed_dev(seed)))
    ops.layernorm_bwd(dy.to(DEV), xd, mean, rstd, w.to(DEV), dx, dw, db, gate=yg,
                      gate_scale=1 / (1 - p), res=res.to(DEV))
    assert rel(dx, xt.grad + res) < 5e-5
    assert rel(dw, wt.grad) < 5e-5
    assert rel(db, bt.grad) < 5e-5


# ------------------------------------------------------------------------------ attention
def attn_ref(qkv, kv, B, L, H, p, seed):
    D = qkv.shape[1] // 3
    dh = D // H
    q, k, v = qkv.float().reshape(B, L, 3, H, dh).permute(2, 0, 3, 1, 4)
    s = (q @ k.transpose(-1, -2)) / math.sqrt(dh)
    allowed = torch.ones(L, L, dtype=torch.bool).tril()[None, None] & (kv != 0)[:, None, None, :]
    row_any = allowed.any(-1, keepdim=True)
    s = s.masked_fill(~allowed, float("-inf")).masked_fill(~row_any, 0.0)
    lse = torch.logsumexp(s, -1).masked_fill(~row_any[..., 0], float("inf"))
    prob = torch.softmax(s, -1) * row_any
    if p > 0:
        prob = prob * keep_mask(seed, (B, H, L, L), p).float() / (1 - p)
    o = (prob @ v).transpose(1, 2).reshape(B * L, D)
    return o, lse.reshape(-1)


def masks(B, L, g):
    lengths = torch.randint(1, L + 1, (B,), generator=g)
    lengths[0] = L
    lengths[1 % B] = 0
    m = (torch.arange(L)[None] < lengths[:, None]).long()
    if B > 2:
        m[2] = m[2].flip(0)            # left-padded row
    return m


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,L,H,Dh", [(6, 8, 4, 8), (16, 50, 4, 32), (4, 64, 2, 64), (3, 1, 4, 16),
                                      (4, 65, 2, 32), (3, 200, 4, 32), (2, 130, 2, 64), (2, 512, 1, 8),
                                      (3, 128, 4, 32), (3, 512, 4, 32), (2, 1000, 2, 32), (2, 2048, 1, 16)])
@pytest.mark.parametrize("p", [0.0, 0.2])
def test_mha_fwd_bwd(gpu_pkg, dtype, B, L, H, Dh, p):
    ops = gpu_pkg.ops
    g = torch.Generator().manual_seed(B * L + Dh)
    D = H * Dh
    qkv = (torch.randn(B * L, 3 * D, generator=g) * 1.5).to(dtype)
    kv = masks(B, L, g)
    seed = 0x1234567890ABCDEF
    qt = qkv.float().clone().requires_grad_(True)
    o_ref, lse_ref = attn_ref(qt, kv, B, L, H, p, seed)
    ctx = torch.empty(B * L, D, device=DEV, dtype=dtype)
    lse = torch.empty(B * H * L, device=DEV)
    sd = seed_dev(seed)
    ops.mha_fwd(qkv.to(DEV), kv.to(DEV), B, L, H, ctx, lse, (p, sd))
    tol = 2e-5 if dtype == torch.float32 else 2e-2
    assert rel(ctx.float(), o_ref) < tol
    fin = torch.isfinite(lse_ref)
    assert torch.equal(torch.isfinite(lse.cpu()), fin)
    assert rel(lse.cpu()[fin], lse_ref[fin]) < (2e-6 if dtype == torch.float32 else 1e-2)
    dctx = torch.randn(B * L, D, generator=g).to(dtype)
    o_ref.backward(dctx.float())
    dqkv = torch.empty(B * L, 3 * D, device=DEV, dtype=dtype)
    ops.mha_bwd(qkv.to(DEV), kv.to(DEV), lse, dctx.to(DEV), B, L, H, dqkv, (p, sd))
    assert rel(dqkv.float(), qt.grad) < (5e-5 if dtype == torch.float32 else 3e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,L,H,Dh", [(6, 8, 1, 128), (5, 50, 2, 96), (3, 20, 1, 256), (4, 33, 3, 12),
                                      (2, 70, 1, 500), (2, 2100, 1, 16), (3, 50, 4, 32)])
@pytest.mark.parametrize("p", [0.0, 0.2])
def test_mha_generic_fwd_bwd(gpu_pkg, dtype, B, L, H, Dh, p):
    """ttmi_mha_generic_fwd / _bwd (ABI 22): the shapes the tuned kernels refuse — head widths
    above 64 or not a multiple of 8, L past TTMI_ATTN_LMAX — against the torch restatement, with
    the same masks (left-padded, empty and full rows) and dropout indices; (3, 50, 4, 32) is a
    tuned shape, where it must agree with ttmi_mha_fwd / _bwd too."""
    ops = gpu_pkg.ops
    g = torch.Generator().manual_seed(7 * B * L + Dh)
    D = H * Dh
    qkv = (torch.randn(B * L, 3 * D, generator=g) * 1.5).to(dtype)
    kv = masks(B, L, g)
    seed = 0x0F1E2D3C4B5A6978
    qt = qkv.float().clone().requires_grad_(True)
    o_ref, lse_ref = attn_ref(qt, kv, B, L, H, p, seed)
    ctx = torch.empty(B * L, D, device=DEV, dtype=dtype)
    lse = torch.empty(B * H * L, device=DEV)
    sd = seed_dev(seed)
    qd, kd = qkv.to(DEV), kv.to(DEV)
    ops.mha_generic_fwd(qd, kd, B, L, H, ctx, lse, (p, sd))
    tol = 2e-5 if dtype == torch.float32 else 2e-2
    assert rel(ctx.float(), o_ref) < tol
    fin = torch.isfinite(lse_ref)
    assert torch.equal(torch.isfinite(lse.cpu()), fin)
    assert rel(lse.cpu()[fin], lse_ref[fin]) < (2e-6 if dtype == torch.float32 else 1e-2)
    dctx = torch.randn(B * L, D, generator=g).to(dtype)
    o_ref.backward(dctx.float())
    dqkv = torch.empty(B * L, 3 * D, device=DEV, dtype=dtype)
    ops.mha_generic_bwd(qd, kd, lse, ctx, dctx.to(DEV), B, L, H, dqkv, (p, sd))
    assert rel(dqkv.float(), qt.grad) < (5e-5 if dtype == torch.float32 else 3e-2)
    if ops.mha_tuned_supported(L, Dh):
        ctx2 = torch.empty_like(ctx)
        lse2 = torch.empty_like(lse)
        ops.mha_fwd(qd, kd, B, L, H, ctx2, lse2, (p, sd))
        assert rel(ctx2.float(), ctx.float()) < tol


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,L,H,Dh", [(6, 8, 4, 8), (16, 50, 4, 32), (4, 64, 2, 64), (5, 150, 4, 32),
                                      (3, 300, 2, 64), (4, 65, 4, 32), (4, 128, 4, 32), (3, 512, 4, 32),
                                      (2, 1000, 2, 32), (2, 2048, 1, 16)])
@pytest.mark.parametrize("p", [0.0, 0.2])
def test_mha_single_query_matches_full_row(gpu_pkg, dtype, B, L, H, Dh, p):
    """ttmi_mha_q1_* (pruned last layer) == the full attention restricted to each
    sequence's last valid row, forward and backward, same dropout masks."""
    ops = gpu_pkg.ops
    g = torch.Generator().manual_seed(B + L + Dh)
    D = H * Dh
    qkv = (torch.randn(B * L, 3 * D, generator=g) * 1.5).to(dtype)
    kv = masks(B, L, g)
    seed = 0xFEEDFACE0102
    lengths = kv.sum(1)
    rows = (torch.arange(B) * L + (lengths - 1).clamp(min=0)).to(torch.int32)
    qt = qkv.float().clone().requires_grad_(True)
    o_ref, lse_ref = attn_ref(qt, kv, B, L, H, p, seed)
    o_sel = o_ref[rows.long()]
    lse_sel = lse_ref.reshape(B, H, L)[torch.arange(B), :, (lengths - 1).clamp(min=0)]
    sd = seed_dev(seed)
    rows_d = torch.empty(B, dtype=torch.int32, device=DEV)
    ops.last_rows(kv.to(DEV), rows_d)
    assert torch.equal(rows_d.cpu(), rows)
    ctx = torch.empty(B, D, device=DEV, dtype=dtype)
    lse = torch.empty(B * H, device=DEV)
    ops.mha_q1_fwd(qkv.to(DEV), kv.to(DEV), rows_d, B, L, H, ctx, lse, (p, sd))
    tol = 2e-5 if dtype == torch.float32 else 2e-2
    assert rel(ctx.float(), o_sel) < tol
    fin = torch.isfinite(lse_sel.reshape(-1))
    assert torch.equal(torch.isfinite(lse.cpu()), fin)
    assert rel(lse.cpu()[fin], lse_sel.reshape(-1)[fin]) < (2e-6 if dtype == torch.float32 else 1e-2)
    dsel = torch.randn(B, D, generator=g).to(dtype)
    o_sel.backward(dsel.float())
    dqkv = torch.empty(B * L, 3 * D, device=DEV, dtype=dtype)
    ops.mha_q1_bwd(qkv.to(DEV), kv.to(DEV), rows_d, lse, dsel.to(DEV), B, L, H, dqkv, (p, sd))
    assert rel(dqkv.float(), qt.grad) < (5e-5 if dtype == torch.float32 else 3e-2)


@pytest.mark.parametrize("D", [96, 130])
def test_last_rows_gather(gpu_pkg, D):
    """ttmi_last_rows_gather == ttmi_last_rows + ttmi_gather_rows (incl. empty histories)."""
    ops = gpu_pkg.ops
    B, L = 37, 50
    g = torch.Generator().manual_seed(D)
    lens = torch.randint(0, L + 1, (B,), generator=g)
    kv = (torch.arange(L)[None] < lens[:, None]).long().to(DEV)
    x = torch.randn(B * L, D, generator=g).to(DEV)
    rows_a = torch.empty(B, dtype=torch.int32, device=DEV)
    ops.last_rows(kv, rows_a)
    rows_b = torch.empty(B, dtype=torch.int32, device=DEV)
    out = torch.empty(B, D, device=DEV)
    ops.last_rows_gather(kv, x, rows_b, out)
    assert torch.equal(rows_a, rows_b)
    assert torch.equal(out, x[rows_a.long()])


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,L,H,Dh,p", [(37, 50, 4, 32, 0.1), (8, 64, 2, 64, 0.0), (5, 7, 2, 8, 0.2),
                                        (9, 100, 4, 32, 0.1)])
def test_mha_q1_gather_fwd(gpu_pkg, dtype, B, L, H, Dh, p):
    """ttmi_mha_q1_gather_fwd == ttmi_last_rows_gather + ttmi_mha_q1_fwd bit for bit (rows,
    gathered residual rows, ctx, lse), incl. empty and full histories."""
    ops = gpu_pkg.ops
    D = H * Dh
    g = torch.Generator().manual_seed(B * L + Dh)
    lens = torch.randint(0, L + 1, (B,), generator=g)
    lens[0], lens[-1] = 0, L
    kv = (torch.arange(L)[None] < lens[:, None]).long().to(DEV)
    qkv = torch.randn(B * L, 3 * D, generator=g).to(dtype).to(DEV)
    x = torch.randn(B * L, D, generator=g).to(DEV)
    sd = seed_dev(0xABCD1234)
    rows_a = torch.empty(B, dtype=torch.int32, device=DEV)
    xr_a = torch.empty(B, D, device=DEV)
    ops.last_rows_gather(kv, x, rows_a, xr_a)
    ctx_a = torch.empty(B, D, device=DEV, dtype=dtype)
    lse_a = torch.empty(B * H, device=DEV)
    ops.mha_q1_fwd(qkv, kv, rows_a, B, L, H, ctx_a, lse_a, (p, sd))
    rows_b = torch.full((B,), -1, dtype=torch.int32, device=DEV)
    xr_b = torch.empty(B, D, device=DEV)
    ctx_b = torch.empty(B, D, device=DEV, dtype=dtype)
    lse_b = torch.empty(B * H, device=DEV)
    ops.mha_q1_gather_fwd(qkv, kv, x, rows_b, xr_b, B, L, H, ctx_b, lse_b, (p, sd))
    torch.cuda.synchronize()
    assert torch.equal(rows_a, rows_b)
    assert torch.equal(xr_a, xr_b)
    assert torch.equal(ctx_a, ctx_b)
    assert torch.equal(lse_a, lse_b)


def test_gather_scatter_rows(gpu_pkg):
    ops = gpu_pkg.ops
    x = torch.randn(500, 96, device=DEV)
    rows = torch.tensor([3, 499, 0, 250], dtype=torch.int32, device=DEV)
    out = torch.empty(4, 96, device=DEV)
    ops.gather_rows(x, rows, out)
    assert torch.equal(out, x[rows.long()])
    dst = torch.zeros(500, 96, device=DEV)
    ops.scatter_add_rows(out, rows, dst)
    ops.scatter_add_rows(out, rows, dst)
    expect = torch.zeros(500, 96, device=DEV)
    expect[rows.long()] = 2 * out
    assert torch.equal(dst, expect)


# ------------------------------------------------------------------------------ embedding
@pytest.mark.parametrize("p,deferred", [(0.0, False), (0.1, False), (0.1, True)])
@pytest.mark.parametrize("B,L,D,V", [(37, 50, 128, 301), (64, 20, 128, 997), (9, 20, 256, 50)])
def test_seq_embed_fwd_bwd(gpu_pkg, p, deferred, B, L, D, V):
    """seq_embed_fwd/bwd vs torch autograd.  deferred (ABI 15): inside deferred_wgrad the LN
    partials are folded by the weight-gradient fold (accumulate bit 2 leaves the workspace
    zero), so two deferred calls in a row must each give the same gradients."""
    ops = gpu_pkg.ops
    g = torch.Generator().manual_seed(9)
    ids = torch.randint(0, V, (B, L), generator=g)
    E = torch.randn(V, D, generator=g)
    P = torch.randn(L, D, generator=g)
    w = torch.randn(D, generator=g)
    b = torch.randn(D, generator=g)
    seed = 77
    Et, Pt, wt, bt = (t.clone().requires_grad_(True) for t in (E, P, w, b))
    x_ref = TF.layer_norm(TF.embedding(ids, Et, padding_idx=0) + Pt[None], (D,), wt, bt, 1e-5)
    if p > 0:
        x_ref = x_ref * keep_mask(seed, (B * L, D), p).float().reshape(B, L, D) / (1 - p)
    x = torch.empty(B * L, D, device=DEV)
    mean = torch.empty(B * L, device=DEV)
    rstd = torch.empty(B * L, device=DEV)
    Ed, Pd, wd, bd = (t.to(DEV) for t in (E, P, w, b))
    sd = seed_dev(seed)
    ops.seq_embed_fwd(ids.to(DEV), Ed, Pd, wd, bd, x, mean, rstd, drop=(p, sd))
    assert rel(x, x_ref.reshape(B * L, D)) < 2e-5
    xe = TF.embedding(ids, E) + P[None]
    assert rel(mean, xe.mean(-1).reshape(-1)) < 1e-5
    assert rel(rstd, 1.0 / torch.sqrt(xe.var(-1, unbiased=False) + 1e-5).reshape(-1)) < 1e-5
    dx = torch.randn(B * L, D, generator=g)
    x_ref.reshape(B * L, D).backward(dx)
    dE = torch.zeros(V, D, device=DEV)
    dP = torch.zeros(L, D, device=DEV)
    dw = torch.zeros(D, device=DEV)
    db = torch.zeros(D, device=DEV)
    if deferred:
        for k in range(2):
            dw.zero_()
            db.zero_()
            with ops.deferred_wgrad():
                ops.seq_embed_bwd(ids.to(DEV), Ed, Pd, wd, mean, rstd, dx.to(DEV), dE, dP, dw, db,
                                  drop=(p, sd), padding_idx=0)
            assert rel(dw, wt.grad) < 5e-5 and rel(db, bt.grad) < 5e-5, k
        dE /= 2
        dP /= 2
    else:
        ops.seq_embed_bwd(ids.to(DEV), Ed, Pd, wd, mean, rstd, dx.to(DEV), dE, dP, dw, db,
                          drop=(p, sd), padding_idx=0)
    assert rel(dE, Et.grad) < 5e-5
    assert dE[0].abs().max().item() == 0.0
    assert rel(dP, Pt.grad) < 5e-5
    assert rel(dw, wt.grad) < 5e-5
    assert rel(db, bt.grad) < 5e-5


@pytest.mark.parametrize("scale", [1.0, 1e-3, 1e-6])
def test_seq_embed_bwd_fixed_point_range(gpu_pkg, scale):
    """The embedding-row scatter adds in int64 fixed point (2^-36 per unit, TTMI_FX_GRAD_SHIFT;
    order-independent, so the sum is bit-reproducible).  Each adder is rounded once, so the
    error bound is absolute: |dE - dE_fp64| <= count(row) * 2^-37 + fp32 rounding, whatever the
    gradient's magnitude.  With the upstream gradient scaled down to 1e-6 (element gradients
    ~1e-8) that is still ~1e-3 relative; the test states the bound per element and checks it
    against a float64 reference (small-gradient regime)."""
    ops = gpu_pkg.ops
    B, L, D, V = 64, 50, 128, 97
    g = torch.Generator().manual_seed(31)
    ids = torch.randint(0, V, (B, L), generator=g)
    E = torch.randn(V, D, generator=g)
    P = torch.randn(L, D, generator=g)
    w = torch.randn(D, generator=g)
    b = torch.randn(D, generator=g)
    Et = E.double().clone().requires_grad_(True)
    x_ref = TF.layer_norm(TF.embedding(ids, Et, padding_idx=0) + P.double()[None], (D,), w.double(),
                          b.double(), 1e-5)
    dx = torch.randn(B * L, D, generator=g) * scale
    x_ref.reshape(B * L, D).backward(dx.double())
    x = torch.empty(B * L, D, device=DEV)
    mean, rstd = torch.empty(B * L, device=DEV), torch.empty(B * L, device=DEV)
    Ed = E.to(DEV)
    ops.seq_embed_fwd(ids.to(DEV), Ed, P.to(DEV), w.to(DEV), b.to(DEV), x, mean, rstd)
    dE = torch.zeros(V, D, device=DEV)
    dP, dw, db = torch.zeros(L, D, device=DEV), torch.zeros(D, device=DEV), torch.zeros(D, device=DEV)
    ops.seq_embed_bwd(ids.to(DEV), Ed, P.to(DEV), w.to(DEV), mean, rstd, dx.to(DEV), dE, dP, dw, db,
                      padding_idx=0)
    cnt = torch.bincount(ids.reshape(-1), minlength=V).double()[:, None]
    ref = Et.grad
    err = (dE.cpu().double() - ref).abs()
    bound = cnt * 2.0 ** -37 * 1.01 + 2e-6 * ref.abs().max() + 1e-7 * ref.abs()
    assert bool((err <= bound).all()), (scale, (err - bound).max().item())
    assert dE[0].abs().max().item() == 0.0


# ------------------------------------------------------------------------------ batchnorm
@pytest.mark.parametrize("ydt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B", [96, 250, 512, 700])   # register kernels (<= 512) and the loop
def test_batchnorm_train_eval(gpu_pkg, ydt, B):
    ops = gpu_pkg.ops
    C = 200
    g = torch.Generator().manual_seed(3)
    z = torch.randn(B, C, generator=g) * 2 + 0.5
    w = torch.randn(C, generator=g)
    b = torch.randn(C, generator=g)
    p, seed = 0.1, 99
    bn = torch.nn.BatchNorm1d(C)
    bn.weight.data.copy_(w)
    bn.bias.data.copy_(b)
    zt = z.clone().requires_grad_(True)
    keep = keep_mask(seed, (B, C), p).float()
    y_ref = torch.relu(bn(zt)) * keep / (1 - p)
    rm = torch.zeros(C, device=DEV)
    rv = torch.ones(C, device=DEV)
    nbt = torch.zeros((), dtype=torch.int64, device=DEV)
    y = torch.empty(B, C, device=DEV, dtype=ydt)
    mean = torch.empty(C, device=DEV)
    rstd = torch.empty(C, device=DEV)
    zd = z.to(DEV)
    ops.batchnorm_fwd(zd, w.to(DEV), b.to(DEV), y, mean, rstd, rm, rv, nbt, relu=True,
                      drop=(p, seed_dev(seed)))
    assert rel(y.float(), y_ref) < (2e-5 if ydt == torch.float32 else 8e-3)
    assert rel(rm, bn.running_mean) < 2e-5 and rel(rv, bn.running_var) < 2e-5
    assert int(nbt) == 1
    dy = torch.randn(B, C, generator=g)
    y_ref.backward(dy)
    yf = torch.empty(B, C, device=DEV)
    ops.batchnorm_fwd(zd, w.to(DEV), b.to(DEV), yf, mean, rstd, None, None, None, relu=True,
                      drop=(p, seed_dev(seed)))
    dz = torch.empty(B, C, device=DEV)
    dw = torch.zeros(C, device=DEV)
    db = torch.zeros(C, device=DEV)
    ops.batchnorm_bwd(dy.to(DEV), zd, w.to(DEV), mean, rstd, yf, dz, dw, db, gate_scale=1 / (1 - p))
    assert rel(dz, zt.grad) < 5e-5
    assert rel(dw, bn.weight.grad) < 5e-5 and rel(db, bn.bias.grad) < 5e-5
    # eval: running statistics
    bn.eval()
    ye = torch.empty(B, C, device=DEV)
    ops.batchnorm_fwd(zd, w.to(DEV), b.to(DEV), ye, None, None, rm, rv, None, relu=False,
                      training=False)
    assert rel(ye, bn(z).detach()) < 2e-5


# ------------------------------------------------------------------------------ AdamW
def test_adamw_matches_torch_semantics(gpu_pkg):
    ops = gpu_pkg.ops
    n = 10007
    g = torch.Generator().manual_seed(11)
    p0 = torch.randn(n, generator=g)
    params = {"w": p0.clone()}
    state = {}
    pd = p0.clone().to(DEV)
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    mirror = torch.empty(n, device=DEV, dtype=torch.bfloat16)
    hyper = torch.tensor([1e-3, 0.9, 0.999, 1e-8, 0.01], dtype=torch.float64, device=DEV)
    step = torch.zeros(1, dtype=torch.int32, device=DEV)
    for _ in range(5):
        gr = torch.randn(n, generator=g)
        ref.adamw_(params, {"w": gr}, state, lr=1e-3)
        ops.step_inc(step)
        gd = gr.to(DEV)
        ops.adamw(pd, gd, m, v, mirror, hyper, step, zero_grad=True)
        assert gd.abs().max().item() == 0.0
    assert rel(pd, params["w"]) < 2e-6
    assert torch.equal(mirror.cpu(), pd.cpu().to(torch.bfloat16))
    assert int(step) == 5


def test_batch_copy(gpu_pkg):
    srcs = [torch.randint(0, 100, (513, 50), device=DEV), torch.randn(7, 3, device=DEV),
            torch.randn(1000, 512, device=DEV)[:, 1:].contiguous()]
    dsts = [torch.empty_like(t) for t in srcs]
    gpu_pkg.ops.batch_copy(dsts, srcs)
    for a, b in zip(dsts, srcs):
        assert torch.equal(a, b)


def test_dropout_seed_kernel_matches_host(gpu_pkg):
    F = gpu_pkg.functional
    step = torch.tensor([12], dtype=torch.int32, device=DEV)
    seeds = torch.zeros(F.N_SITES, dtype=torch.int64, device=DEV)
    gpu_pkg.ops.dropout_seeds(0xABCDEF, step, seeds)
    host = F.seed_table(F.site_seeds(0xABCDEF, 12), "cpu")
    assert torch.equal(seeds.cpu(), host)
    # with the step increment folded in: seeds of step 13, counter left at 13
    gpu_pkg.ops.dropout_seeds(0xABCDEF, step, seeds, inc_step=True)
    assert int(step) == 13
    assert torch.equal(seeds.cpu(), F.seed_table(F.site_seeds(0xABCDEF, 13), "cpu"))


def test_transpose_batch_with_seeds(gpu_pkg):
    """The train step's prologue launch: mirror transposes plus the dropout seeds (same values
    and step increment as dropout_seeds), and the seeds-only form (no matrices)."""
    ops, F = gpu_pkg.ops, gpu_pkg.functional
    srcs = [torch.randn(384, 128, device=DEV).bfloat16(), torch.randn(70, 130, device=DEV).bfloat16()]
    dsts = [torch.empty(t.shape[1], t.shape[0], device=DEV, dtype=torch.bfloat16) for t in srcs]
    step = torch.tensor([40], dtype=torch.int32, device=DEV)
    seeds = torch.zeros(F.N_SITES, dtype=torch.int64, device=DEV)
    ops.transpose_batch(dsts, srcs, (0x5EED, step, seeds, True))
    for d, s_ in zip(dsts, srcs):
        assert torch.equal(d, s_.t())
    assert int(step) == 41
    assert torch.equal(seeds.cpu(), F.seed_table(F.site_seeds(0x5EED, 41), "cpu"))
    ops.transpose_batch([], [], (0x5EED, step, seeds, False))
    assert int(step) == 41
    assert torch.equal(seeds.cpu(), F.seed_table(F.site_seeds(0x5EED, 41), "cpu"))


def test_transpose_batch(gpu_pkg):
    """Batched bf16 transpose (the Wᵀ mirrors of the input-grad GEMMs): ragged shapes."""
    ops = gpu_pkg.ops
    g = torch.Generator().manual_seed(11)
    shapes = [(384, 128), (128, 128), (512, 128), (128, 512), (70, 33), (1, 200)]
    srcs = [torch.randn(r, c, generator=g).to(torch.bfloat16).to(DEV) for r, c in shapes]
    dsts = [torch.empty(c, r, device=DEV, dtype=torch.bfloat16) for r, c in shapes]
    ops.transpose_batch(dsts, srcs)
    torch.cuda.synchronize()
    for s_, d in zip(srcs, dsts):
        assert torch.equal(d.cpu(), s_.t().cpu())


@pytest.mark.parametrize("D,M,K", [(128, 3000, 384), (128, 2048, 512), (128, 100, 128), (128, 512, 256),
                                   (256, 3000, 768), (256, 2048, 1024), (256, 100, 256),
                                   (256, 512, 512), (256, 25600, 1024)])
@pytest.mark.parametrize("with_res,with_next", [(True, True), (False, False), (True, False)])
def test_linear_ln_bwd(gpu_pkg, D, M, K, with_res, with_next):
    """Fused Linear input grad + LayerNorm backward (+ dropout backward) vs torch autograd
    on the same bf16 operands (fp32 math): dx, LN dw/db, and the bf16 dropout output.
    D = 256: the streamed-W panel (panel256_kernel, ABI 19)."""
    ops = gpu_pkg.ops
    g = torch.Generator().manual_seed(M + K + D)
    dh = torch.randn(M, K, generator=g).to(torch.bfloat16)
    wt = (torch.randn(D, K, generator=g) / math.sqrt(K)).to(torch.bfloat16)
    x = torch.randn(M, D, generator=g) * 2 + 0.5
    w = torch.randn(D, generator=g)
    b = torch.randn(D, generator=g)
    res = torch.randn(M, D, generator=g)
    mean = x.mean(1)
    rstd = 1.0 / torch.sqrt(x.var(1, unbiased=False) + 1e-5)
    dY = dh.float() @ wt.float().t()
    xt = x.clone().requires_grad_(True)
    wt_ = w.clone().requires_grad_(True)
    bt_ = b.clone().requires_grad_(True)
    TF.layer_norm(xt, (D,), wt_, bt_, 1e-5).backward(dY)
    dx_ref = xt.grad + (res if with_res else 0.0)
    p, seed = 0.1, 0x77AA
    rows = torch.randperm(3 * M, generator=g)[:M].to(torch.int32)
    keep = keep_mask(seed, (3 * M, D), p).float()[rows.long()]
    dx = torch.empty(M, D, device=DEV)
    dw = torch.full((D,), 0.5, device=DEV)
    db = torch.zeros(D, device=DEV)
    nxt = torch.empty(M, D, device=DEV, dtype=torch.bfloat16) if with_next else None
    ops.linear_ln_bwd(dh.to(DEV), wt.to(DEV), x.to(DEV), mean.to(DEV), rstd.to(DEV), w.to(DEV),
                      dx, dw, db, res=res.to(DEV) if with_res else None, next_=nxt,
                      drop=(p, seed_dev(seed)) if with_next else ops.NO_DROP,
                      drop_rows=rows.to(DEV) if with_next else None)
    torch.cuda.synchronize()
    assert rel(dx, dx_ref) < 2e-5
    assert rel(dw, 0.5 + wt_.grad) < 5e-5
    assert rel(db, bt_.grad) < 5e-5
    if with_next:
        assert rel(nxt.float(), dx_ref * keep / (1 - p)) < 8e-3
    # inside deferred_wgrad the LN sums go to per-workgroup slabs folded in workgroup order:
    # same values (to float reassociation), bit-identical run to run, dx untouched
    outs = []
    for _ in range(2):
        dw2 = torch.full((D,), 0.5, device=DEV)
        db2 = torch.zeros(D, device=DEV)
        dx2 = torch.empty(M, D, device=DEV)
        with ops.deferred_wgrad() as pend:
            ops.linear_ln_bwd(dh.to(DEV), wt.to(DEV), x.to(DEV), mean.to(DEV), rstd.to(DEV),
                              w.to(DEV), dx2, dw2, db2, res=res.to(DEV) if with_res else None)
            assert len(pend.folds) == 2
        outs.append((dw2, db2, dx2))
    torch.cuda.synchronize()
    assert rel(outs[0][0], 0.5 + wt_.grad) < 5e-5 and rel(outs[0][1], bt_.grad) < 5e-5
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    if not with_next:
        assert torch.equal(outs[0][2], dx)


@pytest.mark.parametrize("D,M,K", [(128, 300, 128), (128, 4096, 512), (128, 25600, 128),
                                   (256, 300, 256), (256, 4096, 1024), (256, 25600, 256),
                                   (256, 25600, 1024), (256, 1000, 768)])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_linear_res_ln(gpu_pkg, D, M, K, p):
    """Fused out = res + dropout(x·wᵀ + b) and y = LN(out) (ttmi_linear_res_ln) vs fp32 torch
    on the same bf16 operands: out to fp32 accumulation error, y to bf16 rounding, row stats.
    D = 256: the streamed-W panel (ABI 19)."""
    ops = gpu_pkg.ops
    g = torch.Generator().manual_seed(M + K + D + int(p * 10))
    x = torch.randn(M, K, generator=g).to(torch.bfloat16)
    w = (torch.randn(D, K, generator=g) / math.sqrt(K)).to(torch.bfloat16)
    b = torch.randn(D, generator=g)
    res = torch.randn(M, D, generator=g)
    lw = torch.randn(D, generator=g)
    lb = torch.randn(D, generator=g)
    seed = 0x5EED
    keep = keep_mask(seed, (M, D), p).float() if p > 0 else torch.ones(M, D)
    out_ref = res + (x.float() @ w.float().t() + b) * keep / (1 - p)
    y_ref = TF.layer_norm(out_ref, (D,), lw, lb, 1e-5)
    out = torch.empty(M, D, device=DEV)
    y = torch.empty(M, D, device=DEV, dtype=torch.bfloat16)
    mean = torch.empty(M, device=DEV)
    rstd = torch.empty(M, device=DEV)
    ops.linear_res_ln(x.to(DEV), w.to(DEV), b.to(DEV), res.to(DEV), out, lw.to(DEV), lb.to(DEV),
                      y, mean, rstd, eps=1e-5, drop=(p, seed_dev(seed)) if p > 0 else ops.NO_DROP)
    torch.cuda.synchronize()
    assert rel(out, out_ref) < 2e-5
    assert rel(y.float(), y_ref) < 8e-3
    assert rel(mean, out_ref.mean(1)) < 1e-5
    assert rel(rstd, 1.0 / torch.sqrt(out_ref.var(1, unbiased=False) + 1e-5)) < 1e-4


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_seq_embed_fwd_norm1(gpu_pkg, p):
    """seq_embed_fwd with the first layer's norm1 fused: x unchanged, y1 = bf16(LN1(x))."""
    ops = gpu_pkg.ops
    B, L, D, V = 37, 50, 128, 301
    g = torch.Generator().manual_seed(19)
    ids = torch.randint(0, V, (B, L), generator=g).to(DEV)
    E, P = torch.randn(V, D, generator=g).to(DEV), torch.randn(L, D, generator=g).to(DEV)
    w, b = torch.randn(D, generator=g).to(DEV), torch.randn(D, generator=g).to(DEV)
    w1, b1 = torch.randn(D, generator=g).to(DEV), torch.randn(D, generator=g).to(DEV)
    sd = seed_dev(123)
    M = B * L
    x0, m0, r0 = torch.empty(M, D, device=DEV), torch.empty(M, device=DEV), torch.empty(M, device=DEV)
    ops.seq_embed_fwd(ids, E, P, w, b, x0, m0, r0, drop=(p, sd))
    x = torch.empty(M, D, device=DEV)
    m, r = torch.empty(M, device=DEV), torch.empty(M, device=DEV)
    y1 = torch.empty(M, D, device=DEV, dtype=torch.bfloat16)
    m1, r1 = torch.empty(M, device=DEV), torch.empty(M, device=DEV)
    ops.seq_embed_fwd(ids, E, P, w, b, x, m, r, drop=(p, sd), norm1=(w1, b1, 1e-5, y1, m1, r1))
    torch.cuda.synchronize()
    assert torch.equal(x, x0) and torch.equal(m, m0) and torch.equal(r, r0)
    y_ref = TF.layer_norm(x.cpu(), (D,), w1.cpu(), b1.cpu(), 1e-5)
    assert rel(y1.float(), y_ref) < 8e-3
    assert rel(m1, x.cpu().mean(1)) < 1e-5


@pytest.mark.parametrize("D", [256, 768, 1024])
@pytest.mark.parametrize("with_res", [False, True])
def test_layernorm_bwd_wide_no_sums(gpu_pkg, D, with_res):
    """The frozen-LayerNorm backward (no dw/db, no gate; the text encoder's post-LNs): the
    16-byte-per-lane kernel vs torch autograd, with the residual added (and aliased)."""
    ops = gpu_pkg.ops
    M = 1000
    g = torch.Generator().manual_seed(D + with_res)
    x = torch.randn(M, D, generator=g) * 2 - 0.5
    w = torch.randn(D, generator=g)
    b = torch.randn(D, generator=g)
    xt = x.clone().requires_grad_(True)
    TF.layer_norm(xt, (D,), w, b, 1e-7).backward(dy := torch.randn(M, D, generator=g))
    mean = x.mean(1)
    rstd = 1.0 / torch.sqrt(x.var(1, unbiased=False) + 1e-7)
    res = torch.randn(M, D, generator=g)
    dx = res.clone().to(DEV) if with_res else torch.empty(M, D, device=DEV)
    ops.layernorm_bwd(dy.to(DEV), x.to(DEV), mean.to(DEV), rstd.to(DEV), w.to(DEV), dx, None, None,
                      res=dx if with_res else None)           # res aliases dx
    torch.cuda.synchronize()
    assert rel(dx, xt.grad + (res if with_res else 0.0)) < 5e-5


@pytest.mark.parametrize("H", [192, 768])
def test_deb_ln_fwd(gpu_pkg, H):
    """DeBERTa post-LayerNorm (fp32 copy + bf16 operand with a wider row stride, row stats):
    the scalar (H % 256 != 0) and the 16-byte-per-lane (H = 768) kernels vs torch."""
    ops = gpu_pkg.ops
    M, ld16 = 517, H + 64
    g = torch.Generator().manual_seed(H)
    z = torch.randn(M, H, generator=g) * 3 + 0.25
    w, b = torch.randn(H, generator=g), torch.randn(H, generator=g)
    ref = TF.layer_norm(z, (H,), w, b, 1e-7)
    y32 = torch.empty(M, H, device=DEV)
    y16 = torch.zeros(M, ld16, device=DEV, dtype=torch.bfloat16)
    mean, rstd = torch.empty(M, device=DEV), torch.empty(M, device=DEV)
    ops.deb_ln_fwd(z.to(DEV), w.to(DEV), b.to(DEV), 1e-7, y32, y16[:, :H], mean, rstd)
    torch.cuda.synchronize()
    assert rel(y32, ref) < 2e-5
    assert rel(y16[:, :H].float(), ref) < 8e-3
    assert y16[:, H:].abs().max().item() == 0.0
    assert rel(mean, z.mean(1)) < 1e-5


def test_norm_backward_bf16_copies(gpu_pkg):
    """The optional bf16 copies of LayerNorm / BatchNorm1d backward outputs (dx16 / dz16) equal
    bf16(dx) / bf16(dz) exactly."""
    ops = gpu_pkg.ops
    g = torch.Generator().manual_seed(5)
    M, D = 512, 128
    x = torch.randn(M, D, generator=g).to(DEV)
    w, b = torch.randn(D, generator=g).to(DEV), torch.randn(D, generator=g).to(DEV)
    y = torch.empty(M, D, device=DEV, dtype=torch.bfloat16)
    mean, rstd = torch.empty(M, device=DEV), torch.empty(M, device=DEV)
    ops.layernorm_fwd(x, w, b, y, mean, rstd, relu=True)
    dy = torch.randn(M, D, generator=g).to(DEV)
    dx, dx16 = torch.empty(M, D, device=DEV), torch.empty(M, D, device=DEV, dtype=torch.bfloat16)
    dw, db = torch.zeros(D, device=DEV), torch.zeros(D, device=DEV)
    ops.layernorm_bwd(dy, x, mean, rstd, w, dx, dw, db, gate=y, dx16=dx16)
    assert torch.equal(dx16, dx.to(torch.bfloat16))
    B, C = 300, 96
    z = torch.randn(B, C, generator=g).to(DEV)
    yb = torch.empty(B, C, device=DEV, dtype=torch.bfloat16)
    bm, br = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
    ops.batchnorm_fwd(z, w[:C], b[:C], yb, bm, br, None, None, None, relu=True)
    dyb = torch.randn(B, C, generator=g).to(DEV)
    dz, dz16 = torch.empty(B, C, device=DEV), torch.empty(B, C, device=DEV, dtype=torch.bfloat16)
    ops.batchnorm_bwd(dyb, z, w[:C], bm, br, yb, dz, torch.zeros(C, device=DEV),
                      torch.zeros(C, device=DEV), dz16=dz16)
    assert torch.equal(dz16, dz.to(torch.bfloat16))


@pytest.mark.parametrize("D", [128, 768])            # generic and 16-byte-lane kernels
def test_layernorm_bwd_dropout_copy(gpu_pkg, D):
    """dx16 = bf16(dropout(dx)) with keep index m*D + n (the post-LN residual dropout
    backward fused into the LayerNorm backward) vs the separate dropout kernel's mask."""
    ops = gpu_pkg.ops
    M, p, seed = 700, 0.1, 0x5151
    g = torch.Generator().manual_seed(D)
    x = torch.randn(M, D, generator=g).to(DEV)
    w = torch.randn(D, generator=g).to(DEV)
    mean, rstd = x.mean(1), 1.0 / torch.sqrt(x.var(1, unbiased=False) + 1e-7)
    dy = torch.randn(M, D, generator=g).to(DEV)
    dx = torch.empty(M, D, device=DEV)
    dx16 = torch.empty(M, D, device=DEV, dtype=torch.bfloat16)
    ops.layernorm_bwd(dy, x, mean, rstd, w, dx, None, None, dx16=dx16, drop=(p, seed_dev(seed)))
    ref16 = torch.empty(M, D, device=DEV, dtype=torch.bfloat16)
    ops.dropout_bwd(dx, ref16, None, (p, seed_dev(seed)))
    torch.cuda.synchronize()
    assert torch.equal(dx16, ref16)


def test_deb_ln_fwd_lora_dropout_outputs(gpu_pkg):
    """The post-LN kernel's fused next-layer LoRA inputs equal ttmi_dropout_bwd applied to its
    fp32 output with the same seeds (bit-exact: same values, same keep index)."""
    ops = gpu_pkg.ops
    M, H, p = 333, 768, 0.1
    g = torch.Generator().manual_seed(7)
    z = torch.randn(M, H, generator=g).to(DEV)
    w, b = torch.randn(H, generator=g).to(DEV), torch.randn(H, generator=g).to(DEV)
    y32 = torch.empty(M, H, device=DEV)
    y16 = torch.empty(M, H + 64, device=DEV, dtype=torch.bfloat16)
    mean, rstd = torch.empty(M, device=DEV), torch.empty(M, device=DEV)
    yq = torch.empty(M, H, device=DEV, dtype=torch.bfloat16)
    yv = torch.empty(M, H, device=DEV, dtype=torch.bfloat16)
    sq, sv = seed_dev(0x1234), seed_dev(0x9876)
    ops.deb_ln_fwd(z, w, b, 1e-7, y32, y16[:, :H], mean, rstd, yq=yq, yv=yv, drop_q=(p, sq),
                   drop_v=(p, sv))
    rq = ops.dropout_to(y32, torch.empty(M, H, device=DEV, dtype=torch.bfloat16), (p, sq))
    rv = ops.dropout_to(y32, torch.empty(M, H, device=DEV, dtype=torch.bfloat16), (p, sv))
    torch.cuda.synchronize()
    assert torch.equal(yq, rq) and torch.equal(yv, rv)
    assert not torch.equal(yq, yv)


@pytest.mark.parametrize("M,N,R,pad", [
    (384, 128, 25600, 0), (128, 512, 25600, 0), (128, 128, 25600, 64), (176, 128, 512, 0),
    (72, 200, 1000, 8), (512, 512, 512, 0), (64, 64, 100, 0), (136, 72, 777, 32), (8, 8, 1, 0),
    (128, 128, 7, 0)])
def test_wgrad_deterministic(gpu_pkg, M, N, R, pad):
    """ttmi_wgrad (the nn.Linear weight gradient of every bf16 Linear): dw += dyᵀx over R rows
    and db += Σ dy, with strided operands, partial tiles, short and long R; split partials are
    summed in split order, so two runs (and a graph replay) agree bit for bit."""
    ops = gpu_pkg.ops
    g = torch.Generator().manual_seed(M * 7 + N + R)
    dy_full = torch.randn(R, M + 2 * pad, generator=g).to(torch.bfloat16).to(DEV)
    x_full = torch.randn(R, N + pad, generator=g).to(torch.bfloat16).to(DEV)
    dy = dy_full[:, pad:pad + M]
    x = x_full[:, :N]
    expect = 0.5 + dy.float().t() @ x.float()
    outs = []
    for _ in range(2):
        gw = torch.full((M, N), 0.5, device=DEV)
        gb = torch.full((M,), -1.0, device=DEV)
        ops.linear_dw(dy, x, gw, gb)
        outs.append((gw, gb))
    torch.cuda.synchronize()
    gw, gb = outs[0]
    assert rel(gw, expect) < 5e-5, rel(gw, expect)
    assert rel(gb, -1.0 + dy.float().sum(0)) < 5e-5
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    # a captured replay equals the eager result bit for bit
    gw2 = torch.full((M, N), 0.5, device=DEV)
    gb2 = torch.full((M,), -1.0, device=DEV)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            ops.linear_dw(dy, x, gw2, gb2)
    torch.cuda.current_stream().wait_stream(s)
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(gw2, gw) and torch.equal(gb2, gb)


def test_wgrad_deferred_fold_many(gpu_pkg):
    """deferred_wgrad(): eighteen weight gradients (more than one grouped launch's / fold
    launch's 16 entries) are recorded and computed at the block's flush; equal, bit for bit,
    to the immediate path; defer=False inside the block completes at once."""
    ops = gpu_pkg.ops
    g = torch.Generator().manual_seed(5)
    shapes = [(384, 128, 25600), (128, 128, 2048), (512, 128, 4096), (128, 512, 3000)] * 5
    shapes = shapes[:18]
    ins = [(torch.randn(R, M, generator=g).to(torch.bfloat16).to(DEV),
            torch.randn(R, N, generator=g).to(torch.bfloat16).to(DEV)) for M, N, R in shapes]
    ref_out = []
    for dy, x in ins:
        gw = torch.zeros(dy.shape[1], x.shape[1], device=DEV)
        gb = torch.zeros(dy.shape[1], device=DEV)
        ops.linear_dw(dy, x, gw, gb)
        ref_out.append((gw, gb))
    outs = []
    with ops.deferred_wgrad() as pend:
        for k, (dy, x) in enumerate(ins):
            gw = torch.zeros(dy.shape[1], x.shape[1], device=DEV)
            gb = torch.zeros(dy.shape[1], device=DEV)
            ops.linear_dw(dy, x, gw, gb, defer=(k != 3))
            outs.append((gw, gb))
        torch.cuda.synchronize()
        assert torch.equal(outs[3][0], ref_out[3][0])          # defer=False: already complete
        assert len(pend.items) == 17
    torch.cuda.synchronize()
    for (a, b), (c, d) in zip(outs, ref_out):
        assert torch.equal(a, c) and torch.equal(b, d)


@pytest.mark.parametrize("B,L,K", [(64, 50, 384), (7, 20, 512)])
def test_linear_ln_bwd_gathered_residual(gpu_pkg, B, L, K):
    """res_rows (the pruned layer): res [B, D] row b lands only on row res_rows[b] == the
    un-gathered residual followed by ttmi_scatter_add_rows; the emitted dropout output
    (next) is dropout(dx) of the full rows."""
    ops = gpu_pkg.ops
    D, M = 128, B * L
    g = torch.Generator().manual_seed(B + K)
    dh = torch.randn(M, K, generator=g).to(torch.bfloat16).to(DEV)
    wt = (torch.randn(D, K, generator=g) / math.sqrt(K)).to(torch.bfloat16).to(DEV)
    x = (torch.randn(M, D, generator=g) * 2 + 0.5).to(DEV)
    w = torch.randn(D, generator=g).to(DEV)
    mean, rstd = x.mean(1), 1.0 / torch.sqrt(x.var(1, unbiased=False) + 1e-5)
    lens = torch.randint(0, L + 1, (B,), generator=g)
    rows = (torch.arange(B) * L + (lens - 1).clamp(min=0)).to(torch.int32).to(DEV)
    res = torch.randn(B, D, generator=g).to(DEV)
    p, sd = 0.1, seed_dev(0x5151)
    dx_a = torch.empty(M, D, device=DEV)
    dw_a, db_a = torch.zeros(D, device=DEV), torch.zeros(D, device=DEV)
    ops.linear_ln_bwd(dh, wt, x, mean, rstd, w, dx_a, dw_a, db_a)
    ops.scatter_add_rows(res, rows, dx_a)
    nx_a = torch.empty(M, D, device=DEV, dtype=torch.bfloat16)
    ops.dropout_bwd(dx_a, nx_a, None, (p, sd))
    dx_b = torch.empty(M, D, device=DEV)
    dw_b, db_b = torch.zeros(D, device=DEV), torch.zeros(D, device=DEV)
    nx_b = torch.empty(M, D, device=DEV, dtype=torch.bfloat16)
    ops.linear_ln_bwd(dh, wt, x, mean, rstd, w, dx_b, dw_b, db_b, res=res, res_rows=rows, res_L=L,
                      next_=nx_b, drop=(p, sd))
    torch.cuda.synchronize()
    assert torch.allclose(dx_a, dx_b, rtol=0, atol=1e-6)
    assert rel(dw_a, dw_b) < 1e-5 and rel(db_a, db_b) < 1e-5   # float atomics (no fold here)
    assert (nx_a.float() - nx_b.float()).abs().max().item() <= 1e-2 * nx_a.float().abs().max().item()

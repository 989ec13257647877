"""The fused in_proj + attention forward (ttmi_qkv_attn_fwd, reference user_tower.py:111-116)
against the two launches it replaces — ttmi_linear then ttmi_mha_fwd, themselves parity-tested
against the oracle in test_gpu_kernels.py.  The fused kernel shares the panel GEMM's MFMA order
(ttmi_linear's kernel from M = 2048 rows) and the attention tile code, so qkv (there), ctx and
lse must be bit-identical, on ragged batches (a last
workgroup with fewer sequences), every sequences-per-workgroup packing, empty / left-padded /
full key masks, with and without dropout."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _seed(val):
    v = val - (1 << 64) if val >= (1 << 63) else val
    return torch.tensor([v], dtype=torch.int64, device=DEV)


def _masks(B, L, g):
    lengths = torch.randint(1, L + 1, (B,), generator=g)
    lengths[0] = L
    lengths[1 % B] = 0
    m = (torch.arange(L)[None] < lengths[:, None]).long()
    if B > 2:
        m[2] = m[2].flip(0)            # left-padded row
    return m


@pytest.mark.parametrize("B,L,p", [(512, 50, 0.1), (7, 50, 0.0), (3, 50, 0.1), (33, 64, 0.1),
                                   (21, 20, 0.1), (5, 1, 0.0), (64, 37, 0.2), (9, 56, 0.0)])
def test_qkv_attn_matches_linear_then_mha(gpu_pkg, B, L, p):
    ops = gpu_pkg.ops
    H, D = 4, 128
    assert ops.qkv_attn_supported(torch.bfloat16, L, H, D // H)
    g = torch.Generator().manual_seed(1000 * L + B)
    a = torch.randn(B * L, D, generator=g).to(torch.bfloat16).to(DEV)
    w = (torch.randn(3 * D, D, generator=g) / D ** 0.5).to(torch.bfloat16).to(DEV)
    b = (torch.randn(3 * D, generator=g) * 0.1).to(DEV)
    kv = _masks(B, L, g).to(DEV)
    drop = (p, _seed(0x0DDBA11CAFEF00D5 + L)) if p > 0 else (0.0, None)
    qkv1 = torch.full((B * L, 3 * D), float("nan"), device=DEV, dtype=torch.bfloat16)
    ctx1 = torch.full((B * L, D), float("nan"), device=DEV, dtype=torch.bfloat16)
    lse1 = torch.full((B * H * L,), float("nan"), device=DEV)
    ops.qkv_attn_fwd(a, w, b, kv, B, L, H, qkv1, ctx1, lse1, drop)
    # the projection: within bf16 rounding of the fp32 product; at M >= 2048, where ttmi_linear
    # runs the panel kernel, bit-identical to it (same MFMA order, bias add, rounding)
    ref = a.float() @ w.float().t() + b
    err = (qkv1.float() - ref).abs()
    assert bool((err <= ref.abs() * 2 ** -8 + 1e-5).all()), f"projection off by {err.max().item()}"
    if B * L >= 2048:
        qkv0 = torch.empty_like(qkv1)
        ops.linear(a, w, b, qkv0)
        assert torch.equal(qkv1.view(torch.int16), qkv0.view(torch.int16)), "projection differs"
    # the attention on that projection: bit-identical to ttmi_mha_fwd
    ctx0 = torch.empty_like(ctx1)
    lse0 = torch.empty_like(lse1)
    ops.mha_fwd(qkv1, kv, B, L, H, ctx0, lse0, drop)
    torch.cuda.synchronize()
    assert torch.equal(lse1, lse0), "lse differs"
    assert torch.equal(ctx1.view(torch.int16), ctx0.view(torch.int16)), "context differs"


def test_qkv_attn_refuses_unserved_shapes(gpu_pkg):
    ops = gpu_pkg.ops
    assert not ops.qkv_attn_supported(torch.bfloat16, 50, 4, 64)      # d_model 256
    assert not ops.qkv_attn_supported(torch.bfloat16, 65, 4, 32)      # L > 64
    assert not ops.qkv_attn_supported(torch.float32, 50, 4, 32)
    a = torch.zeros(4 * 65, 128, device=DEV, dtype=torch.bfloat16)
    w = torch.zeros(384, 128, device=DEV, dtype=torch.bfloat16)
    b = torch.zeros(384, device=DEV)
    kv = torch.ones(4, 65, device=DEV, dtype=torch.int64)
    qkv = torch.empty(4 * 65, 384, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(Exception, match="ttmi_qkv_attn_fwd"):
        ops.qkv_attn_fwd(a, w, b, kv, 4, 65, 4, qkv, torch.empty_like(a), torch.empty(4 * 4 * 65, device=DEV))


@pytest.mark.parametrize("B,L,p", [(512, 50, 0.1), (9, 20, 0.0), (4, 64, 0.1)])
def test_q1_proj_gather_matches_full_projection(gpu_pkg, B, L, p):
    """The pruned layer's one-query attention with its query rows projected in the launch
    (ttmi_mha_q1_proj_gather_fwd, K / V from a 256-column projection) against the full
    384-column projection + ttmi_mha_q1_gather_fwd: the gathered rows and residual rows equal,
    the query row within bf16 rounding of the fp32 product, ctx / lse to fp32-accumulation noise."""
    ops = gpu_pkg.ops
    H, D = 4, 128
    g = torch.Generator().manual_seed(77 * L + B)
    a = torch.randn(B * L, D, generator=g).to(torch.bfloat16).to(DEV)
    w = (torch.randn(3 * D, D, generator=g) / D ** 0.5).to(torch.bfloat16).to(DEV)
    b = (torch.randn(3 * D, generator=g) * 0.1).to(DEV)
    x = torch.randn(B * L, D, generator=g).to(DEV)
    kv = _masks(B, L, g).to(DEV)
    kv[1 % B] = 0
    kv[1 % B, 0] = 1                                    # (the gather needs one valid key)
    drop = (p, _seed(0x5EED0F00D + L)) if p > 0 else (0.0, None)
    outs = []
    for proj in (False, True):
        qkv = torch.zeros(B * L, 3 * D, device=DEV, dtype=torch.bfloat16)
        rows = torch.empty(B, device=DEV, dtype=torch.int32)
        xr = torch.empty(B, D, device=DEV)
        ctx = torch.empty(B, D, device=DEV, dtype=torch.bfloat16)
        lse = torch.empty(B * H, device=DEV)
        if proj:
            ops.gemm(a, w[D:], qkv[:, D:], B * L, 2 * D, D, lda=D, a_kmajor=True, ldb=D, b_kmajor=True,
                     ldc=3 * D, bias=b[D:])
            ops.mha_q1_proj_gather_fwd(qkv, kv, a, w[:D], b[:D], x, rows, xr, B, L, H, ctx, lse, drop)
        else:
            ops.linear(a, w, b, qkv)
            ops.mha_q1_gather_fwd(qkv, kv, x, rows, xr, B, L, H, ctx, lse, drop)
        torch.cuda.synchronize()
        outs.append((qkv, rows, xr, ctx, lse))
    (q0, r0, x0, c0, l0), (q1, r1, x1, c1, l1) = outs
    assert torch.equal(r0, r1) and torch.equal(x0, x1)
    rl = r1.long()
    ref = a.float()[rl] @ w.float()[:D].t() + b[:D]
    err = (q1[rl, :D].float() - ref).abs()
    assert bool((err <= ref.abs() * 2 ** -8 + 1e-5).all()), float(err.max())
    assert torch.equal(q1[:, D:], q0[:, D:]) if B * L >= 2048 else True
    assert float((c1.float() - c0.float()).abs().max()) <= 0.02 * float(c0.float().abs().max()) + 1e-3
    fin = torch.isfinite(l0)
    assert torch.equal(fin, torch.isfinite(l1))
    assert float((l1[fin] - l0[fin]).abs().max()) <= 1e-2


@pytest.mark.parametrize("B,L,p", [(512, 50, 0.1), (7, 50, 0.0), (33, 64, 0.1), (21, 20, 0.1)])
def test_mha_bwd_dy_matches_linear_then_mha_bwd(gpu_pkg, B, L, p):
    """ttmi_mha_bwd_dy (dctx = dy·W_o computed in the attention backward) against
    ttmi_linear(dy, W_oᵀ) + ttmi_mha_bwd: bit-identical where the row panel serves the linear
    (M >= 2048), else within bf16 rounding of dctx's accumulation order."""
    ops = gpu_pkg.ops
    H, D = 4, 128
    g = torch.Generator().manual_seed(31 * L + B)
    qkv = (torch.randn(B * L, 3 * D, generator=g) * 1.5).to(torch.bfloat16).to(DEV)
    dy = torch.randn(B * L, D, generator=g).to(torch.bfloat16).to(DEV)
    wot = (torch.randn(D, D, generator=g) / D ** 0.5).to(torch.bfloat16).to(DEV)
    kv = _masks(B, L, g).to(DEV)
    drop = (p, _seed(0xD0D0 + L)) if p > 0 else (0.0, None)
    ctx = torch.empty(B * L, D, device=DEV, dtype=torch.bfloat16)
    lse = torch.empty(B * H * L, device=DEV)
    ops.mha_fwd(qkv, kv, B, L, H, ctx, lse, drop)
    dctx = torch.empty(B * L, D, device=DEV, dtype=torch.bfloat16)
    ops.linear(dy, wot, None, dctx)
    d0 = torch.empty(B * L, 3 * D, device=DEV, dtype=torch.bfloat16)
    ops.mha_bwd(qkv, kv, lse, dctx, B, L, H, d0, drop)
    d1 = torch.full_like(d0, float("nan"))
    ops.mha_bwd_dy(qkv, kv, lse, dy, wot, B, L, H, d1, drop)
    torch.cuda.synchronize()
    if B * L >= 2048:
        assert torch.equal(d1.view(torch.int16), d0.view(torch.int16))
    else:
        err = (d1.float() - d0.float()).abs().max()
        assert float(err) <= 0.02 * float(d0.float().abs().max()) + 1e-3, float(err)


@pytest.mark.parametrize("B,L,p", [(512, 50, 0.1), (7, 50, 0.0), (33, 64, 0.1), (5, 38, 0.1)])
def test_attn_block_matches_qkv_attn_then_res_ln(gpu_pkg, B, L, p):
    """ttmi_attn_block_fwd (in_proj + attention + out_proj + residual + dropout 1 + norm2 in one
    launch) against ttmi_qkv_attn_fwd + ttmi_linear_res_ln: qkv / ctx / lse / x1 bit-identical
    (the same MFMA orders, bias adds and dropout indices; the out-projection as the row panel
    computes it from M = 2048 rows), norm2's outputs to its summation order (1e-5)."""
    ops = gpu_pkg.ops
    H, D = 4, 128
    g = torch.Generator().manual_seed(5 * L + B)
    a = torch.randn(B * L, D, generator=g).to(torch.bfloat16).to(DEV)
    w = (torch.randn(3 * D, D, generator=g) / D ** 0.5).to(torch.bfloat16).to(DEV)
    b = (torch.randn(3 * D, generator=g) * 0.1).to(DEV)
    wo = (torch.randn(D, D, generator=g) / D ** 0.5).to(torch.bfloat16).to(DEV)
    bo = (torch.randn(D, generator=g) * 0.1).to(DEV)
    res = torch.randn(B * L, D, generator=g).to(DEV)
    n2w, n2b = (1 + 0.1 * torch.randn(D, generator=g)).to(DEV), (0.1 * torch.randn(D, generator=g)).to(DEV)
    kv = _masks(B, L, g).to(DEV)
    drop = (p, _seed(0xB10C + L)) if p > 0 else (0.0, None)
    drop1 = (p, _seed(0xB10D + L)) if p > 0 else (0.0, None)
    M = B * L
    bf = dict(device=DEV, dtype=torch.bfloat16)
    outs = []
    for fused in (False, True):
        qkv, ctx = torch.empty(M, 3 * D, **bf), torch.empty(M, D, **bf)
        lse = torch.empty(B * H * L, device=DEV)
        x1, a2 = torch.empty(M, D, device=DEV), torch.empty(M, D, **bf)
        m2, r2 = torch.empty(M, device=DEV), torch.empty(M, device=DEV)
        if fused:
            ops.attn_block_fwd(a, w, b, kv, B, L, H, qkv, ctx, lse, drop, wo, bo, res, n2w, n2b, 1e-5, drop1,
                               x1, a2, m2, r2)
        else:
            ops.qkv_attn_fwd(a, w, b, kv, B, L, H, qkv, ctx, lse, drop)
            ops.linear_res_ln(ctx, wo, bo, res, x1, n2w, n2b, a2, m2, r2, eps=1e-5, drop=drop1)
        torch.cuda.synchronize()
        outs.append((qkv, ctx, lse, x1, a2, m2, r2))
    (q0, c0, l0, x0, a0, mu0, r0), (q1, c1, l1, x1_, a1, mu1, r1) = outs
    assert torch.equal(q1.view(torch.int16), q0.view(torch.int16))
    assert torch.equal(c1.view(torch.int16), c0.view(torch.int16)) and torch.equal(l1, l0)
    if M >= 2048:
        assert torch.equal(x1_, x0)
    else:
        assert float((x1_ - x0).abs().max()) <= 1e-2 * float(x0.abs().max())
    assert float((mu1 - mu0).abs().max()) <= 1e-4 and float(((r1 - r0) / r0).abs().max()) <= 1e-4
    assert float((a1.float() - a0.float()).abs().max()) <= 0.02 * float(a0.float().abs().max())


@pytest.mark.parametrize("B,L,p", [(512, 50, 0.1), (7, 50, 0.0), (33, 64, 0.1), (5, 1, 0.0)])
def test_q1_kv_bwd_and_dy_add_match_full_dqkv(gpu_pkg, B, L, p):
    """ttmi_mha_q1_kv_bwd + ttmi_linear_ln_bwd(K = 256, dy_add) against ttmi_mha_q1_bwd +
    ttmi_linear_ln_bwd(K = 384) for the pruned layer: dqkv's K / V columns and the gathered dq
    bit-identical, a_rows = a_in[rows], dyq = dq·W_q in fp32, and the LN1 backward (dx, the
    emitted bf16 rows, norm1's grads) equal to the K = 384 form to fp32 rounding."""
    ops = gpu_pkg.ops
    H, D = 4, 128
    M = B * L
    g = torch.Generator().manual_seed(91 * L + B)
    qkv = (torch.randn(M, 3 * D, generator=g) * 0.7).to(torch.bfloat16).to(DEV)
    kv = _masks(B, L, g).to(DEV)
    rows = torch.empty(B, dtype=torch.int32, device=DEV)
    ops.last_rows(kv, rows)
    lse, ctx = torch.empty(B * H, device=DEV), torch.empty(B, D, device=DEV, dtype=torch.bfloat16)
    drop = (p, _seed(0x91 + L)) if p > 0 else (0.0, None)
    ops.mha_q1_fwd(qkv, kv, rows, B, L, H, ctx, lse, drop)
    dctx = torch.randn(B, D, generator=g).to(torch.bfloat16).to(DEV)
    w_in = (torch.randn(3 * D, D, generator=g) / D ** 0.5).to(torch.bfloat16).to(DEV)
    wti = w_in.t().contiguous()
    a_in = torch.randn(M, D, generator=g).to(torch.bfloat16).to(DEV)
    dq0 = torch.empty(M, 3 * D, device=DEV, dtype=torch.bfloat16)
    ops.mha_q1_bwd(qkv, kv, rows, lse, dctx, B, L, H, dq0, drop)
    dq1 = torch.zeros(M, 3 * D, device=DEV, dtype=torch.bfloat16)
    dqg, ag = torch.empty(B, D, device=DEV, dtype=torch.bfloat16), torch.empty(B, D, device=DEV, dtype=torch.bfloat16)
    dyq = torch.empty(B, D, device=DEV)
    ops.mha_q1_kv_bwd(qkv, kv, rows, lse, dctx, B, L, H, dq1, drop, wti, a_in, dqg, ag, dyq)
    torch.cuda.synchronize()
    r = rows.long()
    assert torch.equal(dq1[:, D:].view(torch.int16), dq0[:, D:].view(torch.int16))
    assert torch.equal(dqg.view(torch.int16), dq0[r, :D].view(torch.int16))
    assert torch.equal(ag.view(torch.int16), a_in[r].view(torch.int16))
    ref = dqg.float() @ w_in[:D].float()
    assert float((dyq - ref).abs().max()) <= 1e-5 * max(float(ref.abs().max()), 1.0)
    # the LN1 backward both ways
    x = torch.randn(M, D, generator=g).to(DEV)
    mu, rs = x.mean(1), torch.rsqrt(x.var(1, unbiased=False) + 1e-5)
    n1w = (1 + 0.1 * torch.randn(D, generator=g)).to(DEV)
    res = torch.randn(B, D, generator=g).to(DEV)
    outs = []
    for kvo in (False, True):
        dx = torch.empty(M, D, device=DEV)
        nxt = torch.empty(M, D, device=DEV, dtype=torch.bfloat16)
        gw, gb = torch.zeros(D, device=DEV), torch.zeros(D, device=DEV)
        ops.linear_ln_bwd(dq1[:, D:] if kvo else dq0, wti[:, D:] if kvo else wti, x, mu, rs, n1w, dx, gw, gb,
                          res=res, res_rows=rows, res_L=L, next_=nxt, dy_add=dyq if kvo else None)
        torch.cuda.synchronize()
        outs.append((dx, nxt, gw, gb))
    (x0, n0, w0, b0), (x1, n1, w1, b1) = outs
    assert float((x1 - x0).abs().max()) <= 1e-4 * float(x0.abs().max())
    assert float((n1.float() - n0.float()).abs().max()) <= 0.01 * float(n0.float().abs().max())
    assert torch.allclose(w1, w0, rtol=1e-3, atol=1e-4 * float(w0.abs().max()))
    assert torch.allclose(b1, b0, rtol=1e-3, atol=1e-4 * float(b0.abs().max()))

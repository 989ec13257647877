"""The fused feed-forward sub-block forward (ttmi_ffn_block_fwd, reference user_tower.py:37-45 and
the next layer's norm1, :111-116) against the two launches it replaces — ttmi_linear(act=ReLU)
then ttmi_linear_res_ln, themselves parity-tested against the oracle in test_gpu_kernels.py — and
against a torch fp32 restatement.  h shares the FFN1 row panel's fragments and MFMA order (the
kernel ttmi_linear runs from M = 2048 rows): bit-identical there.  FFN2 sums its k-steps in
hidden-unit order, so x2 / y / mean / rstd agree to fp32 rounding (tolerances below)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _seed(val):
    v = val - (1 << 64) if val >= (1 << 63) else val
    return torch.tensor([v], dtype=torch.int64, device=DEV)


def _operands(M, F, g, D=128):
    a = torch.randn(M, D, generator=g).to(torch.bfloat16)
    w1 = (torch.randn(F, D, generator=g) / D ** 0.5).to(torch.bfloat16)
    b1 = torch.randn(F, generator=g) * 0.1
    w2 = (torch.randn(D, F, generator=g) / F ** 0.5).to(torch.bfloat16)
    b2 = torch.randn(D, generator=g) * 0.1
    res = torch.randn(M, D, generator=g)
    lnw = 1 + 0.1 * torch.randn(D, generator=g)
    lnb = 0.1 * torch.randn(D, generator=g)
    return [t.to(DEV) for t in (a, w1, b1, w2, b2, res, lnw, lnb)]


def _run(ops, fused, M, F, ops_in, drop_f, drop2, D=128):
    a, w1, b1, w2, b2, res, lnw, lnb = ops_in
    h = torch.empty(M, F, device=DEV, dtype=torch.bfloat16)
    x2 = torch.empty(M, D, device=DEV)
    y = torch.empty(M, D, device=DEV, dtype=torch.bfloat16)
    mu, rs = torch.empty(M, device=DEV), torch.empty(M, device=DEV)
    if fused:
        ops.ffn_block_fwd(a, w1, b1, w2, b2, res, drop_f, drop2, h, x2, lnw, lnb, 1e-5, y, mu, rs)
    else:
        ops.linear(a, w1, b1, h, act=1, drop=drop_f)
        ops.linear_res_ln(h, w2, b2, res, x2, lnw, lnb, y, mu, rs, eps=1e-5, drop=drop2)
    torch.cuda.synchronize()
    return h, x2, y, mu, rs


@pytest.mark.parametrize("M,F,p", [(25600, 512, 0.1), (2053, 512, 0.0), (2048, 256, 0.1), (7, 512, 0.1),
                                   (113, 256, 0.0), (1, 512, 0.0)])
def test_ffn_block_matches_linear_then_res_ln(gpu_pkg, M, F, p):
    ops = gpu_pkg.ops
    assert ops.ffn_block_supported(torch.bfloat16, 128, F)
    g = torch.Generator().manual_seed(17 * M + F)
    ops_in = _operands(M, F, g)
    drop_f = (p, _seed(0xFF1 + M)) if p > 0 else (0.0, None)
    drop2 = (p, _seed(0xFF2 + M)) if p > 0 else (0.0, None)
    h0, x0, y0, mu0, rs0 = _run(ops, False, M, F, ops_in, drop_f, drop2)
    h1, x1, y1, mu1, rs1 = _run(ops, True, M, F, ops_in, drop_f, drop2)
    if M >= 2048:
        assert torch.equal(h1.view(torch.int16), h0.view(torch.int16))
    else:       # ttmi_linear's small-M GEMM: another MFMA order
        assert float((h1.float() - h0.float()).abs().max()) <= 0.02 * float(h0.float().abs().max())
    # x2 from the fused kernel's own h, restated in fp32 (the FFN2 sum order aside: exact)
    a, w1, b1, w2, b2, res, lnw, lnb = ops_in
    keep2 = (x0 - res) != 0 if p > 0 else None
    ref = h1.float() @ w2.float().t() + b2
    if p > 0:
        ref = torch.where(keep2 | (ref == 0), ref / (1 - p), torch.zeros_like(ref))
    ref = ref + res
    tol = 2e-5 * float(ref.abs().max())
    assert float((x1 - ref).abs().max()) <= max(tol, 1e-5) * 4
    if M >= 2048:
        assert float((x1 - x0).abs().max()) <= max(tol, 1e-5) * 4
    assert float((mu1 - mu0).abs().max()) <= 1e-4 and float(((rs1 - rs0) / rs0).abs().max()) <= 1e-3
    assert float((y1.float() - y0.float()).abs().max()) <= 0.05


def test_ffn_block_no_dropout_vs_torch(gpu_pkg):
    """p = 0 against a torch fp32 restatement of the whole sub-block (h to bf16 rounding)."""
    ops = gpu_pkg.ops
    M, F = 4096, 512
    g = torch.Generator().manual_seed(3)
    ops_in = _operands(M, F, g)
    a, w1, b1, w2, b2, res, lnw, lnb = ops_in
    h, x2, y, mu, rs = _run(ops, True, M, F, ops_in, (0.0, None), (0.0, None))
    h_ref = torch.relu(a.float() @ w1.float().t() + b1)
    assert float((h.float() - h_ref).abs().max()) <= 2 ** -7 * float(h_ref.abs().max())
    x_ref = res + h_ref @ w2.float().t() + b2
    assert float((x2 - x_ref).abs().max()) <= 0.02
    y_ref = torch.nn.functional.layer_norm(x2, (128,), lnw, lnb, 1e-5)
    assert float((y.float() - y_ref).abs().max()) <= 0.03
    assert float((mu - x2.mean(1)).abs().max()) <= 1e-5


def test_ffn_block_refuses_unserved(gpu_pkg):
    ops = gpu_pkg.ops
    assert ops.ffn_block_supported(torch.bfloat16, 256, 1024)
    assert ops.ffn_block_supported(torch.bfloat16, 256, 1024, bwd=True)
    assert ops.ffn_block_supported(torch.bfloat16, 128, 512, bwd=True)
    assert not ops.ffn_block_supported(torch.bfloat16, 256, 512)
    assert not ops.ffn_block_supported(torch.bfloat16, 128, 384)
    assert not ops.ffn_block_supported(torch.float32, 128, 512)


@pytest.mark.parametrize("M,p", [(25600, 0.1), (2053, 0.0), (2048, 0.1), (7, 0.1), (129, 0.0)])
def test_ffn_block_d256(gpu_pkg, M, p):
    """ABI 22: the D = 256, F = 1024 forward (the reference's default width) against
    ttmi_linear(act=ReLU) + ttmi_linear_res_ln.  Its FFN1 fragments sum k in another order than
    the row panel (panel256), so h agrees to bf16 rounding; x2 is checked exactly
    against an fp32 restatement from the launch's own h, y / mean / rstd against the unfused
    pair."""
    ops = gpu_pkg.ops
    D, F = 256, 1024
    g = torch.Generator().manual_seed(41 * M + 3)
    ops_in = _operands(M, F, g, D=D)
    drop_f = (p, _seed(0xDF1 + M)) if p > 0 else (0.0, None)
    drop2 = (p, _seed(0xDF2 + M)) if p > 0 else (0.0, None)
    h0, x0, y0, mu0, rs0 = _run(ops, False, M, F, ops_in, drop_f, drop2, D=D)
    h1, x1, y1, mu1, rs1 = _run(ops, True, M, F, ops_in, drop_f, drop2, D=D)
    # identical dropout masks: zeros in the same places (a kept unit's pre-activation can round
    # to zero in one sum order only: allow a handful)
    z0, z1 = h0 == 0, h1 == 0
    assert int((z0 ^ z1).sum()) <= max(4, M * F // 100000)
    assert float((h1.float() - h0.float()).abs().max()) <= 2 ** -6 * float(h0.float().abs().max())
    a, w1, b1, w2, b2, res, lnw, lnb = ops_in
    ref = h1.float() @ w2.float().t() + b2
    if p > 0:
        keep2 = (x0 - res) != 0
        ref = torch.where(keep2 | (ref == 0), ref / (1 - p), torch.zeros_like(ref))
    ref = ref + res
    tol = 2e-5 * float(ref.abs().max())
    assert float((x1 - ref).abs().max()) <= max(tol, 1e-5) * 4
    assert float((x1 - x0).abs().max()) <= 0.02
    assert float((mu1 - mu0).abs().max()) <= 1e-3 and float(((rs1 - rs0) / rs0).abs().max()) <= 1e-2
    yr = torch.nn.functional.layer_norm(x1, (D,), lnw, lnb, 1e-5)
    assert float((y1.float() - yr).abs().max()) <= 0.03
    assert float((mu1 - x1.mean(1)).abs().max()) <= 1e-5


@pytest.mark.parametrize("M,F,p,D", [(25600, 512, 0.1, 128), (2053, 512, 0.0, 128), (2048, 256, 0.1, 128),
                                     (7, 512, 0.1, 128), (129, 256, 0.0, 128), (25600, 1024, 0.1, 256),
                                     (2053, 1024, 0.0, 256), (7, 1024, 0.1, 256), (129, 1024, 0.1, 256)])
def test_ffn_block_bwd_matches_gated_linear_then_ln_bwd(gpu_pkg, M, F, p, D):
    """ttmi_ffn_block_bwd against ttmi_linear(gate = h) + ttmi_linear_ln_bwd (both row panels from
    M = 2048): dz1 bit-identical there at D = 128; dx1 / dy1 / norm2's weight and bias grads to
    the fp32 rounding of FFN1's input-grad sum order (it sums hidden-unit order).  D = 256, F =
    1,024 (round 6): dz1's k order differs from the panel's too (bf16 rounding)."""
    ops = gpu_pkg.ops
    assert ops.ffn_block_supported(torch.bfloat16, D, F, bwd=True)
    g = torch.Generator().manual_seed(31 * M + F)
    dy2 = (torch.randn(M, D, generator=g) * 0.1).to(torch.bfloat16).to(DEV)
    w2t = (torch.randn(F, D, generator=g) / D ** 0.5).to(torch.bfloat16).to(DEV)
    w1t = (torch.randn(D, F, generator=g) / F ** 0.5).to(torch.bfloat16).to(DEV)
    hv = torch.randn(M, F, generator=g)
    hv[hv < 0.3] = 0.0                                  # the ReLU / dropout zeros
    h = hv.to(torch.bfloat16).to(DEV)
    x1 = torch.randn(M, D, generator=g).to(DEV)
    m2, r2 = x1.mean(1), torch.rsqrt(x1.var(1, unbiased=False) + 1e-5)
    n2w = (1 + 0.1 * torch.randn(D, generator=g)).to(DEV)
    res = torch.randn(M, D, generator=g).to(DEV)
    sf = 1.0 / (1.0 - p) if p > 0 else 1.0
    drop1 = (p, _seed(0xD1 + M)) if p > 0 else (0.0, None)
    outs = []
    for fused in (False, True):
        dz1 = torch.empty(M, F, device=DEV, dtype=torch.bfloat16)
        dx1 = torch.empty(M, D, device=DEV)
        dy1 = torch.empty(M, D, device=DEV, dtype=torch.bfloat16)
        gw, gb = torch.zeros(D, device=DEV), torch.zeros(D, device=DEV)
        if fused:
            ops.ffn_block_bwd(dy2, w2t, w1t, h, sf, dz1, x1, m2, r2, n2w, res, dx1, dy1, drop1, gw, gb)
        else:
            ops.linear(dy2, w2t, None, dz1, gate=h, gate_scale=sf)
            ops.linear_ln_bwd(dz1, w1t, x1, m2, r2, n2w, dx1, gw, gb, res=res, next_=dy1, drop=drop1)
        torch.cuda.synchronize()
        outs.append((dz1, dx1, dy1, gw, gb))
    (z0, x0, y0, w0, b0), (z1, x1_, y1, w1_, b1_) = outs
    if M >= 2048 and F == 512 and D == 128:   # the N = 512 row panel (ttmi_linear serves N = 256 otherwise)
        assert torch.equal(z1.view(torch.int16), z0.view(torch.int16))
    else:
        assert float((z1.float() - z0.float()).abs().max()) <= 0.02 * float(z0.float().abs().max())
    # dx1 against a torch fp32 restatement from the fused kernel's own dz1
    dY = z1.float() @ w1t.float().t()
    xh = (x1 - m2[:, None]) * r2[:, None]
    gg = dY * n2w
    ref = r2[:, None] * (gg - gg.mean(1, keepdim=True) - xh * (gg * xh).mean(1, keepdim=True)) + res
    assert float((x1_ - ref).abs().max()) <= 2e-4 * float(ref.abs().max())
    assert float((x1_ - x0).abs().max()) <= 5e-3 * float(x0.abs().max())
    assert float((y1.float() - y0.float()).abs().max()) <= 0.02 * float(y0.float().abs().max()) + 1e-3
    assert torch.allclose(w1_, (dY * xh).sum(0), rtol=1e-3, atol=1e-3 * float(w1_.abs().max()))
    assert torch.allclose(b1_, dY.sum(0), rtol=1e-3, atol=1e-3 * float(b1_.abs().max()))
    assert torch.allclose(w1_, w0, rtol=1e-2, atol=1e-2 * float(w0.abs().max()))


@pytest.mark.parametrize("M,F,p,pipe", [(25600, 512, 0.1, True), (2053, 512, 0.0, True), (2048, 256, 0.1, True),
                                        (113, 256, 0.1, True), (4100, 512, 0.1, False)])
def test_ffn_block_kv_projection(gpu_pkg, monkeypatch, M, F, p, pipe):
    """ABI 22: the next (pruned) layer's K / V projection inside the FFN block launch.  The
    launch's other outputs match the launch without it (h bit for bit), and kv is the K / V row
    panel's (ttmi_gemm of y against in_proj rows D..3D, + bias) bits from M = 2048 rows; below
    that the small-M GEMM sums in another order (bf16 rounding).  (TTMI_FFN_NOPIPE, the
    unpipelined group loop, is read once per process: A/B runs only.)"""
    ops = gpu_pkg.ops
    if not pipe:
        pytest.skip("TTMI_FFN_NOPIPE is read once per process; the unpipelined loop runs in A/B runs")
    D = 128
    g = torch.Generator().manual_seed(29 * M + F)
    ops_in = _operands(M, F, g)
    wkv = (torch.randn(2 * D, D, generator=g) / D ** 0.5).to(torch.bfloat16).to(DEV)
    bkv = (torch.randn(2 * D, generator=g) * 0.1).to(DEV)
    drop_f = (p, _seed(0xAF1 + M)) if p > 0 else (0.0, None)
    drop2 = (p, _seed(0xAF2 + M)) if p > 0 else (0.0, None)
    h0, x0, y0, mu0, rs0 = _run(ops, True, M, F, ops_in, drop_f, drop2)
    a, w1, b1, w2, b2, res, lnw, lnb = ops_in
    h = torch.empty(M, F, device=DEV, dtype=torch.bfloat16)
    x2 = torch.empty(M, D, device=DEV)
    y = torch.empty(M, D, device=DEV, dtype=torch.bfloat16)
    mu, rs = torch.empty(M, device=DEV), torch.empty(M, device=DEV)
    qkv = torch.full((M, 3 * D), float("nan"), device=DEV, dtype=torch.bfloat16)
    ops.ffn_block_fwd(a, w1, b1, w2, b2, res, drop_f, drop2, h, x2, lnw, lnb, 1e-5, y, mu, rs,
                      kv=(wkv, bkv, qkv[:, D:]))
    torch.cuda.synchronize()
    # h is bit-identical; x2 / LN to fp32 rounding (another instantiation: hipcc contracts the
    # epilogue's a·b + c differently), y to one bf16 step
    assert torch.equal(h0.view(torch.int16), h.view(torch.int16))
    assert float((x2 - x0).abs().max()) <= 1e-6 * float(x0.abs().max())
    assert float((mu - mu0).abs().max()) <= 1e-6 and float(((rs - rs0) / rs0).abs().max()) <= 1e-5
    assert float((y.float() - y0.float()).abs().max()) <= 0.02 * float(y0.float().abs().max())
    assert torch.isnan(qkv[:, :D].float()).all()                  # Q columns untouched
    # the K / V row panel on the launch's own y
    ref = torch.empty(M, 2 * D, device=DEV, dtype=torch.bfloat16)
    ops.gemm(y, wkv, ref, M, 2 * D, D, lda=D, a_kmajor=True, ldb=D, b_kmajor=True, ldc=2 * D, bias=bkv)
    torch.cuda.synchronize()
    got = qkv[:, D:].contiguous()
    if M >= 2048:
        assert torch.equal(got.view(torch.int16), ref.view(torch.int16))
    else:
        assert float((got.float() - ref.float()).abs().max()) <= 0.02 * float(ref.float().abs().max())

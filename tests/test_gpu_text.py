"""cfg-4 text encoder on the GPU (mDeBERTa-v3 + LoRA, reference item_tower.py:41-83).

* Kernel level: ttmi_dis_attn_fwd/bwd against torch fp32 math on the same bf16 inputs
  (disentangled attention with log buckets, padding, partial blocks): ctx within 1e-2 of the
  output's max-abs, dq/dk/dv within 2e-2 (bf16 operands of the backward products), and the
  LoRA contractions HU / PB (PB summed over batch and heads; built here from the explicit
  raw-score gradient) within 2e-2.
* Module level: TextEncoder loaded with the transformers-generated fixture's parameters
  (tests/golden/deberta_tiny.npz) — output within 3e-2 of the fixture (bf16 GEMMs through
  two post-LN layers); LoRA and projection gradients against the fp32 oracle by direction
  (cosine >= 0.99) and norm (within 5 %)."""
import math

import numpy as np
import pytest
import torch

from conftest import load_golden, sub
from oracle import deberta_ref as dref
from oracle import two_tower_ref as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    a = torch.as_tensor(a).detach().double().cpu()
    b = torch.as_tensor(b).detach().double().cpu()
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-30)


def _cos(a, b):
    a = torch.as_tensor(a).detach().double().cpu().flatten()
    b = torch.as_tensor(b).detach().double().cpu().flatten()
    return torch.dot(a, b).item() / (a.norm().item() * b.norm().item() + 1e-30)


def _bf(t):
    return t.to(torch.bfloat16).float()


@pytest.mark.parametrize("B,S,nh,lens,p", [(2, 64, 1, (64, 30), 0.0), (2, 160, 2, (160, 150), 0.0),
                                           (1, 256, 2, (200,), 0.0), (3, 256, 2, (256, 70, 16), 0.0),
                                           (2, 192, 2, (192, 77), 0.1), (2, 97, 1, (97, 41), 0.1),
                                           (1, 131, 2, (120,), 0.1)])
def test_dis_attn_kernels_vs_torch(gpu_pkg, B, S, nh, lens, p):
    """p > 0: attention-probability dropout with the kernels' counter-hash mask, regenerated
    here by oracle.two_tower_ref.hash_keep at index ((b·nh + h)·S + i)·S + j (odd S puts the
    hash pairs across rows)."""
    ops = gpu_pkg.ops
    text = gpu_pkg.text
    cfg = text.TextCfg(hidden=64 * nh, heads=nh)
    g = torch.Generator().manual_seed(S + nh)
    H, npos = 64 * nh, cfg.npos
    q, k, v = (_bf(torch.randn(B, S, H, generator=g)) for _ in range(3))
    posq, posk = _bf(torch.randn(npos, H, generator=g)), _bf(torch.randn(npos, H, generator=g))
    mask = torch.zeros(B, S, dtype=torch.int64)
    for b, L in enumerate(lens):
        mask[b, :L] = 1
    # padded rows get zero upstream gradient in the encoder (masked mean-pool): the kernels'
    # precondition for skipping padded blocks (include/ttmi.h, ttmi_dis_attn_desc)
    dctx = _bf(torch.randn(B, S, H, generator=g)) * mask[:, :, None].to(torch.float32)
    u = torch.randn(npos, 8, generator=g)
    bq = torch.randn(H, 8, generator=g) * 0.1
    delta_t = text._Frozen().delta(S, cfg, "cpu").long()
    dmat = torch.stack([delta_t[i - torch.arange(S) + S - 1] for i in range(S)])   # [S, S]
    scale = 1.0 / math.sqrt(64 * 3)
    # torch reference
    qr, kr, vr = (t.clone().requires_grad_(True) for t in (q, k, v))

    def heads(t):
        return t.view(B, S, nh, 64).permute(0, 2, 1, 3)
    Q, K, V = heads(qr), heads(kr), heads(vr)
    pQ = posq.view(npos, nh, 64).permute(1, 0, 2)
    pK = posk.view(npos, nh, 64).permute(1, 0, 2)
    c2c = Q @ K.transpose(-1, -2)
    c2p = torch.gather(Q @ pK.transpose(-1, -2), -1, dmat.expand(B, nh, S, S))
    p2c = torch.gather(K @ pQ.transpose(-1, -2), -1, dmat.t().expand(B, nh, S, S)).transpose(-1, -2)
    raw = c2c + c2p + p2c
    raw.retain_grad()
    m2 = (mask[:, None, :] * mask[:, :, None]).bool()[:, None]
    sc = (raw * scale).masked_fill(~m2, torch.finfo(torch.float32).min)
    probs = torch.softmax(sc, -1)
    seed = 0x1234_5678_9ABC_DEF1
    if p > 0:
        keep = torch.from_numpy(ref.hash_keep(seed, B * nh * S * S, p)).view(B, nh, S, S)
        probs = probs * keep.float() / (1.0 - p)
    ctx_ref = (probs @ V).permute(0, 2, 1, 3).reshape(B, S, H)
    (ctx_ref * dctx).sum().backward()
    dS = raw.grad                                                       # [B, nh, S, S]
    HU_ref = torch.einsum("bhij,ijc->bjhc", dS, u[dmat])
    KB = torch.einsum("bhjd,hdc->bhjc", K.detach(), bq.view(nh, 64, 8))
    PB_ref = torch.zeros(B, nh, npos, 8)
    contrib = torch.einsum("bhij,bhjc->bhijc", dS, KB).reshape(B, nh, S * S, 8)
    PB_ref.index_add_(2, dmat.reshape(-1), contrib)
    # GPU
    qkv = torch.cat([q, k, v], dim=2).reshape(B * S, 3 * H).to(torch.bfloat16).to(DEV)
    pos = torch.cat([posq, posk], dim=1).to(torch.bfloat16).to(DEV)
    md, dd = mask.to(DEV), delta_t.to(torch.int16).to(DEV)
    ctx = torch.empty(B * S, H, device=DEV, dtype=torch.bfloat16)
    lse = torch.empty(B * nh * S, device=DEV)
    drop = (p, torch.tensor([seed], dtype=torch.int64, device=DEV)) if p > 0 else ops.NO_DROP
    # the per-sequence kernels run in dis_attn_order's order (or batch order without it)
    order = ops.dis_attn_order(md, B, S) if B > 1 and S % 3 != 0 else None
    if order is not None:
        nl = ((mask.cumsum(1) * mask).argmax(1) + 64) // 64 * mask.any(1)
        got = order.cpu().long()
        assert sorted(got.tolist()) == list(range(B))
        assert (nl[got][:-1] >= nl[got][1:]).all(), (nl, got)
    ops.dis_attn(B, S, nh, qkv[:, :H], qkv[:, H:2 * H], qkv[:, 2 * H:], pos[:, :H], pos[:, H:], md,
                 dd, scale, ctx, lse, drop, order=order)
    torch.cuda.synchronize()
    valid = mask.reshape(-1).bool()
    cg = ctx.float().cpu().view(B * S, H)
    cr = ctx_ref.detach().reshape(B * S, H)
    assert rel(cg[valid], cr[valid]) < 1e-2, rel(cg[valid], cr[valid])
    assert torch.isfinite(cg).all()                # pad rows: don't-care, finite
    dqkv = torch.zeros(B * S, 3 * H, device=DEV, dtype=torch.bfloat16)
    hu = torch.zeros(B * S * nh * 8, device=DEV)
    pb = torch.full((npos * 8,), 7.0, device=DEV)         # overwritten
    ops.dis_attn(B, S, nh, qkv[:, :H], qkv[:, H:2 * H], qkv[:, 2 * H:], pos[:, :H], pos[:, H:], md,
                 dd, scale, ctx, lse, drop, dctx=dctx.reshape(B * S, H).to(torch.bfloat16).to(DEV),
                 dq=dqkv[:, :H], dk=dqkv[:, H:2 * H], dv=dqkv[:, 2 * H:], lora_u=u.to(DEV),
                 lora_bq=bq.to(DEV), lora_hu=hu, lora_pb=pb, order=order)
    torch.cuda.synchronize()
    dg = dqkv.float().cpu()
    for name, got, want in (("dq", dg[:, :H], qr.grad), ("dk", dg[:, H:2 * H], kr.grad),
                            ("dv", dg[:, 2 * H:], vr.grad)):
        want = want.reshape(B * S, H)
        assert rel(got, want) < 2e-2, (name, rel(got, want))
    assert rel(hu.cpu().view(B, S, nh, 8), HU_ref) < 2e-2, rel(hu.cpu().view(B, S, nh, 8), HU_ref)
    assert rel(pb.cpu().view(npos, 8), PB_ref.sum((0, 1))) < 2e-2


def test_text_encoder_vs_transformers_fixture(gpu_pkg):
    text = gpu_pkg.text
    z = load_golden("deberta_tiny.npz")
    H, NH, NL, I, V, R, ALPHA, B, S, OUT = z["cfg"].tolist()
    cfg = text.TextCfg(vocab_size=V, hidden=H, layers=NL, heads=NH, intermediate=I, lora_r=R,
                       lora_alpha=ALPHA, lora_dropout=0.0, hidden_dropout=0.0, attn_dropout=0.0)
    enc = text.TextEncoder(embedding_dim=OUT, cfg=cfg).to(DEV)
    enc.projection[2].p = 0.0
    P = {k: torch.tensor(v) for k, v in sub(z, "p/").items()}
    enc.load_state_dict(P)
    enc.train()
    ids, mask = torch.tensor(z["input_ids"]), torch.tensor(z["attention_mask"])
    up = torch.tensor(z["upstream"])
    out = enc(ids.to(DEV), mask.to(DEV))
    (out * up.to(DEV)).sum().backward()
    torch.cuda.synchronize()
    assert rel(out, z["out"]) < 3e-2, rel(out, z["out"])
    # fp32 oracle gradients of the trainable tensors
    Pr = {k: v.clone().requires_grad_(True) for k, v in P.items()}
    dcfg = dref.DebertaCfg(vocab_size=V, hidden=H, layers=NL, heads=NH, intermediate=I, lora_r=R,
                           lora_alpha=ALPHA)
    ref_out = dref.text_encoder_forward(Pr, ids, mask, dcfg)
    (ref_out * up).sum().backward()
    n_checked = 0
    for name, p in enc.named_parameters():
        if not p.requires_grad:
            assert p.grad is None, name
            continue
        gr = Pr[name].grad
        assert _cos(p.grad, gr) > 0.99, (name, _cos(p.grad, gr))
        assert abs(p.grad.norm().item() / gr.norm().item() - 1) < 0.05, name
        n_checked += 1
    assert n_checked == 4 * NL + 4


def test_text_encoder_eval_and_shapes(gpu_pkg):
    """Eval mode (no dropout, no autograd state) equals the train-mode forward with dropout off;
    padded tokens do not influence the pooled output."""
    text = gpu_pkg.text
    cfg = text.TextCfg(vocab_size=300, hidden=128, layers=2, heads=2, intermediate=256,
                       lora_dropout=0.0, hidden_dropout=0.0, attn_dropout=0.0)
    torch.manual_seed(0)
    enc = text.TextEncoder(embedding_dim=16, cfg=cfg).to(DEV)
    enc.projection[2].p = 0.0
    ids = torch.randint(1, 300, (3, 96), device=DEV)
    mask = torch.ones(3, 96, dtype=torch.int64, device=DEV)
    mask[1, 50:] = 0
    enc.eval()
    with torch.no_grad():
        a = enc(ids, mask)
        ids2 = ids.clone()
        ids2[1, 50:] = 7                       # change only padded tokens of row 1
        b = enc(ids2, mask)
    enc.train()
    c = enc(ids, mask)
    assert torch.allclose(a, c, atol=1e-5)
    assert torch.allclose(a[1], b[1], atol=1e-5)


def _cfg4(pkg, B=8, S=96, seed=0, p=0.0):
    from oracle import resnet_ref as rref
    from oracle import two_tower_ref as ref
    text = pkg.text
    tcfg = text.TextCfg(vocab_size=400, hidden=128, layers=2, heads=2, intermediate=256,
                        lora_dropout=p, hidden_dropout=p, attn_dropout=p)
    torch.manual_seed(seed)
    m = pkg.TwoTowerModel(vocab_size=211, tabular_input_dim=32, num_genders=3, num_countries=8,
                          max_seq_len=12, user_embedding_dim=128, item_embedding_dim=128,
                          user_dropout=p, precomputed_modalities=False, with_text=True,
                          text_cfg=tcfg).to(DEV)
    m.item_tower.fusion_layer[3].p = p
    m.item_tower.tabular_encoder.mlp[3].p = p
    m.item_tower.text_encoder.projection[2].p = p
    with torch.no_grad():                         # non-zero LoRA B so every path is live
        for n, prm in m.named_parameters():
            if "lora_B" in n:
                prm.normal_(0.0, 0.02)
    g = torch.Generator().manual_seed(seed + 1)
    batch = ref.synthetic_batch(B, 12, 211, num_countries=8, generator=g)
    del batch["target_modal"]
    batch.update(rref.synthetic_items(B, 32, (64, 96), (64, 64), generator=g))
    ids, mask = dref.synthetic_text(B, S, 400, generator=g)
    batch["target_input_ids"], batch["target_attention_mask"] = ids, mask
    return m, {k: v.to(DEV) for k, v in batch.items()}


def test_cfg4_train_step_graph_equals_eager_and_learns(gpu_pkg):
    """cfg 4 (ResNet-18 x2 + mDeBERTa-LoRA + tabular): TrainStep graph replay equals the
    eager schedule bit for bit for 10 steps (losses and every parameter / buffer: the LoRA
    rank-8 gradient streams and the relative-position sums are int64 fixed point, the conv
    BatchNorm statistics too), the loss falls, and the frozen DeBERTa base never changes."""
    m1, bd = _cfg4(gpu_pkg, seed=3, p=0.1)
    m2, _ = _cfg4(gpu_pkg, seed=3, p=0.1)
    frozen0 = {n: p.detach().clone() for n, p in m1.named_parameters() if not p.requires_grad}
    lora0 = {n: p.detach().clone() for n, p in m1.named_parameters() if "lora_" in n}
    assert frozen0 and all("text_encoder.transformer" in n and "lora_" not in n for n in frozen0)
    s1 = gpu_pkg.TrainStep(m1, lr=1e-3, use_graph=True, seed=5)
    s2 = gpu_pkg.TrainStep(m2, lr=1e-3, use_graph=False, seed=5)
    l1 = [float(s1.step(bd)) for _ in range(10)]
    l2 = [float(s2.step(bd)) for _ in range(10)]
    assert l1 == l2, (l1, l2)
    torch.cuda.synchronize()
    sd1, sd2 = m1.state_dict(), m2.state_dict()
    bad = [k for k in sd1 if not torch.equal(sd1[k], sd2[k])]
    assert not bad, bad[:8]
    assert l1[-1] < l1[0] - 0.2, l1
    for n, p in m1.named_parameters():
        if n in frozen0:
            assert torch.equal(p.detach(), frozen0[n]), n
    names = dict(m1.named_parameters())
    assert len(lora0) == 4 * 2
    for n, v0 in lora0.items():                  # the LoRA matrices train
        assert not torch.equal(names[n].detach(), v0), n


def test_cfg4_module_text_slot_is_text_encoder(gpu_pkg):
    """The module path concatenates the TextEncoder output into the text slot (item_tower.py:147)."""
    m, bd = _cfg4(gpu_pkg, seed=4)
    it = m.item_tower
    it.eval()
    with torch.no_grad():
        t = it.text_encoder(bd["target_input_ids"], bd["target_attention_mask"])
        full = it(images=bd["target_image"], audio=bd["target_audio"],
                  input_ids=bd["target_input_ids"], attention_mask=bd["target_attention_mask"],
                  tabular=bd["target_tabular"])
        zero_text = it.fuse(torch.cat([it.audio_encoder(bd["target_audio"]),
                                       it.visual_encoder(bd["target_image"]),
                                       torch.zeros_like(t), it.tabular_encoder(bd["target_tabular"])], 1))
        with_text = it.fuse(torch.cat([it.audio_encoder(bd["target_audio"]),
                                       it.visual_encoder(bd["target_image"]), t,
                                       it.tabular_encoder(bd["target_tabular"])], 1))
    assert torch.allclose(full, with_text, atol=1e-4)
    assert not torch.allclose(full, zero_text, atol=1e-4)


def _reference_loop(model, dataloader, optimizer, device):
    """The reference's epoch loop body (train.py:41-76) call for call: batch dict moved to the
    device in place, zero_grad(set_to_none), fp16 autocast forward, GradScaler
    scale/backward/step/update, loss.item().  Returns the per-batch losses."""
    model.train()
    scaler = torch.amp.GradScaler("cuda")
    losses = []
    for batch in dataloader:
        for k, v in batch.items():
            if isinstance(v, torch.Tensor):
                batch[k] = v.to(device)
        optimizer.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.float16):
            loss, _, _, _ = model(batch)
        scaler.scale(loss).backward()
        scaler.step(optimizer)
        scaler.update()
        losses.append(loss.item())
        del loss, batch
    return losses


def test_reference_call_site_runs_unchanged(gpu_pkg):
    """Drop-in at the reference call site (train.py:289-302 + train_one_epoch): the DEFAULT
    constructor with the reference's arguments builds the full multimodal item tower (ResNet-18
    audio + visual, mDeBERTa-LoRA text, tabular; tiny text dims here), the batches carry the
    reference keys (plus the ignored target_id / user_id), the last batch is ragged (B = 7,
    no drop_last), and the loop runs under fp16 autocast + GradScaler with torch.optim.AdamW.
    The first batch's loss matches the fp32 oracle of the same model on the same inputs
    (bf16 storage through two ResNet-18s and DeBERTa: 3e-2); every batch gives a finite loss
    and every trainable parameter moves."""
    from oracle import resnet_ref as rref
    from oracle import two_tower_ref as ref
    tcfg = gpu_pkg.text.TextCfg(vocab_size=400, hidden=128, layers=2, heads=2, intermediate=256,
                                lora_dropout=0.0, hidden_dropout=0.0, attn_dropout=0.0)
    dcfg = dref.DebertaCfg(vocab_size=400, hidden=128, layers=2, heads=2, intermediate=256)
    torch.manual_seed(0)
    model = gpu_pkg.TwoTowerModel(vocab_size=211, num_genders=3, num_countries=8,
                                  tabular_input_dim=32, item_embedding_dim=256,
                                  user_embedding_dim=256, use_lora=True, text_cfg=tcfg,
                                  user_dropout=0.0).to(DEV)
    it = model.item_tower
    assert it.with_text and not it.precomputed_modalities
    it.fusion_layer[3].p = 0.0
    it.tabular_encoder.mlp[3].p = 0.0
    it.text_encoder.projection[2].p = 0.0
    loader = []
    for s, B in enumerate((8, 8, 7)):
        g = torch.Generator().manual_seed(40 + s)
        b = ref.synthetic_batch(B, 50, 211, num_countries=8, generator=g)
        del b["target_modal"]
        b.update(rref.synthetic_items(B, 32, (64, 96), (64, 64), generator=g))
        b["target_input_ids"], b["target_attention_mask"] = dref.synthetic_text(B, 64, 400,
                                                                                 generator=g)
        b["target_id"] = torch.arange(B)
        b["user_id"] = b["user_idx"].clone()
        loader.append(b)
    params = {k: v.detach().cpu().clone() for k, v in model.named_parameters()}
    lref = float(ref.two_tower_loss(params, loader[0], running=None, text_cfg=dcfg)[0])
    before = {k: v.detach().clone() for k, v in model.named_parameters() if v.requires_grad}
    opt = torch.optim.AdamW([p for p in model.parameters() if p.requires_grad], lr=1e-4)
    losses = _reference_loop(model, loader, opt, DEV)
    assert len(losses) == 3 and all(math.isfinite(x) for x in losses), losses
    assert abs(losses[0] - lref) < 3e-2, (losses[0], lref)
    moved = [k for k, v in model.named_parameters() if v.requires_grad
             and not torch.equal(v.detach(), before[k])]
    assert len(moved) >= 0.9 * len(before), (len(moved), len(before))


def test_text_encoder_base_dims_vs_oracle(gpu_pkg):
    """cfg 4 at mDeBERTa-v3-base dimensions (hidden 768, 12 heads, 12 layers, FFN 3072, 256
    position buckets, vocab 251,000 — oracle DebertaCfg() defaults), S = 256, B = 2 with one
    full and one 100-token sequence, LoRA B non-zero so every LoRA path is live: output vs the
    fp32 oracle (bf16 storage through 12 layers: 5e-2), and every trainable gradient by
    direction (cosine >= 0.98) and norm (±10 %)."""
    text = gpu_pkg.text
    dcfg = dref.DebertaCfg()
    cfg = text.TextCfg(lora_dropout=0.0, hidden_dropout=0.0, attn_dropout=0.0)
    assert (cfg.hidden, cfg.heads, cfg.layers, cfg.intermediate, cfg.vocab_size,
            cfg.position_buckets) == (dcfg.hidden, dcfg.heads, dcfg.layers, dcfg.intermediate,
                                      dcfg.vocab_size, dcfg.position_buckets)
    g = torch.Generator().manual_seed(21)
    P = dref.init_text_params(dcfg, 128, g, lora_b_std=0.02)
    enc = text.TextEncoder(embedding_dim=128, cfg=cfg).to(DEV)
    enc.projection[2].p = 0.0
    enc.load_state_dict(P)
    enc.train()
    B, S = 2, 256
    ids = torch.randint(1, dcfg.vocab_size, (B, S), generator=g)
    mask = torch.ones(B, S, dtype=torch.int64)
    mask[1, 100:] = 0
    ids = ids * mask
    up = torch.randn(B, 128, generator=g)
    out = enc(ids.to(DEV), mask.to(DEV))
    (out * up.to(DEV)).sum().backward()
    torch.cuda.synchronize()
    train = {n for n, p in enc.named_parameters() if p.requires_grad}
    Pr = {k: (v.clone().requires_grad_(True) if k in train else v) for k, v in P.items()}
    ref_out = dref.text_encoder_forward(Pr, ids, mask, dcfg)
    (ref_out * up).sum().backward()
    assert rel(out, ref_out) < 5e-2, rel(out, ref_out)
    rows = []
    for name, p in enc.named_parameters():
        if name in train:
            gr = Pr[name].grad
            rows.append((name, _cos(p.grad, gr), p.grad.norm().item() / gr.norm().item()))
    for r in rows:
        print("GRAD", *r)
    assert len(rows) == 4 * dcfg.layers + 4
    # measured (MI355X): cosines 0.991-1.000; LoRA-A norms spread ±6 % with one at -8 %
    # (deterministic for this seed: bf16 rounding through 12 layers; the rank-8 contraction
    # dL = dQ·B_q with B ~ N(0, 0.02) sums cancelling terms over every token)
    bad = [r for r in rows if not (r[1] > 0.98 and abs(r[2] - 1) < 0.10)]
    assert not bad, bad

"""Model-level parity on the GPU: the libttmi towers, loss and fused train step against
(a) the golden fixtures produced by the REFERENCE modules and (b) the fp32 CPU oracle.

Tolerances (stated per test):
  * fp32 compute path: 1e-4 relative to the tensor's max-abs for outputs and gradients
    (two transformer layers of fp32-MFMA vs CPU summation order).
  * bf16 compute path (the product default): outputs within 2x (+0.03) of the deviation
    that rounding every GEMM's operands (forward and backward) and the bf16-stored QKV /
    FFN-hidden activations produces in the CPU oracle (``bf16_emulated``); gradients by
    direction and norm (``check_bf16_grad``: boundary flips at fixture batch sizes): ReLU gates that
    flip under rounding make some gradients legitimately 40%+ off in max-abs terms, and this
    bound separates that from kernel bugs.  Plus the north-star bar
    |loss_bf16 - loss_fp32_oracle| <= 1e-3 at the full cfg-2 size (B=512, L=50, D=128,
    V=10136).
"""
import contextlib

import numpy as np
import pytest
import torch

from bf16emu import bf16_linears, check_bf16_grad, cosine, frob, rel
from conftest import load_golden, sub
from oracle import two_tower_ref as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def bf16_emulated(z):
    """(out, grads) of the reference user-tower fixture under bf16 GEMM operands."""
    V, D, L, B, H, n_g, n_c, use_mask = z["cfg"].tolist()
    with bf16_linears():
        params = {k: torch.tensor(v, requires_grad=True) for k, v in sub(z, "p/").items()}
        out = ref.user_tower_forward(
            params, torch.tensor(z["history_ids"]), torch.tensor(z["user_gender"]),
            torch.tensor(z["user_country"]),
            torch.tensor(z["history_mask"]) if use_mask else None, num_heads=H)
        (out * torch.tensor(z["upstream"])).sum().backward()
    return out.detach(), {k: p.grad for k, p in params.items()}


def build_user(pkg, z, dtype):
    V, D, L, B, H, n_g, n_c, use_mask = z["cfg"].tolist()
    m = pkg.SequentialUserEncoder(V, n_g, n_c, D, L, H, 2, 0.0, compute_dtype=dtype).to(DEV)
    m.load_state_dict({k: torch.tensor(v) for k, v in sub(z, "p/").items()})
    return m, use_mask


def frob(a, b):
    a = torch.as_tensor(a).detach().double().cpu().reshape(-1)
    b = torch.as_tensor(b).detach().double().cpu().reshape(-1)
    return ((a - b).norm() / max(b.norm().item(), 1e-30)).item()


def cosine(a, b):
    a = torch.as_tensor(a).detach().double().cpu().reshape(-1)
    b = torch.as_tensor(b).detach().double().cpu().reshape(-1)
    return (a @ b / max((a.norm() * b.norm()).item(), 1e-30)).item()


def check_bf16_grad(k, g, gref, g_emul):
    """bf16 end-to-end gradient check at fixture scale (B = 6-8 users).  A single ReLU gate
    that flips under bf16 rounding re-routes one user's whole gradient path: measured up to
    16% relative Frobenius error on the nomask fixture's embedding gradient (tools/
    diag_prune.py traced it to one pre-ReLU element of the user-fusion MLP; the fp32 path
    matches the reference to 1e-4 on the same inputs).  So the criterion is direction
    (cosine >= 0.97 — a wrong-row / wrong-mask bug fails it) plus a norm cap of 3x the
    emulated bf16 error + 0.25."""
    bound = 3.0 * frob(g_emul, gref) + 0.25
    assert frob(g, gref) <= bound, (k, frob(g, gref), bound)
    if torch.as_tensor(gref).abs().max() > 0:
        assert cosine(g, gref) >= 0.97, (k, cosine(g, gref))


@pytest.mark.parametrize("name", ["user_tower_small.npz", "user_tower_nomask.npz",
                                  "user_tower_leftpad.npz", "user_tower_d128.npz"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_user_tower_vs_reference(gpu_pkg, name, dtype):
    z = load_golden(name)
    m, use_mask = build_user(gpu_pkg, z, dtype)
    ids = torch.tensor(z["history_ids"], device=DEV)
    mask = torch.tensor(z["history_mask"], device=DEV) if use_mask else None
    out = m(ids, torch.tensor(z["user_gender"], device=DEV),
            torch.tensor(z["user_country"], device=DEV), mask)
    if dtype == torch.bfloat16:
        e_out, e_grads = bf16_emulated(z)
        assert rel(out, z["out"]) < 2.0 * rel(e_out, z["out"]) + 0.03
    else:
        assert rel(out, z["out"]) < 1e-4
    (out * torch.tensor(z["upstream"], device=DEV)).sum().backward()
    grads = dict(m.named_parameters())
    for k, gref in sub(z, "g/").items():
        g = grads[k].grad
        if k.endswith("in_proj_bias"):
            # q|k|v slices: the K slice has an identically-zero true gradient (softmax is
            # shift-invariant over keys) — hold it to an absolute bound on the Q/V scale
            q, kk, v = torch.tensor(gref).chunk(3)
            gq, gk, gv = g.cpu().chunk(3)
            scale = max(q.abs().max().item(), v.abs().max().item())
            if dtype == torch.float32:
                assert rel(gq, q) < 1e-4 and rel(gv, v) < 1e-4, k
                assert gk.abs().max().item() <= 1e-4 * scale + 1e-6, k
            else:
                eq, _, ev = e_grads[k].chunk(3)
                check_bf16_grad(k + "[q]", gq, q, eq)
                check_bf16_grad(k + "[v]", gv, v, ev)
                assert gk.abs().max().item() <= 0.05 * scale + 1e-6, k
        elif dtype == torch.float32:
            assert rel(g, gref) < 1e-4, (k, rel(g, gref))
        else:
            check_bf16_grad(k, g, gref, e_grads[k])


@pytest.mark.parametrize("name", ["infonce_b8.npz", "infonce_b64.npz"])
@pytest.mark.parametrize("tag", ["nomask", "mask"])
def test_infonce_vs_reference(gpu_pkg, name, tag):
    z = load_golden(name)
    u = torch.tensor(z["u"], device=DEV, requires_grad=True)
    i = torch.tensor(z["i"], device=DEV, requires_grad=True)
    uid = torch.tensor(z["user_idx"], device=DEV) if tag == "mask" else None
    loss, logits, uh, ih = gpu_pkg.infonce(u, i, uid)
    loss.backward()
    assert abs(loss.item() - float(z[f"{tag}/loss"])) < 2e-6 * max(1.0, abs(float(z[f"{tag}/loss"])))
    assert rel(logits, z[f"{tag}/logits"]) < 2e-6
    assert rel(uh, z[f"{tag}/u_hat"]) < 2e-6
    assert rel(ih, z[f"{tag}/i_hat"]) < 2e-6
    assert rel(u.grad, z[f"{tag}/du"]) < 1e-5
    assert rel(i.grad, z[f"{tag}/di"]) < 1e-5


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_item_fusion_vs_reference(gpu_pkg, dtype):
    z = load_golden("item_fusion.npz")
    D = z["out"].shape[1]
    m = gpu_pkg.MultimodalItemEncoder(precomputed_modalities=True, tabular_input_dim=128, embedding_dim=D,
                                      compute_dtype=dtype).to(DEV)
    m.fusion_layer[3].p = 0.0
    m.load_state_dict({k: torch.tensor(v) for k, v in sub(z, "p/").items()})
    m.train()
    p0 = sub(z, "p/")
    e_grads = None
    if dtype == torch.bfloat16:
        with bf16_linears():
            params = {k: torch.tensor(v, requires_grad=True) for k, v in p0.items()
                      if "running" not in k and "num_batches" not in k}
            eo = ref.item_fusion_forward(params, torch.tensor(z["modal"]))
            (eo * torch.tensor(z["upstream"])).sum().backward()
        e_grads = {k: p.grad for k, p in params.items()}
    out = m.fuse(torch.tensor(z["modal"], device=DEV))
    if dtype == torch.float32:
        assert rel(out, z["out"]) < 1e-4
    else:
        assert rel(out, z["out"]) < 2.0 * rel(eo.detach(), z["out"]) + 0.03
    (out * torch.tensor(z["upstream"], device=DEV)).sum().backward()
    grads = dict(m.named_parameters())
    for k, gref in sub(z, "g/").items():
        if k.startswith("fusion_layer.0.bias"):      # exactly zero in math (BN follows)
            # fp32: ~0; bf16: the row sum of a bf16-rounded dy (sums to 0 in exact math)
            tol = 1e-3 if dtype == torch.float32 else 3e-2
            assert grads[k].grad.abs().max().item() < tol * max(1.0, np.abs(gref).max())
            continue
        if dtype == torch.float32:
            assert rel(grads[k].grad, gref) < 1e-4, (k, rel(grads[k].grad, gref))
        else:
            check_bf16_grad(k, grads[k].grad, gref, e_grads[k])
    after = sub(z, "after/")
    bufs = dict(m.named_buffers())
    for k in ("fusion_layer.1.running_mean", "fusion_layer.1.running_var"):
        assert rel(bufs[k], after[k]) < (1e-4 if dtype == torch.float32 else 1e-2)
    assert int(bufs["fusion_layer.1.num_batches_tracked"]) == 1


def _train_step_model(pkg, z, dtype):
    V, D, L, B, n_g, n_c, n_steps = z["cfg"].tolist()
    m = pkg.TwoTowerModel(precomputed_modalities=True, vocab_size=V, tabular_input_dim=128, num_genders=n_g,
                          num_countries=n_c, max_seq_len=L, user_embedding_dim=D,
                          item_embedding_dim=D, user_dropout=0.0, use_lora=False,
                          compute_dtype=dtype).to(DEV)
    m.item_tower.fusion_layer[3].p = 0.0
    m.load_state_dict({k: torch.tensor(v) for k, v in sub(z, "p0/").items()})
    batches = [{k: torch.tensor(v, device=DEV) for k, v in sub(z, f"batch{s}/").items()}
               for s in range(n_steps)]
    return m, batches, n_steps


DEGENERATE = ("in_proj_bias", "item_tower.fusion_layer.0.")


def _check_params(m, z, n_steps, tol):
    p1 = sub(z, "p1/")
    for k, v in m.state_dict().items():
        if k.endswith("num_batches_tracked"):
            assert int(v) == int(p1[k])
            continue
        err_abs = (v.double().cpu() - torch.tensor(p1[k]).double()).abs().max().item()
        if any(d in k for d in DEGENERATE):
            assert err_abs <= 2e-4 * n_steps + 1e-6, k      # AdamW sign-amplified noise
        elif "running" in k:
            assert err_abs <= 1e-4 + tol * np.abs(p1[k]).max(), k
        else:
            assert err_abs <= tol * max(np.abs(p1[k]).max(), 1e-3), (k, err_abs)


@pytest.mark.parametrize("use_graph", [False, True])
def test_fused_train_step_vs_reference(gpu_pkg, use_graph):
    """TrainStep (flat params, fused AdamW, HIP graph) reproduces the reference's
    train_one_epoch on two batches (fp32 compute path)."""
    z = load_golden("train_step.npz")
    m, batches, n_steps = _train_step_model(gpu_pkg, z, torch.float32)
    step = gpu_pkg.TrainStep(m, lr=1e-4, use_graph=use_graph)
    losses = [float(step.step(b)) for b in batches]
    assert np.abs(np.array(losses) - z["losses"]).max() < 1e-5
    _check_params(m, z, n_steps, 1e-4)


def test_module_path_with_torch_adamw_vs_reference(gpu_pkg):
    """The drop-in path: reference-shaped train_one_epoch + torch.optim.AdamW."""
    z = load_golden("train_step.npz")
    m, batches, n_steps = _train_step_model(gpu_pkg, z, torch.float32)
    opt = torch.optim.AdamW(m.parameters(), lr=1e-4)
    mean = gpu_pkg.train_one_epoch(m, batches, opt, DEV, 1, is_main_process=False)
    assert abs(mean - float(z["mean_loss"])) < 1e-5
    _check_params(m, z, n_steps, 1e-4)


def _cfg2(pkg, dtype, B=512, L=50, D=128, V=10136, p=0.0, seed=0):
    torch.manual_seed(seed)
    m = pkg.TwoTowerModel(precomputed_modalities=True, vocab_size=V, tabular_input_dim=128, num_genders=3,
                          num_countries=64, max_seq_len=L, user_embedding_dim=D,
                          item_embedding_dim=D, user_dropout=p, compute_dtype=dtype).to(DEV)
    m.item_tower.fusion_layer[3].p = p
    g = torch.Generator().manual_seed(seed + 1)
    batch = ref.synthetic_batch(B, L, V, generator=g)
    return m, batch


def _oracle_loss(m, batch, drop=None, p=0.0):
    params = {k: v.detach().cpu() for k, v in m.named_parameters()}
    running = {"running_mean": torch.zeros(512), "running_var": torch.ones(512),
               "num_batches_tracked": torch.zeros((), dtype=torch.long)}
    loss, logits, _, _ = ref.two_tower_loss(params, batch, p_drop=p, drop=drop, running=running)
    return float(loss), logits


@pytest.mark.parametrize("dtype,tol", [(torch.bfloat16, 1e-3), (torch.float32, 1e-5)])
def test_cfg2_loss_parity_full_size(gpu_pkg, dtype, tol):
    """North-star bar: loss within 1e-3 of the fp32 oracle at BASELINE cfg 2 size."""
    m, batch = _cfg2(gpu_pkg, dtype)
    lref, logits_ref = _oracle_loss(m, batch)
    bd = {k: v.to(DEV) for k, v in batch.items()}
    with torch.no_grad():
        loss, logits, _, _ = m(bd)
    assert abs(float(loss) - lref) <= tol, (float(loss), lref)
    assert rel(logits, logits_ref) < (3e-2 if dtype == torch.bfloat16 else 1e-4)


def test_long_history_matches_oracle(gpu_pkg):
    """max_seq_len past 512 (ABI 21 raised TTMI_ATTN_LMAX to 2048; the reference takes any
    length, user_tower.py:5-13): L = 1100 with dropout on through the tiled long-sequence and
    one-query kernels, loss against the oracle's restatement."""
    F = gpu_pkg.functional
    m, batch = _cfg2(gpu_pkg, torch.float32, B=8, L=1100, V=997, p=0.1, seed=5)
    seeds = F.site_seeds(0x10A6, 1)
    lref, _ = _oracle_loss(m, batch, drop=ref.HashDropout(seeds), p=0.1)
    loss, _, _, _ = m({k: v.to(DEV) for k, v in batch.items()}, seeds=F.seed_table(seeds, DEV))
    assert abs(float(loss) - lref) < 1e-4


@pytest.mark.parametrize("D,H,L", [(128, 1, 20), (128, 32, 20), (256, 2, 30)])
def test_generic_head_widths_match_oracle(gpu_pkg, D, H, L):
    """Head widths the tuned attention kernels refuse — d_h = 128 (D = 128 with 1 head, D = 256
    with 2) and d_h = 4, not a multiple of 8 (D = 128 with 32 heads) — which the reference
    accepts (user_tower.py:5-13): the model runs the generic attention on an unpruned last
    layer.  Loss and gradients against the oracle with dropout on."""
    F = gpu_pkg.functional
    torch.manual_seed(11)
    m = gpu_pkg.TwoTowerModel(precomputed_modalities=True, vocab_size=997, tabular_input_dim=128,
                              num_genders=3, num_countries=64, max_seq_len=L, user_embedding_dim=D,
                              item_embedding_dim=D, user_num_heads=H, user_dropout=0.1,
                              compute_dtype=torch.float32).to(DEV)
    m.item_tower.fusion_layer[3].p = 0.1
    assert not m.user_tower.prune_last
    g = torch.Generator().manual_seed(12)
    batch = ref.synthetic_batch(16, L, 997, generator=g)
    seeds = F.site_seeds(0x6E4, 1)
    params = {k: v.detach().cpu() for k, v in m.named_parameters()}
    running = {"running_mean": torch.zeros(512), "running_var": torch.ones(512),
               "num_batches_tracked": torch.zeros((), dtype=torch.long)}
    lref, _, _, _ = ref.two_tower_loss(params, batch, num_heads=H, p_drop=0.1, drop=ref.HashDropout(seeds),
                                       running=running)
    loss, _, _, _ = m({k: v.to(DEV) for k, v in batch.items()}, seeds=F.seed_table(seeds, DEV))
    assert abs(float(loss) - float(lref)) < 1e-4
    loss.backward()
    pr = {k: v.detach().cpu().requires_grad_(True) for k, v in m.named_parameters()}
    lo, _, _, _ = ref.two_tower_loss(pr, batch, num_heads=H, p_drop=0.1, drop=ref.HashDropout(seeds),
                                     running=running)
    lo.backward()
    mine = dict(m.named_parameters())
    for k in ("user_tower.transformer_encoder.layers.0.self_attn.in_proj_weight",
              "user_tower.transformer_encoder.layers.1.self_attn.in_proj_weight",
              "user_tower.item_embedding.weight"):
        a, b = mine[k].grad.detach().double().cpu(), pr[k].grad.double()
        assert float((a - b).abs().max()) <= 1e-3 * float(b.abs().max()), k


@pytest.mark.parametrize("L", [20, 150])
def test_dropout_on_matches_oracle_hash(gpu_pkg, L):
    """Dropout ON (p=0.1 at every site) — kernels' masks vs the oracle's restatement.  L = 150
    runs the long-sequence attention (ttmi_attn_long.hip: tiled full attention in layer 0, the
    one-query kernel in the pruned layer 1)."""
    F = gpu_pkg.functional
    m, batch = _cfg2(gpu_pkg, torch.float32, B=64, L=L, V=997, p=0.1, seed=3)
    seeds = F.site_seeds(0x5EED, 1)
    table = F.seed_table(seeds, DEV)
    lref, _ = _oracle_loss(m, batch, drop=ref.HashDropout(seeds), p=0.1)
    bd = {k: v.to(DEV) for k, v in batch.items()}
    loss, _, _, _ = m(bd, seeds=table)
    assert abs(float(loss) - lref) < 1e-5
    # gradients too: compare the user-tower embedding grad with the oracle's
    loss.backward()
    params = {k: v.detach().cpu().requires_grad_(True) for k, v in m.named_parameters()}
    running = {"running_mean": torch.zeros(512), "running_var": torch.ones(512),
               "num_batches_tracked": torch.zeros((), dtype=torch.long)}
    lo, _, _, _ = ref.two_tower_loss(params, batch, p_drop=0.1, drop=ref.HashDropout(seeds),
                                     running=running)
    lo.backward()
    mine = dict(m.named_parameters())
    # A single ReLU whose input sits within ~1e-7 of zero flips with the summation order: the
    # fp32 oracle itself, with its item embedding perturbed by 2e-7 relative, moves to 7.4e-4
    # (item embedding rows) and 3.3e-3 (linear1 rows) of its unperturbed gradients at L = 20
    # (one token's row, one hidden unit's row).  So all rows but at most 2 are held to 1e-4 and
    # those 2 to 1e-2 (a mask or indexing error moves many rows, or one by O(1)).
    for k in ("user_tower.item_embedding.weight",
              "user_tower.transformer_encoder.layers.0.linear1.weight",
              "user_tower.transformer_encoder.layers.1.self_attn.in_proj_weight",
              "item_tower.fusion_layer.4.weight"):
        a, b = mine[k].grad.detach().double().cpu(), params[k].grad.double()
        rows = (a - b).abs().reshape(a.shape[0], -1).amax(1) / b.abs().max()
        top = rows.sort(descending=True).values
        assert top[2:].max().item() < 1e-4 and top[0].item() < 1e-2, (k, top[:4].tolist())


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_pruned_last_layer_equals_full(gpu_pkg, p):
    """Pruning the last encoder layer to the gathered rows (default) gives the same output
    and parameter gradients as running it on every token (fp32, dropout on/off)."""
    F = gpu_pkg.functional
    outs, grads = [], []
    for prune in (True, False):
        m, batch = _cfg2(gpu_pkg, torch.float32, B=96, L=50, V=997, p=p, seed=5)
        m.user_tower.prune_last = prune
        seeds = F.seed_table(F.site_seeds(0xABC, 3), DEV)
        bd = {k: v.to(DEV) for k, v in batch.items()}
        loss, logits, _, _ = m(bd, seeds=seeds)
        loss.backward()
        outs.append(logits.detach().cpu())
        grads.append({k: v.grad.detach().cpu() for k, v in m.named_parameters()})
    assert rel(outs[0], outs[1]) < 1e-5
    for k in grads[0]:
        if k.endswith("in_proj_bias") or k == "item_tower.fusion_layer.0.bias":
            continue        # identically-zero true gradients (noise vs noise)
        assert rel(grads[0][k], grads[1][k]) < 1e-4, k


def _state_bits(m, step):
    """Every parameter, buffer and AdamW moment of a TrainStep, for bit comparisons."""
    out = {k: v.detach().clone() for k, v in m.state_dict().items()}
    out["__exp_avg"] = step.flat.exp_avg.detach().clone()
    out["__exp_avg_sq"] = step.flat.exp_avg_sq.detach().clone()
    return out


def assert_bit_equal(a, b):
    assert a.keys() == b.keys()
    bad = [k for k in a if not torch.equal(a[k], b[k])]
    assert not bad, bad[:8]


@pytest.mark.parametrize("D,p", [(128, 0.0), (128, 0.1), (256, 0.1)])
def test_cfg2_graph_equals_eager_bitexact(gpu_pkg, D, p):
    """The benchmarked step (cfg 2: B 512, L 50, D 128, V 10,136, bf16) is deterministic: the
    HIP-graph replay and the eager schedule give bit-identical losses, parameters, BatchNorm
    buffers and AdamW moments for 3 steps (every cross-workgroup sum is fixed-order or int64
    fixed point: the embedding scatter, the LN / BN column sums, the split weight gradients).
    D = 256 (the reference's default width) runs the FFN-split user head at its own width."""
    m1, batch = _cfg2(gpu_pkg, torch.bfloat16, D=D, p=p, seed=7)
    m2, _ = _cfg2(gpu_pkg, torch.bfloat16, D=D, p=p, seed=7)
    bd = {k: v.to(DEV) for k, v in batch.items()}
    s1 = gpu_pkg.TrainStep(m1, lr=1e-3, use_graph=True, seed=11)
    s2 = gpu_pkg.TrainStep(m2, lr=1e-3, use_graph=False, seed=11)
    for i in range(3):
        l1, l2 = float(s1.step(bd)), float(s2.step(bd))
        assert l1 == l2, (i, l1, l2)
    torch.cuda.synchronize()
    assert_bit_equal(_state_bits(m1, s1), _state_bits(m2, s2))


@pytest.mark.parametrize("D,H", [(128, 1), (128, 32)])
def test_generic_head_widths_trainstep_graph_equals_eager(gpu_pkg, D, H):
    """TrainStep on head widths the tuned kernels refuse (generic attention, unpruned last layer,
    bf16): graph and eager bit-identical over 3 steps, and the loss falls."""
    def build():
        torch.manual_seed(13)
        m = gpu_pkg.TwoTowerModel(precomputed_modalities=True, vocab_size=997, tabular_input_dim=128,
                                  num_genders=3, num_countries=64, max_seq_len=20, user_embedding_dim=D,
                                  item_embedding_dim=D, user_num_heads=H, user_dropout=0.1,
                                  compute_dtype=torch.bfloat16).to(DEV)
        m.item_tower.fusion_layer[3].p = 0.1
        return m
    g = torch.Generator().manual_seed(14)
    bd = {k: v.to(DEV) for k, v in ref.synthetic_batch(64, 20, 997, generator=g).items()}
    m1, m2 = build(), build()
    s1 = gpu_pkg.TrainStep(m1, lr=3e-3, use_graph=True, seed=5)
    s2 = gpu_pkg.TrainStep(m2, lr=3e-3, use_graph=False, seed=5)
    losses = []
    for i in range(3):
        l1, l2 = float(s1.step(bd)), float(s2.step(bd))
        assert l1 == l2, (i, l1, l2)
        losses.append(l1)
    torch.cuda.synchronize()
    assert_bit_equal(_state_bits(m1, s1), _state_bits(m2, s2))
    assert losses[-1] < losses[0]


def test_train_step_graph_learns(gpu_pkg):
    """bf16, dropout on: 30 graph replays on one batch drive the loss down."""
    m1, batch = _cfg2(gpu_pkg, torch.bfloat16, B=256, p=0.1, seed=7)
    bd = {k: v.to(DEV) for k, v in batch.items()}
    s1 = gpu_pkg.TrainStep(m1, lr=1e-3, use_graph=True, seed=11)
    l1 = [float(s1.step(bd)) for _ in range(30)]
    assert l1[-1] < l1[0] - 0.3, l1


def _grad_from_moments(step, prev_m):
    """The step's fp32 gradient, recovered from AdamW's first moment (m_t = β1 m_{t-1} +
    (1 - β1) g_t; the fused AdamW clears the gradient buffer itself)."""
    m = step.flat.exp_avg.detach().double()
    g = (m - 0.9 * prev_m) / 0.1
    return g, m


@pytest.mark.parametrize("D,p", [(128, 0.0), (128, 0.1), (256, 0.1)])
def test_cfg2_bf16_trainstep_vs_oracle_full_size(gpu_pkg, D, p):
    """The exact benchmarked step — bf16 TrainStep (fused user / item heads, co-launched
    item head, fused InfoNCE with the in-launch combine and loss accumulator, grouped
    weight gradients, fused AdamW) at BASELINE cfg 2 (B 512, L 50, D 128, V 10,136) — against
    the fp32 oracle's train_step (reference src/train.py:41-76 loop body, two_tower.py:68-142,
    AdamW at the reference's lr 1e-4, train.py:302) for 2 steps, dropout off and on (the
    oracle restates the kernels' hash dropout):
      * loss per step within 1e-3 of the fp32 oracle (the north-star bar);
      * step-1 gradients (recovered from AdamW's first moment) by direction and norm against
        the bf16-emulated oracle (check_bf16_grad);
      * the 2-step parameter update by direction: cosine(Δ_gpu, Δ_fp32) at least the bf16
        emulation's cosine − 0.05, norm ratio within 2x the emulation's deviation + 0.05.
    Exactly-zero true gradients (in_proj bias's key third, the bias ahead of BatchNorm) are
    AdamW-amplified noise in every implementation and are skipped.  D = 256 is the reference's
    own default width (src/train.py:289-297, two_tower.py:18,23)."""
    F = gpu_pkg.functional
    base = 11
    m, batch = _cfg2(gpu_pkg, torch.bfloat16, D=D, p=p, seed=21)
    b2 = ref.synthetic_batch(512, 50, 10136, generator=torch.Generator().manual_seed(99))
    batches = [batch, b2]
    p0 = {k: v.detach().cpu().clone() for k, v in m.named_parameters()}
    step = gpu_pkg.TrainStep(m, lr=1e-4, use_graph=True, seed=base)
    losses, grads1 = [], None
    prev_m = torch.zeros_like(step.flat.exp_avg, dtype=torch.float64)
    for i, b in enumerate(batches):
        losses.append(float(step.step({k: v.to(DEV) for k, v in b.items()})))
        g, prev_m = _grad_from_moments(step, prev_m)
        if i == 0:
            grads1 = {k: v.detach().double().cpu().clone() for k, v in step.flat.views(g).items()}
    got = {k: v.detach().cpu().double() for k, v in m.named_parameters()}

    def oracle(emulate):
        params = {k: v.clone() for k, v in p0.items()}
        opt, running, ls, g1 = {}, ref.init_running(), [], None
        for i, b in enumerate(batches):
            drop = ref.HashDropout(F.site_seeds(base, i + 1)) if p > 0 else None
            leaves = {k: v.detach().clone().requires_grad_(True) for k, v in params.items()}
            ctx = bf16_linears() if emulate else contextlib.nullcontext()
            with ctx:
                loss, _, _, _ = ref.two_tower_loss(leaves, b, p_drop=p, drop=drop, running=running)
                loss.backward()
            ls.append(float(loss))
            gr = {k: v.grad for k, v in leaves.items()}
            if i == 0:
                g1 = {k: v.detach().double().clone() for k, v in gr.items()}
            with torch.no_grad():
                ref.adamw_(params, gr, opt, lr=1e-4)
        return ls, g1, {k: v.double() for k, v in params.items()}

    l_ref, g_ref, p_ref = oracle(False)
    l_emu, g_emu, p_emu = oracle(True)
    for i in range(2):
        assert abs(losses[i] - l_ref[i]) <= 1e-3, (i, losses[i], l_ref[i], l_emu[i])
    skip = ("in_proj_bias", "item_tower.fusion_layer.0.bias")
    for k in g_ref:
        if any(s in k for s in skip):
            continue
        check_bf16_grad(k, grads1[k], g_ref[k], g_emu[k])
        d_gpu, d_ref, d_emu = got[k] - p0[k].double(), p_ref[k] - p0[k].double(), p_emu[k] - p0[k].double()
        c_gpu, c_emu = cosine(d_gpu, d_ref), cosine(d_emu, d_ref)
        # AdamW's first steps are near sign(g): a tiny parameter's update direction moves with
        # rounding alone (gender embedding, 48 values: the emulation's own cosine spreads
        # 0.923-0.950 under 2e-7 perturbations, tools/diag_update_spread.py)
        margin = 0.05 if d_ref.numel() >= 1024 else 0.10
        assert c_gpu >= c_emu - margin, (k, c_gpu, c_emu)
        n_gpu, n_emu = d_gpu.norm() / d_ref.norm(), d_emu.norm() / d_ref.norm()
        assert abs(n_gpu - 1) <= 2 * abs(n_emu - 1) + 0.05, (k, float(n_gpu), float(n_emu))


@pytest.mark.parametrize("collide", [False, True])
def test_global_negatives_kernels_simulated_world(gpu_pkg, collide):
    """cfg-5 pieces (l2norm, rectangular row CE fwd/bwd, owner-summed key grads) for two
    simulated ranks in one process vs the reference InfoNCE on the concatenated batch
    (fp32 path: 1e-5 relative)."""
    ops = gpu_pkg.ops
    W, B, D, tau = 2, 64, 128, 0.07
    g = torch.Generator().manual_seed(3)
    u_all = torch.randn(W * B, D, generator=g)
    i_all = torch.randn(W * B, D, generator=g)
    uid = torch.randint(0, 40 if collide else 10**6, (W * B,), generator=g)
    ua, ia = u_all.clone().requires_grad_(True), i_all.clone().requires_grad_(True)
    lref, _, _, _ = ref.infonce(ua, ia, uid, tau)
    lref.backward()
    f32 = dict(device=DEV, dtype=torch.float32)
    uh = [torch.empty(B, D, **f32) for _ in range(W)]
    ih = [torch.empty(B, D, **f32) for _ in range(W)]
    nu = [torch.empty(B, **f32) for _ in range(W)]
    ni = [torch.empty(B, **f32) for _ in range(W)]
    for r in range(W):
        ops.l2norm_fwd(u_all[r * B:(r + 1) * B].to(DEV), uh[r], nu[r])
        ops.l2norm_fwd(i_all[r * B:(r + 1) * B].to(DEV), ih[r], ni[r])
    U, I, UID = torch.cat(uh), torch.cat(ih), uid.to(DEV)
    losses, saved = [], []
    for r in range(W):
        s1, s2 = torch.empty(B, W * B, **f32), torch.empty(B, W * B, **f32)
        l1, l2, ce = torch.empty(B, **f32), torch.empty(B, **f32), torch.empty(2 * B, **f32)
        uq = UID[r * B:(r + 1) * B]
        ops.rowce_fwd(uh[r], I, uq, UID, r * B, 1 / tau, s1, l1, ce[:B])
        ops.rowce_fwd(ih[r], U, uq, UID, r * B, 1 / tau, s2, l2, ce[B:])
        loss = torch.empty(1, **f32)
        ops.sum_scaled(ce, 0.5 / B, loss)
        losses.append(float(loss))
        saved.append((s1, l1, s2, l2, uq))
    assert abs(sum(losses) / W - float(lref)) < 1e-5 * max(1.0, abs(float(lref)))
    dloss = torch.full((1,), 1.0 / W, **f32)
    duh = [torch.empty(B, D, **f32) for _ in range(W)]
    dih = [torch.empty(B, D, **f32) for _ in range(W)]
    dU, dI = torch.zeros(W * B, D, **f32), torch.zeros(W * B, D, **f32)
    for r in range(W):
        s1, l1, s2, l2, uq = saved[r]
        dIr, dUr = torch.empty(W * B, D, **f32), torch.empty(W * B, D, **f32)
        ops.rowce_bwd(uh[r], I, s1, l1, uq, UID, r * B, 1 / tau, dloss, 0.5 / B, duh[r], dIr)
        ops.rowce_bwd(ih[r], U, s2, l2, uq, UID, r * B, 1 / tau, dloss, 0.5 / B, dih[r], dUr)
        dU += dUr          # the reduce-scatter's sum (test harness)
        dI += dIr
    for r in range(W):
        sl = slice(r * B, (r + 1) * B)
        du, di = torch.empty(B, D, **f32), torch.empty(B, D, **f32)
        ops.l2norm_bwd(uh[r], nu[r], duh[r], du, dy2=dU[sl].contiguous())
        ops.l2norm_bwd(ih[r], ni[r], dih[r], di, dy2=dI[sl].contiguous())
        assert rel(du, ua.grad[sl]) < 1e-5
        assert rel(di, ia.grad[sl]) < 1e-5


def test_global_infonce_world1_equals_local(gpu_pkg):
    """functional.infonce_global_fwd/bwd without a process group is the local InfoNCE."""
    F = gpu_pkg.functional
    B, D = 96, 128
    g = torch.Generator().manual_seed(9)
    u, it = torch.randn(B, D, generator=g), torch.randn(B, D, generator=g)
    uid = torch.randint(0, 30, (B,), generator=g)
    ua, ia = u.clone().requires_grad_(True), it.clone().requires_grad_(True)
    lref, sref, _, _ = ref.infonce(ua, ia, uid)
    lref.backward()
    loss, logits, _, _, st = F.infonce_global_fwd(u.to(DEV), it.to(DEV), uid.to(DEV), 0.07)
    assert abs(float(loss) - float(lref)) < 1e-5 * max(1.0, abs(float(lref)))
    assert rel(logits, sref) < 1e-5
    du, di = torch.empty(B, D, device=DEV), torch.empty(B, D, device=DEV)
    F.infonce_global_bwd(st, None, du, di)
    assert rel(du, ua.grad) < 1e-5
    assert rel(di, ia.grad) < 1e-5


@pytest.mark.parametrize("D", [64, 128, 256])
@pytest.mark.parametrize("B", [1, 2, 3, 5, 7, 13, 61])
def test_infonce_ragged_batch(gpu_pkg, B, D):
    """Any B >= 1 (the reference DataLoader keeps its ragged last batch, train.py:259-266):
    the fused kernels' row pitch is then not 16-byte aligned (element loads/stores); fp32
    path vs the reference InfoNCE restatement, with and without collisions."""
    g = torch.Generator().manual_seed(B * 1000 + D)
    u, it = torch.randn(B, D, generator=g), torch.randn(B, D, generator=g)
    for uid in (None, torch.randint(0, max(1, B // 2), (B,), generator=g)):
        ua, ia = u.clone().requires_grad_(True), it.clone().requires_grad_(True)
        lref, sref, _, _ = ref.infonce(ua, ia, uid)
        lref.backward()
        ug, ig = u.to(DEV).requires_grad_(True), it.to(DEV).requires_grad_(True)
        loss, logits, _, _ = gpu_pkg.infonce(ug, ig, None if uid is None else uid.to(DEV))
        loss.backward()
        assert abs(float(loss) - float(lref)) <= 1e-5 * max(1.0, abs(float(lref)))
        assert rel(logits, sref) < 1e-5
        if B > 1:
            assert rel(ug.grad, ua.grad) < 1e-5
            assert rel(ig.grad, ia.grad) < 1e-5
        else:
            assert float(ug.grad.abs().max()) < 1e-6


@pytest.mark.parametrize("D,B", [(128, 64), (128, 7), (96, 64)])
def test_infonce_du16_copy(gpu_pkg, D, B):
    """ttmi_infonce_bwd16: du16 is du rounded to bf16, bit for bit, from the fused finish
    kernel (D % 64 == 0) and from the unfused path's cast (D = 96); with/without collisions."""
    F = gpu_pkg.functional
    g = torch.Generator().manual_seed(D + B)
    u = torch.randn(B, D, generator=g).to(DEV)
    it = torch.randn(B, D, generator=g).to(DEV)
    for uid in (None, torch.randint(0, 10, (B,), generator=g).to(DEV)):
        _, _, _, _, st = F.infonce_fwd(u, it, uid)
        du, di = torch.empty_like(u), torch.empty_like(it)
        du16 = torch.full((B, D), float("nan"), device=DEV, dtype=torch.bfloat16)
        F.infonce_bwd(st, None, du, di, du16)
        assert torch.equal(du16.view(torch.int16), du.bfloat16().view(torch.int16))


@pytest.mark.parametrize("use_graph", [True, False])
def test_trainstep_ragged_last_batch(gpu_pkg, use_graph):
    """TrainStep over batches of 8, 8, 7 and 8 pairs (a new batch shape gets its own static
    buffers and graph; a known one reuses its graph) vs the fp32 oracle's train step."""
    V, D, L = 101, 64, 12
    torch.manual_seed(0)
    m = gpu_pkg.TwoTowerModel(vocab_size=V, tabular_input_dim=128, num_genders=3,
                              num_countries=8, max_seq_len=L, user_embedding_dim=D,
                              item_embedding_dim=D, user_dropout=0.0,
                              compute_dtype=torch.float32, precomputed_modalities=True).to(DEV)
    m.item_tower.fusion_layer[3].p = 0.0
    params = {k: v.detach().cpu().clone() for k, v in m.named_parameters()}
    opt, running = {}, ref.init_running()
    step = gpu_pkg.TrainStep(m, lr=1e-3, use_graph=use_graph)
    for s, B in enumerate((8, 8, 7, 8)):
        b = ref.synthetic_batch(B, L, V, 3, 8, num_users=5,
                                generator=torch.Generator().manual_seed(50 + s))
        loss = float(step.step({k: v.to(DEV) for k, v in b.items()}))
        want = ref.train_step(params, opt, b, lr=1e-3, running=running)
        assert abs(loss - want) <= 2e-5 * max(1.0, abs(want)), (s, B, loss, want)
    assert len(step._entries) == 2
    got = {k: v.detach().cpu() for k, v in m.named_parameters()}
    for k in params:
        if any(d in k for d in DEGENERATE):      # exactly-zero gradients: AdamW ±lr noise
            assert (got[k] - params[k]).abs().max().item() <= 1.01 * 1e-3 * 4, k
        else:
            assert rel(got[k], params[k]) < 2e-4, (k, rel(got[k], params[k]))


def _item_head_inputs(ops, B, g, p):
    """Random item fusion-head weights / input / buffers (bf16 operands) for the fused tests."""
    def bf(*s, scale=1.0):
        return (torch.randn(*s, generator=g) * scale).to(torch.bfloat16).to(DEV)

    def f32(*s, scale=1.0):
        return (torch.randn(*s, generator=g) * scale).to(DEV)
    W = {"fusion_layer.0.weight": bf(512, 512, scale=512 ** -0.5),
         "fusion_layer.4.weight": bf(128, 512, scale=512 ** -0.5)}
    W["fusion_layer.4.weight.T"] = W["fusion_layer.4.weight"].t().contiguous()
    P = {"fusion_layer.0.bias": f32(512, scale=0.1), "fusion_layer.1.weight": 1 + f32(512, scale=0.1),
         "fusion_layer.1.bias": f32(512, scale=0.1), "fusion_layer.4.bias": f32(128, scale=0.1),
         "fusion_layer.5.weight": 1 + f32(128, scale=0.1), "fusion_layer.5.bias": f32(128, scale=0.1)}
    modal = f32(B, 512) * 2 + 0.3
    seeds = torch.tensor([0x7654321], dtype=torch.int64, device=DEV)
    drop = (p, seeds[0:1]) if p > 0 else ops.NO_DROP

    def bufs():
        return {"fusion_layer.1.running_mean": torch.full((512,), 0.2, device=DEV),
                "fusion_layer.1.running_var": torch.full((512,), 1.5, device=DEV),
                "fusion_layer.1.num_batches_tracked": torch.full((), 3, dtype=torch.int64, device=DEV)}
    return W, P, modal, drop, bufs


def _item_head_outs(B):
    f = dict(device=DEV)
    return dict(m16=torch.full((B, 512), 7, dtype=torch.bfloat16, **f), z=torch.full((B, 512), 7., **f),
                bn_mean=torch.full((512,), 7., **f), bn_rstd=torch.full((512,), 7., **f),
                y1=torch.full((B, 512), 7, dtype=torch.bfloat16, **f), y2=torch.full((B, 128), 7., **f),
                out=torch.full((B, 128), 7., **f), m5=torch.full((B,), 7., **f), r5=torch.full((B,), 7., **f))


@pytest.mark.parametrize("B,p,co", [(512, 0.1, False), (300, 0.0, False), (37, 0.1, False),
                                    (512, 0.1, True), (37, 0.1, True)])
def test_user_head_fused_matches_ops(gpu_pkg, B, p, co):
    """ttmi_user_head_fwd (the user tower head in one launch) against the unfused op sequence
    it replaces (functional.user_tower_fwd's pruned-layer path): same dropout masks (same hash,
    same drop_rows indices), fp32 values to 1e-4 of their scale, bf16 values to 1e-2."""
    ops = gpu_pkg.ops
    D, F, M = 128, 512, 7 * B
    g = torch.Generator().manual_seed(B)

    def bf(*s, scale=1.0):
        return (torch.randn(*s, generator=g) * scale).to(torch.bfloat16).to(DEV)

    def f32(*s, scale=1.0):
        return (torch.randn(*s, generator=g) * scale).to(DEV)
    pre = "transformer_encoder.layers.1."
    W = {pre + "self_attn.out_proj.weight": bf(D, D, scale=D ** -0.5),
         pre + "linear1.weight": bf(F, D, scale=D ** -0.5),
         pre + "linear2.weight": bf(D, F, scale=F ** -0.5),
         "fusion_layer.0.weight": bf(D, D + 48, scale=(D + 48) ** -0.5),
         "fusion_layer.3.weight": bf(D, D, scale=D ** -0.5)}
    P = {pre + "self_attn.out_proj.bias": f32(D, scale=0.1), pre + "norm2.weight": 1 + f32(D, scale=0.1),
         pre + "norm2.bias": f32(D, scale=0.1), pre + "linear1.bias": f32(F, scale=0.1),
         pre + "linear2.bias": f32(D, scale=0.1), "gender_embedding.weight": f32(3, 16),
         "country_embedding.weight": f32(11, 32), "fusion_layer.0.bias": f32(D, scale=0.1),
         "fusion_layer.1.weight": 1 + f32(D, scale=0.1), "fusion_layer.1.bias": f32(D, scale=0.1),
         "fusion_layer.3.bias": f32(D, scale=0.1)}
    ctx, res = bf(B, D), f32(B, D)
    drows = torch.randperm(M, generator=g)[:B].to(torch.int32).to(DEV)
    gender = torch.randint(0, 3, (B,), generator=g).to(DEV)
    country = torch.randint(0, 11, (B,), generator=g).to(DEV)
    seeds = torch.tensor([11, -22, 33], dtype=torch.int64, device=DEV)
    drops = tuple((p, seeds[k:k + 1]) if p > 0 else ops.NO_DROP for k in range(3))
    assert ops.user_head_fusable(W, P, pre, D, torch.bfloat16)
    # unfused reference sequence
    x1 = torch.empty(B, D, device=DEV)
    ops.linear(ctx, W[pre + "self_attn.out_proj.weight"], P[pre + "self_attn.out_proj.bias"], x1,
               drop=drops[0], residual=res, drop_rows=drows)
    a2 = torch.empty(B, D, device=DEV, dtype=torch.bfloat16)
    m2, r2 = torch.empty(B, device=DEV), torch.empty(B, device=DEV)
    ops.layernorm_fwd(x1, P[pre + "norm2.weight"], P[pre + "norm2.bias"], a2, m2, r2, eps=1e-5)
    h = torch.empty(B, F, device=DEV, dtype=torch.bfloat16)
    ops.linear(a2, W[pre + "linear1.weight"], P[pre + "linear1.bias"], h, act=1, drop=drops[1],
               drop_rows=drows)
    x2 = torch.empty(B, D, device=DEV)
    ops.linear(h, W[pre + "linear2.weight"], P[pre + "linear2.bias"], x2, drop=drops[2],
               residual=x1, drop_rows=drows)
    comb = torch.empty(B, D + 48, device=DEV, dtype=torch.bfloat16)
    rows = torch.empty(B, device=DEV, dtype=torch.int32)
    ops.user_concat_fwd(x2, None, gender, P["gender_embedding.weight"], country,
                        P["country_embedding.weight"], comb, rows, B, 1)
    z = torch.empty(B, D, device=DEV)
    ops.linear(comb, W["fusion_layer.0.weight"], P["fusion_layer.0.bias"], z)
    az = torch.empty(B, D, device=DEV, dtype=torch.bfloat16)
    mz, rz = torch.empty(B, device=DEV), torch.empty(B, device=DEV)
    ops.layernorm_fwd(z, P["fusion_layer.1.weight"], P["fusion_layer.1.bias"], az, mz, rz,
                      eps=1e-5, relu=True)
    u = torch.empty(B, D, device=DEV)
    ops.linear(az, W["fusion_layer.3.weight"], P["fusion_layer.3.bias"], u)
    want = dict(x1=x1, a2=a2, m2=m2, r2=r2, h=h, comb=comb, rows=rows, z=z, az=az, mz=mz, rz=rz, u=u)
    out = {k: torch.full_like(v, 7) for k, v in want.items()}
    if co:      # ABI 15: the item head's stage A rides in the same launch (idle CUs)
        Wi, Pi, modal, drop_i, bufs = _item_head_inputs(ops, B, g, p)
        iw, ig = _item_head_outs(B), _item_head_outs(B)
        ops.item_head_fwd(modal, Wi, Pi, bufs(), drop_i, 1e-5, iw)
        norms = torch.full((2 * B,), 7., device=DEV)
        uh, ih = torch.full((B, D), 7., device=DEV), torch.full((B, D), 7., device=DEV)
        ig["out_hat"], ig["out_norm"] = ih, norms[B:]          # InfoNCE's l2norm in stage C
        d = ops.item_head_desc(modal, Wi, Pi, bufs(), drop_i, 1e-5, ig)
        ops.user_head_fwd(ctx, res, drows, W, P, pre, gender, country, 1e-5, drops, out, co_item=d,
                          normed=(uh, norms[:B]))
        ops.item_head_fwd_stages(d, 6)
        solo = {k: torch.full_like(v, 7) for k, v in want.items()}
        ops.user_head_fwd(ctx, res, drows, W, P, pre, gender, country, 1e-5, drops, solo)
        torch.cuda.synchronize()
        for k in solo:                       # the user blocks run the same code either way
            assert torch.equal(out[k], solo[k]), k
        for k in ("m16", "z", "y1"):         # stage A (and BN) are the same kernels' arithmetic
            assert torch.equal(ig[k], iw[k]), k
        for k in ("bn_mean", "bn_rstd", "y2", "out", "m5", "r5"):
            assert rel(ig[k], iw[k]) < 1e-6, k
        # the heads' l2norm outputs = F.normalize (eps 1e-12) and the row norms
        for x, xh, nr in ((out["u"], uh, norms[:B]), (ig["out"], ih, norms[B:])):
            assert rel(xh, torch.nn.functional.normalize(x, dim=1)) < 1e-6
            assert rel(nr, x.norm(dim=1)) < 1e-6
        # ttmi_infonce_fwd_pre on them = ttmi_infonce_fwd from the raw rows
        F_ = gpu_pkg.functional
        # (its lse / loss combine runs in the logits launch: arrival counters, reset by the last
        # arrivers, so a second call must agree too)
        l0, lg0, _, _, s0 = F_.infonce_fwd(out["u"], ig["out"], None, 0.07)
        for _ in range(2):
            l1, lg1, _, _, s1 = F_.infonce_fwd(out["u"], ig["out"], None, 0.07, normed=(uh, ih, norms))
            torch.cuda.synchronize()
            assert abs(float(l1) - float(l0)) <= 1e-6 * max(1.0, abs(float(l0)))
            assert rel(lg1, lg0) < 1e-6 and rel(s1.lse, s0.lse) < 1e-6
    else:
        ops.user_head_fwd(ctx, res, drows, W, P, pre, gender, country, 1e-5, drops, out)
    torch.cuda.synchronize()
    assert torch.equal(out["rows"], rows)
    for k in ("x1", "m2", "r2", "z", "mz", "rz", "u"):
        assert rel(out[k], want[k]) < 1e-4 if k in ("x1",) else rel(out[k], want[k]) < 2e-3, k
    for k in ("a2", "h", "comb", "az"):
        assert rel(out[k].float(), want[k].float()) < 1e-2, k
        # masks: dropped (zero) positions agree except where the kept value rounds to zero
        if p > 0 and k == "h":
            zo, zw = out[k] == 0, want[k] == 0
            assert (zo != zw).float().mean().item() < 1e-3


@pytest.mark.parametrize("B,p", [(512, 0.1), (300, 0.0), (37, 0.1), (2, 0.0)])
def test_item_head_fused_matches_ops(gpu_pkg, B, p):
    """ttmi_item_head_fwd (the item late-fusion MLP in three launches) against the unfused op
    sequence of functional.item_fusion_fwd (cast, Linear, BatchNorm+ReLU+dropout, Linear,
    LayerNorm): every saved tensor, the BatchNorm batch statistics and the running buffers."""
    ops = gpu_pkg.ops
    g = torch.Generator().manual_seed(B + 5)

    def bf(*s, scale=1.0):
        return (torch.randn(*s, generator=g) * scale).to(torch.bfloat16).to(DEV)

    def f32(*s, scale=1.0):
        return (torch.randn(*s, generator=g) * scale).to(DEV)
    W = {"fusion_layer.0.weight": bf(512, 512, scale=512 ** -0.5),
         "fusion_layer.4.weight": bf(128, 512, scale=512 ** -0.5)}
    P = {"fusion_layer.0.bias": f32(512, scale=0.1), "fusion_layer.1.weight": 1 + f32(512, scale=0.1),
         "fusion_layer.1.bias": f32(512, scale=0.1), "fusion_layer.4.bias": f32(128, scale=0.1),
         "fusion_layer.5.weight": 1 + f32(128, scale=0.1), "fusion_layer.5.bias": f32(128, scale=0.1)}
    modal = f32(B, 512) * 2 + 0.3
    seeds = torch.tensor([0x1234567], dtype=torch.int64, device=DEV)
    drop = (p, seeds[0:1]) if p > 0 else ops.NO_DROP

    def bufs():
        return {"fusion_layer.1.running_mean": torch.full((512,), 0.2, device=DEV),
                "fusion_layer.1.running_var": torch.full((512,), 1.5, device=DEV),
                "fusion_layer.1.num_batches_tracked": torch.full((), 3, dtype=torch.int64, device=DEV)}
    assert ops.item_head_fusable(W, modal, torch.bfloat16)
    # unfused reference sequence
    bw = bufs()
    m16 = ops.cast_bf16(modal, torch.empty(B, 512, device=DEV, dtype=torch.bfloat16))
    z = torch.empty(B, 512, device=DEV)
    ops.linear(m16, W["fusion_layer.0.weight"], P["fusion_layer.0.bias"], z)
    y1 = torch.empty(B, 512, device=DEV, dtype=torch.bfloat16)
    bm, br = torch.empty(512, device=DEV), torch.empty(512, device=DEV)
    ops.batchnorm_fwd(z, P["fusion_layer.1.weight"], P["fusion_layer.1.bias"], y1, bm, br,
                      bw["fusion_layer.1.running_mean"], bw["fusion_layer.1.running_var"],
                      bw["fusion_layer.1.num_batches_tracked"], relu=True, drop=drop, training=True)
    y2 = torch.empty(B, 128, device=DEV)
    ops.linear(y1, W["fusion_layer.4.weight"], P["fusion_layer.4.bias"], y2)
    out = torch.empty(B, 128, device=DEV)
    m5, r5 = torch.empty(B, device=DEV), torch.empty(B, device=DEV)
    ops.layernorm_fwd(y2, P["fusion_layer.5.weight"], P["fusion_layer.5.bias"], out, m5, r5, eps=1e-5)
    want = dict(m16=m16, z=z, bn_mean=bm, bn_rstd=br, y1=y1, y2=y2, out=out, m5=m5, r5=r5)
    got = {k: torch.full_like(v, 7) for k, v in want.items()}
    bf_ = bufs()
    ops.item_head_fwd(modal, W, P, bf_, drop, 1e-5, got)
    torch.cuda.synchronize()
    assert torch.equal(got["m16"], want["m16"])
    for k in ("z", "bn_mean", "bn_rstd", "y2", "out", "m5", "r5"):
        assert rel(got[k], want[k]) < (1e-5 if k == "z" else 1e-4 if k in ("bn_mean", "bn_rstd") else 2e-3), k
    assert rel(got["y1"].float(), want["y1"].float()) < 1e-2
    if p > 0:     # same dropout mask (zeros agree except where a kept value rounds to zero)
        assert ((got["y1"] == 0) != (want["y1"] == 0)).float().mean().item() < 1e-3
    for k in ("fusion_layer.1.running_mean", "fusion_layer.1.running_var"):
        assert rel(bf_[k], bw[k]) < 1e-5, k
    assert int(bf_["fusion_layer.1.num_batches_tracked"]) == 4


def _item_bwd_case(ops, B, g):
    """LayerNorm(fusion_layer.5)-backward + Linear-4 input-grad inputs and the unfused ops'
    results (ttmi_layernorm_bwd with its bf16 copy, then the dgrad GEMM)."""
    W, P, _, _, _ = _item_head_inputs(ops, B, g, 0.0)
    y2 = (torch.randn(B, 128, generator=g) * 1.5 + 0.2).to(DEV)
    out, m5, r5 = torch.empty(B, 128, device=DEV), torch.empty(B, device=DEV), torch.empty(B, device=DEV)
    ops.layernorm_fwd(y2, P["fusion_layer.5.weight"], P["fusion_layer.5.bias"], out, m5, r5, eps=1e-5)
    dout = torch.randn(B, 128, generator=g).to(DEV)
    dy2, dy2c = torch.empty(B, 128, device=DEV), torch.empty(B, 128, device=DEV, dtype=torch.bfloat16)
    gw, gb = torch.zeros(128, device=DEV), torch.zeros(128, device=DEV)
    ops.layernorm_bwd(dout, y2, m5, r5, P["fusion_layer.5.weight"], dy2, gw, gb, dx16=dy2c)
    dy1 = torch.empty(B, 512, device=DEV)
    ops.linear_dx(dy2c, W["fusion_layer.4.weight"], dy1)
    return dict(W=W, P=P, y2=y2, m5=m5, r5=r5, dout=dout, dy2c=dy2c, dy1=dy1, gw=gw, gb=gb)


def _item_bwd_check(ops, c, dy2, dy1, gw, gb):
    assert rel(dy2.float(), c["dy2c"].float()) < 1e-2
    assert ((dy2.float() - c["dy2c"].float()).abs() >
            2 ** -7 * c["dy2c"].float().abs() + 1e-6).float().mean().item() < 1e-2   # ≤ 1 bf16 ulp
    assert rel(dy1, c["dy1"]) < 5e-3
    assert rel(gw, c["gw"]) < 1e-4 and rel(gb, c["gb"]) < 1e-4


@pytest.mark.parametrize("B", [512, 300, 37, 2])
def test_item_head_bwd_c_matches_ops(gpu_pkg, B):
    """ttmi_item_head_bwd_c (ABI 15) against the ops it replaces in item_fusion_bwd:
    ttmi_layernorm_bwd (dy2, its bf16 copy, the LN weight / bias gradients) and the Linear-4
    input-gradient GEMM (dy1 = dy2·W4)."""
    ops = gpu_pkg.ops
    g = torch.Generator().manual_seed(B + 77)
    c = _item_bwd_case(ops, B, g)
    dy2 = torch.full((B, 128), 7, device=DEV, dtype=torch.bfloat16)
    dy1 = torch.full((B, 512), 7., device=DEV)
    ws = ops.item_head_bwd_ws(B, DEV)
    gw, gb = torch.zeros(128, device=DEV), torch.zeros(128, device=DEV)
    d = ops.item_head_bwd_desc(c["dout"], c["y2"], c["m5"], c["r5"], c["P"]["fusion_layer.5.weight"],
                               c["W"]["fusion_layer.4.weight.T"], dy2, dy1, ws)
    ops.item_head_bwd_c(d)
    ops.ln_sum_folds(ws, (gw, gb), 2, 128)
    torch.cuda.synchronize()
    _item_bwd_check(ops, c, dy2, dy1, gw, gb)


@pytest.mark.parametrize("B,p,co", [(512, 0.1, False), (37, 0.0, False), (512, 0.1, True)])
def test_user_head_bwd_fused_matches_ops(gpu_pkg, B, p, co):
    """ttmi_user_head_bwd against the unfused backward ops it replaces (functional's
    _head_bwd_unfused + _layer_tail_bwd for the pruned layer): dctx, dx1, the bf16 dY operands
    of the deferred weight gradients, the LayerNorm parameter gradients (folded per-block sums)
    and the demographic embedding gradients."""
    ops, F_ = gpu_pkg.ops, gpu_pkg.functional
    D, F, M = 128, 512, 9 * B
    g = torch.Generator().manual_seed(B + 1)

    def bf(*s, scale=1.0):
        return (torch.randn(*s, generator=g) * scale).to(torch.bfloat16).to(DEV)

    def f32(*s, scale=1.0):
        return (torch.randn(*s, generator=g) * scale).to(DEV)
    pre = "transformer_encoder.layers.1."
    names = {pre + "self_attn.out_proj.weight": (D, D), pre + "linear1.weight": (F, D),
             pre + "linear2.weight": (D, F), "fusion_layer.0.weight": (D, D + 48),
             "fusion_layer.3.weight": (D, D)}
    W = {}
    for n, (o, i) in names.items():
        W[n] = bf(o, i, scale=i ** -0.5)
        W[n + ".T"] = W[n].t().contiguous()
    P = {pre + "norm2.weight": 1 + f32(D, scale=0.1), "fusion_layer.1.weight": 1 + f32(D, scale=0.1),
         "gender_embedding.weight": f32(3, 16), "country_embedding.weight": f32(11, 32)}
    for n in ("self_attn.out_proj.bias", "norm2.bias", "linear1.bias", "linear2.bias"):
        P[pre + n] = f32(F if n == "linear1.bias" else D, scale=0.1)
    for n in ("fusion_layer.0.bias", "fusion_layer.1.bias", "fusion_layer.3.bias"):
        P[n] = f32(D, scale=0.1)
    # a forward to get consistent saved values
    ctx, res = bf(B, D), f32(B, D)
    drows = torch.randperm(M, generator=g)[:B].to(torch.int32).to(DEV)
    gender = torch.randint(0, 3, (B,), generator=g).to(DEV)
    country = torch.randint(0, 11, (B,), generator=g).to(DEV)
    seeds = torch.tensor([5, -6, 7], dtype=torch.int64, device=DEV)
    drops = tuple((p, seeds[k:k + 1]) if p > 0 else ops.NO_DROP for k in range(3))
    o = dict(x1=f32(B, D), a2=bf(B, D), m2=f32(B), r2=f32(B), h=bf(B, F), comb=bf(B, D + 48),
             rows=torch.empty(B, dtype=torch.int32, device=DEV), z=f32(B, D), az=bf(B, D),
             mz=f32(B), rz=f32(B), u=f32(B, D))
    ops.user_head_fwd(ctx, res, drows, W, P, pre, gender, country, 1e-5, drops, o)
    du16 = bf(B, D)
    cfg = F_.TowerCfg(D=D, n_layers=2, p_drop=p)

    def grads0():
        return {k: torch.zeros(P[k].shape if k in P else (D, D), device=DEV) for k in (
            "fusion_layer.1.weight", "fusion_layer.1.bias", pre + "norm2.weight", pre + "norm2.bias",
            "gender_embedding.weight", "country_embedding.weight")}
    # unfused: head MLP + concat, then the layer tail
    Gu = grads0()
    for k in ("fusion_layer.3.weight", "fusion_layer.0.weight", pre + "linear2.weight",
              pre + "linear1.weight", pre + "self_attn.out_proj.weight"):
        Gu[k] = torch.zeros(names[k], device=DEV)
        Gu[k.replace("weight", "bias")] = torch.zeros(names[k][0], device=DEV)

    class St:
        pass
    st = St()
    st.ids = torch.zeros(B, 1, dtype=torch.int64, device=DEV)
    st.az, st.z, st.mz, st.rz, st.comb, st.rows = o["az"], o["z"], o["mz"], o["rz"], o["comb"], o["rows"]
    st.gender, st.country = gender, country
    dx = F_._head_bwd_unfused(P, W, st, du16.float(), Gu, cfg, du16, True)
    s = F_.LayerSaved(None, None, None, None, None, ctx, None, o["x1"], o["a2"], o["m2"], o["r2"],
                      o["h"], drows)
    sd = torch.arange(1, 65, dtype=torch.int64, device=DEV) * 7919      # a full site table
    cfg_seeds = sd
    dx1_u, dctx_u, _ = F_._layer_tail_bwd(P, W, s, dx, None, Gu, cfg, cfg_seeds, 1, pre, B, drows,
                                          F, True, D, torch.bfloat16, p)
    # fused
    Gf = grads0()
    site = (F_.site_drop1(1), F_.site_drop2(1))
    dr = tuple((p, sd[k:k + 1]) if p > 0 else ops.NO_DROP for k in site)
    co_d = None
    if co:      # ABI 15: the item head's row-local backward rides in the same launch
        c = _item_bwd_case(ops, B, g)
        idy2 = torch.full((B, 128), 7, device=DEV, dtype=torch.bfloat16)
        idy1 = torch.full((B, 512), 7., device=DEV)
        iws = ops.item_head_bwd_ws(B, DEV)
        co_d = ops.item_head_bwd_desc(c["dout"], c["y2"], c["m5"], c["r5"], c["P"]["fusion_layer.5.weight"],
                                      c["W"]["fusion_layer.4.weight.T"], idy2, idy1, iws)
    head = ops.user_head_bwd(du16, dict(az=o["az"], z=o["z"], mz=o["mz"], rz=o["rz"], h=o["h"],
                                        x1=o["x1"], m2=o["m2"], r2=o["r2"]),
                             drows, W, P, pre, gender, country, F_._scale(p), dr,
                             Gf["gender_embedding.weight"], Gf["country_embedding.weight"],
                             (Gf["fusion_layer.1.weight"], Gf["fusion_layer.1.bias"],
                              Gf[pre + "norm2.weight"], Gf[pre + "norm2.bias"]), co_item=co_d)
    torch.cuda.synchronize()
    if co:
        igw, igb = torch.zeros(128, device=DEV), torch.zeros(128, device=DEV)
        ops.ln_sum_folds(iws, (igw, igb), 2, 128)
        torch.cuda.synchronize()
        _item_bwd_check(ops, c, idy2, idy1, igw, igb)
    assert rel(head["dx1"], dx1_u) < 2e-3
    assert rel(head["dctx"].float(), dctx_u.float()) < 2e-2
    for k in ("fusion_layer.1.weight", "fusion_layer.1.bias", pre + "norm2.weight", pre + "norm2.bias",
              "gender_embedding.weight", "country_embedding.weight"):
        assert rel(Gf[k], Gu[k]) < 2e-3, k


@pytest.mark.parametrize("use_graph,glob", [(True, False), (False, False), (True, True)])
def test_trainstep_loss_sum(gpu_pkg, use_graph, glob):
    """TrainStep.loss_sum (the reference loop's total_loss, src/train.py:68) is the running sum
    of the returned step losses: added inside the InfoNCE logits launch on the cfg-2 path, by
    an add in the step on the global-negatives path; the capture's warm-up step is undone."""
    torch.manual_seed(3)
    m = gpu_pkg.TwoTowerModel(precomputed_modalities=True, vocab_size=1001, tabular_input_dim=128,
                              num_genders=3, num_countries=64, max_seq_len=50, user_embedding_dim=128,
                              item_embedding_dim=128, global_negatives=glob).to(DEV)
    step = gpu_pkg.TrainStep(m, lr=1e-4, use_graph=use_graph)
    total = 0.0
    for s in range(3):
        b = ref.synthetic_batch(64, 50, 1001, generator=torch.Generator().manual_seed(70 + s))
        total += float(step.step({k: v.to(DEV) for k, v in b.items()}))
    torch.cuda.synchronize()
    assert abs(float(step.loss_sum) - total) <= 1e-5 * max(1.0, abs(total)), (float(step.loss_sum), total)

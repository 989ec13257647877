"""Round-4 co-launches (ABI 18): independent item-head work riding on the user tower's
one-query attention grids, and the InfoNCE backward's finish inside its logit-gradient launch.

Each co-launch must equal the separate launches it replaces BIT FOR BIT (the workgroups run
the same device bodies; only the grid they sit on changes), and must stay so on a second call
(the in-launch arrival counters are reset by their last arrivers).
"""
import pytest
import torch

from bf16emu import rel

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _q1_case(B, L, H, Dh, g, dtype=torch.bfloat16):
    D = H * Dh
    qkv = (torch.randn(B * L, 3 * D, generator=g) * 0.5).to(dtype).to(DEV)
    lens = torch.randint(0, L + 1, (B,), generator=g)
    lens[0], lens[-1] = 0, L                                # an empty history and a full one
    kv = (torch.arange(L)[None, :] < lens[:, None]).to(torch.int64).to(DEV)
    x = torch.randn(B * L, D, generator=g).to(DEV)
    return qkv, kv, x


def _item_case(ops, B, g, p):
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
    seeds = torch.tensor([0x5151], dtype=torch.int64, device=DEV)
    drop = (p, seeds[0:1]) if p > 0 else ops.NO_DROP
    return W, P, modal, drop


def _bufs():
    return {"fusion_layer.1.running_mean": torch.full((512,), 0.2, device=DEV),
            "fusion_layer.1.running_var": torch.full((512,), 1.5, device=DEV),
            "fusion_layer.1.num_batches_tracked": torch.full((), 3, dtype=torch.int64, device=DEV)}


def _item_outs(B):
    f = dict(device=DEV)
    return dict(m16=torch.full((B, 512), 7, dtype=torch.bfloat16, **f), z=torch.full((B, 512), 7., **f),
                bn_mean=torch.full((512,), 7., **f), bn_rstd=torch.full((512,), 7., **f),
                y1=torch.full((B, 512), 7, dtype=torch.bfloat16, **f), y2=torch.full((B, 128), 7., **f),
                out=torch.full((B, 128), 7., **f), m5=torch.full((B,), 7., **f), r5=torch.full((B,), 7., **f))


@pytest.mark.parametrize("B,p", [(512, 0.1), (37, 0.0), (2, 0.1)])
def test_q1_gather_item_fwd_equals_separate(gpu_pkg, B, p):
    """ttmi_mha_q1_gather_item_fwd (one-query attention + item stage A on one grid) then item
    stage C alone == ttmi_mha_q1_gather_fwd + ttmi_item_head_fwd, bit for bit (twice: the
    in-launch BatchNorm merge counters are left zero)."""
    ops = gpu_pkg.ops
    L, H, Dh = 50, 4, 32
    g = torch.Generator().manual_seed(B + 3)
    qkv, kv, x = _q1_case(B, L, H, Dh, g)
    seeds = torch.tensor([0x2468ACE], dtype=torch.int64, device=DEV)
    drop = (p, seeds[0:1]) if p > 0 else ops.NO_DROP
    W, P, modal, drop_i = _item_case(ops, B, g, p)

    def q1_outs():
        return (torch.full((B,), -1, dtype=torch.int32, device=DEV), torch.full((B, H * Dh), 7., device=DEV),
                torch.full((B, H * Dh), 7, dtype=torch.bfloat16, device=DEV), torch.full((B * H,), 7., device=DEV))
    rows0, xr0, ctx0, lse0 = q1_outs()
    ops.mha_q1_gather_fwd(qkv, kv, x, rows0, xr0, B, L, H, ctx0, lse0, drop)
    b0, want = _bufs(), _item_outs(B)
    ops.item_head_fwd(modal, W, P, b0, drop_i, 1e-5, want)
    for _ in range(2):
        rows1, xr1, ctx1, lse1 = q1_outs()
        b1, got = _bufs(), _item_outs(B)
        d = ops.item_head_desc(modal, W, P, b1, drop_i, 1e-5, got)
        assert d.bn_part, "the fused BatchNorm statistics apply at B <= 512"
        ops.mha_q1_gather_fwd(qkv, kv, x, rows1, xr1, B, L, H, ctx1, lse1, drop, co_item=d)
        ops.item_head_fwd_stages(d, 6)
        torch.cuda.synchronize()
        for a, b in ((rows1, rows0), (xr1, xr0), (ctx1, ctx0), (lse1, lse0)):
            assert torch.equal(a, b)
        for k in want:
            assert torch.equal(got[k], want[k]), k
        for k in b0:
            assert torch.equal(b1[k], b0[k]), k


@pytest.mark.parametrize("B,p", [(512, 0.1), (37, 0.0), (2, 0.1)])
def test_user_head_item_c_equals_separate(gpu_pkg, B, p):
    """ttmi_user_item_head_fwd_c (user head + item stage C on one grid) and
    ttmi_user_item_head_fwd_ac (user head + item stages A and C on one grid, C waiting for A's
    BatchNorm statistics inside the launch) == the user head alone + item_head_fwd_stages(A, C),
    bit for bit, including InfoNCE's l2norm outputs and the running statistics, on repeated
    calls (the in-launch counts are left zero)."""
    ops = gpu_pkg.ops
    D, F = 128, 512
    g = torch.Generator().manual_seed(B + 9)

    def bf(*s, scale=1.0):
        return (torch.randn(*s, generator=g) * scale).to(torch.bfloat16).to(DEV)

    def f32(*s, scale=1.0):
        return (torch.randn(*s, generator=g) * scale).to(DEV)
    pre = "transformer_encoder.layers.1."
    Wu = {pre + "self_attn.out_proj.weight": bf(D, D, scale=D ** -0.5), pre + "linear1.weight": bf(F, D, scale=D ** -0.5),
          pre + "linear2.weight": bf(D, F, scale=F ** -0.5), "fusion_layer.0.weight": bf(D, D + 48, scale=0.07),
          "fusion_layer.3.weight": bf(D, D, scale=D ** -0.5)}
    Pu = {pre + "self_attn.out_proj.bias": f32(D, scale=0.1), pre + "norm2.weight": 1 + f32(D, scale=0.1),
          pre + "norm2.bias": f32(D, scale=0.1), pre + "linear1.bias": f32(F, scale=0.1),
          pre + "linear2.bias": f32(D, scale=0.1), "gender_embedding.weight": f32(3, 16),
          "country_embedding.weight": f32(11, 32), "fusion_layer.0.bias": f32(D, scale=0.1),
          "fusion_layer.1.weight": 1 + f32(D, scale=0.1), "fusion_layer.1.bias": f32(D, scale=0.1),
          "fusion_layer.3.bias": f32(D, scale=0.1)}
    ctx, res = bf(B, D), f32(B, D)
    drows = torch.randperm(50 * B, generator=g)[:B].to(torch.int32).to(DEV)
    gender = torch.randint(0, 3, (B,), generator=g).to(DEV)
    country = torch.randint(0, 11, (B,), generator=g).to(DEV)
    seeds = torch.tensor([5, -6, 7], dtype=torch.int64, device=DEV)
    drops = tuple((p, seeds[k:k + 1]) if p > 0 else ops.NO_DROP for k in range(3))
    Wi, Pi, modal, drop_i = _item_case(ops, B, g, p)

    def uouts():
        f = dict(device=DEV)
        return dict(x1=torch.full((B, D), 7., **f), a2=torch.full((B, D), 7, dtype=torch.bfloat16, **f),
                    m2=torch.full((B,), 7., **f), r2=torch.full((B,), 7., **f),
                    h=torch.full((B, F), 7, dtype=torch.bfloat16, **f),
                    comb=torch.full((B, D + 48), 7, dtype=torch.bfloat16, **f),
                    rows=torch.full((B,), -1, dtype=torch.int32, **f), z=torch.full((B, D), 7., **f),
                    az=torch.full((B, D), 7, dtype=torch.bfloat16, **f), mz=torch.full((B,), 7., **f),
                    rz=torch.full((B,), 7., **f), u=torch.full((B, D), 7., **f))

    def run(mode):
        uo, io = uouts(), _item_outs(B)
        nrm = torch.full((2 * B,), 7., device=DEV)
        uh, ih = torch.full((B, D), 7., device=DEV), torch.full((B, D), 7., device=DEV)
        io["out_hat"], io["out_norm"] = ih, nrm[B:]
        bufs = _bufs()
        d = ops.item_head_desc(modal, Wi, Pi, bufs, drop_i, 1e-5, io)
        if mode != "AC":
            ops.item_head_fwd_stages(d, 1)                    # stage A (+ the BatchNorm merge)
        if mode == "sep":
            ops.user_head_fwd(ctx, res, drows, Wu, Pu, pre, gender, country, 1e-5, drops, uo,
                              normed=(uh, nrm[:B]))
            ops.item_head_fwd_stages(d, 6)
        else:
            ops.user_head_fwd(ctx, res, drows, Wu, Pu, pre, gender, country, 1e-5, drops, uo,
                              co_item=d, normed=(uh, nrm[:B]), co_stage=mode)
        torch.cuda.synchronize()
        if mode == "AC":      # every in-launch count left zero, no C workgroup's poll timed out
            cnt = ops._zero_ws("ttmi_item_head_bn_counter_bytes", (0,), modal.device)
            assert int(cnt.view(torch.int32).abs().sum()) == 0
        return uo, io, uh, ih, nrm, bufs
    ref = run("sep")
    for mode in ("C", "AC", "AC", "AC"):
        got = run(mode)
        for x, y in zip(ref, got):
            if isinstance(x, dict):
                for k in x:
                    assert torch.equal(x[k], y[k]), (mode, k)
            else:
                assert torch.equal(x, y), mode


@pytest.mark.parametrize("B,p,dt", [(512, 0.1, torch.bfloat16), (37, 0.0, torch.bfloat16),
                                    (300, 0.1, torch.float32)])
def test_q1_bnr_bwd_equals_separate(gpu_pkg, B, p, dt):
    """ttmi_mha_q1_bnr_bwd (one-query backward + the item BatchNorm1d backward on one grid) ==
    ttmi_mha_q1_bwd + ttmi_batchnorm_bwd, bit for bit: dqkv, dz, its bf16 copy, dw, db."""
    ops = gpu_pkg.ops
    L, H, Dh, C = 50, 4, 32, 512
    g = torch.Generator().manual_seed(B + 21)
    qkv, kv, x = _q1_case(B, L, H, Dh, g, dt)
    seeds = torch.tensor([0x13579], dtype=torch.int64, device=DEV)
    drop = (p, seeds[0:1]) if p > 0 else ops.NO_DROP
    rows = torch.empty(B, dtype=torch.int32, device=DEV)
    xr = torch.empty(B, H * Dh, device=DEV)
    ctx = torch.empty(B, H * Dh, dtype=dt, device=DEV)
    lse = torch.empty(B * H, device=DEV)
    ops.mha_q1_gather_fwd(qkv, kv, x, rows, xr, B, L, H, ctx, lse, drop)
    dctx = torch.randn(B, H * Dh, generator=g).to(dt).to(DEV)
    # BatchNorm backward operands (the item head's, B x 512, bf16 gate y1)
    dy = torch.randn(B, C, generator=g).to(DEV)
    z = torch.randn(B, C, generator=g).to(DEV) * 1.3 + 0.2
    w = 1 + 0.1 * torch.randn(C, generator=g).to(DEV)
    mean, rstd = z.mean(0), 1 / (z.var(0, unbiased=False) + 1e-5).sqrt()
    y = torch.relu(torch.randn(B, C, generator=g)).to(torch.bfloat16).to(DEV)

    def run(co):
        dqkv = torch.full((B * L, 3 * H * Dh), 7, dtype=dt, device=DEV)
        dz = torch.full((B, C), 7., device=DEV)
        dz16 = torch.full((B, C), 7, dtype=torch.bfloat16, device=DEV)
        dw, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
        if co:
            d = ops.bn_bwd_desc(dy, z, w, mean, rstd, y, dz, dw, db, gate_scale=1 / 0.9, gated=True, dz16=dz16)
            ops.mha_q1_bwd(qkv, kv, rows, lse, dctx, B, L, H, dqkv, drop, bn=d)
        else:
            ops.mha_q1_bwd(qkv, kv, rows, lse, dctx, B, L, H, dqkv, drop)
            ops.batchnorm_bwd(dy, z, w, mean, rstd, y, dz, dw, db, gate_scale=1 / 0.9, gated=True, dz16=dz16)
        torch.cuda.synchronize()
        return dqkv, dz, dz16, dw, db
    for a, b in zip(run(False), run(True)):
        assert torch.equal(a, b)


@pytest.mark.parametrize("B,D", [(512, 128), (64, 128), (7, 64), (300, 256)])
def test_infonce_bwd_fused_finish_equals_two_launch(gpu_pkg, B, D):
    """ttmi_infonce_bwd_fused (finish by the last arriving key split, sc1 partials) ==
    ttmi_infonce_bwd16 (separate finish kernel) bit for bit, with and without collisions, on
    three consecutive calls (its arrival counters are reset by the last arrivers)."""
    F, ops = gpu_pkg.functional, gpu_pkg.ops
    g = torch.Generator().manual_seed(B * 7 + D)
    u = torch.randn(B, D, generator=g).to(DEV)
    it = torch.randn(B, D, generator=g).to(DEV)
    dloss = torch.tensor([0.73], device=DEV)
    for uid in (None, torch.randint(0, max(B // 3, 1), (B,), generator=g).to(DEV)):
        _, _, _, _, st = F.infonce_fwd(u, it, uid)
        outs = []
        for fused in (False, True, True, True):
            du, di = torch.full_like(u, 7.), torch.full_like(it, 7.)
            du16 = torch.full((B, D), 7, device=DEV, dtype=torch.bfloat16)
            ops.infonce_bwd(st.u_hat, st.i_hat, st.norms, st.logits, st.lse, st.user_idx, st.inv_tau,
                            dloss, du, di, st.ws, du16, fused_finish=fused)
            torch.cuda.synchronize()
            outs.append((du, di, du16))
        for o in outs[1:]:
            for a, b in zip(o, outs[0]):
                assert torch.equal(a, b)
        assert rel(outs[0][0], outs[0][0]) == 0.0


def test_trainstep_grad_sink_off_is_bit_identical(gpu_pkg):
    """TrainStep(grad_sink=False) folds the item-embedding gradient into flat.grad (complete
    gradients between backward and update, for clipping / norms / hooks) and must update the
    parameters bit-identically to the default sink (AdamW converting the fixed-point
    accumulator itself)."""
    from oracle import two_tower_ref as ref
    B, L, V, D = 64, 20, 301, 128
    outs = []
    for sink in (True, False):
        torch.manual_seed(3)
        m = gpu_pkg.TwoTowerModel(precomputed_modalities=True, vocab_size=V, tabular_input_dim=128,
                                  num_genders=3, num_countries=16, max_seq_len=L, user_embedding_dim=D,
                                  item_embedding_dim=D, user_dropout=0.1,
                                  compute_dtype=torch.bfloat16).to(DEV)
        step = gpu_pkg.TrainStep(m, lr=1e-3, grad_sink=sink, seed=5)
        for s in range(2):
            b = ref.synthetic_batch(B, L, V, 3, 16, generator=torch.Generator().manual_seed(70 + s))
            step.step({k: v.to(DEV) for k, v in b.items()})
        torch.cuda.synchronize()
        outs.append({k: v.detach().clone() for k, v in m.named_parameters()})
    for k in outs[0]:
        assert torch.equal(outs[0][k], outs[1][k]), k


@pytest.mark.parametrize("D", [128, 256])
def test_trainstep_fold_in_update_is_bit_identical(gpu_pkg, D, monkeypatch):
    """One process folds the step's weight-gradient partials inside the AdamW launch
    (ttmi_wgrad_batch_plan + ttmi_adamw_folded, ABI 19): the same sums in the same order, the
    same AdamW arithmetic, so the parameters and both moments are bit-identical to the fold
    launch + AdamW launch path (TTMI_FOLD_IN_UPDATE=0), in graph replays and eagerly; and with
    the weight-gradient GEMMs on the main stream and one AdamW launch (no side-stream overlap,
    no item-embedding update of its own: TTMI_WGRAD_EARLY=0, TTMI_ADAM_SPLIT=0)."""
    import importlib
    from oracle import two_tower_ref as ref
    train_mod = importlib.import_module(gpu_pkg.__name__ + ".train")
    B, L, V = 64, 20, 301
    outs = []
    for fold, graph, overlap in ((True, True, True), (False, True, True), (True, False, True),
                                 (True, True, False)):
        monkeypatch.setenv("TTMI_FOLD_IN_UPDATE", "1" if fold else "0")
        monkeypatch.setattr(gpu_pkg.ops, "_WG_EARLY", overlap)
        monkeypatch.setattr(train_mod, "_ADAM_SPLIT", overlap)
        torch.manual_seed(3)
        m = gpu_pkg.TwoTowerModel(precomputed_modalities=True, vocab_size=V, tabular_input_dim=128,
                                  num_genders=3, num_countries=16, max_seq_len=L, user_embedding_dim=D,
                                  item_embedding_dim=D, user_dropout=0.1,
                                  compute_dtype=torch.bfloat16).to(DEV)
        step = gpu_pkg.TrainStep(m, lr=1e-3, seed=5, use_graph=graph)
        assert step.fold_in_update == fold
        for s in range(3):
            b = ref.synthetic_batch(B, L, V, 3, 16, generator=torch.Generator().manual_seed(70 + s))
            step.step({k: v.to(DEV) for k, v in b.items()})
        torch.cuda.synchronize()
        st = {k: v.detach().clone() for k, v in m.named_parameters()}
        st.update({"m/" + k: v.clone() for k, v in step.flat.views(step.flat.exp_avg).items()})
        st.update({"v/" + k: v.clone() for k, v in step.flat.views(step.flat.exp_avg_sq).items()})
        assert step.flat.grad.abs().max().item() == 0.0          # zero_grad covered every slot
        outs.append(st)
    for o in outs[1:]:
        bad = [k for k in outs[0] if not torch.equal(outs[0][k], o[k])]
        assert not bad, bad[:8]


@pytest.mark.parametrize("B,D", [(512, 256), (37, 128), (64, 64)])
def test_infonce_fwd_acc_equals_unfused(gpu_pkg, B, D):
    """ttmi_infonce_fwd_acc (normalise launch + logits launch with the in-launch combine and the
    loss accumulator, ABI 19) == ttmi_infonce_fwd: logits, lse, normalised rows bit for bit; the
    loss to float reassociation; loss_acc += loss; repeated calls (counters left zero)."""
    ops = gpu_pkg.ops
    g = torch.Generator().manual_seed(B + D)
    u = torch.randn(B, D, generator=g).to(DEV)
    it = torch.randn(B, D, generator=g).to(DEV)
    uid = torch.randint(0, max(B // 3, 1), (B,), generator=g).to(DEV)
    f32 = dict(device=DEV, dtype=torch.float32)

    def outs():
        return (torch.empty(B, D, **f32), torch.empty(B, D, **f32), torch.empty(2 * B, **f32),
                torch.empty(B, B, **f32), torch.empty(2 * B, **f32), torch.empty((), **f32),
                torch.empty(ops.infonce_workspace(B, D), device=DEV, dtype=torch.uint8))
    ref = outs()
    ops.infonce_fwd(u, it, uid, 1 / 0.07, *ref)
    acc = torch.full((1,), 0.25, **f32)
    losses = []
    for k in range(2):
        got = outs()
        ops.infonce_fwd_acc(u, it, uid, 1 / 0.07, *got, acc)
        torch.cuda.synchronize()
        for a, b in zip(got[:5], ref[:5]):
            assert torch.equal(a, b)
        # the 2B per-row CE terms are summed per query block, then over blocks (the separate
        # combine sums them per thread, then by a tree): the same terms, another order
        assert abs(float(got[5]) - float(ref[5])) <= 2e-5 * abs(float(ref[5]))
        losses.append(float(got[5]))
    assert losses[0] == losses[1]
    assert abs(float(acc) - (0.25 + sum(losses))) <= 1e-6 * abs(float(acc))
    cnt = ops._zero_ws("ttmi_infonce_counter_bytes", (B,), u.device)
    assert int(cnt.view(torch.int32).abs().sum()) == 0

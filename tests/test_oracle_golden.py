"""Pin the CPU oracle (oracle/two_tower_ref.py) against the golden fixtures produced by
running the reference modules (tools/make_golden.py).  fp32 tolerance: 1e-5 relative
(SURVEY §8d)."""
import numpy as np
import pytest
import torch

from conftest import load_golden, sub
from oracle import two_tower_ref as ref

RTOL, ATOL = 1e-5, 2e-6


def close(a, b, rtol=RTOL, atol=ATOL):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    scale = max(np.abs(b).max(), 1e-30)
    err = np.abs(a - b).max()
    assert err <= atol + rtol * scale, f"max err {err:.3e} vs scale {scale:.3e}"


@pytest.mark.parametrize("name", ["user_tower_small.npz", "user_tower_nomask.npz",
                                  "user_tower_leftpad.npz", "user_tower_d128.npz"])
def test_user_tower_matches_reference(name):
    z = load_golden(name)
    V, D, L, B, H, n_g, n_c, use_mask = z["cfg"].tolist()
    params = {k: torch.tensor(v, requires_grad=True) for k, v in sub(z, "p/").items()}
    out = ref.user_tower_forward(
        params, torch.tensor(z["history_ids"]), torch.tensor(z["user_gender"]),
        torch.tensor(z["user_country"]),
        torch.tensor(z["history_mask"]) if use_mask else None, num_heads=H)
    close(out.detach(), z["out"])
    (out * torch.tensor(z["upstream"])).sum().backward()
    for k, g in sub(z, "g/").items():
        close(params[k].grad, g)


@pytest.mark.parametrize("name", ["infonce_b8.npz", "infonce_b64.npz"])
@pytest.mark.parametrize("tag", ["nomask", "mask"])
def test_infonce_matches_reference(name, tag):
    z = load_golden(name)
    u = torch.tensor(z["u"], requires_grad=True)
    i = torch.tensor(z["i"], requires_grad=True)
    uid = torch.tensor(z["user_idx"]) if tag == "mask" else None
    loss, logits, un, inn = ref.infonce(u, i, uid)
    loss.backward()
    close(loss.detach(), z[f"{tag}/loss"])
    close(logits.detach(), z[f"{tag}/logits"])
    close(un.detach(), z[f"{tag}/u_hat"])
    close(inn.detach(), z[f"{tag}/i_hat"])
    close(u.grad, z[f"{tag}/du"])
    close(i.grad, z[f"{tag}/di"])


def test_item_fusion_matches_reference():
    z = load_golden("item_fusion.npz")
    p0 = sub(z, "p/")
    params = {k: torch.tensor(v, requires_grad=True) for k, v in p0.items()
              if "running" not in k and "num_batches" not in k}
    running = {"running_mean": torch.tensor(p0["fusion_layer.1.running_mean"]),
               "running_var": torch.tensor(p0["fusion_layer.1.running_var"]),
               "num_batches_tracked": torch.tensor(p0["fusion_layer.1.num_batches_tracked"])}
    out = ref.item_fusion_forward(params, torch.tensor(z["modal"]), running=running)
    close(out.detach(), z["out"])
    (out * torch.tensor(z["upstream"])).sum().backward()
    for k, g in sub(z, "g/").items():
        close(params[k].grad, g)
    after = sub(z, "after/")
    close(running["running_mean"], after["fusion_layer.1.running_mean"])
    close(running["running_var"], after["fusion_layer.1.running_var"])
    assert int(running["num_batches_tracked"]) == int(after["fusion_layer.1.num_batches_tracked"])


def test_train_step_matches_reference():
    z = load_golden("train_step.npz")
    V, D, L, B, n_g, n_c, n_steps = z["cfg"].tolist()
    p0 = sub(z, "p0/")
    p1 = sub(z, "p1/")
    buf = ("running_mean", "running_var", "num_batches_tracked")
    params = {k: torch.tensor(v) for k, v in p0.items() if not k.endswith(buf)}
    rk = "item_tower.fusion_layer.1."
    running = {b: torch.tensor(p0[rk + b]) for b in buf}
    state = {}
    losses = []
    for s in range(n_steps):
        batch = {k: torch.tensor(v) for k, v in sub(z, f"batch{s}/").items()}
        losses.append(ref.train_step(params, state, batch, running=running))
    close(np.array(losses), z["losses"])
    # AdamW normalises each element's gradient, so parameters whose true gradient is
    # identically zero turn float noise into +-lr steps: the K slice of in_proj_bias
    # (softmax is shift-invariant over keys) and the Linear feeding BatchNorm (BN removes
    # per-feature shift and scale).  Those are held to 2*lr per step instead.
    degenerate = ("in_proj_bias", "item_tower.fusion_layer.0.")
    for k, v in params.items():
        if any(d in k for d in degenerate):
            close(v, p1[k], rtol=0, atol=2e-4 * n_steps)
        else:
            close(v, p1[k], rtol=1e-5, atol=1e-6)
    # step 2's BN statistics are taken on the output of that degenerate Linear, so they
    # inherit its step-1 deviation.
    for b in buf[:2]:
        close(running[b], p1[rk + b], rtol=1e-5, atol=1e-4)


def test_hash_dropout_rate_and_determinism():
    keep = ref.hash_keep(0x1234_5678_9ABC_DEF0, 1 << 20, 0.1)
    assert abs(keep.mean() - 0.9) < 3e-3
    assert np.array_equal(keep, ref.hash_keep(0x1234_5678_9ABC_DEF0, 1 << 20, 0.1))
    assert ref.hash_keep(7, 1000, 0.0).all()


def test_serving_fixture_vs_oracle():
    """tests/golden/serving.npz (the reference's index_catalog + recommend_for_user, run by
    tools/make_golden_serving.py) restated by the oracle: eval-mode fusion head -> normalise
    (1e-12) -> nan_to_num -> normalise (1e-8) -> dense rows; user tower (eval) on the last 50
    history items -> normalise twice -> scores, padding + history masked -> top-10."""
    import torch.nn.functional as TF
    z = load_golden("serving.npz")
    p = {k[2:]: torch.tensor(v) for k, v in z.items() if k.startswith("p/")}
    ip = {k[len("item_tower."):]: v for k, v in p.items() if k.startswith("item_tower.")}
    up = {k[len("user_tower."):]: v for k, v in p.items() if k.startswith("user_tower.")}
    running = {k[len("fusion_layer.1."):]: v for k, v in ip.items() if k.startswith("fusion_layer.1.")}
    out = ref.item_fusion_forward(ip, torch.tensor(z["modal"]), running=running, eval_mode=True)
    e = TF.normalize(torch.nan_to_num(TF.normalize(out, dim=1), nan=0.0), p=2, dim=1, eps=1e-8)
    dense = torch.zeros_like(torch.tensor(z["dense"]))
    dense[torch.tensor(z["catalogue_ids"])] = e
    assert (dense - torch.tensor(z["dense"])).abs().max().item() < 1e-5
    hist = torch.tensor(z["history"])[-50:][None]
    u = ref.user_tower_forward(up, hist, torch.tensor(z["gender"]), torch.tensor(z["country"]),
                               None, 4, 2)
    u = TF.normalize(TF.normalize(u, dim=1), p=2, dim=1, eps=1e-8)
    s = (u @ torch.tensor(z["dense"]).t())[0]
    s[0] = -float("inf")
    s[hist[0]] = -float("inf")
    v, i = torch.topk(s, 10)
    assert i.tolist() == z["top_ids"].tolist()
    assert np.abs(v.numpy() - z["top_scores"]).max() < 6e-5


@pytest.mark.parametrize("name", ["tabular_t128.npz", "tabular_t37.npz"])
def test_tabular_encoder_matches_reference(name):
    """oracle/resnet_ref.tabular_forward vs the reference's own TabularEncoder
    (item_tower.py:85-98, train mode, dropout off): output, gradients, BN running stats."""
    from oracle import resnet_ref as rref
    z = load_golden(name)
    p0 = sub(z, "p/")
    params = {k: torch.tensor(v, requires_grad=("running" not in k and "num_batches" not in k
                                                and v.dtype.kind == "f"))
              for k, v in p0.items()}
    out = rref.tabular_forward(params, torch.tensor(z["x"]), update_running=True)
    close(out.detach(), z["out"])
    (out * torch.tensor(z["upstream"])).sum().backward()
    for k, g in sub(z, "g/").items():
        close(params[k].grad, g)
    for k, v in sub(z, "after/").items():
        if "running" in k:
            close(params[k], v)

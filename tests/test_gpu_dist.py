"""Data-parallel PRODUCT code at world size 2 on the GPU: two processes share cuda:0 over gloo
(RCCL refuses two ranks on one device; the product's collectives go through ``comm``, which
stages device tensors through the host under gloo — the arithmetic is the same).

* cfg 5 (global in-batch negatives): ``functional.infonce_global_fwd/bwd`` with the real
  all-gather / reduce-scatter, each rank holding 32 of the 64 rows of the reference-generated
  fixture ``infonce_b64.npz`` (two_tower.py:98-140 on the concatenated batch): mean of the
  per-rank losses and each rank's dU/dI vs the fixture (fp32 kernels: 1e-5 relative).
* ``TrainStep`` at N = 2 (graph capture, two-bucket overlapped gradient all-reduce, BN buffer
  broadcast) vs the fp32 CPU oracle of DDP (train.py:300): per step, the average of the two
  ranks' gradients (per-rank BatchNorm statistics), AdamW; rank r's BN running buffers are
  rank 0's at the step start updated with rank r's batch.  Both local negatives and
  ``global_negatives=True`` (oracle: the reference InfoNCE over both ranks' embeddings,
  differentiated through both ranks' towers).  fp32 compute: params 2e-4 relative.
* The bf16 product step at D = 128 (every fused head on its fused path: co-launched user /
  item heads, ``infonce_fwd_pre`` with the loss accumulator, the fused item BatchNorm, the
  overlap hook that flushes the deferred weight gradients at the layer-1 cut) with dropout
  on, local and global negatives.  With the overlap on, the head buckets reduce on comm's
  gloo worker thread (pinned-host staging on a side stream) while the second graph segment
  runs — the concurrency is real, not a synchronous copy.  Run with ``overlap_grad_sync`` on
  and off, the flat
  parameters, AdamW moments and BatchNorm buffers are bit-identical (the step is
  deterministic, so any flush-placement or bucket-split error shows as a bit difference),
  identical on both ranks, and the losses stay within the bf16 emulation's distance of the
  fp32 DDP oracle.
"""
import importlib
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from bf16emu import bf16_linears
from conftest import GOLDEN, PKG_NAME, ROOT
from oracle import two_tower_ref as ref

pytestmark = pytest.mark.gpu
WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _entry(rank, fn, port, args):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        torch.set_num_threads(4)
        fn(rank, *args)
    finally:
        dist.destroy_process_group()


def _run(fn, *args):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    mp.spawn(_entry, args=(fn, _free_port(), args), nprocs=WORLD, join=True)


def rel(a, b):
    a = torch.as_tensor(a).detach().double().cpu()
    b = torch.as_tensor(b).detach().double().cpu()
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-30)


# ------------------------------------------------------------------ cfg 5 loss, product path
def _global_infonce_worker(rank, variant, module_path):
    pkg = importlib.import_module(PKG_NAME)
    F = pkg.functional
    with np.load(os.path.join(GOLDEN, "infonce_b64.npz"), allow_pickle=False) as z:
        g = {k: torch.tensor(z[k]) for k in z.files}
    B = g["u"].shape[0] // WORLD
    sl = slice(rank * B, (rank + 1) * B)
    u = g["u"][sl].cuda()
    it = g["i"][sl].cuda()
    uid = g["user_idx"][sl].cuda() if variant == "mask" else None
    if module_path:       # TwoTowerModel's autograd path (infonce_global), DDP loss scale 1/W
        ua, ia = u.clone().requires_grad_(True), it.clone().requires_grad_(True)
        loss, logits, uh, ih = pkg.infonce_global(ua, ia, uid, 0.07)
        (loss / WORLD).backward()
        du, di = ua.grad, ia.grad
    else:
        loss, logits, uh, ih, st = F.infonce_global_fwd(u, it, uid, 0.07)
        du, di = torch.empty_like(u), torch.empty_like(it)
        dloss = torch.full((1,), 1.0 / WORLD, device="cuda")
        F.infonce_global_bwd(st, dloss, du, di)
    tot = loss.detach().reshape(1).clone()
    dist.all_reduce(tot)
    expect = float(g[variant + "/loss"])
    assert abs(float(tot) / WORLD - expect) <= 1e-5 * max(1.0, abs(expect)), (float(tot), expect)
    assert logits.shape == (B, WORLD * B)
    assert rel(logits, g[variant + "/logits"][sl]) < 1e-5
    assert rel(uh, g[variant + "/u_hat"][sl]) < 1e-6
    assert rel(du, g[variant + "/du"][sl]) < 1e-5, rel(du, g[variant + "/du"][sl])
    assert rel(di, g[variant + "/di"][sl]) < 1e-5, rel(di, g[variant + "/di"][sl])


@pytest.mark.parametrize("variant", ["nomask", "mask"])
@pytest.mark.parametrize("module_path", [False, True])
def test_global_infonce_world2_vs_reference_fixture(variant, module_path):
    _run(_global_infonce_worker, variant, module_path)


# ------------------------------------------------------------------ TrainStep at N = 2
V, D, L, B, NG, NC = 101, 64, 12, 16, 3, 8
STEPS, LR = 2, 1e-3


def _batch(rank, step):
    g = torch.Generator().manual_seed(1000 + 10 * step + rank)
    return ref.synthetic_batch(B, L, V, NG, NC, num_users=6, generator=g)


def _oracle_ddp(params, global_negatives, batch=None, p_drop=0.0, seeds=None):
    """fp32 CPU oracle of STEPS DDP steps at WORLD ranks; returns (params, running per rank,
    mean losses).  ``seeds(rank, step)``: the rank's hash-dropout site seeds (p_drop > 0)."""
    batch = batch or _batch
    params = {k: v.clone() for k, v in params.items()}
    opt = {}
    running = [ref.init_running() for _ in range(WORLD)]
    losses = []
    for s in range(STEPS):
        for r in range(1, WORLD):               # broadcast_buffers: rank 0's at the step start
            running[r] = {k: v.clone() for k, v in running[0].items()}
        leaves = {k: v.detach().clone().requires_grad_(True) for k, v in params.items()}
        up = {k[len("user_tower."):]: v for k, v in leaves.items() if k.startswith("user_tower.")}
        ip = {k[len("item_tower."):]: v for k, v in leaves.items() if k.startswith("item_tower.")}
        us, its, uids = [], [], []
        for r in range(WORLD):
            b = batch(r, s)
            drop = ref.HashDropout(seeds(r, s)) if p_drop > 0 else None
            us.append(ref.user_tower_forward(up, b["history_ids"], b["user_gender"],
                                             b["user_country"], b["history_mask"], 4, 2, p_drop,
                                             drop))
            its.append(ref.item_fusion_forward(ip, b["target_modal"], p_drop, drop, running[r]))
            uids.append(b["user_idx"])
        if global_negatives:
            loss = ref.infonce(torch.cat(us), torch.cat(its), torch.cat(uids))[0]
        else:
            loss = sum(ref.infonce(u, i, d)[0] for u, i, d in zip(us, its, uids)) / WORLD
        loss.backward()
        losses.append(float(loss.detach()))
        with torch.no_grad():
            ref.adamw_(params, {k: v.grad for k, v in leaves.items()}, opt, lr=LR)
    return params, running, losses


# gradients that are exactly 0 in exact arithmetic (the key third of in_proj_bias: softmax
# ignores a per-query shift; the Linear bias ahead of BatchNorm): AdamW turns their rounding
# noise into ±lr steps, so they are held to lr·steps absolute
DEGENERATE = ("in_proj_bias", "item_tower.fusion_layer.0.bias")


def _check_params(got, want):
    for k in want:
        if any(d in k for d in DEGENERATE):
            err = (got[k].double() - want[k].double()).abs().max().item()
            assert err <= 1.01 * LR * STEPS, (k, err)
        else:
            assert rel(got[k], want[k]) < 2e-4, (k, rel(got[k], want[k]))


def _trainstep_worker(rank, global_negatives, use_graph, out):
    pkg = importlib.import_module(PKG_NAME)
    torch.manual_seed(0)
    m = pkg.TwoTowerModel(vocab_size=V, tabular_input_dim=128, num_genders=NG, num_countries=NC,
                          max_seq_len=L, user_embedding_dim=D, item_embedding_dim=D,
                          user_dropout=0.0, compute_dtype=torch.float32,
                          precomputed_modalities=True,
                          global_negatives=global_negatives).cuda()
    m.item_tower.fusion_layer[3].p = 0.0
    p0 = {k: v.detach().cpu().clone() for k, v in m.named_parameters()}
    step = pkg.TrainStep(m, lr=LR, use_graph=use_graph, seed=rank + 1, overlap_grad_sync=True)
    assert step.world == WORLD and step.overlap and step.broadcast_buffers
    assert step.flat.tail_offset < step.flat.numel
    losses = []
    for s in range(STEPS):
        b = {k: v.cuda() for k, v in _batch(rank, s).items()}
        loss = step.step(b).detach().reshape(1).clone()
        dist.all_reduce(loss)
        losses.append(float(loss) / WORLD)
    torch.cuda.synchronize()
    params = {k: v.detach().cpu() for k, v in m.named_parameters()}
    bufs = {k: v.detach().cpu() for k, v in m.named_buffers()}
    # every rank holds the same parameters after the averaged update
    flat = step.flat.data.detach().clone()
    other = flat.clone()
    dist.broadcast(other, 0)
    assert torch.equal(flat, other)
    want, running, wl = _oracle_ddp(p0, global_negatives)
    for s in range(STEPS):
        assert abs(losses[s] - wl[s]) <= 2e-5 * max(1.0, abs(wl[s])), (s, losses[s], wl[s])
    _check_params(params, want)
    for k in ("running_mean", "running_var"):
        got = bufs["item_tower.fusion_layer.1." + k]
        # running_mean carries the pre-BN Linear bias, a degenerate parameter (±lr AdamW
        # noise, see DEGENERATE), scaled by the BN momentum 0.1; without the broadcast rank
        # 1's buffers would be off by ~1e-2 here
        err = (got.double() - running[rank][k].double()).abs().max().item()
        assert err <= 0.1 * 1.01 * LR * STEPS + 1e-5 * running[rank][k].abs().max().item(), \
            (rank, k, err)
    if rank == 0:
        torch.save({"losses": losses}, out)


@pytest.mark.parametrize("global_negatives", [False, True])
@pytest.mark.parametrize("use_graph", [True, False])
def test_trainstep_world2_vs_ddp_oracle(tmp_path, global_negatives, use_graph):
    out = str(tmp_path / "r0.pt")
    _run(_trainstep_worker, global_negatives, use_graph, out)
    assert os.path.exists(out)


# ------------------------------------------------------------------ bf16 product step at N = 2
V16, D16, L16, B16, P16 = 997, 128, 20, 64, 0.1


def _batch16(rank, step):
    g = torch.Generator().manual_seed(2000 + 10 * step + rank)
    return ref.synthetic_batch(B16, L16, V16, NG, NC, num_users=20, generator=g)


def _trainstep_bf16_worker(rank, global_negatives, out):
    pkg = importlib.import_module(PKG_NAME)
    F = pkg.functional
    states = []
    for overlap in (True, False):
        torch.manual_seed(0)
        m = pkg.TwoTowerModel(vocab_size=V16, tabular_input_dim=128, num_genders=NG,
                              num_countries=NC, max_seq_len=L16, user_embedding_dim=D16,
                              item_embedding_dim=D16, user_dropout=P16,
                              compute_dtype=torch.bfloat16, precomputed_modalities=True,
                              global_negatives=global_negatives).cuda()
        m.item_tower.fusion_layer[3].p = P16
        p0 = {k: v.detach().cpu().clone() for k, v in m.named_parameters()}
        step = pkg.TrainStep(m, lr=LR, use_graph=True, seed=rank + 1, overlap_grad_sync=overlap)
        assert step.world == WORLD and step.overlap == overlap and step.broadcast_buffers
        losses = []
        for s in range(STEPS):
            b = {k: v.cuda() for k, v in _batch16(rank, s).items()}
            loss = step.step(b).detach().reshape(1).clone()
            dist.all_reduce(loss)
            losses.append(float(loss) / WORLD)
        torch.cuda.synchronize()
        st = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
        # AdamW moments per parameter (the flat layout differs: overlap puts the late
        # parameters last)
        st.update({"m/" + k: v.cpu().clone() for k, v in step.flat.views(step.flat.exp_avg).items()})
        st.update({"v/" + k: v.cpu().clone() for k, v in step.flat.views(step.flat.exp_avg_sq).items()})
        flat = step.flat.data.detach().clone()
        other = flat.clone()
        dist.broadcast(other, 0)
        assert torch.equal(flat, other)              # both ranks hold the same parameters
        states.append((st, losses))
    (sa, la), (sb, lb) = states
    bad = [k for k in sa if not torch.equal(sa[k], sb[k])]
    assert not bad, ("overlap on/off differ", bad[:8])
    assert la == lb
    seeds = (lambda r, s: F.site_seeds(r + 1, s + 1))
    _, _, wl = _oracle_ddp(p0, global_negatives, _batch16, P16, seeds)
    with bf16_linears():
        _, _, el = _oracle_ddp(p0, global_negatives, _batch16, P16, seeds)
    for s in range(STEPS):
        assert abs(la[s] - wl[s]) <= 2 * abs(el[s] - wl[s]) + 2e-3, (s, la[s], wl[s], el[s])
    if rank == 0:
        torch.save({"losses": la}, out)


@pytest.mark.parametrize("global_negatives", [False, True])
def test_trainstep_world2_bf16_fused_overlap_bitexact(tmp_path, global_negatives):
    out = str(tmp_path / "r0.pt")
    _run(_trainstep_bf16_worker, global_negatives, out)
    assert os.path.exists(out)

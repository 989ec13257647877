"""RCCL on the GPU: the data-parallel code path with the product backend (``nccl`` = RCCL), at
world size 1 on the one-GPU box (RCCL refuses two ranks on one device; the world-2 runs of the
same code are the gloo tests in test_gpu_dist.py).  ``comm.force_dp`` makes a world-1 group run
every collective and the whole data-parallel schedule of ``TrainStep`` (two gradient buckets,
the layer-1 flush, the BN-buffer broadcast carried by the all-reduce, no fold-in-update, no
fixed-point sink), so RCCL executes exactly where an 8-GPU run would call it
(reference: src/train.py:29-35 ``init_process_group("nccl")``, :300 DDP; src/jobs/train.sh:48).

At world size 1 every collective is the identity, so:

* each comm helper returns its input bit for bit, and the out-of-place ones (all-gather,
  reduce-scatter) overwrite a NaN-filled output, which proves the RCCL kernel ran;
* the same collectives recorded inside a HIP graph replay correctly (the captured schedule);
* ``TrainStep`` on the forced schedule — RCCL with the collectives captured into the step's
  graph (one all-reduce, and the two-bucket overlap), RCCL with host cuts between graph
  segments, and gloo (host-staged, segmented) — gives parameters, AdamW moments, BN buffers and
  losses bit-identical to the single-process step, for local and global (cfg 5) negatives.

Each case runs in one fresh spawned process (nothing else has touched the GPU there), which
initialises the process group itself on 127.0.0.1.
"""
import importlib
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG_NAME, ROOT
from oracle import two_tower_ref as ref

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(backend):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group(backend, rank=0, world_size=1)


def _entry(rank, fn, args):
    import sys
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    torch.cuda.set_device(0)
    fn(*args)


def _run(fn, *args):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    mp.spawn(_entry, args=(fn, args), nprocs=1, join=True)


# ------------------------------------------------------------------ the collectives
def _collectives_worker():
    pkg = importlib.import_module(PKG_NAME)
    comm = pkg.comm
    _init("nccl")
    try:
        assert dist.get_backend() == "nccl" and not comm.dp_active()
        comm.force_dp(True)
        assert comm.dp_active() and comm.capturable()
        g = torch.Generator(device="cuda").manual_seed(5)
        flat = torch.randn(300_001, device="cuda", generator=g)
        want = flat.clone()
        # GradSync's bucketed asynchronous all-reduce (many buckets, ragged last one)
        sync = pkg.GradSync(bucket_bytes=4 * 65_536)
        assert sync.active and sync.world == 1
        works = sync.start(flat)
        assert len(works) == 5
        for w in works:
            w.wait()
        torch.cuda.synchronize()
        assert torch.equal(flat, want)
        # out-of-place collectives overwrite a NaN output: the RCCL kernel ran
        out = torch.full_like(flat, float("nan"))
        comm.all_gather_into(out, flat)
        torch.cuda.synchronize()
        assert torch.equal(out, want)
        ids = torch.arange(512, device="cuda", dtype=torch.int64)
        oid = torch.full_like(ids, -1)
        comm.all_gather_into(oid, ids)
        assert torch.equal(oid, ids)
        rs = torch.full_like(flat, float("nan"))
        comm.reduce_scatter_sum(rs, flat)
        torch.cuda.synchronize()
        assert torch.equal(rs, want)
        comm.broadcast(flat, 0)
        assert torch.equal(flat, want)
        # the same collectives recorded in a HIP graph (TrainStep's captured schedule)
        x = torch.randn(70_000, device="cuda", generator=g)
        y = torch.full_like(x, float("nan"))
        z = torch.full_like(x, float("nan"))
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            comm.all_reduce_sum(x)                       # warm the communicator off-capture
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        comm.quiesce_before_capture()                    # as TrainStep does before its capture
        graph = torch.cuda.CUDAGraph()
        # thread-local capture, as TrainStep's: the watchdog may query earlier works meanwhile
        with torch.cuda.graph(graph, capture_error_mode="thread_local"):
            x.mul_(2.0)
            ws = pkg.GradSync(bucket_bytes=4 * 16_384).start(x)
            for w in ws:
                w.wait()
            comm.all_gather_into(y, x)
            comm.reduce_scatter_sum(z, y)
            z.add_(1.0)
        x0 = torch.randn(70_000, device="cuda", generator=g)
        x.copy_(x0)
        y.fill_(float("nan"))
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(x, x0 * 2.0) and torch.equal(y, x0 * 2.0) and torch.equal(z, x0 * 2.0 + 1.0)
    finally:
        comm.force_dp(False)
        dist.destroy_process_group()


def test_rccl_collectives_world1_and_captured():
    _run(_collectives_worker)


# ------------------------------------------------------------------ TrainStep's DP schedule
V16, D16, L16, B16, P16, NG, NC = 997, 128, 20, 64, 0.1, 3, 8
STEPS, LR = 3, 1e-3


def _batch(step):
    g = torch.Generator().manual_seed(3000 + 10 * step)
    return ref.synthetic_batch(B16, L16, V16, NG, NC, num_users=20, generator=g)


def _train(pkg, global_negatives, **kw):
    torch.manual_seed(0)
    m = pkg.TwoTowerModel(vocab_size=V16, tabular_input_dim=128, num_genders=NG, num_countries=NC,
                          max_seq_len=L16, user_embedding_dim=D16, item_embedding_dim=D16,
                          user_dropout=P16, compute_dtype=torch.bfloat16,
                          precomputed_modalities=True, global_negatives=global_negatives).cuda()
    m.item_tower.fusion_layer[3].p = P16
    step = pkg.TrainStep(m, lr=LR, use_graph=True, seed=1, **kw)
    losses = []
    for s in range(STEPS):
        b = {k: v.cuda() for k, v in _batch(s).items()}
        losses.append(step.step(b).detach().clone())
    step.check()
    torch.cuda.synchronize()
    st = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    st.update({"m/" + k: v.cpu().clone() for k, v in step.flat.views(step.flat.exp_avg).items()})
    st.update({"v/" + k: v.cpu().clone() for k, v in step.flat.views(step.flat.exp_avg_sq).items()})
    info = (step.dp, step.capture_collectives, step.overlap, step.fold_in_update,
            step.broadcast_buffers, step._cur.seg.n_graphs)
    return st, [float(x) for x in losses], float(step.loss_sum), info


def _trainstep_worker(global_negatives):
    pkg = importlib.import_module(PKG_NAME)
    comm = pkg.comm
    runs = {}
    _init("nccl")
    try:
        runs["single"] = _train(pkg, global_negatives)          # one process, fused schedule
        comm.force_dp(True)
        runs["rccl_captured"] = _train(pkg, global_negatives)   # default: one all-reduce
        runs["rccl_captured_overlap"] = _train(pkg, global_negatives, overlap_grad_sync=True)
        runs["rccl_segmented"] = _train(pkg, global_negatives, capture_collectives=False,
                                        overlap_grad_sync=True)
    finally:
        comm.force_dp(False)
        dist.destroy_process_group()
    _init("gloo")
    try:
        comm.force_dp(True)
        runs["gloo"] = _train(pkg, global_negatives, overlap_grad_sync=True)
    finally:
        comm.force_dp(False)
        dist.destroy_process_group()
    info = {k: v[3] for k, v in runs.items()}
    # (dp, captured collectives, overlap, fold_in_update, broadcast_buffers, graphs per step)
    assert info["single"][:5] == (False, False, False, True, False) and info["single"][5] == 1, info
    assert info["rccl_captured"][:5] == (True, True, False, False, True), info
    assert info["rccl_captured"][5] == 1, info                 # one graph: collectives inside
    assert info["rccl_captured_overlap"][:5] == (True, True, True, False, True), info
    assert info["rccl_captured_overlap"][5] == 1, info
    assert info["rccl_segmented"][:3] == (True, False, True) and info["rccl_segmented"][5] > 1, info
    assert info["gloo"][:3] == (True, False, True) and info["gloo"][5] > 1, info
    base_st, base_l, base_sum, _ = runs["single"]
    assert all(abs(x) < 20 for x in base_l) and base_l[0] == base_l[0]
    for name, (st, losses, lsum, _) in runs.items():
        assert losses == base_l, (name, losses, base_l)
        assert lsum == base_sum, (name, lsum, base_sum)
        bad = [k for k in base_st if not torch.equal(st[k], base_st[k])]
        assert not bad, (name, bad[:8])


@pytest.mark.parametrize("global_negatives", [False, True])
def test_trainstep_forced_dp_schedule_rccl_bitexact(global_negatives):
    _run(_trainstep_worker, global_negatives)


# ------------------------------------------------------------------ capture refused: segments
def _fallback_worker():
    """If recording the collectives into the step graph fails (untested at world > 1 here: RCCL
    needs a device per rank), TrainStep falls back to graph segments with the collectives
    between them instead of failing the run — same bits as the one-process step."""
    pkg = importlib.import_module(PKG_NAME)
    comm = pkg.comm
    _init("nccl")
    real = comm.all_reduce_sum
    try:
        base = _train(pkg, False)

        def refusing(t, *a, **k):
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("collective refused under capture (test)")
            return real(t, *a, **k)
        comm.force_dp(True)
        comm.all_reduce_sum = refusing
        fb = _train(pkg, False)
    finally:
        comm.all_reduce_sum = real
        comm.force_dp(False)
        dist.destroy_process_group()
    info = fb[3]
    assert info[:2] == (True, False) and info[5] > 1, info     # DP, segments, several graphs
    assert fb[1] == base[1] and fb[2] == base[2]
    bad = [k for k in base[0] if not torch.equal(fb[0][k], base[0][k])]
    assert not bad, bad[:8]


def test_captured_collectives_fall_back_to_segments():
    _run(_fallback_worker)


# ------------------------------------------------------------------ a bad id on the DP schedule
def _bad_id_worker():
    pkg = importlib.import_module(PKG_NAME)
    comm = pkg.comm
    _init("nccl")
    try:
        comm.force_dp(True)
        torch.manual_seed(0)
        m = pkg.TwoTowerModel(vocab_size=V16, tabular_input_dim=128, num_genders=NG,
                              num_countries=NC, max_seq_len=L16, user_embedding_dim=D16,
                              item_embedding_dim=D16, user_dropout=P16,
                              compute_dtype=torch.bfloat16, precomputed_modalities=True).cuda()
        step = pkg.TrainStep(m, lr=LR, seed=1)
        assert step.dp and step.flag_off is not None
        step.step({k: v.cuda() for k, v in _batch(0).items()})
        step.check()
        f = step.flat
        before = [t.clone() for t in (f.data, f.exp_avg, f.exp_avg_sq, f.mirror)]
        b = {k: v.cuda() for k, v in _batch(1).items()}
        b["user_country"] = b["user_country"].clone()
        b["user_country"][3] = NC + 2
        step.step(b)
        torch.cuda.synchronize()
        # the flags rode the gradient all-reduce: the summed slot is 1.0, and nothing moved
        assert float(f.grad_extra[step.flag_off + 2]) == 1.0
        for a, t in zip((f.data, f.exp_avg, f.exp_avg_sq, f.mirror), before):
            assert torch.equal(a, t)
        with pytest.raises(IndexError, match="user_country"):
            step.check()
        step.step({k: v.cuda() for k, v in _batch(2).items()})
        step.check()
        assert not torch.equal(f.data, before[0])
    finally:
        comm.force_dp(False)
        dist.destroy_process_group()


def test_dp_schedule_bad_id_skips_update_on_every_rank():
    _run(_bad_id_worker)


# ------------------------------------------------------------------ cfg 3 on the DP schedule
def _train3(pkg, **kw):
    from oracle import resnet_ref as rref
    torch.manual_seed(7)
    m = pkg.TwoTowerModel(with_text=False, vocab_size=211, tabular_input_dim=32, num_genders=3,
                          num_countries=8, max_seq_len=12, user_embedding_dim=128,
                          item_embedding_dim=128, user_dropout=0.1,
                          precomputed_modalities=False).cuda()
    m.item_tower.fusion_layer[3].p = 0.1
    m.item_tower.tabular_encoder.mlp[3].p = 0.1
    g = torch.Generator().manual_seed(8)
    batch = ref.synthetic_batch(8, 12, 211, num_countries=8, generator=g)
    del batch["target_modal"]
    batch.update(rref.synthetic_items(8, 32, (64, 96), (64, 64), generator=g))
    b = {k: v.cuda() for k, v in batch.items()}
    step = pkg.TrainStep(m, lr=1e-3, seed=11, **kw)
    losses = [float(step.step(b)) for _ in range(2)]
    step.check()
    torch.cuda.synchronize()
    st = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    st["__m"], st["__v"] = step.flat.exp_avg.cpu().clone(), step.flat.exp_avg_sq.cpu().clone()
    return st, losses, step.dp


def _cfg3_worker():
    pkg = importlib.import_module(PKG_NAME)
    comm = pkg.comm
    _init("nccl")
    try:
        sa, la, dpa = _train3(pkg)
        comm.force_dp(True)
        sb, lb, dpb = _train3(pkg)
    finally:
        comm.force_dp(False)
        dist.destroy_process_group()
    assert not dpa and dpb
    assert la == lb, (la, lb)
    bad = [k for k in sa if not torch.equal(sa[k], sb[k])]
    assert not bad, bad[:8]


def test_cfg3_forced_dp_schedule_rccl_bitexact():
    """BASELINE configs[2] (ResNet-18 audio / visual + tabular item tower, BatchNorm2d in train
    mode, dropout on) on the RCCL data-parallel schedule: bit-identical to the one-process step
    (parameters, BN running buffers, AdamW moments, losses)."""
    _run(_cfg3_worker)

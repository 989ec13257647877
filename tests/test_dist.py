"""Multi-process (world_size 2, gloo, CPU) tests of the data-parallel pieces.

* GradSync: the 1/world loss scale + bucketed SUM all-reduce of the flat gradient buffer
  equals DDP's average (reference train.py:300), over buckets smaller than the buffer.
* comm's asynchronous gloo staging: ``GradSync.start`` returns before the peer has issued
  its buckets (the overlap is real), later collectives drain the pending ones first.
* Global negatives (BASELINE cfg 5): the per-rank decomposition the GPU path implements
  (all-gather û, î, user_idx; rank r scores its rows against every rank's; key grads summed
  back to their owners) reproduces the reference InfoNCE on the concatenated batch — loss and
  embedding gradients.  The per-rank math is the oracle restatement (oracle.infonce_rank);
  the collectives are real.  Gloo has no reduce_scatter, so the owner-sum is an all_reduce
  followed by the owner's slice (same result as reduce_scatter_tensor on RCCL).
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import two_tower_ref as ref

WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(fn, *args):
    port = _free_port()
    mp.spawn(_entry, args=(fn, port, args), nprocs=WORLD, join=True)


def _entry(rank, fn, port, args):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        torch.set_num_threads(1)
        fn(rank, *args)
    finally:
        dist.destroy_process_group()


def _grad_sync_worker(rank):
    import importlib
    pkg = importlib.import_module("music-recommendation-multimodal_amd")
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(37, 19), torch.nn.Linear(19, 5))
    flat = pkg.FlatParams(model)
    # params are views into the flat buffer, in the same slots for grads
    views = flat.views(flat.grad)
    for n, p in model.named_parameters():
        assert p.data.data_ptr() == flat.views(flat.data)[n].data_ptr()
    g = torch.Generator().manual_seed(100 + rank)
    local = torch.randn(flat.numel, generator=g)
    sync = pkg.GradSync(bucket_bytes=64 * 4)                 # many buckets
    assert sync.world == WORLD and abs(sync.loss_scale - 1.0 / WORLD) < 1e-12
    flat.grad.copy_(local * sync.loss_scale)                 # the step pre-scales dloss
    sync(flat.grad)
    every = [torch.randn(flat.numel, generator=torch.Generator().manual_seed(100 + r))
             for r in range(WORLD)]
    expect = sum(every) / WORLD
    assert torch.allclose(flat.grad, expect, atol=1e-6)
    assert set(views) == {n for n, _ in model.named_parameters()}


def test_grad_sync_averages_over_buckets():
    _run(_grad_sync_worker)


def _async_staged_worker(rank):
    """comm's asynchronous staging (the gloo path of a device gradient, here forced on host
    tensors): ``start`` returns while the peer has not even issued its buckets, the buckets
    reduce in issue order, and a later collective drains them first."""
    import importlib
    import time
    pkg = importlib.import_module("music-recommendation-multimodal_amd")
    comm = pkg.comm
    comm._FORCE_STAGE = True
    try:
        g = torch.Generator().manual_seed(100 + rank)
        flat = torch.randn(1000, generator=g)
        every = [torch.randn(1000, generator=torch.Generator().manual_seed(100 + r))
                 for r in range(WORLD)]
        sync = pkg.GradSync(bucket_bytes=96 * 4)
        if rank == 1:
            time.sleep(1.0)                      # rank 0's reductions cannot finish before this
        t0 = time.perf_counter()
        works = sync.start(flat)
        issued = time.perf_counter() - t0
        if rank == 0:
            assert issued < 0.5, issued          # did not wait for the peer
            assert not any(w.is_completed() for w in works)
        # a collective issued meanwhile drains the staged buckets first (same order on both)
        tag = torch.tensor([float(rank)])
        comm.broadcast(tag, 0)
        assert all(w.is_completed() for w in works) and float(tag) == 0.0
        for w in works:
            w.wait()
        assert torch.allclose(flat, sum(every), atol=1e-6)
        # the synchronous path agrees bit for bit
        again = every[rank].clone()
        comm.all_reduce_sum(again)
        assert torch.equal(again, flat)
    finally:
        comm._FORCE_STAGE = False


def test_async_staged_all_reduce_overlaps():
    _run(_async_staged_worker)


def _global_negatives_worker(rank, B, D, collide):
    g = torch.Generator().manual_seed(7)
    u_all = torch.randn(WORLD * B, D, generator=g, dtype=torch.float64)
    i_all = torch.randn(WORLD * B, D, generator=g, dtype=torch.float64)
    uid_all = torch.randint(0, 3 * B if collide else 10**6, (WORLD * B,), generator=g)
    sl = slice(rank * B, (rank + 1) * B)
    u = u_all[sl].clone().requires_grad_(True)
    it = i_all[sl].clone().requires_grad_(True)
    # --- the distributed algorithm (as functional.infonce_global_fwd/bwd run it)
    uh = torch.nn.functional.normalize(u, dim=1)
    ih = torch.nn.functional.normalize(it, dim=1)
    U = [torch.empty_like(uh) for _ in range(WORLD)]
    I = [torch.empty_like(ih) for _ in range(WORLD)]
    UID = [torch.empty_like(uid_all[sl]) for _ in range(WORLD)]
    dist.all_gather(U, uh.detach())
    dist.all_gather(I, ih.detach())
    dist.all_gather(UID, uid_all[sl].clone())
    U = torch.cat(U).requires_grad_(True)
    I = torch.cat(I).requires_grad_(True)
    UID = torch.cat(UID)
    loss_r = ref.infonce_rank(uh, ih, U, I, uid_all[sl], UID, rank * B)
    # DDP's 1/world scaling of each rank's loss
    duh, dih, dU, dI = torch.autograd.grad(loss_r / WORLD, [uh, ih, U, I])
    dist.all_reduce(dU)                    # reduce-scatter: owner takes its slice of the sum
    dist.all_reduce(dI)
    torch.autograd.backward([uh, ih], [duh + dU[sl], dih + dI[sl]])
    loss_mean = loss_r.detach().clone()
    dist.all_reduce(loss_mean)
    loss_mean /= WORLD
    # --- the reference on the concatenated global batch
    ua = u_all.clone().requires_grad_(True)
    ia = i_all.clone().requires_grad_(True)
    lref, _, _, _ = ref.infonce(ua, ia, uid_all)
    lref.backward()
    assert abs(float(loss_mean) - float(lref)) < 1e-12
    assert torch.allclose(u.grad, ua.grad[sl], atol=1e-12)
    assert torch.allclose(it.grad, ia.grad[sl], atol=1e-12)


@pytest.mark.parametrize("collide", [False, True])
def test_global_negatives_decomposition(collide):
    _run(_global_negatives_worker, 16, 8, collide)


def test_flat_params_excludes_frozen_text_base():
    """peft freezes the DeBERTa base: FlatParams (and so AdamW) hold only trainable tensors."""
    import importlib
    pkg = importlib.import_module("music-recommendation-multimodal_amd")
    tcfg = pkg.text.TextCfg(vocab_size=50, hidden=64, layers=1, heads=1, intermediate=128)
    m = pkg.TwoTowerModel(vocab_size=31, tabular_input_dim=8, user_embedding_dim=64,
                          item_embedding_dim=64, precomputed_modalities=False, with_text=True,
                          text_cfg=tcfg)
    flat = pkg.FlatParams(m)
    trainable = [n for n, p in m.named_parameters() if p.requires_grad]
    assert flat.names == trainable
    assert any("lora_A" in n for n in flat.names)
    assert not any("text_encoder.transformer" in n and "lora_" not in n for n in flat.names)
    keys = m.state_dict().keys()
    assert "item_tower.text_encoder.transformer.base_model.model.encoder.layer.0.attention.self." \
           "query_proj.lora_B.default.weight" in keys
    assert "item_tower.text_encoder.projection.3.weight" in keys


def test_reference_checkpoint_roundtrip(tmp_path):
    """a reference-keyed checkpoint saved by DDP (``module.`` prefix,
    train.py:329) loads into the framework with dimensions inferred as inference.py:109-128
    does, through torch.load(weights_only=True)."""
    import importlib
    from conftest import load_golden, sub
    pkg = importlib.import_module("music-recommendation-multimodal_amd")
    z = load_golden("train_step.npz")
    V, D, L, B, n_g, n_c, _ = z["cfg"].tolist()
    ref_sd = {"module." + k: torch.tensor(v) for k, v in sub(z, "p0/").items()}
    path = str(tmp_path / "ckpt.pth")
    torch.save(ref_sd, path)
    m = pkg.retrieval.model_from_reference_checkpoint(path, vocab_size=V, num_genders=n_g,
                                                      max_seq_len=L, use_lora=False)
    sd = m.state_dict()
    for k, v in ref_sd.items():
        assert torch.equal(sd[k[len("module."):]].cpu(), v), k
    assert m.user_tower.country_embedding.weight.shape[0] == n_c


def test_reference_checkpoint_infers_dims(tmp_path):
    """Vocabulary, genders, countries, history length, encoder depth and (with a text
    encoder) the DeBERTa shape all come from the checkpoint: a full multimodal state_dict
    with several gender classes round-trips with no dimension passed."""
    import importlib
    pkg = importlib.import_module("music-recommendation-multimodal_amd")
    tcfg = pkg.text.TextCfg(vocab_size=50, hidden=128, layers=2, heads=2, intermediate=256,
                            position_buckets=32)
    torch.manual_seed(0)
    src = pkg.TwoTowerModel(vocab_size=37, tabular_input_dim=9, num_genders=3, num_countries=5,
                            max_seq_len=20, user_embedding_dim=64, item_embedding_dim=64,
                            user_num_layers=3, text_cfg=tcfg)
    path = str(tmp_path / "ckpt.pth")
    torch.save({"module." + k: v for k, v in src.state_dict().items()}, path)
    m = pkg.retrieval.model_from_reference_checkpoint(path)
    assert m.item_tower.with_text and not m.item_tower.precomputed_modalities
    assert m.user_tower.num_layers == 3 and m.user_tower.max_seq_len == 20
    got = m.state_dict()
    for k, v in src.state_dict().items():
        assert torch.equal(got[k], v), k


def _forced_dp_world1_worker(rank):
    """comm.force_dp at world size 1 (the RCCL rehearsal's schedule, here on gloo / CPU): every
    helper runs its collective (identity at one rank), GradSync reports itself active, and
    without force_dp a world-1 group keeps the one-process short cuts."""
    import importlib
    pkg = importlib.import_module("music-recommendation-multimodal_amd")
    comm = pkg.comm
    assert dist.get_world_size() == 1 and not comm.dp_active()
    assert not pkg.GradSync().active
    comm.force_dp(True)
    try:
        assert comm.dp_active() and pkg.GradSync().active and not comm.capturable()
        g = torch.Generator().manual_seed(3)
        x = torch.randn(1001, generator=g)
        want = x.clone()
        works = pkg.GradSync(bucket_bytes=4 * 100).start(x)
        assert len(works) == 11
        for w in works:
            w.wait()
        assert torch.equal(x, want)
        out = torch.full((1001,), float("nan"))
        comm.all_gather_into(out, x)
        assert torch.equal(out, want)
        rs = torch.full((1001,), float("nan"))
        comm.reduce_scatter_sum(rs, x)
        assert torch.equal(rs, want)
        comm.broadcast(x, 0)
        assert torch.equal(x, want)
    finally:
        comm.force_dp(False)
    assert not comm.dp_active()


def test_forced_dp_schedule_at_world1():
    port = _free_port()
    mp.spawn(_forced_dp_world1_entry, args=(port,), nprocs=1, join=True)


def _forced_dp_world1_entry(rank, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        torch.set_num_threads(1)
        _forced_dp_world1_worker(rank)
    finally:
        dist.destroy_process_group()


def _staged_timeout_worker(rank):
    """A staged reduction whose peer is late past TTMI_GLOO_TIMEOUT: wait() raises, and the stager
    refuses later work at once (its worker thread may still be inside the stuck reduction and
    write the pinned buffer later)."""
    import concurrent.futures
    import importlib
    import time
    pkg = importlib.import_module("music-recommendation-multimodal_amd")
    comm = pkg.comm
    comm._FORCE_STAGE = True
    old = comm.STAGED_TIMEOUT_S
    try:
        x = torch.ones(64)
        dist.barrier()                            # both ranks imported: the 1.5 s lateness is relative
        if rank == 0:
            comm.STAGED_TIMEOUT_S = 0.3
            works = pkg.GradSync().start(x)
            with pytest.raises(concurrent.futures.TimeoutError):
                works[0].wait()
            with pytest.raises(RuntimeError, match="timed out earlier"):
                pkg.GradSync().start(x)
            with pytest.raises(RuntimeError, match="timed out earlier"):
                works[0].wait()
        else:
            time.sleep(1.5)                       # late: rank 0's wait gave up meanwhile
            dist.all_reduce(x)                    # completes rank 0's stuck reduction
        dist.barrier()
        if rank == 0:                             # the stuck reduction's thread has returned from
            works[0].fut.result(timeout=60)       # gloo before the group is torn down
    finally:
        comm.STAGED_TIMEOUT_S = old
        comm._FORCE_STAGE = False


def test_staged_all_reduce_timeout_breaks_the_stager():
    _run(_staged_timeout_worker)

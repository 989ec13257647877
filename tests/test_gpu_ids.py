"""Embedding ids outside their tables (reference nn.Embedding raises IndexError,
src/models/user_tower.py:26,30-31) on every batch and every path, without a GPU fault and without
a host sync per step: the device lookups clamp the id and set a device + host-mapped flag
(include/ttmi.h TTMI_IDERR_*, ABI 22); TrainStep.step() / the module forward raise at their
start for an earlier finished launch, TrainStep.check() and train_one_epoch (right after the
forward) right away.  As the reference raises before optimizer.step(), a bad step updates no
parameter: TrainStep's AdamW reads the device flags and skips (parameters, moments and the bf16
mirror bit-identical afterwards), train_one_epoch raises before backward."""
import ctypes

import pytest
import torch

from oracle import two_tower_ref as ref

DEV = "cuda:0"
V, L, B = 997, 50, 64
pytestmark = pytest.mark.gpu


def _model(pkg, dtype=torch.bfloat16, p=0.1):
    torch.manual_seed(0)
    m = pkg.TwoTowerModel(precomputed_modalities=True, vocab_size=V, tabular_input_dim=128,
                          num_genders=3, num_countries=64, max_seq_len=L, user_embedding_dim=128,
                          item_embedding_dim=128, user_dropout=p, compute_dtype=dtype).to(DEV)
    return m


def _batch(seed, key=None, bad=None):
    g = torch.Generator().manual_seed(seed)
    b = {k: v.to(DEV) for k, v in ref.synthetic_batch(B, L, V, generator=g).items()}
    if key is not None:
        t = b[key].clone()
        if key == "history_ids":
            t[5, 0] = bad              # position 0 is inside every history (lengths >= 1)
        else:
            t[5] = bad
        b[key] = t
    return b


BAD = [("user_gender", 3), ("user_country", 64), ("history_ids", V), ("user_gender", -1),
       ("user_country", 1 << 40)]


@pytest.mark.parametrize("key,bad", BAD)
@pytest.mark.parametrize("use_graph", [True, False])
def test_trainstep_bad_id_in_a_later_batch_of_a_captured_shape(gpu_pkg, key, bad, use_graph):
    m = _model(gpu_pkg)
    step = gpu_pkg.TrainStep(m, use_graph=use_graph)
    step.step(_batch(1))                    # this shape's graph is captured here
    step.check()
    step.step(_batch(2, key, bad))          # same shape: replays the captured graph
    with pytest.raises(IndexError, match=key):
        step.check()
    step.check()                            # the flags were cleared by the raise
    step.step(_batch(3))
    step.check()
    assert all(torch.isfinite(p).all() for p in m.parameters())


@pytest.mark.parametrize("key,bad", BAD[:3])
def test_trainstep_next_step_raises_without_sync(gpu_pkg, key, bad):
    m = _model(gpu_pkg)
    step = gpu_pkg.TrainStep(m, use_graph=True)
    step.step(_batch(1))
    step.step(_batch(2, key, bad))
    torch.cuda.synchronize()                # the bad step has finished ...
    with pytest.raises(IndexError, match=key):
        step.step(_batch(3))                # ... so the next step() raises at its start


@pytest.mark.parametrize("key,bad", BAD[:3])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_module_forward_bad_id(gpu_pkg, key, bad, dtype):
    m = _model(gpu_pkg, dtype)
    loss, _, _, _ = m(_batch(1))
    loss.backward()
    loss, _, _, _ = m(_batch(2, key, bad))  # runs on the clamped id, no fault
    loss.backward()
    assert torch.isfinite(loss).all()
    torch.cuda.synchronize()
    with pytest.raises(IndexError, match=key):
        m(_batch(3))
    with torch.no_grad():                   # cleared: eval helpers run again
        u = m.get_user_embedding(_batch(3)["history_ids"])
    assert torch.isfinite(u).all()


def test_train_one_epoch_raises_at_the_bad_batch(gpu_pkg):
    m = _model(gpu_pkg)
    opt = torch.optim.AdamW(m.parameters(), lr=1e-4)
    gpu_pkg.train.train_one_epoch(m, [_batch(1)], opt, DEV, epoch=0)
    before = {k: v.detach().clone() for k, v in m.named_parameters()}
    loader = [_batch(2, "user_country", 64), _batch(3)]
    with pytest.raises(IndexError, match="user_country"):
        gpu_pkg.train.train_one_epoch(m, loader, opt, DEV, epoch=0)
    for k, v in m.named_parameters():       # raised before backward / optimizer.step()
        assert torch.equal(v.detach(), before[k]), k


def _flat_state(step):
    f = step.flat
    return [t.detach().clone() for t in (f.data, f.exp_avg, f.exp_avg_sq) +
            ((f.mirror,) if f.mirror is not None else ())]


@pytest.mark.parametrize("key,bad", BAD[:3] + [("history_ids", -7)])
@pytest.mark.parametrize("use_graph", [True, False])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_trainstep_bad_batch_updates_nothing(gpu_pkg, key, bad, use_graph, dtype):
    """AdamW's skip_if: the step that met the bad id leaves parameters, moments and the bf16
    mirror bit-identical (also the fixed-point item-embedding gradient and the folded weight
    gradients are consumed, so the next good step is exactly a normal step)."""
    m = _model(gpu_pkg, dtype)
    step = gpu_pkg.TrainStep(m, use_graph=use_graph)
    step.step(_batch(1))
    step.check()
    before = _flat_state(step)
    step.step(_batch(2, key, bad))
    torch.cuda.synchronize()
    for a, b in zip(_flat_state(step), before):
        assert torch.equal(a, b)
    assert not step.flat.grad.any()          # the gradient was still cleared
    with pytest.raises(IndexError, match=key):
        step.check()
    step.step(_batch(3))                     # a good step updates again
    step.check()
    assert not torch.equal(step.flat.data, before[0])
    # ... exactly as a run that never saw the bad batch (Adam's step count aside, which the
    # skipped step advanced): compare against a twin stepped on batches 1 and 3 only, with its
    # step counter advanced once
    twin_m = _model(gpu_pkg, dtype)
    twin = gpu_pkg.TrainStep(twin_m, use_graph=use_graph)
    twin.step(_batch(1))
    torch.cuda.synchronize()
    twin.step_t.add_(1)
    twin.step(_batch(3))
    twin.check()
    # dropout seeds are drawn from (seed, step count): the same masks in both runs.  (The fp32
    # path's split-K weight gradients add with float atomics, so only bf16 is bit-reproducible.)
    if dtype == torch.bfloat16:
        for a, b in zip(_flat_state(step), _flat_state(twin)):
            assert torch.equal(a, b)


def test_catalogue_indexer_bad_target_id(gpu_pkg):
    m = _model(gpu_pkg, p=0.0)
    g = torch.Generator().manual_seed(4)
    modal = torch.randn(B, 512, generator=g).to(DEV)
    ids = torch.arange(1, B + 1, device=DEV)
    ids[7] = V + 5
    ix = gpu_pkg.retrieval.CatalogueIndexer(m, V)
    with pytest.raises(IndexError, match="target_id"):
        ix.index([{"target_id": ids, "target_modal": modal}])
    assert torch.isfinite(ix.dense).all()


def test_flags_are_host_mapped(gpu_pkg):
    """The flags are read without a device sync: the hipHostMalloc mapping was accepted."""
    ops = gpu_pkg.ops
    ops.id_err_ptr(torch.empty(1, device=DEV))
    f = ops._IDF[torch.device(DEV).index]
    assert f.host is not None and f.dptr is not None
    assert isinstance(f.host, ctypes.Array)
    # the device block's pointer slot (byte 32) holds the host array's device address
    assert int(f.dev.view(torch.int64)[4]) != 0

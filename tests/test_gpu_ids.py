"""Embedding ids outside their tables (reference nn.Embedding raises IndexError,
src/models/user_tower.py:26,30-31) on every batch and every path, without a GPU fault and without
a host sync per step: the device lookups clamp the id and set a host-mapped flag
(include/ttmi.h TTMI_IDERR_*); TrainStep.step() / the module forward raise at their start for an
earlier finished launch, TrainStep.check() and train_one_epoch (after loss.item()) right away."""
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
    loader = [_batch(1), _batch(2, "user_country", 64), _batch(3)]
    with pytest.raises(IndexError, match="user_country"):
        gpu_pkg.train.train_one_epoch(m, loader, opt, DEV, epoch=0)


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

"""Global retrieval on the GPU: the radix-select top-K kernel against
torch.topk (values exact, indices exact when scores are distinct; ties resolved to the lower
index), the padding-column exclusion, and the full metrics path against the metrics the
reference's calculate_metrics_global produced (tests/golden/retrieval.npz).  Ranks are
integers: a fp32 summation-order difference may flip a near-tie, so the metrics are allowed
one user's worth of difference."""
import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("R,V,K", [(7, 100, 10), (33, 10136, 20), (5, 3001, 64), (3, 64, 64), (4, 16384, 20),
                                    (4, 16385, 20), (3, 40000, 50)])
def test_topk_rows_vs_torch(gpu_pkg, R, V, K):
    ops = gpu_pkg.ops
    g = torch.Generator().manual_seed(V + K)
    s = torch.randn(R, V, generator=g)
    val = torch.empty(R, K, device=DEV)
    idx = torch.empty(R, K, device=DEV, dtype=torch.int64)
    ops.topk_rows(s.to(DEV), K, val, idx)
    rv, ri = torch.topk(s, K, dim=1)
    assert torch.equal(val.cpu(), rv)
    assert torch.equal(idx.cpu(), ri)
    # padding column excluded
    s2 = s.clone()
    s2[:, 0] = 100.0
    ops.topk_rows(s2.to(DEV), K, val, idx, skip_first=True)
    s3 = s2.clone()
    s3[:, 0] = -float("inf")
    rv, ri = torch.topk(s3, K, dim=1)
    assert torch.equal(idx.cpu(), ri) and torch.equal(val.cpu(), rv)


@pytest.mark.parametrize("V", [10136, 30000])
def test_topk_rows_one_exponent(gpu_pkg, V):
    """Scores in [1, 2): one exponent, so the first radix digit is the same for every key and
    the histogram's wave aggregation carries the whole pass (LDS-staged and global rows)."""
    ops = gpu_pkg.ops
    g = torch.Generator().manual_seed(V)
    s = 1.0 + torch.rand(6, V, generator=g)
    val = torch.empty(6, 20, device=DEV)
    idx = torch.empty(6, 20, device=DEV, dtype=torch.int64)
    ops.topk_rows(s.to(DEV), 20, val, idx, skip_first=True)
    s[:, 0] = -float("inf")
    nv, ri = torch.sort(-s, dim=1, stable=True)         # ties (a few here): lower index first
    assert torch.equal(val.cpu(), -nv[:, :20]) and torch.equal(idx.cpu(), ri[:, :20])


def test_topk_rows_ties_lower_index_first(gpu_pkg):
    ops = gpu_pkg.ops
    s = torch.zeros(2, 500)
    s[0, 10:20] = 1.0           # 10 tied best
    s[1, ::7] = 2.0             # 72 tied best, K = 16
    val = torch.empty(2, 16, device=DEV)
    idx = torch.empty(2, 16, device=DEV, dtype=torch.int64)
    ops.topk_rows(s.to(DEV), 16, val, idx)
    assert idx[0, :10].cpu().tolist() == list(range(10, 20))
    assert idx[0, 10:].cpu().tolist() == list(range(0, 6))          # then the zeros, in order
    assert idx[1].cpu().tolist() == list(range(0, 7 * 16, 7))


def test_retrieval_metrics_vs_reference_fixture(gpu_pkg):
    retrieval = gpu_pkg.retrieval
    z = load_golden("retrieval.npz")
    users, items = torch.tensor(z["users"]).to(DEV), torch.tensor(z["items"]).to(DEV)
    targets = torch.tensor(z["targets"]).to(DEV)
    n = users.shape[0]

    class Stub:
        def __init__(self):
            self.i = 0

        def eval(self):
            return self

        def get_user_embedding(self, history_ids, history_mask, user_gender, user_country):
            out = users[self.i:self.i + history_ids.shape[0]]
            self.i += history_ids.shape[0]
            return out
    B = 48
    loader = [{"history_ids": torch.ones(B, 5, dtype=torch.long),
               "history_mask": torch.ones(B, 5, dtype=torch.long),
               "user_gender": torch.zeros(B, dtype=torch.long),
               "user_country": torch.zeros(B, dtype=torch.long),
               "target_id": targets[b * B:(b + 1) * B].cpu()} for b in range(n // B)]
    res = retrieval.calculate_metrics_global(Stub(), loader, items, DEV, k_list=[10, 20])
    for k, v in res.items():
        assert abs(v - float(z["metric/" + k])) <= 1.0 / n + 1e-6, (k, v, float(z["metric/" + k]))


def test_global_evaluator_graph_matches_eager(gpu_pkg):
    """GlobalEvaluator's graph replay vs the eager path: two batches of one size (one capture,
    restaged inputs), a batch of another size (a second capture), and a replay after an in-place
    weight update (the cached bf16 operands are refreshed into the captured buffers)."""
    torch.manual_seed(0)
    V, D = 2000, 128
    m = gpu_pkg.TwoTowerModel(precomputed_modalities=True, vocab_size=V, tabular_input_dim=128, num_genders=3, num_countries=8,
                              max_seq_len=50, user_embedding_dim=D, item_embedding_dim=D,
                              user_num_heads=4, compute_dtype=torch.bfloat16).to(DEV).eval()
    g = torch.Generator().manual_seed(2)
    items = torch.nn.functional.normalize(torch.randn(V, D, generator=g), dim=1).to(DEV)

    def batch(B):
        lens = torch.randint(1, 51, (B,), generator=g)
        ids = torch.randint(1, V, (B, 50), generator=g)
        ids[torch.arange(50)[None, :] >= lens[:, None]] = 0
        return {"history_ids": ids, "history_mask": (ids != 0).long(),
                "user_gender": torch.randint(0, 3, (B,), generator=g),
                "user_country": torch.randint(0, 8, (B,), generator=g),
                "target_id": torch.randint(1, V, (B,), generator=g)}
    rt = gpu_pkg.retrieval
    ev = rt.GlobalEvaluator(m, items, 20)
    eager = rt.GlobalEvaluator(m, items, 20, use_graph=False)
    assert ev.use_graph
    for b in (batch(64), batch(64), batch(37)):
        # targets taken from the eager top-20 so the ranks are informative
        with torch.no_grad():
            u = m.get_user_embedding(b["history_ids"].to(DEV), b["history_mask"].to(DEV),
                                     b["user_gender"].to(DEV), b["user_country"].to(DEV))
        top = rt.topk_items(u, items, 20)[1].cpu()
        b["target_id"][::2] = top[::2, 5]
        r_graph = ev.ranks(b).clone()
        assert torch.equal(r_graph.cpu(), eager.ranks(b).cpu())
        assert (r_graph[::2] < 20).float().mean() > 0.9
    assert len(ev._graphs) == 2
    with torch.no_grad():
        m.user_tower.transformer_encoder.layers[0].linear1.weight.mul_(-1.0)
        m.user_tower.fusion_layer[3].weight.mul_(0.5)
    b = batch(64)
    assert torch.equal(ev.ranks(b).cpu(), eager.ranks(b).cpu())
    assert len(ev._graphs) == 2


def test_recommend_matches_oracle_inference(gpu_pkg):
    """Serving (inference.py:254-310): last-50 history, normalised user embedding, padding and
    history excluded, top-10 — fp32 model vs the oracle's user tower + torch ops."""
    from oracle import two_tower_ref as ref
    torch.manual_seed(0)
    V, D, L = 997, 64, 60
    m = gpu_pkg.TwoTowerModel(precomputed_modalities=True, vocab_size=V, tabular_input_dim=128, num_genders=3, num_countries=8,
                              max_seq_len=50, user_embedding_dim=D, item_embedding_dim=D,
                              compute_dtype=torch.float32).to(DEV)
    g = torch.Generator().manual_seed(1)
    hist = torch.randint(1, V, (6, L), generator=g)
    hist[2, :30] = 0                                         # left part padding
    gender = torch.randint(0, 3, (6,), generator=g)
    country = torch.randint(0, 8, (6,), generator=g)
    items = torch.nn.functional.normalize(torch.randn(V, D, generator=g), dim=1)
    val, idx = gpu_pkg.retrieval.recommend(m, hist.to(DEV), items.to(DEV), k=10,
                                           user_gender=gender.to(DEV), user_country=country.to(DEV))
    p = {k[len("user_tower."):]: v.detach().cpu() for k, v in m.named_parameters()
         if k.startswith("user_tower.")}
    h = hist[:, -50:]
    u = ref.user_tower_forward(p, h, gender, country, None, 4, 2)
    u = torch.nn.functional.normalize(torch.nn.functional.normalize(u, dim=1), p=2, dim=1, eps=1e-8)
    s = u @ items.t()
    s[:, 0] = -float("inf")
    for r in range(6):
        s[r, h[r]] = -float("inf")
    rv, ri = torch.topk(s, 10, dim=1)
    assert torch.equal(idx.cpu(), ri)
    assert torch.allclose(val.cpu(), rv, atol=1e-4)
    assert not any(int(i) in set(h[r].tolist()) for r in range(6) for i in idx[r].cpu())


def test_global_evaluator_after_trainstep_rehomes_params(gpu_pkg):
    """An evaluator built BEFORE TrainStep (which re-homes every parameter into its flat
    buffer, new storages) and used again after training steps scores with the trained weights:
    its graphs are keyed by the cached operand buffers and recaptured when they change."""
    from oracle import two_tower_ref as ref
    torch.manual_seed(0)
    V, D = 500, 128
    m = gpu_pkg.TwoTowerModel(precomputed_modalities=True, vocab_size=V, tabular_input_dim=128,
                              num_genders=3, num_countries=8, max_seq_len=50,
                              user_embedding_dim=D, item_embedding_dim=D).to(DEV)
    g = torch.Generator().manual_seed(4)
    items = torch.nn.functional.normalize(torch.randn(V, D, generator=g), dim=1).to(DEV)
    rt = gpu_pkg.retrieval
    ev = rt.GlobalEvaluator(m, items, 20)
    b = ref.synthetic_batch(64, 50, V, 3, 8, generator=g)
    b["target_id"] = torch.randint(1, V, (64,), generator=g)
    ev.ranks(b)
    step = gpu_pkg.TrainStep(m, lr=1e-2)
    m.train()
    tb = {k: v.to(DEV) for k, v in ref.synthetic_batch(64, 50, V, 3, 8, generator=g).items()}
    for _ in range(3):
        step.step(tb)
    torch.cuda.synchronize()
    eager = rt.GlobalEvaluator(m, items, 20, use_graph=False)
    with torch.no_grad():
        u = m.get_user_embedding(b["history_ids"].to(DEV), b["history_mask"].to(DEV),
                                 b["user_gender"].to(DEV), b["user_country"].to(DEV))
    b["target_id"][::2] = rt.topk_items(u, items, 20)[1].cpu()[::2, 3]
    got = ev.ranks(b).clone()
    assert torch.equal(got.cpu(), eager.ranks(b).cpu())
    assert (got[::2] < 20).float().mean() > 0.9


def _oracle_index(item_out, ids, V):
    e = torch.nn.functional.normalize(item_out, dim=1)                    # get_item_embedding
    e = torch.nan_to_num(e, nan=0.0)
    e = torch.nn.functional.normalize(e, p=2, dim=1, eps=1e-8)
    dense = torch.zeros(V, e.shape[1])
    dense[ids] = e
    return dense


def _randomise_bn(m, g):
    with torch.no_grad():
        for n, b in m.named_buffers():
            if n.endswith("running_mean"):
                b.copy_(torch.randn(b.shape, generator=g) * 0.1)
            elif n.endswith("running_var"):
                b.copy_(0.5 + torch.rand(b.shape, generator=g))


@pytest.mark.parametrize("use_graph", [True, False])
def test_catalogue_indexer_precomputed_vs_oracle(gpu_pkg, use_graph):
    """compute_all_item_embeddings / index_catalog (evaluate_metrics.py:24-104): fp32 fusion head
    in eval mode (BatchNorm on running statistics), three batches (8, 8, 5 items; a ragged
    last batch gets its own graph), 15 ids never indexed: rows match the oracle to 1e-5, row 0
    and unseen rows are 0, and a second pass is bit-identical."""
    from oracle import two_tower_ref as ref
    torch.manual_seed(0)
    V, D = 37, 64
    m = gpu_pkg.TwoTowerModel(precomputed_modalities=True, vocab_size=V, tabular_input_dim=128,
                              user_embedding_dim=D, item_embedding_dim=D,
                              compute_dtype=torch.float32).to(DEV)
    g = torch.Generator().manual_seed(6)
    _randomise_bn(m, g)
    ids = torch.randperm(V - 1, generator=g)[:21] + 1
    modal = torch.randn(21, 512, generator=g)
    loader = [{"target_id": ids[s:s + 8], "target_modal": modal[s:s + 8]} for s in (0, 8, 16)]
    ix = gpu_pkg.retrieval.CatalogueIndexer(m, V, use_graph=use_graph)
    dense = ix.index(loader).clone()
    p = {k[len("item_tower."):]: v.detach().cpu() for k, v in m.named_parameters()
         if k.startswith("item_tower.")}
    running = {k[len("item_tower.fusion_layer.1."):]: v.detach().cpu()
               for k, v in m.named_buffers() if k.startswith("item_tower.fusion_layer.1.")}
    out = ref.item_fusion_forward(p, modal, running=running, eval_mode=True)
    want = _oracle_index(out, ids, V)
    assert (dense[0] == 0).all()
    seen = torch.zeros(V, dtype=torch.bool)
    seen[ids] = True
    assert (dense.cpu()[~seen] == 0).all()
    assert (dense.cpu() - want).abs().max().item() < 1e-5
    again = ix.index(loader)
    assert torch.equal(again, dense)
    if use_graph:
        assert len(ix._graphs) == 2


def test_catalogue_indexer_follows_rehomed_parameters(gpu_pkg):
    """Graphs captured before a TrainStep re-homes the item tower's parameters and buffers into
    its flat storage (and trains them) must not replay the freed old storage: the index after
    training equals a fresh indexer's (key the graph cache on the operand
    storages)."""
    torch.manual_seed(1)
    V, D = 37, 64
    m = gpu_pkg.TwoTowerModel(precomputed_modalities=True, vocab_size=V, tabular_input_dim=128,
                              user_embedding_dim=D, item_embedding_dim=D,
                              compute_dtype=torch.float32).to(DEV)
    g = torch.Generator().manual_seed(8)
    ids = torch.randperm(V - 1, generator=g)[:16] + 1
    modal = torch.randn(16, 512, generator=g)
    loader = [{"target_id": ids[s:s + 8], "target_modal": modal[s:s + 8]} for s in (0, 8)]
    ix = gpu_pkg.retrieval.CatalogueIndexer(m, V)
    before = ix.index(loader).clone()
    from oracle import two_tower_ref as ref
    step = gpu_pkg.TrainStep(m, lr=1e-2, use_graph=False)
    # the model's demographic tables have the reference's default single row each
    b = ref.synthetic_batch(8, 12, V, 1, 1, generator=torch.Generator().manual_seed(9))
    for _ in range(3):
        step.step({k: v.to(DEV) for k, v in b.items()})
    torch.cuda.synchronize()
    after = ix.index(loader).clone()
    fresh = gpu_pkg.retrieval.CatalogueIndexer(m, V).index(loader)
    assert torch.equal(after, fresh)
    assert not torch.equal(after, before)


def test_catalogue_indexer_raw_items_vs_oracle(gpu_pkg):
    """The index over raw item inputs (ResNet-18 audio + visual, tabular, zero text slot,
    fusion head) in eval mode vs the oracle item tower in eval mode (bf16 storage: 3e-2 on the
    unit rows)."""
    from oracle import resnet_ref as rref
    torch.manual_seed(0)
    V, D, T = 29, 128, 32
    m = gpu_pkg.TwoTowerModel(vocab_size=V, tabular_input_dim=T, user_embedding_dim=D,
                              item_embedding_dim=D, with_text=False).to(DEV)
    g = torch.Generator().manual_seed(8)
    _randomise_bn(m, g)
    ids = torch.arange(1, 17)
    items = rref.synthetic_items(16, T, (32, 64), (32, 32), generator=g)
    loader = [{"target_id": ids[s:s + 8], **{k: v[s:s + 8] for k, v in items.items()}}
              for s in (0, 8)]
    dense = gpu_pkg.retrieval.CatalogueIndexer(m, V).index(loader)
    p = {k[len("item_tower."):]: v.detach().cpu() for k, v in m.state_dict().items()
         if k.startswith("item_tower.")}
    running = {k[len("fusion_layer.1."):]: v for k, v in p.items()
               if k.startswith("fusion_layer.1.")}
    out = rref.item_tower_raw_forward(p, items, running=running, eval_mode=True)
    want = _oracle_index(out, ids, V)
    err = (dense.cpu() - want).abs().max().item()
    assert err < 3e-2, err
    assert (dense[17:] == 0).all() and (dense[0] == 0).all()


def _serving_model(pkg):
    from conftest import sub
    z = load_golden("serving.npz")
    V, D, L, n_g, n_c = z["cfg"].tolist()
    m = pkg.TwoTowerModel(precomputed_modalities=True, vocab_size=V, tabular_input_dim=128,
                          num_genders=n_g, num_countries=n_c, max_seq_len=L,
                          user_embedding_dim=D, item_embedding_dim=D,
                          compute_dtype=torch.float32).to(DEV)
    m.load_state_dict({k: torch.tensor(v) for k, v in sub(z, "p/").items()})
    return m.eval(), z


def test_catalogue_index_vs_reference_index_catalog(gpu_pkg):
    """The dense item index vs the REFERENCE's own index_catalog (inference.py:137-209, run by
    tools/make_golden_serving.py on the reference model with the fusion head on precomputed
    modality embeddings, eval-mode BatchNorm): every row to 1e-5, batches of 16 as there."""
    m, z = _serving_model(gpu_pkg)
    ids = torch.tensor(z["catalogue_ids"])
    modal = torch.tensor(z["modal"])
    loader = [{"target_id": ids[s:s + 16], "target_modal": modal[s:s + 16]}
              for s in range(0, len(ids), 16)]
    dense = gpu_pkg.retrieval.compute_all_item_embeddings(m, loader, m.user_tower.item_embedding.num_embeddings)[0]
    want = torch.tensor(z["dense"])
    assert dense.shape == want.shape
    assert (dense.cpu() - want).abs().max().item() < 1e-5


def test_recommend_vs_reference_recommend_for_user(gpu_pkg):
    """Serving vs the REFERENCE's own recommend_for_user (inference.py:213-300): a user with
    63 history items (the last 50 used and masked), the reference's dense index, top-10 ids
    identical and scores to its printed 4 decimals."""
    m, z = _serving_model(gpu_pkg)
    hist = torch.tensor(z["history"])[None]
    val, idx = gpu_pkg.retrieval.recommend(
        m, hist.to(DEV), torch.tensor(z["dense"]).to(DEV), k=10,
        user_gender=torch.tensor(z["gender"]).to(DEV), user_country=torch.tensor(z["country"]).to(DEV))
    assert idx[0].cpu().tolist() == z["top_ids"].tolist()
    assert np.abs(val[0].cpu().numpy() - z["top_scores"]).max() < 6e-5

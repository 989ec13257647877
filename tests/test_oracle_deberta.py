"""The cfg-4 text-encoder oracle (oracle/deberta_ref.py) against the golden fixture that
transformers' own DebertaV2Model produced (tools/make_golden_deberta.py): last_hidden_state,
TextEncoder output and gradients.  LoRA is checked through the merged weight: the fixture's
gradient G of the merged W + s·B·A gives dL/dW_base = G, dL/dA = s·Bᵀ·G, dL/dB = s·G·Aᵀ."""
import numpy as np
import torch

from conftest import load_golden, sub
from oracle import deberta_ref as dref

PRE = "transformer.base_model.model."


def _cfg(z):
    H, NH, NL, I, V, R, ALPHA, B, S, OUT = z["cfg"].tolist()
    return dref.DebertaCfg(vocab_size=V, hidden=H, layers=NL, heads=NH, intermediate=I,
                           lora_r=R, lora_alpha=ALPHA), OUT


def test_relative_buckets_match_transformers_formula():
    cfg = dref.DebertaCfg()
    d = dref.rel_index(256, cfg)
    assert d[0, 0] == 256 and d[5, 0] == 261 and d[0, 5] == 251
    assert d.min() >= 0 and d.max() < 512
    # log buckets beyond |rel| >= 128 (mid): monotone and odd-symmetric
    rel = dref.relative_position(256, cfg)
    assert torch.equal(rel, -rel.t())
    assert rel[255, 0] == 192 and rel[128, 0] == 128 and rel[127, 0] == 127


def test_deberta_oracle_vs_transformers_fixture():
    z = load_golden("deberta_tiny.npz")
    cfg, _ = _cfg(z)
    p = {k: torch.tensor(v, requires_grad=True) for k, v in sub(z, "p/").items()}
    ids = torch.tensor(z["input_ids"])
    mask = torch.tensor(z["attention_mask"])
    hs = dref.deberta_forward(p, ids, mask, cfg, PRE)
    assert np.abs(hs.detach().numpy() - z["last_hidden"]).max() < 2e-5
    out = dref.text_encoder_forward(p, ids, mask, cfg, PRE)
    assert np.abs(out.detach().numpy() - z["out"]).max() < 2e-5
    (out * torch.tensor(z["upstream"])).sum().backward()
    g = sub(z, "g/")
    s = cfg.lora_scale

    def close(a, b, name):
        b = torch.as_tensor(b)
        err = (a.detach() - b).abs().max().item() / max(b.abs().max().item(), 1e-12)
        assert err < 1e-4, (name, err)

    for i in range(cfg.layers):
        L = f"encoder.layer.{i}.attention.self."
        for proj in ("query_proj", "value_proj"):
            G = torch.tensor(g[L + proj + ".weight"])
            A = p[PRE + L + proj + ".lora_A.default.weight"]
            Bm = p[PRE + L + proj + ".lora_B.default.weight"]
            close(p[PRE + L + proj + ".base_layer.weight"].grad, G, proj)
            close(p[PRE + L + proj + ".base_layer.bias"].grad, g[L + proj + ".bias"], proj + "b")
            close(A.grad, s * Bm.detach().t() @ G, proj + ".lora_A")
            close(Bm.grad, s * G @ A.detach().t(), proj + ".lora_B")
        close(p[PRE + L + "key_proj.weight"].grad, g[L + "key_proj.weight"], "key_proj")
    close(p[PRE + "encoder.rel_embeddings.weight"].grad, g["encoder.rel_embeddings.weight"], "rel")

"""GPU diagnostic: bf16 vs fp32-reference error per gradient, pruned vs unpruned last layer."""
import importlib, sys
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import torch
from conftest import load_golden, sub
pkg = importlib.import_module("music-recommendation-multimodal_amd")
import test_gpu_model as t
for name in ("user_tower_small.npz", "user_tower_d128.npz"):
    z = load_golden(name)
    e_out, e_g = t.bf16_emulated(z)
    res = {}
    for prune in (True, False):
        m, use_mask = t.build_user(pkg, z, torch.bfloat16)
        m.prune_last = prune
        ids = torch.tensor(z["history_ids"], device="cuda")
        mask = torch.tensor(z["history_mask"], device="cuda") if use_mask else None
        out = m(ids, torch.tensor(z["user_gender"], device="cuda"), torch.tensor(z["user_country"], device="cuda"), mask)
        (out * torch.tensor(z["upstream"], device="cuda")).sum().backward()
        res[prune] = {k: t.rel(p.grad, z["g/" + k]) for k, p in m.named_parameters()}
        res[prune]["out"] = t.rel(out, z["out"])
    print(name)
    for k in res[True]:
        em = t.rel(e_g[k], z["g/" + k]) if k != "out" else t.rel(e_out, z["out"])
        print(f"  {k:60s} pruned {res[True][k]:.4f} full {res[False][k]:.4f} emul {em:.4f}")

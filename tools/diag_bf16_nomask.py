import importlib, sys
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import torch
from conftest import load_golden
pkg = importlib.import_module("music-recommendation-multimodal_amd")
import test_gpu_model as t
z = load_golden("user_tower_nomask.npz")
print("ids", z["history_ids"].tolist())
e_out, e_g = t.bf16_emulated(z)
k = "item_embedding.weight"
ref = torch.tensor(z["g/" + k])
print("emul rel", t.rel(e_g[k], ref))
for prune in (True, False):
    for dt in (torch.bfloat16, torch.float32):
        m, use_mask = t.build_user(pkg, z, dt)
        m.prune_last = prune
        ids = torch.tensor(z["history_ids"], device="cuda")
        out = m(ids, torch.tensor(z["user_gender"], device="cuda"), torch.tensor(z["user_country"], device="cuda"), None)
        (out * torch.tensor(z["upstream"], device="cuda")).sum().backward()
        g = dict(m.named_parameters())[k].grad.cpu()
        err = (g - ref).abs().max(1).values
        top = torch.topk(err, 4)
        print(f"prune={prune} {dt}: rel {t.rel(g, ref):.4f} out {t.rel(out, z['out']):.4f} worst rows {top.indices.tolist()} {[round(v,4) for v in top.values.tolist()]}")
        for r in top.indices.tolist()[:2]:
            print("   row", r, "gpu", [round(v,4) for v in g[r,:6].tolist()], "ref", [round(v,4) for v in ref[r,:6].tolist()], "emul", [round(v,4) for v in e_g[k][r,:6].tolist()])

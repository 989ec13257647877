"""GPU diagnostic: the fp32 cfg-2 model's gradients at B 64, L 20 with dropout on, dumped for
an A/B of TTMI_SEQ_VEC (run twice, then compare with --compare)."""
import importlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
if "--compare" in sys.argv:
    a = torch.load(sys.argv[2], weights_only=True)
    b = torch.load(sys.argv[3], weights_only=True)
    for k in a:
        d = (a[k] - b[k]).abs()
        if d.max() > 0:
            idx = (d == d.max()).nonzero()[0].tolist()
            rows = (d.reshape(d.shape[0], -1).amax(1) > 0).nonzero().flatten().tolist() if d.dim() > 1 else []
            print(f"{k}: max diff {d.max().item():.3e} at {idx}, ref max {a[k].abs().max().item():.3e}, "
                  f"rows differing {len(rows)}: {rows[:20]}")
    sys.exit(0)
from oracle import two_tower_ref as ref
pkg = importlib.import_module("music-recommendation-multimodal_amd")
F = pkg.functional
torch.manual_seed(3)
m = pkg.TwoTowerModel(precomputed_modalities=True, vocab_size=997, tabular_input_dim=128, num_genders=3,
                      num_countries=64, max_seq_len=20, user_embedding_dim=128, item_embedding_dim=128,
                      user_dropout=0.1, compute_dtype=torch.float32).cuda()
m.item_tower.fusion_layer[3].p = 0.1
batch = ref.synthetic_batch(64, 20, 997, generator=torch.Generator().manual_seed(4))
seeds = F.site_seeds(0x5EED, 1)
table = F.seed_table(seeds, "cuda")
loss, _, _, _ = m({k: v.cuda() for k, v in batch.items()}, seeds=table)
loss.backward()
out = {k: v.grad.detach().cpu() for k, v in m.named_parameters() if v.grad is not None}
out["loss"] = loss.detach().cpu().reshape(1)
ut = m.user_tower
ids_d = batch["history_ids"].cuda()
M = ids_d.numel()
x = torch.empty(M, 128, device="cuda")
mu = torch.empty(M, device="cuda")
rs = torch.empty(M, device="cuda")
pkg.ops.seq_embed_fwd(ids_d, ut.item_embedding.weight.detach(), ut.position_embedding.weight.detach(),
                      ut.layer_norm.weight.detach(), ut.layer_norm.bias.detach(), x, mu, rs,
                      drop=(0.1, table[F.SITE_EMB:F.SITE_EMB + 1]))
torch.cuda.synchronize()
out["x_se"], out["mu_se"], out["rs_se"] = x.cpu(), mu.cpu(), rs.cpu()
ids = batch["history_ids"]
print("ids min/max", int(ids.min()), int(ids.max()), "dtype", ids.dtype, "contig", ids.is_contiguous())
torch.save(out, sys.argv[1])

"""Diagnostic (GPU, not a test): which parameters of the forced data-parallel schedule at world
size 1 (comm.force_dp, RCCL) differ from the single-process step after one and two steps, and by
how much.  Dropout off, bf16.  Usage: python tools/diag_dp_bits.py"""
import importlib
import os
import socket
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import two_tower_ref as ref  # noqa: E402

pkg = importlib.import_module("music-recommendation-multimodal_amd")
V, D, L, B, NG, NC = 997, 128, 20, 64, 3, 8


def batch(s):
    g = torch.Generator().manual_seed(3000 + 10 * s)
    return {k: v.cuda() for k, v in ref.synthetic_batch(B, L, V, NG, NC, num_users=20, generator=g).items()}


def run(steps, **kw):
    torch.manual_seed(0)
    m = pkg.TwoTowerModel(vocab_size=V, tabular_input_dim=128, num_genders=NG, num_countries=NC,
                          max_seq_len=L, user_embedding_dim=D, item_embedding_dim=D, user_dropout=0.0,
                          compute_dtype=torch.bfloat16, precomputed_modalities=True).cuda()
    m.item_tower.fusion_layer[3].p = 0.0
    st = pkg.TrainStep(m, lr=1e-3, seed=1, **kw)
    for s in range(steps):
        st.step(batch(s))
    torch.cuda.synchronize()
    g = {k: v.detach().clone() for k, v in m.state_dict().items()}
    return g


def main():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    for steps in (1, 2):
        for name, env in (("fold_in_update=0", {"TTMI_FOLD_IN_UPDATE": "0"}), ("default", {})):
            os.environ.update(env)
            pkg.comm.force_dp(False)
            a = run(steps, grad_sink=name == "default")
            pkg.comm.force_dp(True)
            b = run(steps)
            pkg.comm.force_dp(False)
            os.environ.pop("TTMI_FOLD_IN_UPDATE", None)
            bad = [(k, (a[k].double() - b[k].double()).abs().max().item()) for k in a
                   if not torch.equal(a[k], b[k])]
            print(f"steps={steps} single[{name}] vs dp: {len(bad)} of {len(a)} differ")
            for k, d in bad[:40]:
                print(f"   {k}: max|diff| {d:.3e}")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

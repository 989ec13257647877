"""Launches the cfg-2 feed-forward sub-block (M = 25,600, D = 128, F = 512, dropout 0.1) as the
fused ttmi_ffn_block_fwd and as the FFN1 row panel + ttmi_linear_res_ln pair, 10 times each, for
rocprofv3 counter passes (tools/gpu.sh kcounters tools/micro/ffn_run.py ffn)."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
ops = importlib.import_module("music-recommendation-multimodal_amd").ops
dev = "cuda"
M, D, F = 25600, 128, 512
g = torch.Generator().manual_seed(0)
a = torch.randn(M, D, generator=g).to(torch.bfloat16).to(dev)
w1 = (torch.randn(F, D, generator=g) * 0.05).to(torch.bfloat16).to(dev)
w2 = (torch.randn(D, F, generator=g) * 0.05).to(torch.bfloat16).to(dev)
b1, b2 = torch.zeros(F, device=dev), torch.zeros(D, device=dev)
res = torch.randn(M, D, generator=g).to(dev)
lnw, lnb = torch.ones(D, device=dev), torch.zeros(D, device=dev)
seed = torch.tensor([7], dtype=torch.int64, device=dev)
drop = (0.1, seed)
h = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
x2 = torch.empty(M, D, device=dev)
y = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
mu, rs = torch.empty(M, device=dev), torch.empty(M, device=dev)
for _ in range(10):
    ops.ffn_block_fwd(a, w1, b1, w2, b2, res, drop, drop, h, x2, lnw, lnb, 1e-5, y, mu, rs)
for _ in range(10):
    ops.linear(a, w1, b1, h, act=1, drop=drop)
    ops.linear_res_ln(h, w2, b2, res, x2, lnw, lnb, y, mu, rs, eps=1e-5, drop=drop)
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
ev[0].record()
for _ in range(50):
    ops.ffn_block_fwd(a, w1, b1, w2, b2, res, drop, drop, h, x2, lnw, lnb, 1e-5, y, mu, rs)
ev[1].record()
for _ in range(50):
    ops.linear(a, w1, b1, h, act=1, drop=drop)
    ops.linear_res_ln(h, w2, b2, res, x2, lnw, lnb, y, mu, rs, eps=1e-5, drop=drop)
ev[2].record()
torch.cuda.synchronize()
print(f"fused {ev[0].elapsed_time(ev[1]) * 20:.2f} us   pair {ev[1].elapsed_time(ev[2]) * 20:.2f} us")

"""Weight-gradient shapes of the cfg-2 step: torch.mm (hipBLASLt) dyᵀ·x vs ttmi_wgrad, timed
under rocprofv3 (kernel durations) — a yardstick for the wgrad kernel."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pkg = importlib.import_module("music-recommendation-multimodal_amd")
ops = pkg.ops
for M, N, R in ((384, 128, 25600), (128, 128, 25600), (512, 128, 25600), (128, 512, 25600)):
    dy = torch.randn(R, M, device="cuda").bfloat16()
    x = torch.randn(R, N, device="cuda").bfloat16()
    gw = torch.zeros(M, N, device="cuda")
    gb = torch.zeros(M, device="cuda")
    for _ in range(20):
        torch.mm(dy.t(), x)
        torch.mm(dy.t().float(), x.float()) if False else None
        ops.linear_dw(dy, x, gw, gb)
    torch.cuda.synchronize()
    print(M, N, R, "done", flush=True)

#!/usr/bin/env python3
"""Row-panel GEMM time against the row count (GPU diagnostic, not a test).

Times ops.linear at the cfg-2 shapes (N x K = 512 x 128 FFN1, 384 x 128 in_proj, 128 x 512
FFN2) for M = 256 .. 51,200 rows, each call replayed 20x inside one HIP graph, so the fixed
per-launch cost (W staging, first A loads, launch) separates from the per-row cost.
Usage: python tools/panel_scale.py
"""
import importlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module("music-recommendation-multimodal_amd")
sys.path.insert(0, os.path.join(ROOT, "tools"))
from gemm_profile import timed  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    for (N, K, act) in ((512, 128, 1), (384, 128, 0), (128, 512, 0), (128, 128, 0)):
        w = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
        b = torch.zeros(N, device=dev)
        for M in (256, 1024, 4096, 12800, 25600, 51200):
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            us = timed(lambda: pkg.ops.linear(x, w, b, out, act=act))
            mb = (M * K * 2 + M * N * 2) / 1e6
            print(f"N={N} K={K} M={M:6d}: {us:7.2f} us  {mb / us:6.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()

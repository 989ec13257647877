#!/usr/bin/env python3
"""Calibration (GPU diagnostic): library GEMM and plain fill/copy at the hot-path sizes."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tools.gemm_profile import timed  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    M = 25600
    for N, K in ((384, 128), (512, 128), (128, 512), (128, 128)):
        a = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = torch.randn(N, K, device=dev).to(torch.bfloat16)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        us = timed(lambda: torch.mm(a, w.t(), out=out))
        by = (M * K + N * K + M * N) * 2
        print(f"torch.mm     M={M} N={N} K={K}: {us:7.2f} us {by / us / 1e3:7.1f} GB/s", flush=True)
    for mb in (6.5, 19.7, 26.2, 52.4):
        n = int(mb * 1e6 / 2)
        x = torch.empty(n, device=dev, dtype=torch.bfloat16)
        y = torch.empty(n, device=dev, dtype=torch.bfloat16)
        us = timed(lambda: x.fill_(1.0))
        us2 = timed(lambda: y.copy_(x))
        print(f"fill {mb:5.1f} MB: {us:7.2f} us {mb * 1e6 / us / 1e3:7.1f} GB/s | copy: {us2:7.2f} us "
              f"{2 * mb * 1e6 / us2 / 1e3:7.1f} GB/s (r+w)", flush=True)
    e = torch.empty(1, device=dev)
    print(f"empty-ish kernel (fill 1 float): {timed(lambda: e.fill_(0.0)):.2f} us")


if __name__ == "__main__":
    main()

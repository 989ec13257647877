"""The encoder's long weight gradients of the cfg-2 step (R = B·L = 25,600 rows) as ONE grouped
wgrad launch (ops.deferred_wgrad), and the same GEMMs through torch.mm (hipBLASLt) for a
yardstick; run under rocprofv3 (--kernel-trace --stats, or --pmc passes) for per-kernel
durations / traffic.  usage: python tools/wgrad_shapes.py [--dim 128|256] [--reps N]"""
import argparse
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pkg = importlib.import_module("music-recommendation-multimodal_amd")
ops = pkg.ops

ap = argparse.ArgumentParser()
ap.add_argument("--dim", type=int, default=128)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--blas", type=int, default=1)
a = ap.parse_args()
D, R = a.dim, 25600
# (M = dW rows = dy width, N = dW cols = x width): layer-1 in_proj, out_proj, linear1, linear2,
# layer-2 K/V in_proj rows
shapes = [(3 * D, D), (D, D), (4 * D, D), (D, 4 * D), (2 * D, D)]
g = torch.Generator(device="cuda").manual_seed(0)
ops_in = []
for M, N in shapes:
    dy = torch.randn(R, M, device="cuda", generator=g).bfloat16()
    x = torch.randn(R, N, device="cuda", generator=g).bfloat16()
    ops_in.append((dy, x, torch.zeros(M, N, device="cuda"), torch.zeros(M, device="cuda")))
for _ in range(a.reps):
    with ops.deferred_wgrad():
        for dy, x, gw, gb in ops_in:
            ops.linear_dw(dy, x, gw, gb)
    if a.blas:
        for dy, x, gw, gb in ops_in:
            torch.mm(dy.t(), x)
torch.cuda.synchronize()
for dy, x, gw, gb in ops_in:                  # one clean group, checked against fp32 torch
    gw.zero_()
    gb.zero_()
with ops.deferred_wgrad():
    for dy, x, gw, gb in ops_in:
        ops.linear_dw(dy, x, gw, gb)
err = max(float(((gw - dy.float().t() @ x.float()).abs().max()) / (dy.float().t() @ x.float()).abs().max())
          for dy, x, gw, gb in ops_in)
print(f"max |err| / max |ref| over the group: {err:.2e}", flush=True)
assert err < 1e-4, "wgrad group mismatch"
ab = sum(R * (M + N) * 2 for M, N in shapes)
fl = sum(2 * R * M * N for M, N in shapes)
print(f"D={D}: {len(shapes)} GEMMs, algorithmic {ab / 1e6:.1f} MB, {fl / 1e9:.2f} GF per group", flush=True)

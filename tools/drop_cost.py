"""GPU diagnostic: what the dropout mask costs the attention and feed-forward kernels at cfg 2
(B = 512, L = 50, D = 128, H = 4): device time per launch with p = 0.1 against p = 0 (HIP
events over 50 launches).  python tools/drop_cost.py"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pkg = importlib.import_module("music-recommendation-multimodal_amd")
ops = pkg.ops
DEV = "cuda"


def timeit(fn, n=50):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / n


def main():
    B, L, D, H = 512, 50, 128, 4
    M = B * L
    g = torch.Generator().manual_seed(0)
    bf = lambda *s, sc=0.05: (torch.randn(*s, generator=g) * sc).to(torch.bfloat16).to(DEV)
    f32 = lambda *s, sc=1.0: (torch.randn(*s, generator=g) * sc).to(DEV)
    seed = torch.tensor([7], dtype=torch.int64, device=DEV)
    kv = (torch.arange(L)[None] < torch.randint(1, L + 1, (B, 1), generator=g)).long().to(DEV)
    a1, w_in, b_in = bf(M, D, sc=1.0), bf(3 * D, D), f32(3 * D, sc=0.1)
    qkv = torch.empty(M, 3 * D, device=DEV, dtype=torch.bfloat16)
    ctx = torch.empty(M, D, device=DEV, dtype=torch.bfloat16)
    lse = torch.empty(B * H * L, device=DEV)
    dctx, dqkv = bf(M, D, sc=0.1), torch.empty(M, 3 * D, device=DEV, dtype=torch.bfloat16)
    for p in (0.0, 0.1):
        drop = (p, seed) if p > 0 else (0.0, None)
        t1 = timeit(lambda: ops.qkv_attn_fwd(a1, w_in, b_in, kv, B, L, H, qkv, ctx, lse, drop))
        t2 = timeit(lambda: ops.mha_fwd(qkv, kv, B, L, H, ctx, lse, drop))
        t3 = timeit(lambda: ops.mha_bwd(qkv, kv, lse, dctx, B, L, H, dqkv, drop))
        print(f"p={p}: qkv_attn_fwd {t1:6.2f} us   mha_fwd {t2:6.2f} us   mha_bwd {t3:6.2f} us", flush=True)


if __name__ == "__main__":
    main()

"""Time ttmi_dis_attn_fwd/bwd at the cfg-4 shape (B=256, S=256, 12 heads, d_head 64, LoRA
contractions on) with HIP events; prints per-launch us and effective TFLOP/s (kernel MFMA
work: fwd 6·64³·2 per 64x64 block pair, bwd 13·64³·2)."""
import importlib
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pkg = importlib.import_module("music-recommendation-multimodal_amd")
ops, text = pkg.ops, pkg.text
if os.environ.get("TTMI_LIB"):          # experiment builds (tools only; the product loads lib/)
    pkg.lib.load(os.environ["TTMI_LIB"])


def main(B=256, S=256, nh=12, reps=5):
    dev = "cuda"
    H, cfg = 64 * nh, text.TextCfg()
    g = torch.Generator(device="cpu").manual_seed(0)
    qkv = torch.randn(B * S, 3 * H, generator=g).to(torch.bfloat16).to(dev)
    pos = torch.randn(cfg.npos, 2 * H, generator=g).to(torch.bfloat16).to(dev)
    lengths = torch.randint(16, S + 1, (B,), generator=g)
    mask = (torch.arange(S)[None] < lengths[:, None]).long().to(dev)
    delta = text._Frozen().delta(S, cfg, dev)
    ctx = torch.empty(B * S, H, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B * nh * S, device=dev)
    dctx = torch.randn(B * S, H, generator=g).to(torch.bfloat16).to(dev)
    dqkv = torch.empty(B * S, 3 * H, device=dev, dtype=torch.bfloat16)
    u = torch.randn(cfg.npos, 8, device=dev)
    bq = torch.randn(H, 8, device=dev) * 0.02
    hu = torch.empty(B * S * nh * 8, device=dev)
    pb = torch.empty(B * nh * cfg.npos * 8, device=dev)
    scale = 1 / math.sqrt(192)
    drop = (0.1, torch.tensor([12345], dtype=torch.int64, device=dev))
    order = ops.dis_attn_order(mask, B, S)

    def fwd():
        ops.dis_attn(B, S, nh, qkv[:, :H], qkv[:, H:2 * H], qkv[:, 2 * H:], pos[:, :H], pos[:, H:],
                     mask, delta, scale, ctx, lse, drop, order=order)

    def bwd():
        ops.dis_attn(B, S, nh, qkv[:, :H], qkv[:, H:2 * H], qkv[:, 2 * H:], pos[:, :H], pos[:, H:],
                     mask, delta, scale, ctx, lse, drop, dctx=dctx, dq=dqkv[:, :H],
                     dk=dqkv[:, H:2 * H], dv=dqkv[:, 2 * H:], lora_u=u, lora_bq=bq, lora_hu=hu,
                     lora_pb=pb, order=order)
    def bwd_nolora():
        ops.dis_attn(B, S, nh, qkv[:, :H], qkv[:, H:2 * H], qkv[:, 2 * H:], pos[:, :H], pos[:, H:],
                     mask, delta, scale, ctx, lse, drop, dctx=dctx, dq=dqkv[:, :H],
                     dk=dqkv[:, H:2 * H], dv=dqkv[:, 2 * H:], order=order)
    pairs = B * nh * (S // 64) ** 2
    cases = (("fwd", fwd, 6), ("bwd", bwd, 13), ("bwd-nolora", bwd_nolora, 13))
    if os.environ.get("ATTN_FWD_ONLY"):
        cases = cases[:1]
    for name, fn, units in cases:
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        fl = pairs * units * 64 ** 3 * 2
        print(f"dis_attn_{name}: {us:9.1f} us  {fl / us / 1e6:7.1f} TF/s (kernel MFMA work)", flush=True)


if __name__ == "__main__":
    main()

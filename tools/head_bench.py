"""Time ttmi_user_head_fwd alone (cfg-2 shapes, B = 512, dropout on); with a HEAD_STAMP build
(TTMI_LIB) also print the per-phase s_memtime stamps of workgroups 0-3."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pkg = importlib.import_module("music-recommendation-multimodal_amd")
if os.environ.get("TTMI_LIB"):
    pkg.lib.load(os.environ["TTMI_LIB"])
ops = pkg.ops


def main(B=512, D=128, F=512):
    dev = "cuda"
    g = torch.Generator(device="cpu").manual_seed(0)

    def bf(*s):
        return (torch.randn(*s, generator=g) * 0.05).to(torch.bfloat16).to(dev)

    def f32(*s):
        return (torch.randn(*s, generator=g) * 0.1).to(dev)
    pre = "l."
    W = {pre + "self_attn.out_proj.weight": bf(D, D), pre + "linear1.weight": bf(F, D),
         pre + "linear2.weight": bf(D, F), "fusion_layer.0.weight": bf(D, D + 48),
         "fusion_layer.3.weight": bf(D, D)}
    P = {pre + "self_attn.out_proj.bias": f32(D), pre + "norm2.weight": f32(D), pre + "norm2.bias": f32(D),
         pre + "linear1.bias": f32(F), pre + "linear2.bias": f32(D), "gender_embedding.weight": f32(3, 16),
         "country_embedding.weight": f32(11, 32), "fusion_layer.0.bias": f32(D),
         "fusion_layer.1.weight": f32(D), "fusion_layer.1.bias": f32(D), "fusion_layer.3.bias": f32(D)}
    ctx, res = bf(B, D), f32(B, D)
    drows = torch.arange(B, dtype=torch.int32, device=dev) * 50
    gender = torch.randint(0, 3, (B,), generator=g).to(dev)
    country = torch.randint(0, 11, (B,), generator=g).to(dev)
    seeds = torch.tensor([1, 2, 3], dtype=torch.int64, device=dev)
    drops = tuple((0.1, seeds[k:k + 1]) for k in range(3))
    o = dict(x1=f32(B, D), a2=bf(B, D), m2=f32(B), r2=f32(B), h=bf(B, F), comb=bf(B, D + 48),
             rows=torch.empty(B, dtype=torch.int32, device=dev), z=f32(B, D), az=bf(B, D),
             mz=f32(B), rz=f32(B), u=f32(B, D))

    def fn():
        ops.user_head_fwd(ctx, res, drows, W, P, pre, gender, country, 1e-5, drops, o)
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(100):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"user_head_fwd: {e0.elapsed_time(e1) * 10:.2f} us per launch (back-to-back)")
    if os.environ.get("TTMI_LIB"):
        fn()
        torch.cuda.synchronize()
        st = o["rz"][:32].view(4, 8)[:, 1:7].cpu()
        print("stamps (cycles since start; prologue, S1+LN2, FFN1, FFN2, fusion0+LN, end):")
        print(st)

    # backward (fused ttmi_user_head_bwd) on the forward's saved values
    W2 = dict(W)
    for n in list(W):
        W2[n + ".T"] = W[n].t().contiguous()
    du16 = bf(B, D)
    dG, dC = torch.zeros(3, 16, device=dev), torch.zeros(11, 32, device=dev)
    lg = tuple(torch.zeros(D, device=dev) for _ in range(4))

    def fb():
        return ops.user_head_bwd(du16, o, drows, W2, P, pre, gender, country, 1 / 0.9,
                                 (drops[0], drops[2]), dG, dC, lg)
    fb()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(100):
        fb()
    e1.record()
    torch.cuda.synchronize()
    print(f"user_head_bwd: {e0.elapsed_time(e1) * 10:.2f} us per launch + fold (back-to-back)")
    if os.environ.get("TTMI_LIB"):
        r = fb()
        torch.cuda.synchronize()
        st = r["dx1"][0, :32].view(4, 8)[:, 1:8].cpu()
        print("bwd stamps (prologue, dz, dcomb, dy2, dz1, dx1, end):")
        print(st)


if __name__ == "__main__":
    main()

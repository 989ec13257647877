"""GPU diagnostic: launch time of the user head with the item head's stages co-launched
(tests/test_gpu_colaunch.py's B = 512 case): 'sep' (stage A, user head, stage C), 'C' (stage A,
user head + C) and 'AC' (user head + A + C, C polling A's statistics in-launch)."""
import importlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
pkg = importlib.import_module("music-recommendation-multimodal_amd")
if os.environ.get("TTMI_LIB"):
    pkg.lib.load(os.environ["TTMI_LIB"])
import test_gpu_colaunch as T  # noqa: E402

ops = pkg.ops
DEV = "cuda"
B, D, F = 512, 128, 512
g = torch.Generator().manual_seed(B + 9)


def bf(*s, scale=1.0):
    return (torch.randn(*s, generator=g) * scale).to(torch.bfloat16).to(DEV)


def f32(*s, scale=1.0):
    return (torch.randn(*s, generator=g) * scale).to(DEV)


pre = "transformer_encoder.layers.1."
Wu = {pre + "self_attn.out_proj.weight": bf(D, D, scale=D ** -0.5), pre + "linear1.weight": bf(F, D, scale=D ** -0.5),
      pre + "linear2.weight": bf(D, F, scale=F ** -0.5), "fusion_layer.0.weight": bf(D, D + 48, scale=0.07),
      "fusion_layer.3.weight": bf(D, D, scale=D ** -0.5)}
Pu = {pre + "self_attn.out_proj.bias": f32(D, scale=0.1), pre + "norm2.weight": 1 + f32(D, scale=0.1),
      pre + "norm2.bias": f32(D, scale=0.1), pre + "linear1.bias": f32(F, scale=0.1),
      pre + "linear2.bias": f32(D, scale=0.1), "gender_embedding.weight": f32(3, 16),
      "country_embedding.weight": f32(11, 32), "fusion_layer.0.bias": f32(D, scale=0.1),
      "fusion_layer.1.weight": 1 + f32(D, scale=0.1), "fusion_layer.1.bias": f32(D, scale=0.1),
      "fusion_layer.3.bias": f32(D, scale=0.1)}
ctx, res = bf(B, D), f32(B, D)
drows = torch.randperm(50 * B, generator=g)[:B].to(torch.int32).to(DEV)
gender = torch.randint(0, 3, (B,), generator=g).to(DEV)
country = torch.randint(0, 11, (B,), generator=g).to(DEV)
seeds = torch.tensor([5, -6, 7], dtype=torch.int64, device=DEV)
drops = tuple((0.1, seeds[k:k + 1]) for k in range(3))
Wi, Pi, modal, drop_i = T._item_case(ops, B, g, 0.1)
uo = dict(x1=f32(B, D), a2=bf(B, D), m2=f32(B), r2=f32(B), h=bf(B, F), comb=bf(B, D + 48),
          rows=torch.empty(B, dtype=torch.int32, device=DEV), z=f32(B, D), az=bf(B, D), mz=f32(B), rz=f32(B),
          u=f32(B, D))
io = T._item_outs(B)
bufs = T._bufs()
d = ops.item_head_desc(modal, Wi, Pi, bufs, drop_i, 1e-5, io)


def run(mode):
    if mode != "AC":
        ops.item_head_fwd_stages(d, 1)
    if mode == "sep":
        ops.user_head_fwd(ctx, res, drows, Wu, Pu, pre, gender, country, 1e-5, drops, uo)
        ops.item_head_fwd_stages(d, 6)
    elif mode == "user":
        ops.user_head_fwd(ctx, res, drows, Wu, Pu, pre, gender, country, 1e-5, drops, uo)
    else:
        ops.user_head_fwd(ctx, res, drows, Wu, Pu, pre, gender, country, 1e-5, drops, uo, co_item=d,
                          co_stage=mode)


for mode in ("user", "sep", "C", "AC", "A"):
    for _ in range(3):
        run(mode)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        run(mode)
    e1.record()
    torch.cuda.synchronize()
    cnt = ops._zero_ws("ttmi_item_head_bn_counter_bytes", (0,), modal.device)
    print(f"{mode:5s} {e0.elapsed_time(e1) / 20 * 1000:8.1f} us per call; counters {cnt.view(torch.int32)[:12].tolist()}",
          flush=True)

if os.environ.get("TTMI_LIB", "").endswith("libttmi_stamp.so"):     # phase stamps of one AC launch
    import ctypes
    import numpy as np
    lib = pkg.lib._lib
    lib.ttmi_dbg_stamps_head.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    NB, NW, NP = 512, 16, 8
    buf = (ctypes.c_uint64 * (NB * NW * NP))()
    for mode in ("AC", "C"):
        run(mode)
        torch.cuda.synchronize()
        lib.ttmi_dbg_stamps_head(buf, NB * NW * NP)
        run(mode)
        assert lib.ttmi_dbg_stamps_head(buf, NB * NW * NP) == 0
        a = np.array(buf, dtype=np.float64).reshape(NB, NW, NP)[:, 0, :]
        nu, na = 32, (256 if mode == "AC" else 0)
        tot = nu + na + 32
        t0 = a[:tot, 0][a[:tot, 0] > 0].min()
        rel = (a - t0) / 100.0

        def show(name, rows, phases):
            for k in phases:
                v = rel[rows, k][a[rows, k] > 0]
                if v.size:
                    print(f"{mode:3s} {name:6s} p{k}: min {v.min():7.2f} med {np.median(v):7.2f} max {v.max():7.2f} (n={v.size})")
        if mode == "AC":
            show("A", slice(0, na), range(3))
            show("user", slice(na, na + nu), range(7))
            show("C", slice(na + nu, tot), (0, 3, 4))
        else:
            show("user", slice(0, nu), range(7))
            show("C", slice(nu, tot), (0, 3, 4))

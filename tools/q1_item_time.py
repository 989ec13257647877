"""GPU diagnostic: what the pruned layer's one-query launch (q1_item_fwd_kernel) spends its time
on — the one-query attention waves alone, item head stage A alone, and both on one grid — at
cfg 2 (B = 512, L = 50, D = 128, H = 4), timed with HIP events over 50 replays of a captured graph.
    python tools/q1_item_time.py"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pkg = importlib.import_module("music-recommendation-multimodal_amd")
if os.environ.get("TTMI_LIB"):
    pkg.lib.load(os.environ["TTMI_LIB"])
ops = pkg.ops
dev = "cuda"
B, L, D, H = 512, 50, 128, 4
M = B * L
g = torch.Generator().manual_seed(0)


def bf(*s, sc=0.05):
    return (torch.randn(*s, generator=g) * sc).to(torch.bfloat16).to(dev)


def f32(*s, sc=1.0):
    return (torch.randn(*s, generator=g) * sc).to(dev)


qkv = bf(M, 3 * D, sc=1.0)
lens = torch.randint(1, L + 1, (B, 1), generator=g)
kv = (torch.arange(L)[None] < lens).long().to(dev)
a_in, wq, bq = bf(M, D, sc=1.0), bf(D, D), f32(D, sc=0.1)
x = f32(M, D)
rows = torch.empty(B, dtype=torch.int32, device=dev)
x_rows, ctx = torch.empty(B, D, device=dev), torch.empty(B, D, device=dev, dtype=torch.bfloat16)
lse = torch.empty(B * H, device=dev)
seed = torch.tensor([5], dtype=torch.int64, device=dev)
drop = (0.1, seed)
modal = f32(B, 512)
W = {"fusion_layer.0.weight": bf(512, 512), "fusion_layer.4.weight": bf(D, 512)}
P = {"fusion_layer.0.bias": f32(512, sc=0.1), "fusion_layer.1.weight": 1 + f32(512, sc=0.1),
     "fusion_layer.1.bias": f32(512, sc=0.1), "fusion_layer.4.bias": f32(D, sc=0.1),
     "fusion_layer.5.weight": 1 + f32(D, sc=0.1), "fusion_layer.5.bias": f32(D, sc=0.1)}
bufs = {"fusion_layer.1.running_mean": torch.zeros(512, device=dev),
        "fusion_layer.1.running_var": torch.ones(512, device=dev),
        "fusion_layer.1.num_batches_tracked": torch.zeros((), dtype=torch.int64, device=dev)}
out = {"m16": torch.empty(B, 512, device=dev, dtype=torch.bfloat16), "z": torch.empty(B, 512, device=dev),
       "bn_mean": torch.empty(512, device=dev), "bn_rstd": torch.empty(512, device=dev),
       "y1": torch.empty(B, 512, device=dev, dtype=torch.bfloat16), "y2": torch.empty(B, D, device=dev),
       "out": torch.empty(B, D, device=dev), "m5": torch.empty(B, device=dev), "r5": torch.empty(B, device=dev)}
desc = ops.item_head_desc(modal, W, P, bufs, drop, 1e-5, out)


def run_q1(co):
    ops.mha_q1_proj_gather_fwd(qkv, kv, a_in, wq, bq, x, rows, x_rows, B, L, H, ctx, lse, drop,
                               co_item=desc if co else None)


cases = {"q1 waves alone": lambda: run_q1(False),
         "item stage A alone": lambda: ops.item_head_fwd_stages(desc, 1),
         "q1 + item A, one grid": lambda: run_q1(True)}
for name, fn in cases.items():
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):
            for _ in range(10):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    gr.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        gr.replay()
    e1.record()
    torch.cuda.synchronize()
    print(f"{name:28s} {e0.elapsed_time(e1) * 1e3 / 50:7.2f} us per launch (graph, 50 back to back)", flush=True)

if os.environ.get("TTMI_LIB"):          # the diagnostic stamp build: item stage A's phases
    import ctypes
    import numpy as np
    lib = pkg.lib._lib
    lib.ttmi_dbg_stamps_head.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    NB, NW, NP = 512, 16, 8
    buf = (ctypes.c_uint64 * (NB * NW * NP))()
    for rep in range(2):
        lib.ttmi_dbg_stamps_head(buf, NB * NW * NP)
        if os.environ.get("STAMP_BUSY"):
            torch.cuda._sleep(int(os.environ["STAMP_BUSY"]))
        ops.item_head_fwd_stages(desc, 1)
        torch.cuda.synchronize()
        assert lib.ttmi_dbg_stamps_head(buf, NB * NW * NP) == 0
    a = np.array(buf, dtype=np.float64).reshape(NB, NW, NP)[:, :, :7]
    live = a[:, :, 0] > 0
    t0 = a[:, :, 0][live].min()
    rel = (a - t0) / 100.0
    for k, nm in enumerate(("start", "z stored", "end (last arrivers)", "stats stored + retired",
                            "arrival counted", "partials loaded (last)", "merged (last)")):
        v = rel[:, :, k][live & (a[:, :, k] > 0)]
        print(f"item A stamp {nm:30s} median {np.median(v):6.2f}  max {v.max():6.2f} us  (n={v.size})")

#!/usr/bin/env python3
"""Per-call GEMM timing for one cfg-2 train step (GPU diagnostic, not a test).

Records every ops.gemm call of one eager TrainStep, then replays each call alone and times it
with HIP events on the current stream.  For accumulate (weight-gradient) calls it also sweeps
split_k.  Usage: python tools/gemm_profile.py [--sweep]
"""
import importlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module("music-recommendation-multimodal_amd")
import bench  # noqa: E402

calls = []
_orig = pkg.ops.gemm


def rec(A, B, C, M, N, K, **kw):
    calls.append((A, B, C, M, N, K, dict(kw)))
    return _orig(A, B, C, M, N, K, **kw)


def timed(fn, iters=20):
    """Average device time of fn() over `iters` launches captured in one HIP graph."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(gr, stream=s):
            for _ in range(iters):
                fn()
    torch.cuda.synchronize()
    gr.replay()
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    gr.replay()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    sweep = "--sweep" in sys.argv
    only_wgrad = "--wgrad" in sys.argv
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = pkg.TwoTowerModel(precomputed_modalities=True, vocab_size=bench.V, tabular_input_dim=128, num_genders=3,
                              num_countries=64, max_seq_len=bench.L, user_embedding_dim=bench.D,
                              item_embedding_dim=bench.D, user_num_heads=bench.H,
                              user_dropout=0.1, compute_dtype=torch.bfloat16).to(dev)
    step = pkg.TrainStep(model, lr=1e-4, use_graph=False, seed=1)
    batch = bench.synthetic_batches(1, 512, 0, dev)[0]
    step.step(batch)
    torch.cuda.synchronize()
    pkg.ops.gemm = rec
    step.step(batch)
    torch.cuda.synchronize()
    pkg.ops.gemm = _orig
    tot = 0.0
    print(f"{len(calls)} gemm calls")
    for (A, B, C, M, N, K, kw) in calls:
        if only_wgrad and not (kw.get("accumulate") and K > 4096):
            continue
        us = timed(lambda: _orig(A, B, C, M, N, K, **kw))
        tot += us
        fl = 2.0 * M * N * K
        by = (M * K + N * K) * A.element_size() + M * N * C.element_size()
        tag = f"M={M:6d} N={N:4d} K={K:6d} ak={int(kw['a_kmajor'])} bk={int(kw['b_kmajor'])} " \
              f"acc={int(kw.get('accumulate', False))} {str(A.dtype)[6:]}"
        extra = ""
        if sweep and kw.get("accumulate") and kw.get("act", 0) == 0:
            res = []
            for s in (8, 16, 24, 32, 48, 64):
                kw2 = dict(kw, split_k=s)
                res.append(f"{s}:{timed(lambda: _orig(A, B, C, M, N, K, **kw2)):.1f}")
            extra = " sweep " + " ".join(res)
        print(f"{us:8.2f} us  {fl / us / 1e6:7.1f} TF/s  {by / us / 1e3:7.1f} GB/s  {tag}{extra}")
    print(f"total {tot:.1f} us")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""GPU diagnostic (not a test): where the cfg-2 step's weight-gradient flush spends its time.
Runs one eager cfg-2 TrainStep with WgradPending.flush wrapped to keep its descriptors, then
times (HIP events, 50 reps each) the grouped GEMM launch alone, the whole fold launch, and
every fold segment alone (S, M, N, units printed)."""
import ctypes
import importlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module("music-recommendation-multimodal_amd")
import bench  # noqa: E402

ops = pkg.ops
lib = pkg.lib
dev = torch.device("cuda", 0)
captured = []
_orig = ops.WgradPending.flush


def flush(self):
    captured.append((list(self.items), list(self.folds)))
    _orig(self)


ops.WgradPending.flush = flush


def timeit(fn, reps=20, replays=10):
    """Device time per call: `reps` calls captured in one HIP graph, replayed (the host launch
    cost of a ctypes call would otherwise dominate these few-microsecond kernels)."""
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(replays):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / (reps * replays) * 1e3


def main():
    torch.manual_seed(0)
    m = pkg.TwoTowerModel(vocab_size=bench.V, tabular_input_dim=128, num_genders=bench.N_GENDERS,
                          num_countries=bench.N_COUNTRIES, max_seq_len=bench.L, user_embedding_dim=128,
                          item_embedding_dim=128, user_num_heads=bench.H, user_dropout=0.1,
                          compute_dtype=torch.bfloat16, precomputed_modalities=True).to(dev)
    step = pkg.TrainStep(m, lr=1e-4, use_graph=False, seed=1)
    batch = bench.synthetic_batches(1, 512, seed=0, device=dev)[0]
    step.step(batch)
    torch.cuda.synchronize()
    WD = lib.WgradDesc
    for fi, (items, folds) in enumerate(captured):
        arr = (ctypes.POINTER(WD) * max(len(items), 1))(*[ctypes.pointer(d) for d, *_ in items])
        fds = [f for f, *_ in folds]
        farr = (lib.FoldDesc * max(len(fds), 1))(*fds)
        none = (lib.FoldDesc * 1)()
        print(f"flush {fi}: {len(items)} GEMMs, {len(fds)} fold segments", flush=True)
        if items:
            t = timeit(lambda: ops.call("ttmi_wgrad_batch", len(items), arr, 0, none, ops._s()))
            print(f"  grouped GEMMs (+ their split folds): {t:7.2f} us")
        if fds:
            t = timeit(lambda: ops.call("ttmi_wgrad_batch", 0, arr, len(fds), farr, ops._s()))
            print(f"  fold launch, extra segments only: {t:7.2f} us")
        for j, f in enumerate(fds):
            one = (lib.FoldDesc * 1)(f)
            t = timeit(lambda: ops.call("ttmi_wgrad_batch", 0, arr, 1, one, ops._s()))
            print(f"  seg {j:2d}: S {f.S:5d} M {f.M:6d} N {f.N:4d} acc {f.accumulate} fx {f.fx_shift:2d}"
                  f"  {t:7.2f} us", flush=True)
        for k, (d, *_) in enumerate(items):
            one = (ctypes.POINTER(WD) * 1)(ctypes.pointer(d))
            t = timeit(lambda: ops.call("ttmi_wgrad_batch", 1, one, 0, none, ops._s()))
            print(f"  gemm {k:2d}: M {d.M:4d} N {d.N:4d} R {d.R:6d}  {t:7.2f} us", flush=True)


if __name__ == "__main__":
    main()

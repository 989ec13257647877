"""Micro-benchmark: ttmi_wgrad + fold on the cfg-2 big weight-gradient shapes, each alone
(HIP events, 50 reps), and torch.sum over an [S, M*N] slab of the same bytes for scale."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pkg = importlib.import_module("music-recommendation-multimodal_amd")
ops = pkg.ops
dev = "cuda"


def timeit(fn, reps=50):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


for M, N, R in ((384, 128, 25600), (128, 128, 25600), (512, 128, 25600), (128, 512, 25600),
                (512, 512, 512), (128, 176, 512)):
    dy = torch.randn(R, M, device=dev).bfloat16()
    x = torch.randn(R, N, device=dev).bfloat16()
    gw = torch.zeros(M, N, device=dev)
    gb = torch.zeros(M, device=dev)
    t_all = timeit(lambda: ops.linear_dw(dy, x, gw, gb))
    pend_t = []

    def stage1():
        with ops.deferred_wgrad() as p:
            ops.linear_dw(dy, x, gw, gb)
            pend_t.append(p.items[:])
            p.items = []
    t1 = timeit(stage1)
    d = pend_t[-1]
    S = (d[0][1].numel() // 4) // (M * N) if d else 1
    slab = torch.randn(max(S, 1), M * N, device=dev)
    t_sum = timeit(lambda: slab.sum(0))
    t_atomic = timeit(lambda: ops.gemm(dy, x, gw, M, N, R, lda=M, a_kmajor=False, ldb=N,
                                       b_kmajor=False, ldc=N, accumulate=True, rowsum_a=gb))
    print(f"M={M} N={N} R={R}: wgrad+fold {t_all:6.1f} us, stage1 {t_1:6.1f}" if False else
          f"M={M} N={N} R={R} S~{S}: wgrad+fold {t_all:6.1f} us  stage1 {t1:6.1f} us  "
          f"torch.sum(slab) {t_sum:6.1f} us  atomic path {t_atomic:6.1f} us", flush=True)

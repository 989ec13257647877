"""Token-GEMM shapes of the cfg-4 text encoder (M = 256·256 tokens): the 256x256 LDS-DMA
tile kernel vs the generic 128x128 kernel (TTMI_NO_BIG) vs torch.matmul (hipBLASLt, no
epilogue), HIP-event timed in one process on the same random operands."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pkg = importlib.import_module("music-recommendation-multimodal_amd")
ops = pkg.ops


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    dev = "cuda"
    M = 65536
    g = torch.Generator(device=dev).manual_seed(0)
    for name, N, K, epi in (("qkv", 2304, 832, "bias"), ("out", 768, 768, "res"),
                            ("ffn1", 3072, 768, "bias"), ("ffn1g", 3072, 768, "gelu"),
                            ("ffn2", 768, 3072, "res"),
                            ("dpre", 3072, 768, "gelu'"), ("dxn", 768, 2304, "res")):
        A = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        W = (torch.rand(N, K, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        bias = torch.randn(N, device=dev, generator=g)
        kw, C = {}, torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        if epi == "bias":
            kw = dict(bias=bias)
        elif epi == "gelu":
            kw = dict(bias=bias, act=2, pre_out=torch.empty(M, N, device=dev, dtype=torch.bfloat16))
        elif epi == "res":
            C = torch.empty(M, N, device=dev)
            kw = dict(bias=bias, residual=torch.randn(M, N, device=dev, generator=g), ld_res=N)
        else:
            kw = dict(act=3, gate=torch.randn(M, N, device=dev, generator=g).to(torch.bfloat16), ld_gate=N)

        def ours():
            ops.gemm(A, W, C, M, N, K, lda=K, a_kmajor=True, ldb=K, b_kmajor=True, ldc=N, **kw)
        ref = A.float() @ W.float().t()
        fl = 2.0 * M * N * K
        t_big = timed(ours)
        os.environ["TTMI_NO_BIG"] = "1"
        t_old = timed(ours)
        del os.environ["TTMI_NO_BIG"]
        t_blas = timed(lambda: torch.matmul(A, W.t()))
        print(f"{name:5s} M={M} N={N:5d} K={K:5d} {epi:6s} big {t_big:8.1f} us {fl/t_big/1e6:7.1f} TF/s | "
              f"128x128 {t_old:8.1f} us {fl/t_old/1e6:7.1f} | hipBLASLt {t_blas:8.1f} us {fl/t_blas/1e6:7.1f}",
              flush=True)
        del ref


if __name__ == "__main__":
    main()

"""ResNet-18 gradient-parity diagnostic for test_resnet18_vs_oracle's BatchNorm margin.

For each size it runs the bf16-storage emulation (tests/test_gpu_cnn.py) under every fp32
accumulation order in EMU_ORDERS and prints, per parameter, the spread of the emulations'
gradient cosine against the fp32 oracle: that spread is what the choice of summation order
alone does to a bf16 pipeline.  With a GPU it also prints the GPU's cosine (both conv kernel
families, TTMI_CONV_DMA = 0 / 1) against the worst emulation.
Usage: python tools/diag_resnet_margin.py [--cpu-only]"""
import importlib
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, ".."))
import test_gpu_cnn as T  # noqa: E402

pkg = importlib.import_module("music-recommendation-multimodal_amd")
gpu = torch.cuda.is_available() and "--cpu-only" not in sys.argv
if gpu:
    pkg.lib.load()
for in_ch, H, W, N in ((1, 128, 256, 4), (3, 224, 224, 4)):
    torch.manual_seed(in_ch)
    net0 = pkg.cnn.ResNet18(in_ch, 128)
    sd0 = {k: v.detach().clone() for k, v in net0.state_dict().items()}
    g = torch.Generator().manual_seed(11)
    x = torch.randn(N, in_ch, H, W, generator=g)
    up = torch.randn(N, 128, generator=g)

    def leaf():
        return {k: (v.clone().requires_grad_(True) if v.is_floating_point() and "running" not in k
                    else v.clone()) for k, v in sd0.items()}
    Pr = leaf()
    (T.rref.resnet18_forward(Pr, x, update_running=True) * up).sum().backward()
    cos = {}
    for order in T.EMU_ORDERS:
        Pe = leaf()
        (T.resnet18_bf16_emulation(Pe, x, order=order) * up).sum().backward()
        for n in Pe:
            if Pe[n].requires_grad:
                cos.setdefault(n, []).append(T._cos(Pe[n].grad, Pr[n].grad))
    rows = sorted(((max(c) - min(c), n, c) for n, c in cos.items()), reverse=True)
    print(f"{in_ch}x{H}x{W} N={N}: widest emulation spreads over {len(T.EMU_ORDERS)} accumulation orders")
    for sp, n, c in rows[:8]:
        print(f"  {n:36s} spread {sp:.4f}  cos " + " ".join(f"{v:.4f}" for v in c))
    if not gpu:
        continue
    for dma in ("0", "1"):
        os.environ["TTMI_CONV_DMA"] = dma
        net = pkg.cnn.ResNet18(in_ch, 128).to("cuda")
        net.load_state_dict(sd0)
        (net(x.to("cuda")) * up.to("cuda")).sum().backward()
        torch.cuda.synchronize()
        d = sorted((T._cos(p.grad, Pr[n].grad) - min(cos[n]), n) for n, p in net.named_parameters())
        print(f"  GPU dma={dma}: worst (gpu cos - worst emulation cos):",
              ", ".join(f"{n} {v:+.4f}" for v, n in d[:4]), flush=True)

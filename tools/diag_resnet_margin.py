"""Per-parameter gradient cosine margins of the GPU ResNet-18 against the bf16 emulation's, at
the full audio size (1x128x256) for batch 4 and 8 and both conv kernel families (diagnostic for
test_resnet18_vs_oracle's margin).  Usage: python tools/diag_resnet_margin.py"""
import importlib
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, ".."))
import test_gpu_cnn as T  # noqa: E402

pkg = importlib.import_module("music-recommendation-multimodal_amd")
pkg.lib.load()
for in_ch, H, W, N in ((1, 128, 256, 4), (1, 128, 256, 8), (3, 224, 224, 4)):
    torch.manual_seed(in_ch)
    net0 = pkg.cnn.ResNet18(in_ch, 128)
    sd0 = {k: v.detach().clone() for k, v in net0.state_dict().items()}
    g = torch.Generator().manual_seed(11)
    x = torch.randn(N, in_ch, H, W, generator=g)
    up = torch.randn(N, 128, generator=g)

    def leaf():
        return {k: (v.clone().requires_grad_(True) if v.is_floating_point() and "running" not in k
                    else v.clone()) for k, v in sd0.items()}
    Pe, Pr = leaf(), leaf()
    (T.resnet18_bf16_emulation(Pe, x) * up).sum().backward()
    (T.rref.resnet18_forward(Pr, x, update_running=True) * up).sum().backward()
    for dma in ("0", "1"):
        os.environ["TTMI_CONV_DMA"] = dma
        net = pkg.cnn.ResNet18(in_ch, 128).to("cuda")
        net.load_state_dict(sd0)
        out = net(x.to("cuda"))
        (out * up.to("cuda")).sum().backward()
        torch.cuda.synchronize()
        rows = []
        for name, p in net.named_parameters():
            cr = T._cos(p.grad, Pr[name].grad)
            ce = T._cos(Pe[name].grad, Pr[name].grad)
            rows.append((cr - ce, name, cr, ce))
        rows.sort()
        print(f"{in_ch}x{H}x{W} N={N} dma={dma}: worst", [f"{n} {cr:.3f} vs emu {ce:.3f} ({d:+.3f})"
                                                        for d, n, cr, ce in rows[:3]], flush=True)

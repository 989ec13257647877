"""cfg-3 full-size loss deviation per conv path (diagnostic for test_cfg3_two_tower_vs_oracle):
the GPU loss for register / LDS-DMA conv kernels x padded / space-to-depth stem next to the fp32
oracle loss and the bf16-emulation loss.  Usage: python tools/diag_cfg3_loss.py"""
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
for B, mel, cover in ((4, (128, 256), (224, 224)), (8, (64, 96), (64, 64))):
    m, batch = T._cfg3(pkg, B=B, mel=mel, cover=cover)
    params = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in m.named_parameters()}
    lref = float(T.ref.two_tower_loss(params, batch, running=None)[0])
    orig = T.rref.resnet18_forward
    T.rref.resnet18_forward = T.resnet18_bf16_emulation
    try:
        pe = {k: v.detach().cpu().clone() for k, v in m.named_parameters()}
        lemu = float(T.ref.two_tower_loss(pe, batch, running=None)[0])
    finally:
        T.rref.resnet18_forward = orig
    bd = {k: v.to(T.DEV) for k, v in batch.items()}
    print(f"B={B} cover={cover}: oracle {lref:.5f}  emu {lemu:.5f} (dev {abs(lemu - lref):.5f})", flush=True)
    for dma in ("0", "1"):
        for s2d in (False, True):
            os.environ["TTMI_CONV_DMA"] = dma
            pkg.cnn.STEM_S2D = s2d
            m2, _ = T._cfg3(pkg, B=B, mel=mel, cover=cover)
            with torch.no_grad():
                loss = float(m2(bd)[0])
            print(f"   dma={dma} s2d={int(s2d)}: gpu {loss:.5f} (dev {abs(loss - lref):.5f})", flush=True)

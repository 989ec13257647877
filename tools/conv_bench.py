"""Per-layer timing of the implicit-GEMM conv (FWD / DGRAD / WGRAD) on the cfg-3 ResNet-18
shapes at B=256 (visual 3x224x224, audio 1x128x256): TFLOP/s per launch with HIP events.
Usage: python tools/conv_bench.py [--batch 256] [--reps 10] [--only visual|audio]"""
import argparse
import importlib
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pkg = importlib.import_module("music-recommendation-multimodal_amd")
ops = pkg.ops
cnn = pkg.cnn


def shapes(in_ch, H, W):
    out = []
    h, w = H, W
    for sp in cnn.resnet18_convs(in_ch):
        out.append(sp)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", default=None)
    ap.add_argument("--wg", default="8:2", help="comma list of WGRAD LDS-DMA <waves>:<stages>")
    ap.add_argument("--ft", default="256:3", help="comma list of FWD/DGRAD LDS-DMA <rows>:<stages>")
    ap.add_argument("--modes", default="fwd,dgrad,wgrad")
    args = ap.parse_args()
    dev = torch.device("cuda")
    N = args.batch
    total = {}
    for name, in_ch, H, W in (("visual", 3, 224, 224), ("audio", 1, 128, 256)):
        if args.only and args.only != name:
            continue
        # walk the network to get each conv's input size
        Hc, Wc = H, W
        hw = {}
        specs = cnn.resnet18_convs(in_ch)
        Ho, Wo = ops.conv_out_hw(Hc, Wc, 7, 2, 3)
        hw[specs[0].name] = (Hc, Wc)
        Hc, Wc = ops.conv_out_hw(Ho, Wo, 3, 2, 1)
        for sp in specs[1:]:
            if sp.name.endswith("conv1.weight") or "downsample" in sp.name:
                hw[sp.name] = (Hc, Wc)
                if sp.name.endswith("conv1.weight"):
                    H1, W1 = ops.conv_out_hw(Hc, Wc, sp.k, sp.stride, sp.pad)
            else:
                hw[sp.name] = (H1, W1)
                Hc, Wc = H1, W1
        for sp in specs:
            h, w = hw[sp.name]
            stem = sp.cin < 8
            C = cnn.stem_s2d_cp(sp.cin) if stem else sp.cin
            Ho, Wo = ops.conv_out_hw(h, w, sp.k, sp.stride, sp.pad)
            x = torch.randn(N, h // 2 if stem else h, w // 2 if stem else w, C, device=dev).to(torch.bfloat16)
            dy = torch.randn(N, Ho, Wo, sp.cout, device=dev).to(torch.bfloat16)
            kk = 4 if stem else sp.k
            wf = torch.randn(sp.cout, kk, kk, C, device=dev).to(torch.bfloat16)
            wd = torch.randn(C, sp.k, sp.k, sp.cout, device=dev).to(torch.bfloat16)
            y = torch.empty(N, Ho, Wo, sp.cout, device=dev, dtype=torch.bfloat16)
            cs = torch.zeros(ops.CONV_STAT_REPS, sp.cout, device=dev, dtype=torch.int64)
            cq = torch.zeros(ops.CONV_STAT_REPS, sp.cout, device=dev, dtype=torch.int64)
            dx = torch.empty(N, h, w, C, device=dev, dtype=torch.bfloat16) if not stem else None
            dw = torch.zeros(sp.cout, sp.cin, sp.k, sp.k, device=dev)
            fl = 2.0 * N * Ho * Wo * sp.cout * sp.cin * sp.k * sp.k
            row = []
            for mode, mname in ((ops.FWD, "fwd"), (ops.DGRAD, "dgrad"), (ops.WGRAD, "wgrad")):
                if mode == ops.DGRAD and sp.cin < 8:
                    row.append("      -     ")
                    continue

                md = {ops.FWD: ops.STEM_FWD, ops.WGRAD: ops.STEM_WGRAD}.get(mode, mode) if stem else mode

                def run():
                    if mode == ops.FWD:
                        ops.conv2d(md, N, h, w, C, sp.cin, sp.cout, sp.k, sp.stride, sp.pad,
                                   x=x, w=wf, out=y, colsum=cs, colsumsq=cq)
                    elif mode == ops.DGRAD:
                        ops.conv2d(mode, N, h, w, C, sp.cin, sp.cout, sp.k, sp.stride, sp.pad,
                                   dy=dy, w=wd, out=dx)
                    else:
                        ops.conv2d(md, N, h, w, C, sp.cin, sp.cout, sp.k, sp.stride, sp.pad,
                                   x=x, dy=dy, out=dw)
                if mname not in args.modes.split(","):
                    continue
                variants = [("0", None)] + [("1", w) for w in (args.wg if mode == ops.WGRAD else args.ft).split(",")]
                for var, wg in variants:
                    os.environ["TTMI_CONV_DMA"] = var
                    if wg:
                        os.environ["TTMI_CONV_WG" if mode == ops.WGRAD else "TTMI_CONV_FT"] = wg
                    run()
                    torch.cuda.synchronize()
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(args.reps):
                        run()
                    e1.record()
                    torch.cuda.synchronize()
                    us = e0.elapsed_time(e1) * 1e3 / args.reps
                    key = mname + (("/dma" + (wg or "")) if var == "1" else "/reg")
                    total[key] = total.get(key, 0.0) + us
                    row.append(f"{key} {us:7.1f}us {fl / us / 1e6:6.1f}TF")
                for k in ("TTMI_CONV_DMA", "TTMI_CONV_WG", "TTMI_CONV_FT"):
                    os.environ.pop(k, None)
            print(f"{name:6s} {sp.name:28s} {h:3d}x{w:<3d} {sp.cin:3d}->{sp.cout:3d} k{sp.k}s{sp.stride} "
                  f"GF={fl / 1e9:6.1f} | " + " | ".join(row), flush=True)
    print("totals (us):", {k: round(v, 1) for k, v in total.items()})


if __name__ == "__main__":
    main()

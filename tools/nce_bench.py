#!/usr/bin/env python3
"""InfoNCE kernel timing at cfg-2 size (GPU diagnostic)."""
import importlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module("music-recommendation-multimodal_amd")
from tools.gemm_profile import timed  # noqa: E402


def main():
    F, ops = pkg.functional, pkg.ops
    dev = torch.device("cuda", 0)
    for B in (512, 1024, 2048):
        D = 128
        u = torch.randn(B, D, device=dev)
        it = torch.randn(B, D, device=dev)
        uid = torch.randint(0, 840, (B,), device=dev)
        loss, logits, uh, ih, st = F.infonce_fwd(u, it, uid)
        du, di = torch.empty_like(u), torch.empty_like(it)
        t_f = timed(lambda: ops.infonce_fwd(u, it, uid, 1 / 0.07, st.u_hat, st.i_hat, st.norms,
                                            st.logits, st.lse, loss, st.ws))
        t_b = timed(lambda: F.infonce_bwd(st, None, du, di))
        print(f"B={B}: fwd {t_f:.2f} us  bwd {t_b:.2f} us", flush=True)


if __name__ == "__main__":
    main()

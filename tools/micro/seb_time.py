"""Time ttmi_seq_embed_bwd alone at the cfg-2 shape (B 512, L 50, D 128, V 10136, dropout 0.1),
against whichever library TTMI_LIB names (e.g. the -DTTMI_DIAG_NOATOM diagnostic build, whose
kernel skips the embedding-row fixed-point scatter).  GPU diagnostic."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
pkg = importlib.import_module("music-recommendation-multimodal_amd")
pkg.lib.load(os.environ.get("TTMI_LIB", pkg.lib.LIB_PATH))
ops = pkg.ops
dev = "cuda"
B, L, D, V = 512, 50, 128, 10136
g = torch.Generator().manual_seed(0)
lens = torch.randint(1, L + 1, (B,), generator=g)
ids = torch.randint(1, V, (B, L), generator=g)
ids[torch.arange(L)[None] >= lens[:, None]] = 0
ids = ids.to(dev)
E = (torch.randn(V, D, generator=g) * 0.05).to(dev)
P = (torch.randn(L, D, generator=g) * 0.05).to(dev)
w = torch.ones(D, device=dev)
mean = torch.zeros(B * L, device=dev)
rstd = torch.ones(B * L, device=dev)
dx = torch.randn(B * L, D, generator=g).to(dev)
dE, dP = torch.zeros(V, D, device=dev), torch.zeros(L, D, device=dev)
dw, db = torch.zeros(D, device=dev), torch.zeros(D, device=dev)
seed = torch.tensor([7], dtype=torch.int64, device=dev)
with ops.deferred_wgrad():
    for _ in range(3):
        ops.seq_embed_bwd(ids, E, P, w, mean, rstd, dx, dE, dP, dw, db, drop=(0.1, seed))
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
n = 200
with ops.deferred_wgrad():
    torch.cuda._sleep(100000)
    a.record()
    for _ in range(n):
        ops.seq_embed_bwd(ids, E, P, w, mean, rstd, dx, dE, dP, dw, db, drop=(0.1, seed))
    b.record()
torch.cuda.synchronize()
print(f"{os.environ.get('TTMI_LIB', 'libttmi.so')}: seq_embed_bwd {a.elapsed_time(b) * 1000 / n:.2f} us/launch "
      f"(tokens {int((ids != 0).sum())} of {B * L})")

if os.environ.get("SEB_STAMPS"):       # the stamp build: 0 start, 1.. pass k starts (SEB_R of them, up to 7)
    import ctypes
    import numpy as np
    NB, NW, NP = 512, 16, 8
    fn = pkg.lib._lib.ttmi_dbg_stamps_norm
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    buf = (ctypes.c_uint64 * (NB * NW * NP))()
    with ops.deferred_wgrad():
        fn(buf, NB * NW * NP)
        torch.cuda._sleep(200000)
        ops.seq_embed_bwd(ids, E, P, w, mean, rstd, dx, dE, dP, dw, db, drop=(0.1, seed))
    torch.cuda.synchronize()
    fn(buf, NB * NW * NP)
    a_ = np.array(buf, dtype=np.float64).reshape(NB, NW, NP)[:, :8, :]
    live = a_[:, :, 0] > 0
    t0 = a_[:, :, 0][live].min()
    for k in range(8):
        v = (a_[:, :, k][live] - t0) / 100.0
        print(f"  phase {k}: median {np.median(v):6.2f} max {v.max():6.2f} us (first 512 blocks)")

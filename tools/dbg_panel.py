"""EXPERIMENT: per-wave phase timestamps (s_memrealtime, 100 MHz) of one LN-backward panel launch."""
import ctypes, importlib, os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pkg = importlib.import_module("music-recommendation-multimodal_amd")
ops = pkg.ops
M, K, D = 25600, 512, 128
dh = torch.randn(M, K, device="cuda").bfloat16()
wt = (torch.randn(D, K, device="cuda") / 20).bfloat16()
x = torch.randn(M, D, device="cuda"); mean = x.mean(1); rstd = torch.rsqrt(x.var(1) + 1e-5)
w = torch.randn(D, device="cuda"); res = torch.randn(M, D, device="cuda")
dx = torch.empty(M, D, device="cuda"); nxt = torch.empty(M, D, device="cuda", dtype=torch.bfloat16)
dw = torch.zeros(D, device="cuda"); db = torch.zeros(D, device="cuda")
seed = torch.zeros(1, dtype=torch.int64, device="cuda")
for it in range(3):
    with ops.deferred_wgrad():
        ops.linear_ln_bwd(dh, wt, x, mean, rstd, w, dx, dw, db, res=res, next_=nxt, drop=(0.1, seed))
    torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * (256 * 8 * 6))()
lib = pkg.lib._lib
lib.ttmi_dbg_dump(buf)
a = np.array(buf, dtype=np.float64).reshape(256, 8, 6)
a = a[:229, :7]
t0 = a[:, :, 0].min()
r = (a - t0) / 100.0   # microseconds (100 MHz)
names = ["start", "W staged", "after sync", "MFMA done", "epi done", "end sync"]
for k in range(6):
    print(f"{names[k]:12s} min {r[:,:,k].min():7.2f} med {np.median(r[:,:,k]):7.2f} max {r[:,:,k].max():7.2f} us")

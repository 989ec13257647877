"""Per-wave phase timings (s_memrealtime stamps, 100 MHz) of the cfg-2 row-panel launches and
the fused user head, from the diagnostic build (tools/stamp_build.sh).  GPU diagnostic:
    TTMI_LIB=music-recommendation-multimodal_amd/lib/diag/libttmi_stamp.so python tools/stamp_phases.py
Phases (panel_kernel): 0 start, 1 W DMA issued, 2 W in LDS (after the barrier), 3 first
tile's first column group MFMAs done, 4 first tile done, 5 all tiles done, 6 end.
Phases (qkv_attn_fwd): 0 start, 1 W group 0 in LDS, 2 projection done, 3 attention done.
Phases (ffn_block_fwd): 0 start, 1 group 0 in LDS, 2-5 hidden groups 0-3 done, 6 end.
Phases (user_head_fwd, the FFN-split kernel): 0 start, 1 prologue, 2 out-proj + LN2, 3 FFN1
slice, 4 FFN2 partial, 5 handoff done (the last arriver), 6 x2, 7 end."""
import ctypes
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pkg = importlib.import_module("music-recommendation-multimodal_amd")
pkg.lib.load(os.environ["TTMI_LIB"])
ops = pkg.ops
NB, NW, NP = 512, 16, 8
lib = pkg.lib._lib
for tu in ("gemm", "head", "infonce", "attn", "ffn"):
    getattr(lib, "ttmi_dbg_stamps_" + tu).argtypes = [ctypes.c_void_p, ctypes.c_int64]
buf = (ctypes.c_uint64 * (NB * NW * NP))()


def stamps(fn, name, nph=7, tu="gemm"):
    dump = getattr(lib, "ttmi_dbg_stamps_" + tu)
    fn()
    torch.cuda.synchronize()
    dump(buf, NB * NW * NP)                         # clear
    if os.environ.get("STAMP_BUSY"):   # keep every XCD busy up to the measured launch
        torch.cuda._sleep(int(os.environ["STAMP_BUSY"]))
    fn()
    assert dump(buf, NB * NW * NP) == 0
    a = np.array(buf, dtype=np.float64).reshape(NB, NW, NP)[:, :, :nph]
    live = a[:, :, 0] > 0
    t0 = a[:, :, 0][live].min()
    rel = (a - t0) / 100.0                          # microseconds
    cols = []
    for k in range(nph):
        v = rel[:, :, k][live & (a[:, :, k] > 0)]
        cols.append(f"{np.median(v):6.2f}/{v.max():6.2f}" if v.size else "   -   ")
    print(f"{name:34s} " + "  ".join(cols), flush=True)
    if os.environ.get("STAMP_XCD"):    # start-time spread by XCD (block id % 8)
        blk = np.arange(NB)
        for x in range(8):
            sel = (blk % 8 == x)[:, None] & live
            v = rel[:, :, 0][sel]
            e = rel[:, :, nph - 1][sel & (a[:, :, nph - 1] > 0)]
            if v.size:
                print(f"    xcd {x}: start min {v.min():5.2f} med {np.median(v):5.2f} max {v.max():5.2f}  "
                      f"end med {np.median(e) if e.size else 0:6.2f} max {e.max() if e.size else 0:6.2f}  n={v.size}")


def main():
    dev = "cuda"
    M, D = 25600, 128
    g = torch.Generator(device="cpu").manual_seed(0)

    def bf(*s, sc=0.05):
        return (torch.randn(*s, generator=g) * sc).to(torch.bfloat16).to(dev)

    def f32(*s, sc=1.0):
        return (torch.randn(*s, generator=g) * sc).to(dev)
    seed = torch.tensor([7], dtype=torch.int64, device=dev)
    drop = (0.1, seed)
    a1 = bf(M, D, sc=1.0)
    print("phase medians / max in us:  " + "  ".join(f"p{k}" + " " * 10 for k in range(7)))
    w_in, b_in = bf(3 * D, D), f32(3 * D, sc=0.1)
    qkv = torch.empty(M, 3 * D, device=dev, dtype=torch.bfloat16)
    stamps(lambda: ops.linear(a1, w_in, b_in, qkv), "qkv fwd 384x128")
    # the fused in_proj + attention (phases: 0 start, 1 W group 0 in LDS, 2 projection done,
    # 3 attention done)
    kvm = (torch.arange(50)[None] < torch.randint(1, 51, (512, 1), generator=g)).long().to(dev)
    ctxq = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    lseq = torch.empty(512 * 4 * 50, device=dev)
    stamps(lambda: ops.qkv_attn_fwd(a1, w_in, b_in, kvm, 512, 50, 4, qkv, ctxq, lseq, drop),
           "qkv + attention fwd", nph=4, tu="attn")
    # the fused feed-forward sub-block (phases: 0 start, 1 group 0 in LDS, 2-5 groups 0-3 done
    # (after the next group's wait), 6 end)
    w1f, b1f, w2f, b2f = bf(512, D), f32(512, sc=0.1), bf(D, 512), f32(D, sc=0.1)
    x1f, hf, x2f = f32(M, D), torch.empty(M, 512, device=dev, dtype=torch.bfloat16), torch.empty(M, D, device=dev)
    yf, muf, rsf = torch.empty(M, D, device=dev, dtype=torch.bfloat16), torch.empty(M, device=dev), torch.empty(M, device=dev)
    lnwf, lnbf = f32(D), f32(D)
    stamps(lambda: ops.ffn_block_fwd(a1, w1f, b1f, w2f, b2f, x1f, drop, drop, hf, x2f, lnwf, lnbf, 1e-5, yf, muf, rsf),
           "ffn block fwd", nph=7, tu="ffn")
    w = np.array(buf, dtype=np.float64).reshape(NB, NW, NP)[:, :8, 7]
    w = w[w > 0] / 100.0
    if w.size:
        print(f"    group-seam wait per wave (us): median {np.median(w):.2f}  max {w.max():.2f}")
    nod = (0.0, None)
    stamps(lambda: ops.ffn_block_fwd(a1, w1f, b1f, w2f, b2f, x1f, nod, nod, hf, x2f, lnwf, lnbf, 1e-5, yf, muf, rsf),
           "ffn block fwd, no dropout", nph=7, tu="ffn")
    # its backward (phases: 0 start, 1 prologue done, 2-5 hidden groups 0-3 done, 6 end, 7 the
    # LayerNorm backward's row stores issued)
    dy2f, w2tf, w1tf = bf(M, D, sc=0.1), bf(512, D), bf(D, 512)
    dz1f, dx1f, dy1f = torch.empty(M, 512, device=dev, dtype=torch.bfloat16), torch.empty(M, D, device=dev), \
        torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    gwf, gbf = torch.zeros(D, device=dev), torch.zeros(D, device=dev)
    stamps(lambda: ops.ffn_block_bwd(dy2f, w2tf, w1tf, hf, 1 / 0.9, dz1f, x1f, muf, rsf, lnwf, x2f, dx1f, dy1f,
                                     drop, gwf, gbf), "ffn block bwd (p7: row stores issued)", nph=8, tu="ffn")
    if os.environ.get("STAMP_FFN_ONLY"):
        return
    wo, bo = bf(D, D), f32(D, sc=0.1)
    x, x1 = f32(M, D), torch.empty(M, D, device=dev)
    lnw, lnb = 1 + f32(D, sc=0.1), f32(D, sc=0.1)
    a2, mu, rs = torch.empty(M, D, device=dev, dtype=torch.bfloat16), torch.empty(M, device=dev), torch.empty(M, device=dev)
    stamps(lambda: ops.linear_res_ln(a1, wo, bo, x, x1, lnw, lnb, a2, mu, rs, drop=drop), "out-proj + res + LN 128x128")
    w1, b1 = bf(4 * D, D), f32(4 * D, sc=0.1)
    h = torch.empty(M, 4 * D, device=dev, dtype=torch.bfloat16)
    stamps(lambda: ops.linear(a2, w1, b1, h, act=1, drop=drop), "FFN1 512x128 relu drop")
    w2, b2 = bf(D, 4 * D), f32(D, sc=0.1)
    x2 = torch.empty(M, D, device=dev)
    stamps(lambda: ops.linear_res_ln(h, w2, b2, x1, x2, lnw, lnb, a2, mu, rs, drop=drop), "FFN2 128x512 + res + LN")
    dqkv = bf(M, 3 * D, sc=1.0)
    w_in_t = bf(D, 3 * D)
    dx = torch.empty(M, D, device=dev)
    nxt = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    dw, db = torch.zeros(D, device=dev), torch.zeros(D, device=dev)

    def lnbwd(dh, wt):
        with ops.deferred_wgrad():
            ops.linear_ln_bwd(dh, wt, x, mu, rs, lnw, dx, dw, db, res=x1, next_=nxt, drop=drop)
    stamps(lambda: lnbwd(dqkv, w_in_t), "qkv dgrad + LN bwd K=384")
    dy2 = bf(M, D, sc=1.0)
    w2t = bf(4 * D, D)
    dz1 = torch.empty(M, 4 * D, device=dev, dtype=torch.bfloat16)
    stamps(lambda: ops.linear(dy2, w2t, None, dz1, gate=h, gate_scale=1 / 0.9), "FFN2 dgrad 512x128 gated")
    w1t = bf(D, 4 * D)
    stamps(lambda: lnbwd(dz1, w1t), "FFN1 dgrad + LN bwd K=512")
    dctx = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    stamps(lambda: ops.linear(dy2, bf(D, D), None, dctx), "out-proj dgrad 128x128")
    # the fused user head (B = 512): phases of ttmi_user_head_fwd's stages
    B, F = 512, 512
    pre = "l."
    W = {pre + "self_attn.out_proj.weight": bf(D, D), pre + "linear1.weight": bf(F, D),
         pre + "linear2.weight": bf(D, F), "fusion_layer.0.weight": bf(D, D + 48),
         "fusion_layer.3.weight": bf(D, D)}
    P = {pre + "self_attn.out_proj.bias": f32(D, sc=0.1), pre + "norm2.weight": f32(D), pre + "norm2.bias": f32(D),
         pre + "linear1.bias": f32(F, sc=0.1), pre + "linear2.bias": f32(D, sc=0.1),
         "gender_embedding.weight": f32(3, 16), "country_embedding.weight": f32(11, 32),
         "fusion_layer.0.bias": f32(D, sc=0.1), "fusion_layer.1.weight": f32(D), "fusion_layer.1.bias": f32(D),
         "fusion_layer.3.bias": f32(D, sc=0.1)}
    ctx, res = bf(B, D, sc=1.0), f32(B, D)
    drows = torch.arange(B, dtype=torch.int32, device=dev) * 50
    gender = torch.randint(0, 3, (B,), generator=g).to(dev)
    country = torch.randint(0, 11, (B,), generator=g).to(dev)
    seeds = torch.tensor([1, 2, 3], dtype=torch.int64, device=dev)
    drops = tuple((0.1, seeds[k:k + 1]) for k in range(3))
    o = dict(x1=f32(B, D), a2=bf(B, D), m2=f32(B), r2=f32(B), h=bf(B, F), comb=bf(B, D + 48),
             rows=torch.empty(B, dtype=torch.int32, device=dev), z=f32(B, D), az=bf(B, D),
             mz=f32(B), rz=f32(B), u=f32(B, D))
    stamps(lambda: ops.user_head_fwd(ctx, res, drows, W, P, pre, gender, country, 1e-5, drops, o),
           "user head fwd (B=512)", nph=8, tu="head")
    # InfoNCE at B = 512 (phases: fwd 0 start, 1 Q staged, 2 logit tiles done, 3 partials
    # retired, 4 arrival counted, 5 block combine done, 6 final combine; bwd 0 start,
    # 1 G.V MFMAs done, 2 partials retired, 3 arrival counted, 4 finish done)
    F_ = pkg.functional
    u, it = f32(B, D), f32(B, D)
    uid = torch.randint(0, 840, (B,), generator=g).to(dev)
    _, _, _, _, st = F_.infonce_fwd(u, it, uid)
    loss = torch.empty((), device=dev)
    stamps(lambda: ops.infonce_fwd_pre(uid, st.inv_tau, st.u_hat, st.i_hat, st.norms, st.logits, st.lse,
                                       loss, st.ws),
           "infonce fwd (B=512)", tu="infonce")
    du, di = torch.empty(B, D, device=dev), torch.empty(B, D, device=dev)
    du16 = torch.empty(B, D, device=dev, dtype=torch.bfloat16)
    stamps(lambda: ops.infonce_bwd(st.u_hat, st.i_hat, st.norms, st.logits, st.lse, uid, st.inv_tau, None,
                                   du, di, st.ws, du16), "infonce bwd fused (B=512)", nph=5, tu="infonce")


if __name__ == "__main__":
    main()

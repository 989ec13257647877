#!/usr/bin/env python3
"""Throughput of the MI355X two-tower training step (BASELINE.json metric).

Workload (BASELINE cfg 2, the configuration the metric is quoted on): SASRec user tower
(L=50, D=128, 4 heads, 2 layers, V=10,136 item vocabulary) + late-fusion item head on
precomputed 512-d modality embeddings + symmetric in-batch InfoNCE, B=512 pairs per GPU,
bf16 operands / fp32 accumulation, dropout 0.1 on (reference defaults), AdamW lr 1e-4.
One step = forward + backward + AdamW over one synthetic batch already resident in HBM.

Multi-GPU: one process per GPU (torchrun), per-GPU batch fixed (weak scaling), gradients
averaged with RCCL all-reduce; value = pairs of all ranks / max-over-ranks time.

``--config 3`` measures BASELINE configs[2] instead (full item tower on raw 128x256 mels,
224x224 covers and tabular features, B=256; its roofline is the implicit-GEMM conv);
``--config 4`` adds the mDeBERTa-v3-base + LoRA lyrics encoder (configs[3], S=256; its
roofline is the text encoder's token GEMMs).

Extra fields: "roofline" for the dominant kernel (timed live with HIP events on the launch
stream) and "cpu_baseline" (the fp32 CPU oracle timed on this host, rank 0 at N=1).
"""
from __future__ import annotations

import argparse
import glob
import importlib
import json
import os
import socket
import subprocess
import sys
import time
from typing import Optional

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
PKG = "music-recommendation-multimodal_amd"
pkg = None          # imported in main(), after the --gpus N launcher has spawned its ranks

V, L, D, H = 10136, 50, 128, 4
N_GENDERS, N_COUNTRIES, N_USERS = 3, 64, 840
PEAK_BF16_TFLOPS = 2500.0       # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0


def synthetic_batches(n: int, B: int, seed: int, device):
    """SURVEY §8(d) synthetic inputs, generated on the host then moved to HBM once."""
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(n):
        lengths = torch.randint(1, L + 1, (B,), generator=g)
        mask = (torch.arange(L)[None] < lengths[:, None]).long()
        ids = torch.randint(1, V, (B, L), generator=g) * mask
        out.append({
            "history_ids": ids.to(device), "history_mask": mask.to(device),
            "user_gender": torch.randint(0, N_GENDERS, (B,), generator=g).to(device),
            "user_country": torch.randint(0, N_COUNTRIES, (B,), generator=g).to(device),
            "user_idx": torch.randint(0, N_USERS, (B,), generator=g).to(device),
            "target_modal": torch.randn(B, 512, generator=g).to(device),
        })
    return out


MEL, COVER, TAB = (128, 256), (224, 224), 128
# SURVEY §8 rows a7/a8 (FlopCounterMode on the torchvision topology): fwd+bwd FLOPs per sample
RESNET_FLOPS_PER_SAMPLE = 6.75e9 + 10.65e9


def add_raw_items(batches, seed: int, device):
    """cfg 3 item inputs (BASELINE configs[2]): N(0,1) mels [B,1,128,256], covers
    [B,3,224,224] and tabular features [B,128], replacing the precomputed embeddings."""
    g = torch.Generator().manual_seed(seed + 7)
    for b in batches:
        B = b["history_ids"].shape[0]
        del b["target_modal"]
        b["target_audio"] = torch.randn(B, 1, *MEL, generator=g).to(device)
        b["target_image"] = torch.randn(B, 3, *COVER, generator=g).to(device)
        b["target_tabular"] = torch.randn(B, TAB, generator=g).to(device)
    return batches


TEXT_S, TEXT_V = 256, 251000
# mDeBERTa-v3-base fwd 50.7 GF + dX-only bwd 53.2 GF per sample, + 14.5 GF per
# batch for the relative-table projections
TEXT_FLOPS_PER_SAMPLE, TEXT_FLOPS_PER_BATCH = 103.9e9, 14.5e9


def add_text(batches, seed: int, device):
    """cfg 4 lyrics: tokens ~U[1, 251000), lengths ~U[16, 256], prefix mask."""
    g = torch.Generator().manual_seed(seed + 11)
    for b in batches:
        B = b["history_ids"].shape[0]
        lengths = torch.randint(16, TEXT_S + 1, (B,), generator=g)
        mask = (torch.arange(TEXT_S)[None] < lengths[:, None]).long()
        ids = torch.randint(1, TEXT_V, (B, TEXT_S), generator=g) * mask
        b["target_input_ids"] = ids.to(device)
        b["target_attention_mask"] = mask.to(device)
    return batches


def step_flops(B: int, pruned: bool = True) -> float:
    """Algorithmic FLOPs of one train step (fwd + bwd = 3x fwd GEMM/attention FLOPs).

    pruned=True is SURVEY §8(d)'s F_min (76.3 MF/pair): the last encoder layer computes K/V
    for every token but Q, attention, out_proj and the FFN only for each sequence's last
    valid row (the only row the user tower reads; output-identical)."""
    M = B * L
    full = 24 * M * D * D + 4 * B * L * L * D
    last = 4 * M * D * D + 20 * B * D * D + 4 * B * L * D if pruned else full
    user_head = 2 * B * (D + 48) * D + 2 * B * D * D
    item_head = 2 * B * 512 * 512 + 2 * B * 512 * D
    loss = 2 * B * B * D
    return 3.0 * (full + last + user_head + item_head + loss)


def record_step(step, batch) -> None:
    """One eager forward + backward of ``step`` for a probe to record its launch mix: no
    collectives, and the fold that TrainStep leaves to AdamW (fold_in_update) switched off, so
    every deferred partial is folded and its persistent workspace re-zeroed here; the flat
    gradient is cleared afterwards.  (The step counter and BatchNorm running statistics advance
    as in a step: the probes run after the timed region.)"""
    keep = step.fold_in_update
    step.fold_in_update = False
    try:
        step._fwd_bwd(step._stage(batch), lambda fn: None)
    finally:
        step.fold_in_update = keep
    step._fold = step._fx = None
    step.flat.grad.zero_()


def _wgrad_call(kw) -> bool:
    return kw.get("accumulate") and not kw["a_kmajor"] and not kw["b_kmajor"]


def probe_dominant(step, batch, device, iters: int = 20):
    """Roofline of the dominant kernel family, the deterministic weight-gradient GEMMs: the
    step's 13 nn.Linear weight gradients (five over 25,600 rows, eight over 512), computed as
    one grouped launch (wgrad_group_kernel) whose split partials the step folds inside its
    AdamW launch (ttmi_wgrad_batch_plan + ttmi_adamw_folded).  One eager forward+backward
    records the exact call mix of a step; the mix, inside one deferred_wgrad(defer_fold=True)
    block as in the step, so the replay is the group launch alone, is captured into a HIP graph
    and replayed `iters` times between HIP events on the launch stream: avg_us = device time of
    the launch / GEMMs.
    Algorithmic bytes per launch: both bf16 operands once (R x (M + N) x 2) plus the fp32
    gradient tile (M x N x 4)."""
    ops = pkg.ops
    calls = []
    orig = ops.linear_dw

    def rec(dy, x, gw, gb=None, split_k=0, defer=True):
        if dy.dtype == torch.bfloat16:
            calls.append((dy, x, gw, gb))
        return orig(dy, x, gw, gb, split_k, defer)

    ops.linear_dw = rec
    try:
        record_step(step, batch)
    finally:
        ops.linear_dw = orig
    torch.cuda.synchronize(device)

    def mix():
        with ops.deferred_wgrad(defer_fold=True):      # GEMMs only: the fold is AdamW's
            for dy, x, gw, gb in calls:
                orig(dy, x, gw, gb)

    side = torch.cuda.Stream(device)
    side.wait_stream(torch.cuda.current_stream(device))
    with torch.cuda.stream(side):
        mix()                                          # warm
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=side):
            mix()
    torch.cuda.current_stream(device).wait_stream(side)
    torch.cuda.synchronize(device)
    st = torch.cuda.current_stream(device)
    g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(iters):
        g.replay()
    e1.record(st)
    torch.cuda.synchronize(device)
    n = max(len(calls), 1)
    sec = e0.elapsed_time(e1) / 1e3 / (iters * n)
    shapes = [(dy.shape[0], dy.shape[1], x.shape[1]) for dy, x, _, _ in calls]
    by = sum(R * (M + N) * 2 + M * N * 4 for R, M, N in shapes) / n
    fl = sum(2.0 * M * N * R for R, M, N in shapes) / n
    gbs = by / sec / 1e9
    # PMC bytes of the family's launch per step (tools/traffic.py), shared out over the step's
    # weight-gradient GEMMs like avg_us
    tg = read_traffic("wgrad_group_kernel")
    traffic = round(tg / n) if tg is not None else None
    return {"kernel": f"ttmi_wgrad_batch_plan: the step's {len(calls)} weight-gradient GEMMs as "
                      "one wgrad_group_kernel launch (deterministic split partials, folded inside "
                      "the step's AdamW launch), graph-replayed; per-GEMM figures",
            "bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(gbs / PEAK_HBM_GBS, 4), "traffic": traffic,
            "avg_us": round(sec * 1e6, 2), "launches_per_step": len(calls),
            "bytes_per_launch": round(by), "flops_per_launch": round(fl),
            "mfma_tflops": round(fl / sec / 1e12, 1)}


def probe_panels(step, batch, device, iters: int = 20, min_rows: int = 4096):
    """Roofline of the second kernel family, the row-panel GEMMs over the encoder's B·L rows
    (panel_kernel / panel256_kernel: QKV, out-proj + residual + LayerNorm, FFN, and their input
    gradients with the LayerNorm backward fused).  As probe_dominant: one eager forward +
    backward records the step's calls of ops.gemm (input-grad / forward GEMMs, weight gradients
    excluded), ops.linear_res_ln and ops.linear_ln_bwd over >= min_rows rows; the mix is
    captured into a HIP graph and replayed between HIP events on the launch stream.
    Algorithmic bytes per launch: every tensor operand once (activations, weights, residual,
    gate, outputs, LayerNorm statistics), i.e. the bytes the launch cannot avoid moving."""
    ops = pkg.ops
    calls = []
    names = ("gemm", "linear_res_ln", "linear_ln_bwd")
    orig = {n: getattr(ops, n) for n in names}

    def wrap(n):
        def rec(*a, **kw):
            rows = a[3] if n == "gemm" else a[0].shape[0]
            if rows >= min_rows and not (n == "gemm" and _wgrad_call(kw)):
                calls.append((n, a, dict(kw)))
            return orig[n](*a, **kw)
        return rec

    for n in names:
        setattr(ops, n, wrap(n))
    try:
        record_step(step, batch)
    finally:
        for n in names:
            setattr(ops, n, orig[n])
    torch.cuda.synchronize(device)
    if not calls:
        return None

    def mix():
        for n, a, kw in calls:
            orig[n](*a, **kw)

    side = torch.cuda.Stream(device)
    side.wait_stream(torch.cuda.current_stream(device))
    with ops.deferred_wgrad():                # LayerNorm-backward partials: folded at exit
        with torch.cuda.stream(side):
            mix()                                          # warm
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=side):
                mix()
    torch.cuda.current_stream(device).wait_stream(side)
    torch.cuda.synchronize(device)
    st = torch.cuda.current_stream(device)
    g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(iters):
        g.replay()
    e1.record(st)
    torch.cuda.synchronize(device)
    n = len(calls)
    sec = e0.elapsed_time(e1) / 1e3 / (iters * n)
    by = fl = 0.0
    for name, a, kw in calls:
        seen = set()
        for t in list(a) + list(kw.values()):
            if isinstance(t, torch.Tensor) and (t.data_ptr(), t.numel()) not in seen:
                seen.add((t.data_ptr(), t.numel()))
                by += t.numel() * t.element_size()
        if name == "gemm":
            fl += 2.0 * a[3] * a[4] * a[5]
        else:
            fl += 2.0 * a[0].shape[0] * a[1].numel()
    by, fl = by / n, fl / n
    gbs = by / sec / 1e9
    return {"kernel": "row-panel GEMMs over the encoder rows (forward QKV / out-proj+res+LN / "
                      "FFN, input grads with the fused LayerNorm backward), graph-replayed; "
                      "per-launch figures",
            "bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(gbs / PEAK_HBM_GBS, 4), "traffic": None,
            "avg_us": round(sec * 1e6, 2), "launches_per_step": n,
            "bytes_per_launch": round(by), "flops_per_launch": round(fl),
            "mfma_tflops": round(fl / sec / 1e12, 1)}


def probe_conv(step, batch, device, iters: int = 3):
    """cfg 3 roofline of the dominant kernel, the implicit-GEMM conv (conv_tile_kernel: FWD,
    DGRAD and WGRAD launches of both ResNet-18s).  As probe_dominant: one eager forward +
    backward records the step's conv launch mix, which is replayed between HIP events on
    the launch stream.  Algorithmic FLOPs per launch: 2·N·Ho·Wo·Co·Cin·k² (the same for all
    three modes; Cin is the real input width, not the padded stem width)."""
    ops = pkg.ops
    calls = []
    orig = ops.conv2d

    def rec(mode, N, H, W, C, Cin, Co, k, stride, pad, **kw):
        calls.append(((mode, N, H, W, C, Cin, Co, k, stride, pad), dict(kw)))
        return orig(mode, N, H, W, C, Cin, Co, k, stride, pad, **kw)

    ops.conv2d = rec
    try:
        record_step(step, batch)
    finally:
        ops.conv2d = orig
    torch.cuda.synchronize(device)
    for a, kw in calls:                                # warm
        orig(*a, **kw)
    st = torch.cuda.current_stream(device)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(iters):
        for a, kw in calls:
            orig(*a, **kw)
    e1.record(st)
    torch.cuda.synchronize(device)
    n = max(len(calls), 1)
    sec = e0.elapsed_time(e1) / 1e3 / (iters * n)
    fl = 0.0
    for (mode, N, H, W, C, Cin, Co, k, stride, pad), _ in calls:
        Ho, Wo = ops.conv_out_hw(H, W, k, stride, pad)
        fl += 2.0 * N * Ho * Wo * Co * Cin * k * k
    fl /= n
    tf = fl / sec / 1e12
    return {"kernel": "conv_tile_kernel (implicit-GEMM conv FWD/DGRAD/WGRAD, per-step launch "
                      "mix of both ResNet-18s)",
            "bound": "mfma", "achieved": round(tf, 2), "peak": PEAK_BF16_TFLOPS,
            "unit": "TFLOP/s", "frac": round(tf / PEAK_BF16_TFLOPS, 4),
            "traffic": read_traffic("conv_tile_kernel"), "avg_us": round(sec * 1e6, 2),
            "launches_per_step": len(calls), "flops_per_launch": round(fl)}


def probe_text_gemm(step, batch, device, iters: int = 3):
    """cfg 4 roofline of the dominant kernel family, the text encoder's GEMMs (gemm_kernel:
    QKV / out-proj / FFN forward and their input-gradient GEMMs).  As probe_dominant: one eager
    forward + backward records the bf16 GEMMs with M >= 4096 rows (the token-parallel ones),
    which are replayed between HIP events on the launch stream.  Algorithmic FLOPs per launch:
    2·M·N·K."""
    ops = pkg.ops
    calls = []
    orig = ops.gemm

    def rec(A, B_, C, M, N, K, **kw):
        if A.dtype == torch.bfloat16 and M >= 4096 and N >= 512 and K >= 512:
            calls.append((A, B_, C, M, N, K, dict(kw)))
        return orig(A, B_, C, M, N, K, **kw)

    ops.gemm = rec
    try:
        record_step(step, batch)
    finally:
        ops.gemm = orig
    torch.cuda.synchronize(device)
    for c in calls:
        orig(*c[:6], **c[6])
    st = torch.cuda.current_stream(device)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(iters):
        for c in calls:
            orig(*c[:6], **c[6])
    e1.record(st)
    torch.cuda.synchronize(device)
    n = max(len(calls), 1)
    sec = e0.elapsed_time(e1) / 1e3 / (iters * n)
    fl = sum(2.0 * M * N * K for (_, _, _, M, N, K, _) in calls) / n
    tf = fl / sec / 1e12
    return {"kernel": "gemm_big_kernel (256x256 LDS-DMA tiles: the text-encoder token GEMMs, QKV+LoRA, "
                      "out-proj, FFN, and their input-gradient GEMMs; per-step launch mix)",
            "bound": "mfma", "achieved": round(tf, 2), "peak": PEAK_BF16_TFLOPS,
            "unit": "TFLOP/s", "frac": round(tf / PEAK_BF16_TFLOPS, 4),
            "traffic": read_traffic("gemm_big_kernel"), "avg_us": round(sec * 1e6, 2),
            "launches_per_step": len(calls), "flops_per_launch": round(fl)}


def cpu_baseline_cfg4(B: int, budget_s: float = 20.0):
    """fp32 CPU oracle cfg-4 train step: cfg 3 + the mDeBERTa-v3-base + LoRA oracle."""
    from oracle import two_tower_ref as ref
    from oracle import resnet_ref as rref
    from oracle import deberta_ref as dref
    threads = torch.get_num_threads()
    g = torch.Generator().manual_seed(0)
    dcfg = dref.DebertaCfg()
    text = dref.init_text_params(dcfg, 128, g, lora_b_std=0.02)
    params = {k: v for k, v in text.items() if "lora_" in k or k.startswith("projection.")}
    frozen = {k: v for k, v in text.items() if k not in params}
    ids, mask = dref.synthetic_text(B, TEXT_S, TEXT_V, generator=g)
    x = {"ids": ids, "mask": mask}
    out_w = torch.randn(128, generator=g)

    def text_step():                       # text encoder fwd + dX/LoRA bwd dominates cfg 4
        leaves = {k: v.detach().requires_grad_(True) for k, v in params.items()}
        out = dref.text_encoder_forward({**frozen, **leaves}, x["ids"], x["mask"], dcfg)
        (out * out_w).sum().backward()
    rate_t, med, tot = _cpu_protocol(text_step, B, warmup=1, timed=5)
    c3 = cpu_baseline_cfg3(8, budget_s)
    value = 1.0 / (1.0 / rate_t + 1.0 / c3["value"])
    return {"value": round(value, 4), "unit": "user-item pairs/s", "cores": threads, "kind": "port",
            **_cpu_host(),
            "sample": f"1 warm-up + 5 timed mDeBERTa-v3-base + LoRA fwd+bwd steps at B={B}, "
                      f"S={TEXT_S} (median {med:.2f} s; fewer steps than BASELINE.md §2's 3 + 10 "
                      f"to keep the sample near 20 s) combined per pair with the cfg-3 oracle "
                      f"rate ({c3['value']} pairs/s: {c3['sample']}); fp32 torch-CPU oracle"}


def _traffic_lookup(name: str, only: Optional[str] = None):
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*traffic*.json")), reverse=True):
        if only is not None and path != only:
            continue
        try:                                   # newest round's file that measured `name`
            with open(path) as f:
                v = json.load(f).get(name, {}).get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            continue
        if v is not None:
            return path, v
    return None, None


def traffic_file(name: str) -> Optional[str]:
    """The committed PMC summary read_traffic(name) takes its figure from."""
    return _traffic_lookup(name)[0]


def read_traffic(name: str, only: Optional[str] = None):
    """Per-launch HBM bytes of `name` from the committed rocprofv3 PMC summary
    (profiles/*traffic*.json, written by tools/traffic.py; `only`: that file alone), or None."""
    return _traffic_lookup(name, only)[1]


def _cpu_host() -> dict:
    """nproc and the CPU model name of this host (BASELINE.md §2 asks for both)."""
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"nproc": os.cpu_count(), "cpu_model": model}


def _cpu_protocol(step, B: int, warmup: int = 3, timed: int = 10):
    """`warmup` untimed steps, then `timed` steps; pairs/s = B / median step
    time.  Threads = torch's intra-op pool (the box exports OMP_NUM_THREADS = 16, its CPU
    share beside one GPU; `nproc` reports the whole machine's CPUs, which this process is not
    allotted), recorded as `cores`."""
    for _ in range(warmup):
        step()
    times = []
    for _ in range(timed):
        t0 = time.perf_counter()
        step()
        times.append(time.perf_counter() - t0)
    med = sorted(times)[len(times) // 2]
    return B / med, med, sum(times)


def cpu_baseline(B: int, budget_s: float = 20.0):
    """fp32 CPU oracle (oracle/two_tower_ref.py) cfg-2 train step on this host's cores."""
    from oracle import two_tower_ref as ref
    threads = torch.get_num_threads()
    g = torch.Generator().manual_seed(0)
    params = ref.init_params(V, D=D, generator=g)
    batch = ref.synthetic_batch(B, L, V, generator=g)
    running = ref.init_running()
    state = {}
    drop = ref.TorchDropout()
    rate, med, tot = _cpu_protocol(
        lambda: ref.train_step(params, state, batch, p_drop=0.1, drop=drop, running=running), B)
    return {"value": round(rate, 2), "unit": "user-item pairs/s", "cores": threads,
            "kind": "port", **_cpu_host(),
            "sample": f"3 warm-up + 10 timed full cfg-2 steps (B={B}, L={L}, D={D}, V={V}, "
                      f"dropout 0.1) of the fp32 torch-CPU oracle; median step {med:.3f} s, "
                      f"{tot:.1f} s timed"}


def cpu_baseline_cfg3(B: int, budget_s: float = 20.0):
    """fp32 CPU oracle cfg-3 train step (two ResNet-18s + tabular + fusion + user tower)."""
    from oracle import two_tower_ref as ref
    from oracle import resnet_ref as rref
    threads = torch.get_num_threads()
    g = torch.Generator().manual_seed(0)
    params = ref.init_params(V, generator=g)
    for k, v in rref.init_resnet18(1, 128, g, "item_tower.audio_encoder.backbone.").items():
        params[k] = v
    for k, v in rref.init_resnet18(3, 128, g, "item_tower.visual_encoder.backbone.").items():
        params[k] = v
    pt = "item_tower.tabular_encoder.mlp."
    params.update({pt + "0.weight": torch.randn(256, TAB, generator=g) * 0.05,
                   pt + "0.bias": torch.zeros(256), pt + "1.weight": torch.ones(256),
                   pt + "1.bias": torch.zeros(256),
                   pt + "4.weight": torch.randn(128, 256, generator=g) * 0.05,
                   pt + "4.bias": torch.zeros(128)})
    params = {k: v for k, v in params.items() if "running" not in k}
    batch = ref.synthetic_batch(B, L, V, generator=g)
    del batch["target_modal"]
    batch.update(rref.synthetic_items(B, TAB, MEL, COVER, generator=g))
    state = {}
    drop = ref.TorchDropout()
    rate, med, tot = _cpu_protocol(
        lambda: ref.train_step(params, state, batch, p_drop=0.1, drop=drop), B)
    return {"value": round(rate, 3), "unit": "user-item pairs/s", "cores": threads,
            "kind": "port", **_cpu_host(),
            "sample": f"3 warm-up + 10 timed cfg-3 steps at B={B} (full 128x256 mels, 224x224 "
                      f"covers) of the fp32 torch-CPU oracle; median step {med:.3f} s, "
                      f"{tot:.1f} s timed"}


def main_eval(args, world, rank, device):
    """Global retrieval evaluation throughput (evaluate_metrics.py:107-192): per step one batch
    of users -> user tower (eval) -> scores against the dense V=10,136 catalogue -> top-20 ->
    target ranks (Recall/NDCG inputs).  Users/s over all ranks; roofline of the top-K kernel
    (algorithmic bytes: the [B, V] fp32 score block read once)."""
    B = args.batch or 512
    K = 20
    torch.manual_seed(1234 + rank)
    model = pkg.TwoTowerModel(precomputed_modalities=True, vocab_size=V, tabular_input_dim=128, num_genders=N_GENDERS,
                              num_countries=N_COUNTRIES, max_seq_len=L, user_embedding_dim=D,
                              item_embedding_dim=D, user_num_heads=H, user_dropout=0.1,
                              compute_dtype=torch.bfloat16).to(device).eval()
    batches = synthetic_batches(4, B, seed=rank, device=device)
    g = torch.Generator().manual_seed(rank + 3)
    items = torch.nn.functional.normalize(torch.randn(V, D, generator=g), dim=1).to(device)
    items[0] = 0.0
    targets = [torch.randint(1, V, (B,), generator=g).to(device) for _ in batches]
    rt = pkg.retrieval
    ev = rt.GlobalEvaluator(model, items, K)            # one HIP graph replay per batch
    ev_batches = [dict(b, target_id=t) for b, t in zip(batches, targets)]

    def step(i):
        return ev.ranks(ev_batches[i % len(ev_batches)])

    with torch.no_grad():
        for i in range(max(args.warmup, 1)):
            step(i)
        torch.cuda.synchronize(device)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        for i in range(args.steps):
            step(i)
        torch.cuda.synchronize(device)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(device)
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], device=device, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t)
        roof = None
        if rank == 0:                                    # top-K kernel, live, on its stream
            u = model.get_user_embedding(batches[0]["history_ids"], batches[0]["history_mask"],
                                         batches[0]["user_gender"], batches[0]["user_country"])
            sc = rt.score_catalogue(u, items)
            val = torch.empty(B, K, device=device)
            idx = torch.empty(B, K, device=device, dtype=torch.int64)
            st = torch.cuda.current_stream(device)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            pkg.ops.topk_rows(sc, K, val, idx, skip_first=True)
            e0.record(st)
            for _ in range(20):
                pkg.ops.topk_rows(sc, K, val, idx, skip_first=True)
            e1.record(st)
            torch.cuda.synchronize(device)
            sec = e0.elapsed_time(e1) / 1e3 / 20
            by = B * V * 4 + B * K * 12
            gbs = by / sec / 1e9
            roof = {"kernel": "topk_rows_kernel (radix-select top-20 over the [B, V] fp32 scores)",
                    "bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                    "frac": round(gbs / PEAK_HBM_GBS, 4), "traffic": read_traffic("topk_rows_kernel"),
                    "avg_us": round(sec * 1e6, 2), "bytes_per_launch": by}
    cpu = None
    if rank == 0 and world == 1 and not args.skip_cpu:
        from oracle import two_tower_ref as ref
        from oracle import retrieval_ref as rr
        gc = torch.Generator().manual_seed(0)
        params = ref.init_params(V, generator=gc)
        up = {k[len("user_tower."):]: v for k, v in params.items() if k.startswith("user_tower.")}
        cb = ref.synthetic_batch(B, L, V, generator=gc)
        it_cpu, tg = items.cpu(), targets[0].cpu()
        n, t0 = 0, time.perf_counter()
        while True:
            with torch.no_grad():
                u = ref.user_tower_forward(up, cb["history_ids"], cb["user_gender"],
                                           cb["user_country"], cb["history_mask"], H, 2)
                rr.retrieval_metrics(torch.nn.functional.normalize(u, dim=1), it_cpu, tg, (10, 20))
            n += 1
            cel = time.perf_counter() - t0
            if cel >= args.cpu_budget or n >= 30:
                break
        cpu = {"value": round(n * B / cel, 2), "unit": "users/s",
               "cores": torch.get_num_threads(), "kind": "port",
               "sample": f"{n} eval batches of {B} users (fp32 oracle user tower + torch.topk "
                         f"over V={V}), {cel:.1f} s"}
    if rank == 0:
        line = {
            "metric": "users/sec (global retrieval eval: user tower + catalogue scores + top-20 "
                      "+ target rank), V=10136, batch=512",
            "value": round(world * B * args.steps / el, 1), "unit": "users/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(el / max(args.steps, 1) * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16+fp32",
            "data": "synthetic histories and catalogue embeddings, random-init weights",
            "config": {"workload": "eval: SURVEY 8(f) rank 2, evaluate_metrics.py:107-192",
                       "global_batch": world * B, "catalogue": V, "k": K,
                       "parallelism": f"dp{world}", "graph": True},
            "roofline": roof, "cpu_baseline": cpu}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main_prep(args, world, rank, device):
    """Item-modality preprocessing throughput (dataset.tex:23,38): per step
    one batch of B items -> mel spectrogram of a 65,024-sample 22.05 kHz clip (128 frames x 128
    mels, dB, min-max) + 300x300 uint8 cover -> 224x224 ImageNet-normalised NCHW.  Items/s over
    all ranks; roofline of the FFT/mel kernel (algorithmic bytes: waveform read + mel write)."""
    B = args.batch or 256
    N = 65024
    prep = pkg.preprocess
    mel = prep.MelSpectrogram(device=device)
    cov = prep.CoverTransform(224)
    g = torch.Generator(device=device).manual_seed(rank)
    waves = [torch.randn(B, N, device=device, generator=g) * 0.1 for _ in range(2)]
    covers = [torch.randint(0, 256, (B, 300, 300, 3), device=device, generator=g, dtype=torch.uint8)
              for _ in range(2)]

    def step(i):
        mel(waves[i % 2])
        cov(covers[i % 2])

    for i in range(max(args.warmup, 1)):
        step(i)
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t)
    roof = None
    if rank == 0:                                        # mel_power kernel, live, on its stream
        st = torch.cuda.current_stream(device)
        out = torch.empty(B, 128, 1 + N // 512, device=device)
        mel.power(waves[0], out)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(10):
            mel.power(waves[0], out)
        e1.record(st)
        torch.cuda.synchronize(device)
        sec = e0.elapsed_time(e1) / 1e3 / 10
        F = 1 + N // 512
        by = B * (N * 4 + 128 * F * 4)
        gbs = by / sec / 1e9
        roof = {"kernel": "mel_power_kernel (per-frame 2048-point LDS FFT + sparse Slaney filterbank)",
                "bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(gbs / PEAK_HBM_GBS, 4), "traffic": read_traffic("mel_power_kernel"),
                "avg_us": round(sec * 1e6, 2), "bytes_per_launch": by,
                "note": "frames overlap 4x (hop 512 of 2048): each sample is read by 4 workgroups"}
    cpu = None
    if rank == 0 and world == 1 and not args.skip_cpu:
        from oracle import prep_ref as pr
        import numpy as np
        w = waves[0][:8].cpu().numpy()
        c = covers[0][:8].cpu().numpy()
        n, t0c = 0, time.perf_counter()
        while True:
            pr.log_mel(w[n % 8])
            pr.cover_transform(c[n % 8])
            n += 1
            cel = time.perf_counter() - t0c
            if cel >= min(args.cpu_budget, 15.0) or n >= 64:
                break
        cpu = {"value": round(n / cel, 2), "unit": "items/s", "cores": 1, "kind": "port",
               "sample": f"{n} items (float64 numpy oracle: 65,024-sample log-mel + 300->224 cover), "
                         f"{cel:.1f} s"}
    if rank == 0:
        line = {
            "metric": "items/sec (GPU item preprocessing: 22.05 kHz clip -> 128x128 log-mel in [0,1] "
                      "+ 300x300 cover -> 224x224 ImageNet-normalised), batch=256",
            "value": round(world * B * args.steps / el, 1), "unit": "items/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(el / max(args.steps, 1) * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32 (u8 covers)",
            "data": "synthetic waveforms and covers",
            "config": {"workload": "prep: SURVEY 8(f) rank 1, dataset.tex:23,38", "global_batch": world * B,
                       "samples_per_clip": N, "parallelism": f"dp{world}"},
            "roofline": roof, "cpu_baseline": cpu}
        print(json.dumps(line), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv=None, poll_s: float = 0.2, script=None) -> int:
    """`bench.py --gpus N` without a launcher: one fresh child process per rank (the reference's
    `torchrun --nproc_per_node`, src/jobs/train.sh:48), env RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_ADDR=127.0.0.1 / MASTER_PORT.  This parent makes no GPU call and imports nothing that
    does (the package is imported in main() after this returns); it forwards rank 0's stdout
    (the JSON line) and, if any rank fails, stops the others (their exact PIDs) and returns
    that rank's exit code."""
    argv = sys.argv[1:] if argv is None else argv
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__), *argv], env=env,
                                      stdout=subprocess.PIPE if r == 0 else None, text=True))
    rc = 0
    out = []
    try:
        import threading
        reader = threading.Thread(target=lambda: out.extend(procs[0].stdout), daemon=True)
        reader.start()
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    for q in live:
                        q.terminate()
            time.sleep(poll_s)
        reader.join(timeout=10)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for line in out:
        sys.stdout.write(line)
    sys.stdout.flush()
    if rc == 0:
        rows = [json.loads(l) for l in out if l.startswith("{")]
        if not rows or rows[-1].get("n_gpus") != n:
            print(f"bench.py: expected one JSON line with n_gpus={n} from rank 0", file=sys.stderr)
            return 1
    return rc if rc >= 0 else 128 - rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=None,
                    help="per-GPU pairs (default: 512 for cfg 2, 256 for cfg 3)")
    ap.add_argument("--config", default="2", choices=("2", "3", "4", "5", "eval", "prep"),
                    help="2 = BASELINE cfg 2 (the metric's configuration); 3 = full item "
                         "tower on raw mels/covers/tabular (BASELINE configs[2]); 4 = cfg 3 + "
                         "mDeBERTa-LoRA lyrics, S=256 (BASELINE configs[3]); 5 = cfg 2 with "
                         "global in-batch negatives (all-gather of every rank's embeddings, "
                         "BASELINE configs[4]); eval = global "
                         "retrieval evaluation over the catalogue (SURVEY 8f rank 2)")
    ap.add_argument("--dim", type=int, default=128,
                    help="d_model of both towers (128 = BASELINE cfg 2; 256 = the reference's "
                         "own default, src/train.py:289-297)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--ddp-schedule", action="store_true",
                    help="run the data-parallel schedule even at --gpus 1: a world-1 process group "
                         "(TTMI_DIST_BACKEND, default nccl = RCCL) whose collectives all run "
                         "(comm.force_dp): the per-rank cost of DDP without the wire")
    ap.add_argument("--overlap-grad-sync", action="store_true",
                    help="data-parallel schedule: two gradient buckets, the first all-reduced "
                         "while layer 0 and the input block are differentiated")
    ap.add_argument("--no-capture-collectives", action="store_true",
                    help="data-parallel schedule: collectives between graph segments (host cuts) "
                         "instead of inside the step's graph")
    ap.add_argument("--skip-cpu", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    args = ap.parse_args()
    global D, pkg
    D = args.dim

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: n_gpus must equal "
                         f"the ranks that run (launch with --nproc-per-node {args.gpus}, or drop "
                         f"WORLD_SIZE and let --gpus spawn the ranks)")
    pkg = importlib.import_module(PKG)
    rank = int(os.environ.get("RANK", "0"))
    # one rank per GPU; ranks beyond the visible GPU count share them (a multi-rank rehearsal
    # on a 1-GPU box, with TTMI_DIST_BACKEND=gloo since RCCL wants distinct devices)
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1)
    if world > 1 or args.ddp_schedule:
        torch.cuda.set_device(local)
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        dist.init_process_group(os.environ.get("TTMI_DIST_BACKEND", "nccl"))
        if args.ddp_schedule:
            pkg.comm.force_dp(True)
    device = torch.device("cuda", local)
    if args.config == "eval":
        return main_eval(args, world, rank, device)
    if args.config == "prep":
        return main_prep(args, world, rank, device)
    cfg4 = args.config == "4"
    cfg5 = args.config == "5"
    cfg3 = args.config == "3" or cfg4                    # cfg 4 = cfg 3 + text
    B = args.batch or (256 if cfg3 else 512)

    torch.manual_seed(1234 + rank)
    model = pkg.TwoTowerModel(vocab_size=V, tabular_input_dim=128, num_genders=N_GENDERS,
                              num_countries=N_COUNTRIES, max_seq_len=L, user_embedding_dim=D,
                              item_embedding_dim=D, user_num_heads=H, user_dropout=0.1,
                              compute_dtype=torch.bfloat16,
                              precomputed_modalities=not cfg3, with_text=cfg4,
                              global_negatives=cfg5).to(device)
    if world > 1:   # identical replicas, as DDP broadcasts from rank 0
        for t in list(model.parameters()) + list(model.buffers()):
            dist.broadcast(t.data, 0)
    step = pkg.TrainStep(model, lr=1e-4, use_graph=not args.no_graph, seed=rank + 1,
                         capture_collectives=False if args.no_capture_collectives else None,
                         overlap_grad_sync=True if args.overlap_grad_sync else None)
    batches = synthetic_batches(2 if cfg3 else 4, B, seed=rank, device=device)
    if cfg3:
        batches = add_raw_items(batches, rank, device)
    if cfg4:
        batches = add_text(batches, rank, device)

    # warm-up runs the exact timed-loop ops.  The step losses are summed on the device by the
    # step itself (TrainStep.loss_sum: inside the InfoNCE logits launch on cfg 2, an add in
    # the captured graph otherwise), read once after the timed region.
    for i in range(max(args.warmup, 1)):
        step.step(batches[i % len(batches)])
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    step.loss_sum.zero_()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step.step(batches[i % len(batches)])
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    el = time.perf_counter() - t0
    step.check()                  # an id outside its table in any timed step raises here
    if world > 1:
        t = torch.tensor([el], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t)
    mean_loss = float(step.loss_sum) / max(args.steps, 1)

    roof = roof_panel = None
    if rank == 0:
        if cfg4:
            roof = probe_text_gemm(step, batches[0], device)
        elif cfg3:
            roof = probe_conv(step, batches[0], device)
        else:
            roof = probe_dominant(step, batches[0], device)
            try:
                roof_panel = probe_panels(step, batches[0], device)
            except Exception as exc:           # a probe must never sink the bench line
                print(f"probe_panels: {exc!r}", file=sys.stderr)
    cpu = None
    if rank == 0 and world == 1 and not args.skip_cpu:
        if cfg4:
            cpu = cpu_baseline_cfg4(2, args.cpu_budget)
        elif cfg3:
            cpu = cpu_baseline_cfg3(8, args.cpu_budget)
        else:
            cpu = cpu_baseline(B, args.cpu_budget)

    if rank == 0:
        pairs = world * B * args.steps
        value = pairs / el
        ms = el / max(args.steps, 1) * 1e3
        flops = step_flops(B) + (RESNET_FLOPS_PER_SAMPLE * B if cfg3 else 0.0) + \
            ((TEXT_FLOPS_PER_SAMPLE * B + TEXT_FLOPS_PER_BATCH) if cfg4 else 0.0) + \
            (2.0 * world * B * D * 3 * B if cfg5 else 0.0)     # +2·C·D·3 per pair
        step_tf = flops * args.steps / el / 1e12 * world
        workload = (f"cfg2: SASRec L=50 D={D} H=4 x2 layers + late-fusion head on "
                    "precomputed 512-d modality embeddings + in-batch InfoNCE; "
                    "fwd+bwd+AdamW, dropout 0.1")
        if cfg5:
            workload = (f"cfg5: cfg2 with global in-batch negatives: all-gather of u_hat, i_hat, "
                        f"user_idx over {world} rank(s), {world * B} negatives per row, "
                        f"reduce-scatter of the key gradients; fwd+bwd+AdamW, dropout 0.1")
        if cfg4:
            workload = ("cfg4: cfg3 item tower + mDeBERTa-v3-base (12 layers, H=768, random init) "
                        "with LoRA r=8 on query/value, lyrics S=256 (lengths U[16,256]); "
                        "fwd+bwd+AdamW, dropout 0.1; 1 GPU (BASELINE quotes DDP x8)")
        elif cfg3:
            workload = ("cfg3: SASRec L=50 D=128 H=4 x2 layers + item tower on raw inputs "
                        "(ResNet-18 on 1x128x256 mels, ResNet-18 on 3x224x224 covers, tabular "
                        "MLP T=128, zero text slot) + late-fusion head + in-batch InfoNCE; "
                        "fwd+bwd+AdamW, dropout 0.1, BN train mode")
        line = {
            "metric": "user-item pairs/sec (train step) at batch=512 d=128; 1/2/4/8 MI355X scaling",
            "value": round(value, 1), "unit": "user-item pairs/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16", "data": "synthetic (SURVEY §8d distributions), random-init weights",
            "config": {"workload": workload,
                       "global_batch": world * B, "per_gpu_batch": B, "seq_len": L,
                       "vocab": V, "d_model": D, "parallelism": f"dp{world}",
                       "graph": not args.no_graph,
                       "schedule": ("ddp" if step.dp else "single-process") +
                                   (f" ({dist.get_backend()}, "
                                    f"{'two buckets' if step.overlap else 'one all-reduce'}, collectives "
                                    f"{'captured in the step graph' if step.capture_collectives else 'between graph segments'}, "
                                    f"{step._cur.seg.n_graphs if step._cur.seg else 0} graph(s) per step)"
                                    if step.dp else "")},
            "roofline": roof,
            "roofline_panel": roof_panel,
            "step_mfma": {"achieved": round(step_tf, 3), "peak": PEAK_BF16_TFLOPS,
                          "unit": "TFLOP/s", "frac": round(step_tf / PEAK_BF16_TFLOPS, 5),
                          "flops_per_step_per_gpu": flops,
                          "flops": "F_min (pruned last layer, SURVEY 8d)" +
                                   (" + ResNet-18 fwd+bwd 17.4 GF/pair (SURVEY a7/a8)"
                                    if cfg3 else "") +
                                   (" + mDeBERTa-LoRA 103.9 GF/pair + 14.5 GF/batch (SURVEY a9)"
                                    if cfg4 else "")},
            "cpu_baseline": cpu,
            "mean_loss": round(mean_loss, 5),
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""Data-pipeline kernels on the GPU against the float64 oracle
(oracle/prep_ref.py, pinned to torch.stft / torch antialiased interpolate on the CPU):

* ttmi_mel_power within 1e-5 of the oracle's mel power (relative to each clip's max),
  ttmi_mel_db_minmax within 2e-4 absolute in [0, 1] units (fp32 FFT vs float64), a silent
  clip -> zeros;
* ttmi_cover_prep within 1e-4 of the oracle (fp32 NCHW) and bf16 rounding for the NHWC-8
  stem operand;
* DeviceCollator / DevicePrefetcher: a MultimodalDataset batch staged to HBM and
  transformed there feeds TwoTowerModel's raw-input (cfg-3) forward."""
import importlib

import numpy as np
import pytest
import torch

from oracle import prep_ref as pr

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("N", [65024, 130560, 5000])
def test_mel_kernels_vs_oracle(gpu_pkg, N):
    P = gpu_pkg.preprocess
    g = np.random.default_rng(N)
    t = np.arange(N) / 22050
    waves = np.stack([
        0.3 * np.sin(2 * np.pi * 440 * t) + 0.01 * g.standard_normal(N),
        g.standard_normal(N) * np.linspace(0, 1, N),
        np.zeros(N),
    ]).astype(np.float32)
    mel = P.MelSpectrogram(device=DEV)
    x = torch.from_numpy(waves).to(DEV)
    pw = mel.power(x).cpu().numpy()
    out = mel(x).cpu().numpy()
    F = 1 + N // 512
    assert out.shape == (3, 1, 128, F)
    fb = pr.mel_filters()
    for b in range(2):
        ref_pw = fb @ pr.stft_power(waves[b])
        assert np.abs(pw[b] - ref_pw).max() <= 1e-5 * ref_pw.max()
        assert np.abs(out[b, 0] - pr.log_mel(waves[b])).max() < 2e-4
    assert np.all(out[2] == 0)


@pytest.mark.parametrize("hw", [(300, 300), (32, 32), (480, 640)])
def test_cover_prep_vs_oracle(gpu_pkg, hw):
    P = gpu_pkg.preprocess
    g = np.random.default_rng(hw[0])
    imgs = g.integers(0, 256, (2, *hw, 3), dtype=np.uint8)
    nchw, nhwc8 = P.CoverTransform(224)(torch.from_numpy(imgs).to(DEV), nchw=True, nhwc8=True)
    for b in range(2):
        want = pr.cover_transform(imgs[b])
        assert np.abs(nchw[b].cpu().numpy() - want).max() < 1e-4
        got8 = nhwc8[b].float().cpu().numpy()
        assert np.abs(got8[..., :3].transpose(2, 0, 1) - want).max() < 2e-2
        assert np.all(got8[..., 3:] == 0)


def test_device_collator_feeds_raw_item_tower(gpu_pkg, tmp_path):
    from PIL import Image
    D = gpu_pkg.data
    df = D.synthetic_interactions(40, 64, 600, seed=5)
    mapper = D.item_id_mapper_from(df)
    img_dir, aud_dir = tmp_path / "covers", tmp_path / "mels"
    img_dir.mkdir()
    aud_dir.mkdir()
    g = np.random.default_rng(0)
    for i, tid in enumerate(df["track_id"].unique()[:32]):
        Image.fromarray(g.integers(0, 256, (300, 300, 3), dtype=np.uint8)).save(img_dir / f"{tid}.jpg")
        np.save(aud_dir / f"{tid}.npy", g.random((128, 128)).astype(np.float32))
    ds = D.MultimodalDataset(df, mapper, img_dir=str(img_dir), audio_dir=str(aud_dir))
    loader = torch.utils.data.DataLoader(ds, batch_size=16, shuffle=True, collate_fn=D.collate,
                                         generator=torch.Generator().manual_seed(0))
    coll = D.DeviceCollator(DEV)
    m = gpu_pkg.TwoTowerModel(with_text=False, vocab_size=len(mapper) + 1, tabular_input_dim=ds.tabular_data.shape[1],
                              num_genders=len(ds.encoders["gender_encoder"].classes_),
                              num_countries=len(ds.encoders["country_encoder"].classes_),
                              user_embedding_dim=128, item_embedding_dim=128,
                              precomputed_modalities=False).to(DEV)
    host = next(iter(loader))
    u8 = host["target_image_u8"].to(DEV).contiguous()
    dev = coll(host)
    assert dev["target_image"].shape == (16, 3, 224, 224)
    assert dev["target_audio"].shape == (16, 1, 128, 128)
    assert torch.equal(dev["target_image"], gpu_pkg.preprocess.CoverTransform(224)(u8))
    assert torch.equal(dev["target_audio"][:, 0].cpu(), host["target_audio_raw"])
    n = 0
    for dev in D.DevicePrefetcher(loader, coll):
        loss, logits, u, it = m(dev)
        loss.backward()
        assert torch.isfinite(loss) and logits.shape == (16, 16)
        n += 1
        if n == 2:
            break
    assert n == 2


def test_cfg1_loader_batches_through_hip_train_step(gpu_pkg):
    """BASELINE configs[0] on the HIP path: MultimodalDataset batches (batch 4, history 20,
    100 users x 1k items, 32 x 32 stub mels / covers) through the fused TrainStep (user tower,
    ResNet-18 audio + visual, tabular, fusion head, InfoNCE with the collision mask, AdamW),
    step for step against the fp32 oracle's train step from the same parameters (bf16
    storage through two ResNet-18s at B = 4: 3e-2 on the loss)."""
    import math
    from oracle import resnet_ref as rr
    from oracle import two_tower_ref as ref
    from oracle import prep_ref as pr
    from test_prep_oracle import _dataset
    D = gpu_pkg.data
    df, mapper, ds = _dataset()
    loader = torch.utils.data.DataLoader(ds, batch_size=4, shuffle=True, collate_fn=D.collate,
                                         generator=torch.Generator().manual_seed(0))
    T = ds.tabular_data.shape[1]
    torch.manual_seed(0)
    m = gpu_pkg.TwoTowerModel(vocab_size=len(mapper) + 1, tabular_input_dim=T,
                              num_genders=len(ds.encoders["gender_encoder"].classes_),
                              num_countries=len(ds.encoders["country_encoder"].classes_),
                              max_seq_len=20, user_embedding_dim=128, item_embedding_dim=128,
                              user_dropout=0.0, with_text=False).to(DEV)
    m.item_tower.fusion_layer[3].p = 0.0
    m.item_tower.tabular_encoder.mlp[3].p = 0.0
    P = {k: v.detach().cpu().clone() for k, v in m.named_parameters()}
    state, running = {}, ref.init_running()
    step = gpu_pkg.TrainStep(m, lr=1e-4)
    for i, b in enumerate(loader):
        img = torch.stack([torch.from_numpy(pr.cover_transform(x.numpy(), size=32)).float()
                           for x in b["target_image_u8"]])
        batch = {k: b[k] for k in ("history_ids", "history_mask", "user_gender", "user_country",
                                   "user_idx")}
        batch.update({"target_audio": b["target_audio_raw"].float().unsqueeze(1).contiguous(),
                      "target_image": img, "target_tabular": b["target_tabular"].float()})
        got = float(step.step({k: v.to(DEV) for k, v in batch.items()}))
        want = ref.train_step(P, state, batch, running=running)
        assert math.isfinite(got) and abs(got - want) < 3e-2, (i, got, want)
        if i == 3:
            break

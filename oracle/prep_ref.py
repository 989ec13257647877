"""ORACLE — test infrastructure only (see oracle/__init__.py).

float64 numpy restatement of the item-modality transforms of the reference's (missing)
``src/data/dataset.py`` as ``report/chapters/dataset.tex`` states them.  The arithmetic lives
in third-party libraries absent from this image; their published algorithms are restated:

* ``log_mel`` — dataset.tex:23 ("ventana FFT de 2048, hop 512, 128 bandas Mel, potencia a dB,
  Min-Max a [0, 1]") with librosa 0.11.0 (reference ``uv.lock:1923``) defaults:
  ``feature.melspectrogram(sr=22050, center=True, pad_mode='constant', window='hann'
  (periodic, scipy get_window fftbins=True), power=2.0, htk=False, norm='slaney')`` and
  ``power_to_db(ref=np.max, amin=1e-10, top_db=80.0)``.  The STFT leg is pinned to
  ``torch.stft``; the Slaney mel scale to its closed-form known answers (tests/test_prep_oracle).
* ``resize_aa`` — dataset.tex:38 (resize to 224 x 224): torchvision 0.24.1 ``Resize`` on
  tensors = antialiased bilinear (PIL's triangle filter), align_corners=False; pinned to
  ``torch.nn.functional.interpolate(mode='bilinear', antialias=True)``.

Parity against the reference itself is unpinned: its dataset module is not in the snapshot.
"""
from __future__ import annotations

import math

import numpy as np

F_SP, MIN_LOG_HZ = 200.0 / 3, 1000.0
MIN_LOG_MEL, LOGSTEP = MIN_LOG_HZ / F_SP, math.log(6.4) / 27.0


def hz_to_mel(f):
    """librosa.hz_to_mel(htk=False): linear below 1 kHz, logarithmic above (Slaney)."""
    f = np.asarray(f, dtype=np.float64)
    out = f / F_SP
    log = f >= MIN_LOG_HZ
    out = np.where(log, MIN_LOG_MEL + np.log(np.where(log, f, MIN_LOG_HZ) / MIN_LOG_HZ) / LOGSTEP, out)
    return out


def mel_to_hz(m):
    m = np.asarray(m, dtype=np.float64)
    return np.where(m >= MIN_LOG_MEL, MIN_LOG_HZ * np.exp(LOGSTEP * (m - MIN_LOG_MEL)), F_SP * m)


def mel_filters(sr=22050, n_fft=2048, n_mels=128, fmin=0.0, fmax=None):
    """librosa.filters.mel(norm='slaney', htk=False) in float64."""
    fmax = sr / 2.0 if fmax is None else fmax
    n_bins = 1 + n_fft // 2
    weights = np.zeros((n_mels, n_bins))
    fftfreqs = np.arange(n_bins) * (sr / n_fft)
    mel_f = mel_to_hz(np.linspace(hz_to_mel(fmin), hz_to_mel(fmax), n_mels + 2))
    for i in range(n_mels):
        lo, ce, hi = mel_f[i], mel_f[i + 1], mel_f[i + 2]
        for k, f in enumerate(fftfreqs):
            up = (f - lo) / (ce - lo)
            down = (hi - f) / (hi - ce)
            weights[i, k] = max(0.0, min(up, down))
        weights[i] *= 2.0 / (hi - lo)
    return weights


def stft_power(y, n_fft=2048, hop=512):
    """|STFT|² [1 + n_fft/2, 1 + len/hop]: zero-padded centre frames, periodic Hann."""
    y = np.asarray(y, dtype=np.float64)
    pad = n_fft // 2
    yp = np.concatenate([np.zeros(pad), y, np.zeros(pad)])
    n_frames = 1 + len(y) // hop
    win = 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(n_fft) / n_fft)
    frames = np.stack([yp[f * hop:f * hop + n_fft] * win for f in range(n_frames)], 1)
    spec = np.fft.rfft(frames, axis=0)
    return np.abs(spec) ** 2


def power_to_db(S, amin=1e-10, top_db=80.0):
    """librosa.power_to_db(S, ref=np.max, amin, top_db)."""
    log_spec = 10.0 * np.log10(np.maximum(amin, S)) - 10.0 * np.log10(np.maximum(amin, S.max()))
    return np.maximum(log_spec, log_spec.max() - top_db)


def minmax(x):
    lo, hi = x.min(), x.max()
    return (x - lo) / (hi - lo) if hi > lo else np.zeros_like(x)


def log_mel(y, sr=22050, n_fft=2048, hop=512, n_mels=128):
    """dataset.tex:23 pipeline for one clip -> [n_mels, 1 + len/hop] in [0, 1]."""
    mel = mel_filters(sr, n_fft, n_mels) @ stft_power(y, n_fft, hop)
    return minmax(power_to_db(mel))


def _aa_weights(in_size, out_size):
    """Per output index: (first input index, normalised triangle-filter weights)."""
    scale = in_size / out_size
    support = scale if scale >= 1.0 else 1.0
    invscale = 1.0 / scale if scale >= 1.0 else 1.0
    out = []
    for o in range(out_size):
        center = scale * (o + 0.5)
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size)
        w = np.array([max(0.0, 1.0 - abs((j + xmin - center + 0.5) * invscale)) for j in range(xmax - xmin)])
        tot = w.sum()
        out.append((xmin, w / tot if tot != 0 else w))
    return out


def resize_aa(img, out_h, out_w):
    """img float [H, W, C] -> [out_h, out_w, C]: separable antialiased bilinear."""
    img = np.asarray(img, dtype=np.float64)
    H, W, C = img.shape
    tmp = np.zeros((H, out_w, C))
    for ox, (x0, w) in enumerate(_aa_weights(W, out_w)):
        tmp[:, ox] = np.tensordot(w, img[:, x0:x0 + len(w)], axes=([0], [1]))
    out = np.zeros((out_h, out_w, C))
    for oy, (y0, w) in enumerate(_aa_weights(H, out_h)):
        out[oy] = np.tensordot(w, tmp[y0:y0 + len(w)], axes=([0], [0]))
    return out


def cover_transform(img_u8, size=224, mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225)):
    """uint8 HWC -> [3, size, size] ImageNet-normalised (ToTensor, Resize, Normalize)."""
    x = resize_aa(np.asarray(img_u8, dtype=np.float64) / 255.0, size, size)
    x = (x - np.asarray(mean)) / np.asarray(std)
    return x.transpose(2, 0, 1)

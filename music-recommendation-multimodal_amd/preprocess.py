"""GPU preprocessing of the item modalities (the transforms of the
reference's missing ``src/data/dataset.py`` as ``report/chapters/dataset.tex`` states them).

* ``MelSpectrogram`` — ``dataset.tex:23``: mono 22.05 kHz audio, STFT with a 2048-sample window
  and hop 512, 128 mel bands, power -> dB, min-max to [0, 1].  The arithmetic is librosa 0.11's
  (``uv.lock:1923``; absent here): ``melspectrogram(center=True, pad_mode='constant',
  window='hann', power=2, htk=False, norm='slaney')`` then ``power_to_db(ref=np.max,
  amin=1e-10, top_db=80)``.  On the GPU: one workgroup per frame runs the 2048-point FFT in
  LDS and applies the sparse filterbank (``ttmi_mel_power``), one per clip the dB and min-max
  (``ttmi_mel_db_minmax``).
* ``CoverTransform`` — ``dataset.tex:38``: resize to 224 x 224 and ImageNet normalisation
  (torchvision ``Resize`` -> antialiased bilinear, ``Normalize``), from uint8 HWC covers.  It
  can emit the ResNet stem's bf16 NHWC-8 operand directly.

Host-side table building (window, twiddles, Slaney filterbank) is plain numpy run once; every
per-sample operation is a HIP kernel (no CPU fallback: the calls raise if libttmi is absent).
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import numpy as np
import torch
from torch import Tensor

from . import lib as _L

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


# ------------------------------------------------------------------ Slaney mel scale (host)
def _hz_to_mel(f: np.ndarray) -> np.ndarray:
    f = np.asarray(f, dtype=np.float64)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, math.log(6.4) / 27.0
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-300) / min_log_hz) / logstep,
                    f / f_sp)


def _mel_to_hz(m: np.ndarray) -> np.ndarray:
    m = np.asarray(m, dtype=np.float64)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, math.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), f_sp * m)


def mel_filterbank(sr: int, n_fft: int, n_mels: int, fmin: float = 0.0,
                   fmax: Optional[float] = None) -> np.ndarray:
    """[n_mels, 1 + n_fft/2] float32 triangular filters, Slaney-normalised (librosa.filters.mel
    with htk=False, norm='slaney')."""
    fmax = sr / 2.0 if fmax is None else fmax
    fft_f = np.linspace(0, sr / 2.0, 1 + n_fft // 2)
    mel_f = _mel_to_hz(np.linspace(_hz_to_mel(fmin), _hz_to_mel(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = mel_f[:, None] - fft_f[None, :]
    lower = -ramps[:-2] / fdiff[:-1, None]
    upper = ramps[2:] / fdiff[1:, None]
    w = np.maximum(0.0, np.minimum(lower, upper))
    w *= (2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels]))[:, None]
    return w.astype(np.float32)


class MelSpectrogram:
    """Waveforms [B, N] fp32 (22.05 kHz mono) -> normalised log-mel [B, 1, n_mels, 1 + N//hop]."""

    def __init__(self, sr: int = 22050, n_fft: int = 2048, hop: int = 512, n_mels: int = 128,
                 fmin: float = 0.0, fmax: Optional[float] = None, top_db: float = 80.0,
                 amin: float = 1e-10, device="cuda"):
        if n_fft != 2048:
            raise ValueError("MelSpectrogram: the FFT kernel is built for n_fft = 2048 (dataset.tex:23)")
        self.sr, self.n_fft, self.hop, self.n_mels = sr, n_fft, hop, n_mels
        self.top_db, self.amin = top_db, amin
        n = np.arange(n_fft)
        win = (0.5 - 0.5 * np.cos(2 * np.pi * n / n_fft)).astype(np.float32)     # periodic Hann
        k = np.arange(n_fft // 2)
        tw = np.stack([np.cos(-2 * np.pi * k / n_fft), np.sin(-2 * np.pi * k / n_fft)], 1)
        fb = mel_filterbank(sr, n_fft, n_mels, fmin, fmax)
        start, length, off, packed = [], [], [], []
        for m in range(n_mels):
            nz = np.nonzero(fb[m])[0]
            s0, s1 = (int(nz[0]), int(nz[-1]) + 1) if nz.size else (0, 0)
            start.append(s0)
            length.append(s1 - s0)
            off.append(sum(length[:-1]))
            packed.append(fb[m, s0:s1])
        self.filterbank = fb
        dev = torch.device(device)
        self.window = torch.from_numpy(win).to(dev)
        self.twiddle = torch.from_numpy(tw.astype(np.float32)).contiguous().to(dev)
        self.band_start = torch.tensor(start, dtype=torch.int32, device=dev)
        self.band_len = torch.tensor(length, dtype=torch.int32, device=dev)
        self.band_off = torch.tensor(off, dtype=torch.int32, device=dev)
        self.band_w = torch.from_numpy(np.concatenate(packed).astype(np.float32)).to(dev)

    def frames(self, n_samples: int) -> int:
        return 1 + n_samples // self.hop

    def power(self, wave: Tensor, out: Optional[Tensor] = None) -> Tensor:
        """Mel power spectrogram [B, n_mels, F] (before dB)."""
        if wave.dim() != 2 or wave.dtype != torch.float32 or wave.stride(1) != 1:
            raise ValueError("MelSpectrogram: waveforms must be fp32 [B, N] with unit column stride")
        B, N = wave.shape
        F = self.frames(N)
        if out is None:
            out = torch.empty(B, self.n_mels, F, device=wave.device)
        _L.call("ttmi_mel_power", B, N, wave.data_ptr(), wave.stride(0), self.hop, self.n_mels,
                self.window.data_ptr(), self.twiddle.data_ptr(), self.band_start.data_ptr(),
                self.band_len.data_ptr(), self.band_off.data_ptr(), self.band_w.data_ptr(),
                out.data_ptr(), torch.cuda.current_stream().cuda_stream)
        return out

    def __call__(self, wave: Tensor) -> Tensor:
        mel = self.power(wave)
        B = mel.shape[0]
        _L.call("ttmi_mel_db_minmax", B, mel[0].numel(), self.amin, self.top_db, mel.data_ptr(),
                torch.cuda.current_stream().cuda_stream)
        return mel.unsqueeze(1)


class CoverTransform:
    """uint8 covers [B, H, W, 3] (device) -> ImageNet-normalised [B, 3, size, size] fp32 and/or
    the ResNet stem's bf16 NHWC-8 operand [B, size, size, 8]."""

    def __init__(self, size: int = 224, mean: Tuple[float, ...] = IMAGENET_MEAN,
                 std: Tuple[float, ...] = IMAGENET_STD):
        self.size = size
        self.mean = (ctypes_floats(mean))
        self.std = (ctypes_floats(std))

    def __call__(self, img: Tensor, nchw: bool = True, nhwc8: bool = False):
        if img.dim() != 4 or img.shape[3] != 3 or img.dtype != torch.uint8 or not img.is_contiguous():
            raise ValueError("CoverTransform: need contiguous uint8 [B, H, W, 3]")
        B, H, W, _ = img.shape
        S = self.size
        o1 = torch.empty(B, 3, S, S, device=img.device) if nchw else None
        o2 = torch.empty(B, S, S, 8, device=img.device, dtype=torch.bfloat16) if nhwc8 else None
        _L.call("ttmi_cover_prep", B, H, W, img.data_ptr(), H * W * 3, S, S, self.mean, self.std,
                None if o1 is None else o1.data_ptr(), None if o2 is None else o2.data_ptr(),
                torch.cuda.current_stream().cuda_stream)
        if nchw and nhwc8:
            return o1, o2
        return o1 if nchw else o2


def ctypes_floats(v):
    import ctypes
    return (ctypes.c_float * len(v))(*[float(x) for x in v])

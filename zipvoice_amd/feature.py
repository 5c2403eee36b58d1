"""Prompt feature extraction: drop-ins for the reference's ``VocosFbank`` and
``BigVGANFbank``.

Reference: ``zipvoice/utils/feature.py:36-120``.  ``VocosFbank.extract`` runs
torchaudio ``MelSpectrogram(sample_rate=24000, n_fft=1024, hop_length=256,
n_mels=100, center=True, power=1)`` (hann window, reflect padding, HTK mel
scale, no filter normalisation), then ``clamp(min=1e-7).log()``, transposes to
(frames, n_mels) and trims / replicate-pads to lhotse's
``compute_num_frames`` (``(num_samples + hop // 2) // hop``).  Stereo
(``num_channels=2``, the Dialog-Stereo model) extracts each channel and
concatenates the mels (``:87-103``); mono input with two channels is averaged.

The compute runs in the engine's ``zv_fbank_*`` kernel (one workgroup per 8
frames: reflect-padded windowed frames in LDS, exact-twiddle fp32 DFT
magnitudes, mel projection and log in the same workgroup).  The mel filterbank
is the torchaudio formula (``melscale_fbanks``, restated below with the same
torch float32 ops; torchaudio itself is not installed here).

``BigVGANFbank`` (``feature.py:133-204``, ``_bigvgan_mel_feature.py:42-111``)
is the same kernel configured for NVIDIA's BigVGAN mel: reflect pad
``(n_fft - hop) / 2`` and ``center=False``, magnitude ``sqrt(|X|^2 + 1e-9)``,
the Slaney mel filterbank of ``librosa.filters.mel`` (restated in
``slaney_mel_fbanks``; librosa is not installed here), ``log(clamp(1e-5))``,
and replicate padding of the last STFT frame up to the lhotse frame count.
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass
from typing import Optional, Tuple, Union

import numpy as np
import torch

from . import engine as _eng


@dataclass
class VocosFbankConfig:
    sampling_rate: int = 24000
    n_mels: int = 100
    n_fft: int = 1024
    hop_length: int = 256


def melscale_fbanks(n_freqs: int, f_min: float, f_max: float, n_mels: int,
                    sample_rate: int) -> torch.Tensor:
    """torchaudio.functional.melscale_fbanks(norm=None, mel_scale="htk"):
    triangular filters on the HTK mel scale, (n_freqs, n_mels) float32."""
    all_freqs = torch.linspace(0, sample_rate // 2, n_freqs)
    m_min = 2595.0 * math.log10(1.0 + (f_min / 700.0))
    m_max = 2595.0 * math.log10(1.0 + (f_max / 700.0))
    m_pts = torch.linspace(m_min, m_max, n_mels + 2)
    f_pts = 700.0 * (10.0 ** (m_pts / 2595.0) - 1.0)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts.unsqueeze(0) - all_freqs.unsqueeze(1)
    zero = torch.zeros(1)
    down_slopes = (-1.0 * slopes[:, :-2]) / f_diff[:-1]
    up_slopes = slopes[:, 2:] / f_diff[1:]
    return torch.max(zero, torch.min(down_slopes, up_slopes))


def _hz_to_mel_slaney(f: np.ndarray) -> np.ndarray:
    """librosa.hz_to_mel(htk=False): linear below 1 kHz (200/3 Hz per mel),
    logarithmic above (27 mels per factor 6.4)."""
    f = np.asarray(f, np.float64)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, math.log(6.4) / 27.0
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-30) / min_log_hz) / logstep,
                    f / f_sp)


def _mel_to_hz_slaney(m: np.ndarray) -> np.ndarray:
    m = np.asarray(m, np.float64)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, math.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), f_sp * m)


def slaney_mel_fbanks(sr: int, n_fft: int, n_mels: int, fmin: float = 0.0,
                      fmax: Optional[float] = None) -> np.ndarray:
    """librosa.filters.mel(sr, n_fft, n_mels, fmin, fmax, htk=False, norm="slaney")
    restated (float64 ramps, float32 result), returned transposed as
    (n_fft // 2 + 1, n_mels) like ``melscale_fbanks``."""
    fmax = float(sr) / 2 if fmax is None else float(fmax)
    fftfreqs = np.fft.rfftfreq(n=n_fft, d=1.0 / sr)
    mel_f = _mel_to_hz_slaney(np.linspace(_hz_to_mel_slaney(fmin), _hz_to_mel_slaney(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    w = np.zeros((n_mels, n_fft // 2 + 1), np.float32)
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        w[i] = np.maximum(0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
    w *= enorm[:, None]
    return np.ascontiguousarray(w.T)


def compute_num_frames(num_samples: int, hop: int) -> int:
    """lhotse.utils.compute_num_frames for duration = num_samples / sr and
    frame_shift = hop / sr: (num_samples + hop // 2) // hop."""
    return int((num_samples + hop // 2) // hop)


class VocosFbank:
    """Mirror of the reference's VocosFbank (feature.py:36-120) on the GPU."""

    name = "VocosFbank"

    # engine front-end variant (zv_fbank_configure): frame-0 sample offset, magnitude
    # epsilon, log floor
    _frame_offset = None            # n_fft // 2: centred STFT
    _mag_eps = 0.0
    _log_floor = 1e-7

    def __init__(self, num_channels: int = 1, device: Optional[Union[str, torch.device]] = None):
        assert num_channels in (1, 2)
        self.config = VocosFbankConfig()
        self.num_channels = num_channels
        c = self.config
        self._sr, self._n_fft, self._hop, self._n_mels = c.sampling_rate, c.n_fft, c.hop_length, c.n_mels
        self.window = torch.hann_window(c.n_fft, dtype=torch.float32)
        self.fb = melscale_fbanks(c.n_fft // 2 + 1, 0.0, float(c.sampling_rate // 2), c.n_mels,
                                  c.sampling_rate).contiguous()
        self._device = torch.device(device) if device is not None else None
        self._h = None
        self._lib = None

    # ------------------------------------------------------------------ lhotse API
    @property
    def frame_shift(self) -> float:
        return self._hop / self._sr

    def feature_dim(self, sampling_rate: int) -> int:
        return self._n_mels

    @property
    def device(self):
        return self._device

    def _handle(self, device: torch.device):
        if not torch.cuda.is_available():
            raise RuntimeError("zipvoice_amd feature extraction needs a ROCm GPU; no CPU fallback")
        if self._h is None:
            self._lib = _eng.load_library()
            w = np.ascontiguousarray(self.window.numpy(), np.float32)
            fb = np.ascontiguousarray(np.asarray(self.fb), np.float32)
            with torch.cuda.device(device):
                h = self._lib.zv_fbank_create(self._n_fft, self._hop, self._n_mels,
                                              w.ctypes.data_as(ctypes.c_void_p),
                                              fb.ctypes.data_as(ctypes.c_void_p))
            if not h:
                raise RuntimeError(self._lib.zv_last_error().decode())
            off = self._n_fft // 2 if self._frame_offset is None else self._frame_offset
            if self._lib.zv_fbank_configure(h, off, self._mag_eps, self._log_floor) != 0:
                err = self._lib.zv_last_error().decode()
                self._lib.zv_fbank_destroy(h)
                raise RuntimeError(err)
            self._h = h
            self._device = device
        return self._h

    def __del__(self):
        if getattr(self, "_h", None) and self._lib is not None:
            try:
                torch.cuda.synchronize(self._device)
            except Exception:
                pass
            self._lib.zv_fbank_destroy(self._h)
            self._h = None

    def extract_batch(self, wavs: torch.Tensor, lens: torch.Tensor,
                      num_frames: Optional[int] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """Batched mono extraction on device: wavs (B, N) fp32 (padded), lens (B,)
        sample counts -> (features (B, T, n_mels), frame counts (B,)).  Each row is
        what ``extract`` returns for that utterance alone."""
        dev = wavs.device if wavs.is_cuda else (self._device or torch.device("cuda"))
        h = self._handle(dev)
        wavs = wavs.to(dev, torch.float32).contiguous()
        B, N = wavs.shape
        hop = self._hop
        lens_cpu = [int(v) for v in lens.cpu().tolist()]
        pad = self._n_fft // 2 if self._frame_offset is None else self._frame_offset
        if min(lens_cpu) <= pad:
            raise ValueError(f"reflect padding needs more than {pad} samples per utterance")
        if max(lens_cpu) > N:
            raise ValueError("lens exceed the padded waveform length")
        nfr = torch.tensor([compute_num_frames(n, hop) for n in lens_cpu], dtype=torch.int64)
        T = int(num_frames if num_frames is not None else nfr.max())
        out = torch.empty((B, T, self._n_mels), dtype=torch.float32, device=dev)
        ln = torch.tensor(lens_cpu, dtype=torch.int32, device=dev)
        _eng._check(self._lib.zv_fbank_extract(h, _eng._ptr(wavs), N, _eng._ptr(ln), B, T,
                                               _eng._ptr(out), self._n_mels, _eng._stream()))
        return out, nfr.to(dev)

    def extract(self, samples: Union[np.ndarray, torch.Tensor], sampling_rate: int
                ) -> Union[np.ndarray, torch.Tensor]:
        """feature.py:66-117: (channels, N) or (N,) samples -> (T, n_mels * num_channels)."""
        expected_sr = self._sr
        assert sampling_rate == expected_sr, (
            f"Mismatched sampling rate: extractor expects {expected_sr}, got {sampling_rate}")
        is_numpy = not isinstance(samples, torch.Tensor)
        src_device = None if is_numpy else samples.device
        x = torch.from_numpy(np.asarray(samples)) if is_numpy else samples
        if x.dim() == 1:
            x = x.unsqueeze(0)
        else:
            assert x.dim() == 2, x.shape
        if self.num_channels == 1:
            if x.shape[0] == 2:
                x = x.mean(dim=0, keepdim=True)
        else:
            assert x.shape[0] == 2, x.shape
        x = x.float()
        n = x.shape[1]
        lens = torch.full((x.shape[0],), n, dtype=torch.int64)
        feats, _ = self.extract_batch(x.to(self._device or "cuda"), lens)   # (C, T, n_mels)
        mel = feats.permute(1, 0, 2).reshape(feats.shape[1], -1)          # (T, C * n_mels)
        if is_numpy:
            return mel.cpu().numpy()
        return mel if src_device.type == "cuda" else mel.to(src_device)


@dataclass
class BigVGANFbankConfig:
    """feature.py:120-130 (BigVGANFbankConfig)."""
    n_fft: int = 1024
    num_mels: int = 100
    sampling_rate: int = 24000
    hop_size: int = 256
    win_size: int = 1024
    fmin: int = 0
    fmax: Optional[int] = None


class BigVGANFbank(VocosFbank):
    """Mirror of the reference's BigVGANFbank (feature.py:133-204) on the GPU:
    ``bigvgan_mel_spectrogram`` (_bigvgan_mel_feature.py:42-111) = reflect pad
    (n_fft - hop) / 2, STFT center=False with a hann window, sqrt(|X|^2 + 1e-9),
    Slaney mel filterbank, log(clamp(1e-5)); (T, n_mels * channels) trimmed or
    replicate-padded (last frame) to lhotse's frame count."""

    name = "BigVGANFbank"
    _mag_eps = 1e-9
    _log_floor = 1e-5

    def __init__(self, num_channels: int = 1, device: Optional[Union[str, torch.device]] = None):
        assert num_channels in (1, 2)
        self.config = BigVGANFbankConfig()
        self.num_channels = num_channels
        c = self.config
        assert c.win_size == c.n_fft, "the engine frames with win_size == n_fft"
        self._sr, self._n_fft, self._hop, self._n_mels = c.sampling_rate, c.n_fft, c.hop_size, c.num_mels
        self._frame_offset = (c.n_fft - c.hop_size) // 2
        self.window = torch.hann_window(c.win_size, dtype=torch.float32)
        self.fb = slaney_mel_fbanks(c.sampling_rate, c.n_fft, c.num_mels, c.fmin, c.fmax)
        self._device = torch.device(device) if device is not None else None
        self._h = None
        self._lib = None


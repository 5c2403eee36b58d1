"""ORACLE — test infrastructure only, never the product path.

(BigVGANFbank: see ``bigvgan_fbank`` below.)

numpy restatement of the reference's prompt feature extractor
``VocosFbank.extract`` (zipvoice/utils/feature.py:36-120): torchaudio
MelSpectrogram(24 kHz, n_fft 1024, hop 256, 100 mels, center=True, reflect
padding, power=1, periodic hann window, HTK mel scale, norm None) ->
clamp(1e-7).log() -> (frames, n_mels) trimmed to lhotse compute_num_frames.
torchaudio and lhotse are not installed: the STFT is pinned against
torch.stft in tests/test_fbank_oracle.py; the filterbank is the caller's
(zipvoice_amd.feature.melscale_fbanks, the torchaudio formula).
"""
import numpy as np


def vocos_fbank(x: np.ndarray, window: np.ndarray, fb: np.ndarray, n_fft: int = 1024,
                hop: int = 256) -> np.ndarray:
    """x: (N,) samples -> (compute_num_frames(N), n_mels) log-mel (float32)."""
    x = np.asarray(x, np.float64)
    n = x.shape[0]
    xp = np.pad(x, (n_fft // 2, n_fft // 2), mode="reflect")
    nfr = 1 + n // hop
    idx = np.arange(nfr)[:, None] * hop + np.arange(n_fft)[None]
    frames = xp[idx] * window.astype(np.float64)
    mag = np.abs(np.fft.rfft(frames, axis=1))
    mel = mag @ fb.astype(np.float64)
    logmel = np.log(np.maximum(mel, 1e-7))
    keep = (n + hop // 2) // hop
    return logmel[:keep].astype(np.float32)


def bigvgan_fbank(x: np.ndarray, window: np.ndarray, fb: np.ndarray, n_fft: int = 1024,
                  hop: int = 256) -> np.ndarray:
    """BigVGANFbank.extract (zipvoice/utils/feature.py:161-204) for one channel:
    ``mel_spectrogram`` (_bigvgan_mel_feature.py:42-111) = reflect pad
    (n_fft - hop) // 2 both sides, frames with center=False, periodic hann window,
    sqrt(|X|^2 + 1e-9), mel projection, log(clamp(1e-5)); then the lhotse frame
    count (num_samples + hop // 2) // hop, trimming or replicating the last frame
    (feature.py:193-201).  x: (N,) -> (frames, n_mels) float32."""
    x = np.asarray(x, np.float64)
    n = x.shape[0]
    p = (n_fft - hop) // 2
    xp = np.pad(x, (p, p), mode="reflect")
    nst = 1 + (xp.shape[0] - n_fft) // hop
    idx = np.arange(nst)[:, None] * hop + np.arange(n_fft)[None]
    spec = np.fft.rfft(xp[idx] * window.astype(np.float64), axis=1)
    mag = np.sqrt(spec.real ** 2 + spec.imag ** 2 + 1e-9)
    logmel = np.log(np.maximum(mag @ fb.astype(np.float64), 1e-5))
    keep = (n + hop // 2) // hop
    if nst >= keep:
        logmel = logmel[:keep]
    else:
        logmel = np.concatenate([logmel, np.repeat(logmel[-1:], keep - nst, axis=0)])
    return logmel.astype(np.float32)

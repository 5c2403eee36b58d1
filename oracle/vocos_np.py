"""ORACLE — test infrastructure only, never the product path.

CPU (numpy, fp32) restatement of the vocoder the reference calls after
sampling: ``wav = vocoder.decode(pred_features).squeeze(1).clamp(-1, 1)``
(``zipvoice/bin/infer_zipvoice.py:374-378``, dialog stereo
``infer_zipvoice_dialog.py:483-488``) with ``vocoder = Vocos.from_pretrained(
"charactr/vocos-mel-24khz")`` (``infer_zipvoice.py:249-260``).

The arithmetic lives in the third-party ``vocos`` package (``requirements.txt:7``,
unpinned; the published release is vocos 0.1.0), which is NOT present in
``/root/reference`` nor installed here.  This module restates that package's
published algorithm for the mel-24khz configuration:

* ``Vocos.decode``                     vocos/pretrained.py  (backbone -> head)
* ``VocosBackbone.forward``            vocos/models.py      (embed Conv1d k7 -> LayerNorm ->
                                                             8 x ConvNeXtBlock -> final LayerNorm)
* ``ConvNeXtBlock.forward``            vocos/modules.py     (dwconv k7 -> LayerNorm -> Linear ->
                                                             GELU -> Linear -> gamma * x + residual)
* ``ISTFTHead.forward``                vocos/heads.py       (Linear dim -> n_fft+2, mag = clip(exp, 1e2),
                                                             S = mag * (cos p + i sin p))
* ``ISTFT.forward`` (padding="same")   vocos/spectral_ops.py (irfft * window, overlap-add over
                                                             (T-1)*hop + win, trim (win-hop)/2 per
                                                             side, divide by the squared-window envelope)

Parity status: the network composition is "parity unpinned" (package absent,
no reference fixture exists); the primitives are pinned in
``tests/test_vocos_oracle.py`` against the torch ops vocos calls
(``torch.fft.irfft`` + ``F.fold`` and ``torch.istft``, ``F.layer_norm``,
``F.gelu``, ``F.conv1d``).  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import this module.
"""
from __future__ import annotations

from typing import Dict, Optional, Sequence

import numpy as np

F32 = np.float32


def layer_norm(x: np.ndarray, w: np.ndarray, b: np.ndarray, eps: float = 1e-6) -> np.ndarray:
    """nn.LayerNorm(dim, eps=1e-6) over the last axis (biased variance)."""
    x64 = x.astype(np.float64)
    mu = x64.mean(-1, keepdims=True)
    var = ((x64 - mu) ** 2).mean(-1, keepdims=True)
    return (((x64 - mu) / np.sqrt(var + eps)) * w + b).astype(F32)


def gelu(x: np.ndarray) -> np.ndarray:
    """nn.GELU() (exact, erf form)."""
    from scipy.special import erf
    x64 = x.astype(np.float64)
    return (0.5 * x64 * (1.0 + erf(x64 / np.sqrt(2.0)))).astype(F32)


def conv1d_same(x: np.ndarray, w: np.ndarray, b: np.ndarray, length: int) -> np.ndarray:
    """Conv1d(Cin, Cout, k, padding=k//2) on (T, Cin) -> (T, Cout) for one
    utterance of `length` frames (zero padding outside [0, length))."""
    T, Cin = x.shape[0], x.shape[1]
    Cout, _, k = w.shape
    pad = k // 2
    xp = np.zeros((length + 2 * pad, Cin), F32)
    xp[pad:pad + length] = x[:length]
    out = np.zeros((length, Cout), np.float64)
    for tap in range(k):
        out += xp[tap:tap + length].astype(np.float64) @ w[:, :, tap].T.astype(np.float64)
    out += b
    return out.astype(F32)


def dwconv_same(x: np.ndarray, w: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Depthwise Conv1d(C, C, k, padding=k//2, groups=C) on (T, C)."""
    T, C = x.shape
    k = w.shape[-1]
    pad = k // 2
    xp = np.zeros((T + 2 * pad, C), np.float64)
    xp[pad:pad + T] = x
    out = np.zeros((T, C), np.float64)
    for tap in range(k):
        out += xp[tap:tap + T] * w[:, 0, tap]
    return (out + b).astype(F32)


def istft_same(re: np.ndarray, im: np.ndarray, window: np.ndarray, hop: int) -> np.ndarray:
    """ISTFT(padding="same") of one utterance: re/im (T, n_fft/2+1) -> (T*hop,).
    irfft (C2R: imaginary parts of DC and Nyquist ignored), times the window,
    overlap-add, trim (win-hop)/2 per side, divide by the squared-window envelope."""
    T, nb = re.shape
    n_fft = window.shape[0]
    frames = np.fft.irfft(re.astype(np.float64) + 1j * im.astype(np.float64), n=n_fft, axis=1)
    frames = frames * window.astype(np.float64)
    out_size = (T - 1) * hop + n_fft
    y = np.zeros(out_size, np.float64)
    env = np.zeros(out_size, np.float64)
    w2 = window.astype(np.float64) ** 2
    for f in range(T):
        y[f * hop:f * hop + n_fft] += frames[f]
        env[f * hop:f * hop + n_fft] += w2
    pad = (n_fft - hop) // 2
    y, env = y[pad:out_size - pad], env[pad:out_size - pad]
    assert (env > 1e-11).all()
    return (y / env).astype(F32)


class VocosOracle:
    """Vocos mel-24khz decode with a given state dict (vocos key names)."""

    def __init__(self, sd: Dict[str, np.ndarray], num_layers: int = 8, hop: int = 256):
        self.sd = {k: np.asarray(v, F32) for k, v in sd.items()}
        self.num_layers = num_layers
        self.hop = hop

    def backbone(self, mel_tc: np.ndarray) -> np.ndarray:
        """VocosBackbone.forward on one utterance, mel (T, n_mels) -> (T, dim)."""
        s = self.sd
        T = mel_tc.shape[0]
        x = conv1d_same(mel_tc, s["backbone.embed.weight"], s["backbone.embed.bias"], T)
        x = layer_norm(x, s["backbone.norm.weight"], s["backbone.norm.bias"])
        for i in range(self.num_layers):
            p = f"backbone.convnext.{i}."
            h = dwconv_same(x, s[p + "dwconv.weight"], s[p + "dwconv.bias"])
            h = layer_norm(h, s[p + "norm.weight"], s[p + "norm.bias"])
            h = (h.astype(np.float64) @ s[p + "pwconv1.weight"].T.astype(np.float64)
                 + s[p + "pwconv1.bias"]).astype(F32)
            h = gelu(h)
            h = (h.astype(np.float64) @ s[p + "pwconv2.weight"].T.astype(np.float64)
                 + s[p + "pwconv2.bias"]).astype(F32)
            x = (x + s[p + "gamma"] * h).astype(F32)
        return layer_norm(x, s["backbone.final_layer_norm.weight"],
                          s["backbone.final_layer_norm.bias"])

    def head(self, x: np.ndarray) -> np.ndarray:
        """ISTFTHead.forward on one utterance, (T, dim) -> (T*hop,)."""
        s = self.sd
        o = (x.astype(np.float64) @ s["head.out.weight"].T.astype(np.float64)
             + s["head.out.bias"]).astype(F32)
        nb = o.shape[1] // 2
        mag = np.minimum(np.exp(o[:, :nb]), F32(1e2)).astype(F32)
        p = o[:, nb:]
        re = (mag * np.cos(p)).astype(F32)
        im = (mag * np.sin(p)).astype(F32)
        return istft_same(re, im, s["head.istft.window"], self.hop)

    def decode(self, mel: np.ndarray, lens: Optional[Sequence[int]] = None) -> np.ndarray:
        """Vocos.decode on (B, n_mels, T) -> (B, T*hop); with `lens`, utterance b
        is decoded on its own first lens[b] frames (as the reference does, one
        sentence per call) and the tail is zero."""
        B, _, T = mel.shape
        out = np.zeros((B, T * self.hop), F32)
        for b in range(B):
            L = T if lens is None else int(lens[b])
            out[b, :L * self.hop] = self.head(self.backbone(mel[b, :, :L].T))
        return out


def postprocess_features(pred: np.ndarray, feat_scale: float = 0.1,
                         feat_bias: float = 0.0) -> np.ndarray:
    """infer_zipvoice.py:374: pred (B, T, C) -> (B, C, T) / feat_scale - feat_bias."""
    return (np.transpose(pred, (0, 2, 1)) / F32(feat_scale) - F32(feat_bias)).astype(F32)

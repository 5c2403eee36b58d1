"""ORACLE — test infrastructure only, never the product path.

numpy (float64) restatement of the BigVGAN-v2 vocoder the reference loads for
``feature.type == "bigvgan_v2"`` (zipvoice/bin/infer_zipvoice.py:261-269:
``bigvgan.BigVGAN.from_pretrained('nvidia/bigvgan_v2_24khz_100band_256x',
use_cuda_kernel=False)``, ``remove_weight_norm()``, ``decode(features) = forward``).
The arithmetic lives in the third-party ``bigvgan`` package (NVIDIA BigVGAN v2,
bigvgan.py / activations.py / alias_free_activation/torch/{filter,resample,act}.py),
which is absent here, as are its weights: this restates the published algorithm,
and parity of the network is UNPINNED (anchored only on the reference's call site:
mel (B, 100, T) -> wav (B, 1, 256 T), clamp(-1, 1) at the end for
use_tanh_at_final = False).

Network (config bigvgan_v2_24khz_100band_256x):
  conv_pre Conv1d(100, 1536, 7, pad 3)
  6 x [ ConvTranspose1d(C, C/2, k_i, u_i, pad (k_i - u_i)/2),
        mean over 3 AMPBlock1(C/2, k in (3, 7, 11), dilations (1, 3, 5)) ]
  Activation1d(SnakeBeta(24)) -> conv_post Conv1d(24, 1, 7, pad 3, no bias) -> clamp(-1, 1)
AMPBlock1: for d: x = x + c2(a2(c1(a1(x)))), c1 dilated by d, c2 dilation 1 ("same" pads).
Activation1d (anti-aliased): UpSample1d(2) -> SnakeBeta -> DownSample1d(2), both with the
12-tap kaiser-sinc low-pass (cutoff 0.25, half width 0.3) and replicate padding.
SnakeBeta (alpha_logscale): x + 1 / (exp(beta) + 1e-9) * sin(x exp(alpha))^2.
"""
import math

import numpy as np

CONFIG = dict(num_mels=100, upsample_rates=(4, 4, 2, 2, 2, 2),
              upsample_kernel_sizes=(8, 8, 4, 4, 4, 4), upsample_initial_channel=1536,
              resblock_kernel_sizes=(3, 7, 11), resblock_dilation_sizes=((1, 3, 5),) * 3,
              use_tanh_at_final=False, use_bias_at_final=False)


def kaiser_sinc_filter1d(cutoff: float, half_width: float, kernel_size: int) -> np.ndarray:
    """alias_free_activation/torch/filter.py: kaiser-windowed sinc low-pass, unit DC gain."""
    even = kernel_size % 2 == 0
    half_size = kernel_size // 2
    delta_f = 4 * half_width
    A = 2.285 * (half_size - 1) * math.pi * delta_f + 7.95
    if A > 50.0:
        beta = 0.1102 * (A - 8.7)
    elif A >= 21.0:
        beta = 0.5842 * (A - 21) ** 0.4 + 0.07886 * (A - 21.0)
    else:
        beta = 0.0
    window = np.kaiser(kernel_size, beta)          # == torch.kaiser_window(periodic=False)
    time = (np.arange(-half_size, half_size) + 0.5) if even else (np.arange(kernel_size) - half_size)
    f = 2 * cutoff * window * np.sinc(2 * cutoff * time)
    return f / f.sum()


def anti_alias_filter(ratio: int = 2) -> np.ndarray:
    ks = int(6 * ratio // 2) * 2
    return kaiser_sinc_filter1d(0.5 / ratio, 0.6 / ratio, ks)


def conv1d(x, w, b, dilation=1, padding=0):
    """x (Cin, T), w (Cout, Cin, k) -> (Cout, T + 2 pad - d (k - 1)); zero padding."""
    cout, cin, k = w.shape
    xp = np.pad(x, ((0, 0), (padding, padding)))
    T = xp.shape[1] - dilation * (k - 1)
    cols = np.stack([xp[:, i * dilation:i * dilation + T] for i in range(k)], 1)   # (Cin, k, T)
    y = w.reshape(cout, cin * k) @ cols.reshape(cin * k, T)
    return y + b[:, None] if b is not None else y


def conv_transpose1d(x, w, b, stride, padding):
    """x (Cin, T), w (Cin, Cout, k) -> (Cout, (T - 1) stride - 2 pad + k)."""
    cin, cout, k = w.shape
    T = x.shape[1]
    full = np.zeros((cout, (T - 1) * stride + k))
    prod = np.einsum("ct,cok->okt", x, w)           # (Cout, k, T)
    for j in range(k):
        full[:, j:j + (T - 1) * stride + 1:stride] += prod[:, j]
    y = full[:, padding:full.shape[1] - padding]
    return y + b[:, None] if b is not None else y


def activation1d_snakebeta(x, log_alpha, log_beta, filt):
    """Activation1d(SnakeBeta(alpha_logscale=True)) with ratio 2 (act.py / resample.py)."""
    ratio, ks = 2, filt.shape[0]
    C, T = x.shape
    # UpSample1d: replicate pad, ratio * conv_transpose(stride ratio) with the filter, crop
    pad = ks // ratio - 1
    pad_left = pad * ratio + (ks - ratio) // 2
    pad_right = pad * ratio + (ks - ratio + 1) // 2
    xp = np.pad(x, ((0, 0), (pad, pad)), mode="edge")
    full = np.zeros((C, (xp.shape[1] - 1) * ratio + ks))
    for j in range(ks):
        full[:, j:j + (xp.shape[1] - 1) * ratio + 1:ratio] += xp * filt[j]
    y = ratio * full[:, pad_left:full.shape[1] - pad_right]
    # SnakeBeta
    a = np.exp(log_alpha)[:, None]
    bt = np.exp(log_beta)[:, None]
    y = y + 1.0 / (bt + 1e-9) * np.sin(y * a) ** 2
    # DownSample1d = LowPassFilter1d(stride ratio): replicate pad (k/2 - even, k/2), strided conv
    pl, pr = ks // 2 - int(ks % 2 == 0), ks // 2
    yp = np.pad(y, ((0, 0), (pl, pr)), mode="edge")
    n_out = (yp.shape[1] - ks) // ratio + 1
    z = np.zeros((C, n_out))
    for j in range(ks):
        z += yp[:, j:j + (n_out - 1) * ratio + 1:ratio] * filt[j]
    return z


def bigvgan_forward(mel: np.ndarray, sd: dict, cfg: dict = CONFIG) -> np.ndarray:
    """mel (n_mels, T) -> wav (T * prod(upsample_rates),), one utterance."""
    g = {k: np.asarray(v, np.float64) for k, v in sd.items()}
    filt = anti_alias_filter(2)
    x = conv1d(np.asarray(mel, np.float64), g["conv_pre.weight"], g["conv_pre.bias"], padding=3)
    nk = len(cfg["resblock_kernel_sizes"])
    for i, (u, k) in enumerate(zip(cfg["upsample_rates"], cfg["upsample_kernel_sizes"])):
        x = conv_transpose1d(x, g[f"ups.{i}.0.weight"], g[f"ups.{i}.0.bias"], u, (k - u) // 2)
        xs = None
        for j, (ks, dil) in enumerate(zip(cfg["resblock_kernel_sizes"], cfg["resblock_dilation_sizes"])):
            p = f"resblocks.{i * nk + j}."
            y = x
            for n, d in enumerate(dil):
                a1, a2 = f"{p}activations.{2 * n}.act.", f"{p}activations.{2 * n + 1}.act."
                t = activation1d_snakebeta(y, g[a1 + "alpha"], g[a1 + "beta"], filt)
                t = conv1d(t, g[f"{p}convs1.{n}.weight"], g[f"{p}convs1.{n}.bias"], d, (ks * d - d) // 2)
                t = activation1d_snakebeta(t, g[a2 + "alpha"], g[a2 + "beta"], filt)
                t = conv1d(t, g[f"{p}convs2.{n}.weight"], g[f"{p}convs2.{n}.bias"], 1, (ks - 1) // 2)
                y = t + y
            xs = y if xs is None else xs + y
        x = xs / nk
    x = activation1d_snakebeta(x, g["activation_post.act.alpha"], g["activation_post.act.beta"], filt)
    x = conv1d(x, g["conv_post.weight"], g.get("conv_post.bias"), padding=3)
    x = np.tanh(x) if cfg["use_tanh_at_final"] else np.clip(x, -1.0, 1.0)
    return x[0].astype(np.float32)

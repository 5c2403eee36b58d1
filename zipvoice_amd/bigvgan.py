"""Drop-in BigVGAN-v2 vocoder (the reference's ``feature.type == "bigvgan_v2"`` path).

The reference loads ``bigvgan.BigVGAN.from_pretrained('nvidia/bigvgan_v2_24khz_100band_256x',
use_cuda_kernel=False)``, calls ``remove_weight_norm()`` and binds ``decode = forward``
(``zipvoice/bin/infer_zipvoice.py:261-269``); the features come from
:class:`zipvoice_amd.feature.BigVGANFbank` (``zipvoice/utils/feature.py:133-204``).
This module mirrors that surface (``BigVGAN.from_pretrained`` on a local directory,
``load_state_dict``, ``remove_weight_norm``, ``decode``) with the compute in the HIP
engine (``zv_bigvgan_*`` in ``include/zipvoice_hip.h``, ``csrc/zv_bigvgan.inc``):
MFMA GEMMs over im2col operands for every Conv1d, a GEMM + gather for each
ConvTranspose1d, and one fused kernel for the anti-aliased SnakeBeta activation
(2x kaiser-sinc upsample -> snake -> 12-tap low-pass downsample) that writes the next
conv's operand directly.

The ``bigvgan`` package and its checkpoint are absent offline: parity is against the
numpy restatement in ``oracle/bigvgan_np.py`` ("parity unpinned" w.r.t. the package);
tests and benchmarks use :func:`synthetic_bigvgan_state_dict`.
"""
from __future__ import annotations

import ctypes
import json
import os
import zlib
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Dict, Optional, Tuple

import numpy as np
import torch

from . import engine as _eng


@dataclass
class BigVGANConfig:
    """bigvgan_v2_24khz_100band_256x config.json (the generator fields)."""
    num_mels: int = 100
    upsample_initial_channel: int = 1536
    upsample_rates: Tuple[int, ...] = (4, 4, 2, 2, 2, 2)
    upsample_kernel_sizes: Tuple[int, ...] = (8, 8, 4, 4, 4, 4)
    resblock_kernel_sizes: Tuple[int, ...] = (3, 7, 11)
    resblock_dilation_sizes: Tuple[Tuple[int, ...], ...] = ((1, 3, 5), (1, 3, 5), (1, 3, 5))
    resblock: str = "1"
    activation: str = "snakebeta"
    snake_logscale: bool = True
    use_tanh_at_final: bool = False
    use_bias_at_final: bool = False
    sampling_rate: int = 24000

    @property
    def hop_length(self) -> int:
        return int(np.prod(self.upsample_rates))

    @classmethod
    def from_json(cls, path: str) -> "BigVGANConfig":
        with open(path) as f:
            h = json.load(f)
        if str(h.get("resblock", "1")) != "1":
            raise NotImplementedError("only AMPBlock1 (resblock '1') is supported")
        if h.get("activation", "snakebeta") != "snakebeta":
            raise NotImplementedError("only the snakebeta activation is supported")
        return cls(num_mels=h["num_mels"], upsample_initial_channel=h["upsample_initial_channel"],
                   upsample_rates=tuple(h["upsample_rates"]),
                   upsample_kernel_sizes=tuple(h["upsample_kernel_sizes"]),
                   resblock_kernel_sizes=tuple(h["resblock_kernel_sizes"]),
                   resblock_dilation_sizes=tuple(tuple(d) for d in h["resblock_dilation_sizes"]),
                   snake_logscale=bool(h.get("snake_logscale", True)),
                   use_tanh_at_final=bool(h.get("use_tanh_at_final", True)),
                   use_bias_at_final=bool(h.get("use_bias_at_final", True)),
                   sampling_rate=h.get("sampling_rate", 24000))


def bigvgan_state_shapes(cfg: BigVGANConfig) -> "OrderedDict[str, tuple]":
    """Tensor names / shapes of a weight-norm-removed BigVGAN generator."""
    d: "OrderedDict[str, tuple]" = OrderedDict()
    C = cfg.upsample_initial_channel
    d["conv_pre.weight"] = (C, cfg.num_mels, 7)
    d["conv_pre.bias"] = (C,)
    nk = len(cfg.resblock_kernel_sizes)
    for i, (u, k) in enumerate(zip(cfg.upsample_rates, cfg.upsample_kernel_sizes)):
        d[f"ups.{i}.0.weight"] = (C, C // 2, k)
        d[f"ups.{i}.0.bias"] = (C // 2,)
        C //= 2
        for j, ks in enumerate(cfg.resblock_kernel_sizes):
            p = f"resblocks.{i * nk + j}."
            for n in range(len(cfg.resblock_dilation_sizes[j])):
                d[f"{p}convs1.{n}.weight"] = (C, C, ks)
                d[f"{p}convs1.{n}.bias"] = (C,)
            for n in range(len(cfg.resblock_dilation_sizes[j])):
                d[f"{p}convs2.{n}.weight"] = (C, C, ks)
                d[f"{p}convs2.{n}.bias"] = (C,)
            for a in range(2 * len(cfg.resblock_dilation_sizes[j])):
                d[f"{p}activations.{a}.act.alpha"] = (C,)
                d[f"{p}activations.{a}.act.beta"] = (C,)
    d["activation_post.act.alpha"] = (C,)
    d["activation_post.act.beta"] = (C,)
    d["conv_post.weight"] = (1, C, 7)
    if cfg.use_bias_at_final:
        d["conv_post.bias"] = (1,)
    return d


def synthetic_bigvgan_state_dict(cfg: BigVGANConfig = BigVGANConfig(), seed: int = 0
                                 ) -> "OrderedDict[str, np.ndarray]":
    """Deterministic weights (numpy PCG64 per tensor name) scaled so activations stay
    O(1) through all stages: unit-gain conv_pre / transposed convs, AMP residual branches
    at ~0.3 gain, log-alpha / log-beta in [-0.3, 0.3], conv_post output std ~0.3
    (well inside the final clamp)."""
    out: "OrderedDict[str, np.ndarray]" = OrderedDict()
    for k, shape in bigvgan_state_shapes(cfg).items():
        rng = np.random.Generator(np.random.PCG64([seed, zlib.crc32(("bigvgan." + k).encode())]))
        n = int(np.prod(shape))

        def uni(a):
            return (a * (2.0 * rng.random(n, dtype=np.float64) - 1.0)).astype(np.float32)

        if k.endswith(".alpha") or k.endswith(".beta"):
            v = uni(0.3)
        elif k.endswith(".bias"):
            v = uni(0.05)
        elif k == "conv_pre.weight":
            v = uni(np.sqrt(3.0 / (shape[1] * shape[2])) * 0.5)
        elif k.startswith("ups."):
            u = cfg.upsample_rates[int(k.split(".")[1])]
            v = uni(np.sqrt(3.0 / (shape[0] * shape[2] / u)))
        elif ".convs1." in k:
            v = uni(np.sqrt(3.0 / (shape[1] * shape[2])))
        elif ".convs2." in k:
            v = uni(np.sqrt(3.0 / (shape[1] * shape[2])) * 0.3)
        elif k == "conv_post.weight":
            v = uni(np.sqrt(3.0 / (shape[1] * shape[2])) * 0.15)
        else:
            raise KeyError(k)
        out[k] = v.reshape(shape)
    return out


def remove_weight_norm_state(sd: Dict[str, np.ndarray]) -> Dict[str, np.ndarray]:
    """Fold weight-norm pairs into plain weights (what ``remove_weight_norm()`` does):
    ``X.weight_g`` / ``X.weight_v`` (torch.nn.utils.weight_norm) or
    ``X.parametrizations.weight.original0`` / ``original1`` (parametrize API) ->
    ``X.weight = g * v / ||v||``, the norm taken over every dim but 0."""
    out = {}
    pairs = {}
    for k, v in sd.items():
        if k.endswith(".weight_g") or k.endswith(".weight_v"):
            pairs.setdefault(k[:-9], {})[k[-1]] = v
        elif k.endswith(".parametrizations.weight.original0"):
            pairs.setdefault(k[:-34], {})["g"] = v
        elif k.endswith(".parametrizations.weight.original1"):
            pairs.setdefault(k[:-34], {})["v"] = v
        else:
            out[k] = v
    for base, gv in pairs.items():
        if set(gv) != {"g", "v"}:
            raise KeyError(f"incomplete weight-norm pair for {base}")
        v = np.asarray(gv["v"], np.float64)
        g = np.asarray(gv["g"], np.float64)
        norm = np.sqrt((v.reshape(v.shape[0], -1) ** 2).sum(1)).reshape((-1,) + (1,) * (v.ndim - 1))
        out[base + ".weight"] = (g.reshape(norm.shape) * v / norm).astype(np.float32)
    return out


def _is_filter(k: str) -> bool:
    return k.endswith(".upsample.filter") or k.endswith(".downsample.lowpass.filter")


class ZvBigVGANConfig(ctypes.Structure):
    _fields_ = [("precision", ctypes.c_int), ("num_mels", ctypes.c_int),
                ("upsample_initial_channel", ctypes.c_int), ("num_upsamples", ctypes.c_int),
                ("upsample_rates", ctypes.c_int * 8), ("upsample_kernel_sizes", ctypes.c_int * 8),
                ("num_kernels", ctypes.c_int), ("resblock_kernel_sizes", ctypes.c_int * 3),
                ("resblock_dilation_sizes", (ctypes.c_int * 3) * 3),
                ("snake_logscale", ctypes.c_int), ("use_tanh_at_final", ctypes.c_int),
                ("use_bias_at_final", ctypes.c_int)]


def _check_state(cfg: BigVGANConfig, sd: Dict[str, np.ndarray]) -> Dict[str, np.ndarray]:
    want = bigvgan_state_shapes(cfg)
    body = {k: v for k, v in sd.items() if not _is_filter(k)}
    missing = [k for k in want if k not in body]
    unexpected = [k for k in body if k not in want]
    if missing or unexpected:
        raise KeyError(f"bigvgan state dict mismatch: missing={missing[:5]}, "
                       f"unexpected={unexpected[:5]}")
    for k, s in want.items():
        if tuple(np.shape(body[k])) != tuple(s):
            raise ValueError(f"shape mismatch for {k}: {np.shape(body[k])} vs {s}")
    return sd


class BigVGAN:
    """Mirror of ``bigvgan.BigVGAN`` (inference).  ``precision="fp32"`` (default) runs
    the GEMMs as split bf16x3 products; ``"bf16"`` plain bf16 MFMA operands."""

    def __init__(self, cfg: BigVGANConfig = BigVGANConfig(), precision: str = "fp32"):
        if len(cfg.upsample_rates) > 8 or len(cfg.resblock_kernel_sizes) > 3:
            raise NotImplementedError("at most 8 upsampling stages and 3 AMP kernels")
        if any(len(d) != 3 for d in cfg.resblock_dilation_sizes):
            raise NotImplementedError("AMPBlock1 uses exactly 3 dilations")
        if precision not in _eng.PRECISION_ID:
            raise ValueError(f"precision must be one of {list(_eng.PRECISION_ID)}")
        self.cfg = cfg
        self.h_cfg = cfg
        self.precision = precision
        self._state: Optional[Dict[str, np.ndarray]] = None
        self.h = None
        self.device = torch.device("cpu")
        self.lib = None

    @classmethod
    def from_pretrained(cls, model_id: str, use_cuda_kernel: bool = False,
                        precision: str = "fp32") -> "BigVGAN":
        """Local directory with config.json + bigvgan_generator.pt ({'generator': sd});
        the Hub is not reachable offline.  ``use_cuda_kernel`` is accepted for API
        parity (the fused activation here is always the HIP kernel)."""
        if not os.path.isdir(model_id):
            raise RuntimeError(f"cannot fetch {model_id!r}: no network; pass a local directory "
                               "with config.json and bigvgan_generator.pt")
        voc = cls(BigVGANConfig.from_json(os.path.join(model_id, "config.json")), precision)
        blob = torch.load(os.path.join(model_id, "bigvgan_generator.pt"), map_location="cpu",
                          weights_only=True)
        voc.load_state_dict(blob.get("generator", blob))
        return voc

    def load_state_dict(self, state_dict, strict: bool = True):
        sd = {k: (v.detach().cpu().float().numpy() if isinstance(v, torch.Tensor)
                  else np.asarray(v, np.float32)) for k, v in state_dict.items()}
        self._state = _check_state(self.cfg, remove_weight_norm_state(sd))
        if self.h is not None:
            self._upload()
        return self

    def load_synthetic(self, seed: int = 0):
        return self.load_state_dict(synthetic_bigvgan_state_dict(self.cfg, seed))

    def remove_weight_norm(self):
        """Weight norm is folded when the state dict is loaded."""
        return self

    def _upload(self):
        if not torch.cuda.is_available():
            raise RuntimeError("zipvoice_amd BigVGAN needs a ROCm GPU (MI355X); no CPU fallback")
        self.lib = _eng.load_library()
        if self.h:
            self.lib.zv_bigvgan_destroy(self.h)
            self.h = None
        c = self.cfg
        cc = ZvBigVGANConfig(precision=_eng.PRECISION_ID[self.precision], num_mels=c.num_mels,
                             upsample_initial_channel=c.upsample_initial_channel,
                             num_upsamples=len(c.upsample_rates),
                             num_kernels=len(c.resblock_kernel_sizes),
                             snake_logscale=int(c.snake_logscale),
                             use_tanh_at_final=int(c.use_tanh_at_final),
                             use_bias_at_final=int(c.use_bias_at_final))
        for i, (u, k) in enumerate(zip(c.upsample_rates, c.upsample_kernel_sizes)):
            cc.upsample_rates[i] = u
            cc.upsample_kernel_sizes[i] = k
        for j, ks in enumerate(c.resblock_kernel_sizes):
            cc.resblock_kernel_sizes[j] = ks
            for n, d in enumerate(c.resblock_dilation_sizes[j]):
                cc.resblock_dilation_sizes[j][n] = d
        with torch.cuda.device(self.device):
            h = self.lib.zv_bigvgan_create(ctypes.byref(cc))
            if not h:
                raise RuntimeError(self.lib.zv_last_error().decode())
            self.h = h
            for k, v in self._state.items():
                a = np.ascontiguousarray(v, np.float32)
                _eng._check(self.lib.zv_bigvgan_set_weight(h, k.encode(),
                                                           a.ctypes.data_as(ctypes.c_void_p), a.size))
            _eng._check(self.lib.zv_bigvgan_finalize(h))

    def to(self, device):
        device = torch.device(device)
        if device.type != "cuda":
            raise RuntimeError("zipvoice_amd BigVGAN runs on the GPU only (no CPU fallback)")
        if device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        if self._state is None:
            raise RuntimeError("load_state_dict() before .to(device)")
        self.device = device
        self._upload()
        return self

    def eval(self):
        return self

    def __del__(self):
        h = getattr(self, "h", None)
        if h and self.lib is not None:
            try:
                torch.cuda.synchronize(self.device)
            except Exception:
                pass
            self.lib.zv_bigvgan_destroy(h)
            self.h = None

    def _run(self, x: torch.Tensor, layout: int, feat_scale: float, feat_bias: float,
             lens: Optional[torch.Tensor]) -> torch.Tensor:
        if self.h is None:
            raise RuntimeError("vocoder not on a device: call .to('cuda')")
        x = x.to(self.device, torch.float32).contiguous()
        B = x.shape[0]
        T = x.shape[2] if layout == 0 else x.shape[1]
        C = x.shape[1] if layout == 0 else x.shape[2]
        if C != self.cfg.num_mels:
            raise ValueError(f"expected {self.cfg.num_mels} mel channels, got {C}")
        ln = None
        if lens is not None:
            ln = lens.to(self.device, torch.int32).contiguous()
            if ln.shape != (B,):
                raise ValueError("lens must have shape (B,)")
        wav = torch.empty((B, T * self.cfg.hop_length), dtype=torch.float32, device=self.device)
        _eng._check(self.lib.zv_bigvgan_decode(
            self.h, _eng._ptr(x), layout, float(feat_scale), float(feat_bias), _eng._ptr(ln),
            B, T, _eng._ptr(wav), _eng._stream()))
        return wav

    @torch.inference_mode()
    def __call__(self, mel: torch.Tensor) -> torch.Tensor:
        """BigVGAN.forward: mel (B, num_mels, T) -> audio (B, 1, T * hop)."""
        if mel.dim() != 3:
            raise ValueError("mel must be (B, num_mels, T)")
        return self._run(mel, 0, 1.0, 0.0, None).unsqueeze(1)

    forward = __call__
    decode = __call__           # infer_zipvoice.py:266-269

    def decode_features(self, pred_features: torch.Tensor, lens: Optional[torch.Tensor] = None,
                        feat_scale: float = 0.1, feat_bias: float = 0.0,
                        clamp: bool = True) -> torch.Tensor:
        """The reference's post-sampling step on device (infer_zipvoice.py:374-378):
        pred (B, T, num_mels) -> wav (B, T*hop); the network's own final clamp makes the
        reference's ``clamp(-1, 1)`` a no-op, so ``clamp`` is accepted for API parity."""
        return self._run(pred_features, 1, feat_scale, feat_bias, lens)

    def device_bytes(self) -> int:
        return int(self.lib.zv_bigvgan_device_bytes(self.h)) if self.h else 0

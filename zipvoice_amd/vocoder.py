"""Drop-in vocoder for the reference's post-sampling step.

The reference loads the third-party Vocos vocoder (``get_vocoder``,
``zipvoice/bin/infer_zipvoice.py:249-273``) and calls
``vocoder.decode(pred_features).squeeze(1).clamp(-1, 1)`` on the generated
features after ``pred_features.permute(0, 2, 1) / feat_scale - feat_bias``
(``infer_zipvoice.py:374-378``; dialog-stereo decodes each channel,
``infer_zipvoice_dialog.py:483-488``).  This module mirrors that API
(``Vocos.from_hparams`` / ``load_state_dict`` / ``decode``, ``get_vocoder``)
with the compute in the HIP engine's vocoder (``zv_vocoder_*`` in
``include/zipvoice_hip.h``): MFMA GEMMs for the embed conv (im2col), the
ConvNeXt pointwise layers, the ISTFT head and the irfft (a real DFT basis GEMM),
plus row kernels for LayerNorm / depthwise conv and a gather overlap-add.

State-dict keys are vocos' own (``backbone.*``, ``head.*``; the
``feature_extractor.*`` buffers of a full Vocos checkpoint are accepted and
ignored).  No pretrained vocoder can be fetched offline: ``from_pretrained``
needs a local directory; tests and the benchmark use
:func:`synthetic_vocos_state_dict`.
"""
from __future__ import annotations

import ctypes
import os
import zlib
from collections import OrderedDict
from dataclasses import dataclass
from typing import Dict, Optional

import numpy as np
import torch

from . import engine as _eng


@dataclass
class VocosConfig:
    """vocos-mel-24khz config.yaml (backbone / head init_args)."""
    n_mels: int = 100
    dim: int = 512
    intermediate_dim: int = 1536
    num_layers: int = 8
    n_fft: int = 1024
    hop_length: int = 256
    padding: str = "same"
    sample_rate: int = 24000

    @classmethod
    def from_yaml(cls, path: str) -> "VocosConfig":
        import yaml
        with open(path) as f:
            y = yaml.safe_load(f)
        bb = y["backbone"]["init_args"]
        hd = y["head"]["init_args"]
        if "vocos.heads.ISTFTHead" not in y["head"]["class_path"]:
            raise NotImplementedError(f"unsupported vocos head {y['head']['class_path']}")
        if bb.get("adanorm_num_embeddings"):
            raise NotImplementedError("AdaLayerNorm (bandwidth-conditioned) vocos is not supported")
        fe = y.get("feature_extractor", {}).get("init_args", {})
        return cls(n_mels=bb["input_channels"], dim=bb["dim"],
                   intermediate_dim=bb["intermediate_dim"], num_layers=bb["num_layers"],
                   n_fft=hd["n_fft"], hop_length=hd["hop_length"],
                   padding=hd.get("padding", "same"), sample_rate=fe.get("sample_rate", 24000))


def vocos_state_shapes(cfg: VocosConfig) -> "OrderedDict[str, tuple]":
    C, I = cfg.dim, cfg.intermediate_dim
    d: "OrderedDict[str, tuple]" = OrderedDict()
    d["backbone.embed.weight"] = (C, cfg.n_mels, 7)
    d["backbone.embed.bias"] = (C,)
    d["backbone.norm.weight"] = (C,)
    d["backbone.norm.bias"] = (C,)
    for i in range(cfg.num_layers):
        p = f"backbone.convnext.{i}."
        d[p + "dwconv.weight"] = (C, 1, 7)
        d[p + "dwconv.bias"] = (C,)
        d[p + "norm.weight"] = (C,)
        d[p + "norm.bias"] = (C,)
        d[p + "pwconv1.weight"] = (I, C)
        d[p + "pwconv1.bias"] = (I,)
        d[p + "pwconv2.weight"] = (C, I)
        d[p + "pwconv2.bias"] = (C,)
        d[p + "gamma"] = (C,)
    d["backbone.final_layer_norm.weight"] = (C,)
    d["backbone.final_layer_norm.bias"] = (C,)
    d["head.out.weight"] = (cfg.n_fft + 2, C)
    d["head.out.bias"] = (cfg.n_fft + 2,)
    d["head.istft.window"] = (cfg.n_fft,)
    return d


def hann_window(n: int) -> np.ndarray:
    """torch.hann_window(n) (periodic), float32."""
    return torch.hann_window(n, dtype=torch.float32).numpy()


def synthetic_vocos_state_dict(cfg: VocosConfig = VocosConfig(), seed: int = 0
                               ) -> "OrderedDict[str, np.ndarray]":
    """Deterministic vocos weights (numpy PCG64 per tensor name) with realistic
    scales: unit-variance activations after each LayerNorm, layer scale ~1/8 (the
    vocos init 1/num_layers), head log-magnitudes ~N(-1, 1) and phases spanning
    several periods."""
    out: "OrderedDict[str, np.ndarray]" = OrderedDict()
    nb = cfg.n_fft // 2 + 1
    for k, shape in vocos_state_shapes(cfg).items():
        rng = np.random.Generator(np.random.PCG64([seed, zlib.crc32(("vocos." + k).encode())]))
        n = int(np.prod(shape))

        def uni(lo, hi):
            return (lo + (hi - lo) * rng.random(n, dtype=np.float32)).astype(np.float32)

        if k == "head.istft.window":
            v = hann_window(cfg.n_fft)
        elif k.endswith("gamma"):
            v = uni(0.05, 0.2)
        elif k.endswith("norm.weight") or k.endswith("final_layer_norm.weight"):
            v = uni(0.8, 1.2)
        elif k == "head.out.weight":
            a = float(np.sqrt(3.0 / shape[1]))
            v = uni(-a, a).reshape(shape)
            v[nb:] *= 3.0                      # phases: several radians
            v = v.reshape(-1)
        elif k == "head.out.bias":
            v = np.concatenate([uni(-1.5, 0.0)[:nb], uni(-3.0, 3.0)[nb:]])
        elif k.endswith("dwconv.weight"):
            a = float(np.sqrt(3.0 / 7))
            v = uni(-a, a)
        elif k == "backbone.embed.weight":
            a = float(np.sqrt(3.0 / (shape[1] * shape[2])))
            v = uni(-a, a)
        elif k.endswith(".weight"):
            a = float(np.sqrt(3.0 / shape[1]))
            v = uni(-a, a)
        elif k.endswith(".bias"):
            v = uni(-0.1, 0.1)
        else:
            raise KeyError(k)
        out[k] = np.asarray(v, np.float32).reshape(shape)
    return out


class ZvVocoderConfig(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("precision", "n_mels", "dim", "intermediate_dim",
                                            "num_layers", "n_fft", "hop", "embed_kernel",
                                            "dw_kernel")]


def load_library():
    return _eng.load_library()


def _check_state(cfg: VocosConfig, sd: Dict[str, np.ndarray]) -> Dict[str, np.ndarray]:
    want = vocos_state_shapes(cfg)
    sd = {k: v for k, v in sd.items() if not k.startswith("feature_extractor.")}
    missing = [k for k in want if k not in sd]
    unexpected = [k for k in sd if k not in want]
    if missing or unexpected:
        raise KeyError(f"vocos state dict mismatch: missing={missing[:5]}, "
                       f"unexpected={unexpected[:5]}")
    for k, s in want.items():
        if tuple(np.shape(sd[k])) != tuple(s):
            raise ValueError(f"shape mismatch for {k}: {np.shape(sd[k])} vs {s}")
    return sd


class Vocos:
    """Mirror of ``vocos.Vocos`` (inference): from_hparams / load_state_dict / to /
    decode.  ``precision="fp32"`` (default) runs every GEMM as split bf16x3
    products (wav within 1e-4 RMS of an fp32 reference); ``"bf16"`` plain bf16
    MFMA operands."""

    def __init__(self, cfg: VocosConfig = VocosConfig(), precision: str = "fp32"):
        if cfg.padding != "same":
            raise NotImplementedError("only ISTFT padding='same' (vocos-mel-24khz) is supported")
        if precision not in _eng.PRECISION_ID:
            raise ValueError(f"precision must be one of {list(_eng.PRECISION_ID)}")
        self.cfg = cfg
        self.precision = precision
        self._state: Optional[Dict[str, np.ndarray]] = None
        self.h = None
        self.device = torch.device("cpu")
        self.lib = None

    @classmethod
    def from_hparams(cls, config_path: str, precision: str = "fp32") -> "Vocos":
        return cls(VocosConfig.from_yaml(config_path), precision=precision)

    @classmethod
    def from_pretrained(cls, repo_id: str, precision: str = "fp32") -> "Vocos":
        """Local directory holding config.yaml + pytorch_model.bin (or
        model.safetensors).  Hub downloads are not available offline."""
        if not os.path.isdir(repo_id):
            raise RuntimeError(
                f"cannot fetch {repo_id!r}: no network; pass a local directory with "
                "config.yaml and pytorch_model.bin (get_vocoder(vocos_local_path=...))")
        voc = cls.from_hparams(os.path.join(repo_id, "config.yaml"), precision=precision)
        st = os.path.join(repo_id, "model.safetensors")
        if os.path.exists(st):
            from safetensors.numpy import load_file
            sd = load_file(st)
        else:
            blob = torch.load(os.path.join(repo_id, "pytorch_model.bin"), map_location="cpu",
                              weights_only=True)
            sd = {k: v.float().numpy() for k, v in blob.items()}
        voc.load_state_dict(sd)
        return voc

    def load_state_dict(self, state_dict, strict: bool = True):
        sd = {k: (v.detach().cpu().float().numpy() if isinstance(v, torch.Tensor)
                  else np.asarray(v, np.float32)) for k, v in state_dict.items()}
        self._state = _check_state(self.cfg, sd)
        if self.h is not None:
            self._upload()
        return self

    def load_synthetic(self, seed: int = 0):
        return self.load_state_dict(synthetic_vocos_state_dict(self.cfg, seed))

    def _upload(self):
        if not torch.cuda.is_available():
            raise RuntimeError("zipvoice_amd vocoder needs a ROCm GPU (MI355X); no CPU fallback")
        self.lib = load_library()
        if self.h:
            self.lib.zv_vocoder_destroy(self.h)
            self.h = None
        c = ZvVocoderConfig(precision=_eng.PRECISION_ID[self.precision], n_mels=self.cfg.n_mels,
                            dim=self.cfg.dim, intermediate_dim=self.cfg.intermediate_dim,
                            num_layers=self.cfg.num_layers, n_fft=self.cfg.n_fft,
                            hop=self.cfg.hop_length, embed_kernel=7, dw_kernel=7)
        with torch.cuda.device(self.device):
            h = self.lib.zv_vocoder_create(ctypes.byref(c))
            if not h:
                raise RuntimeError(self.lib.zv_last_error().decode())
            self.h = h
            for k, v in self._state.items():
                a = np.ascontiguousarray(v, np.float32)
                _eng._check(self.lib.zv_vocoder_set_weight(h, k.encode(),
                                                           a.ctypes.data_as(ctypes.c_void_p), a.size))
            _eng._check(self.lib.zv_vocoder_finalize(h))

    def to(self, device):
        device = torch.device(device)
        if device.type != "cuda":
            raise RuntimeError("zipvoice_amd vocoder runs on the GPU only (no CPU fallback)")
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
            self.lib.zv_vocoder_destroy(h)
            self.h = None

    def _run(self, x: torch.Tensor, layout: int, feat_scale: float, feat_bias: float,
             lens: Optional[torch.Tensor], clamp: bool) -> torch.Tensor:
        if self.h is None:
            raise RuntimeError("vocoder not on a device: call .to('cuda')")
        x = x.to(self.device, torch.float32).contiguous()
        B = x.shape[0]
        T = x.shape[2] if layout == 0 else x.shape[1]
        C = x.shape[1] if layout == 0 else x.shape[2]
        if C != self.cfg.n_mels:
            raise ValueError(f"expected {self.cfg.n_mels} mel channels, got {C}")
        ln = None
        if lens is not None:
            ln = lens.to(self.device, torch.int32).contiguous()
            if ln.shape != (B,):
                raise ValueError("lens must have shape (B,)")
        wav = torch.empty((B, T * self.cfg.hop_length), dtype=torch.float32, device=self.device)
        _eng._check(self.lib.zv_vocoder_decode(
            self.h, _eng._ptr(x), layout, float(feat_scale), float(feat_bias), _eng._ptr(ln),
            B, T, _eng._ptr(wav), int(clamp), _eng._stream()))
        return wav

    @torch.inference_mode()
    def decode(self, features_input: torch.Tensor) -> torch.Tensor:
        """Vocos.decode: mel (B, n_mels, T) -> audio (B, T * hop)."""
        if features_input.dim() != 3:
            raise ValueError("features_input must be (B, n_mels, T)")
        return self._run(features_input, 0, 1.0, 0.0, None, False)

    def decode_features(self, pred_features: torch.Tensor, lens: Optional[torch.Tensor] = None,
                        feat_scale: float = 0.1, feat_bias: float = 0.0,
                        clamp: bool = True) -> torch.Tensor:
        """The reference's post-sampling step fused on device
        (infer_zipvoice.py:374-378): pred (B, T, n_mels) -> wav (B, T*hop) with
        ``permute / feat_scale - feat_bias``, per-utterance lengths (``lens``,
        as separate per-sentence calls would decode), and ``clamp(-1, 1)``."""
        return self._run(pred_features, 1, feat_scale, feat_bias, lens, clamp)

    def device_bytes(self) -> int:
        return int(self.lib.zv_vocoder_device_bytes(self.h)) if self.h else 0


def get_vocoder(vocos_local_path: Optional[str] = None, type: str = "vocos",
                precision: str = "fp32"):
    """Mirror of infer_zipvoice.py:249-273 ("vocos" / "bigvgan_v2"; a local directory
    stands in for the Hub id)."""
    if type == "vocos":
        if vocos_local_path:
            voc = Vocos.from_hparams(f"{vocos_local_path}/config.yaml", precision=precision)
            blob = torch.load(f"{vocos_local_path}/pytorch_model.bin", weights_only=True,
                              map_location="cpu")
            voc.load_state_dict(blob)
            return voc
        return Vocos.from_pretrained("charactr/vocos-mel-24khz", precision=precision)
    if type == "bigvgan_v2":                       # infer_zipvoice.py:261-269
        from .bigvgan import BigVGAN
        return BigVGAN.from_pretrained(vocos_local_path or "nvidia/bigvgan_v2_24khz_100band_256x",
                                       use_cuda_kernel=False, precision=precision)
    raise NotImplementedError(f"Unsupported vocoder type: {type}")

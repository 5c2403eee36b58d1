"""ctypes binding of libzipvoice_hip.so (the C ABI declared in include/zipvoice_hip.h).

PyTorch-ROCm is used only for device memory, streams and distributed plumbing:
every tensor handed to the engine is a contiguous device buffer whose pointer
crosses the C ABI; all arithmetic of the hot path runs in the engine's HIP
kernels.  There is no CPU fallback: if the library or a GPU is missing, the
constructor raises.
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, Optional

import numpy as np
import torch  # noqa: F401  (imported first so the engine shares torch's HIP runtime)

from .config import ModelConfig
from .weights import check_state_dict

LIB_NAME = "libzipvoice_hip.so"
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)
# the same engine built with IEEE fp16 MFMA operands (csrc/build.py VARIANTS)
LIB_F16_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libzipvoice_hip_f16.so")
MAX_STACKS = 8
VARIANT_ID = {"zipvoice": 0, "zipvoice_distill": 1, "zipvoice_dialog": 2,
              "zipvoice_dialog_stereo": 3}
PRECISION_ID = {"fp32": 0, "bf16": 1}      # vocoder / BigVGAN precisions (main library)
# decoder precision modes: name -> (library, zv_precision).  "fp16" is the parity-grade fast
# mode: fp16 MFMA operands in the decoder layers, split products for the decoder's input /
# output projections, the attention-score projections and the text encoder (ZV_MIXED in the
# fp16 library)
# "fp8": the BASELINE C5 mode - the decoder layers' feed-forward, convolution-module and
# NonlinAttention output linears on block-scaled MX-fp8 MFMA (ZV_FP8, main library)
MODES = {"fp32": ("bf16", 0), "bf16": ("bf16", 1), "fp16": ("f16", 2),
         "fp16_plain": ("f16", 1), "bf16_mixed": ("bf16", 2), "fp8": ("bf16", 3)}


class ZvConfig(ctypes.Structure):
    _fields_ = [
        ("variant", ctypes.c_int), ("precision", ctypes.c_int), ("feat_dim", ctypes.c_int),
        ("num_stacks", ctypes.c_int),
        ("downsampling_factor", ctypes.c_int * MAX_STACKS),
        ("num_layers", ctypes.c_int * MAX_STACKS),
        ("cnn_module_kernel", ctypes.c_int * MAX_STACKS),
        ("fm_decoder_dim", ctypes.c_int), ("fm_decoder_feedforward_dim", ctypes.c_int),
        ("fm_decoder_num_heads", ctypes.c_int),
        ("text_encoder_num_layers", ctypes.c_int), ("text_encoder_feedforward_dim", ctypes.c_int),
        ("text_encoder_cnn_module_kernel", ctypes.c_int),
        ("text_encoder_num_heads", ctypes.c_int), ("text_encoder_dim", ctypes.c_int),
        ("time_embed_dim", ctypes.c_int), ("text_embed_dim", ctypes.c_int),
        ("query_head_dim", ctypes.c_int), ("value_head_dim", ctypes.c_int),
        ("pos_head_dim", ctypes.c_int), ("pos_dim", ctypes.c_int),
        ("vocab_size", ctypes.c_int), ("pad_id", ctypes.c_int), ("spk_a_id", ctypes.c_int),
        ("spk_b_id", ctypes.c_int),
    ]


# symbol name -> (restype, argtypes); must match include/zipvoice_hip.h
_P = ctypes.c_void_p
_I = ctypes.c_int
_F = ctypes.c_float
SIGNATURES = {
    "zv_last_error": (ctypes.c_char_p, []),
    "zv_version": (ctypes.c_char_p, []),
    "zv_create": (_P, [ctypes.POINTER(ZvConfig)]),
    "zv_destroy": (None, [_P]),
    "zv_set_weight": (_I, [_P, ctypes.c_char_p, _P, ctypes.c_int64]),
    "zv_finalize": (_I, [_P]),
    "zv_reserve": (_I, [_P, _I, _I]),
    "zv_device_bytes": (ctypes.c_int64, [_P]),
    "zv_profile": (_I, [_I]),
    "zv_bench_gemm": (_I, [_I, _I, _I, _I, _I, _I, ctypes.POINTER(ctypes.c_float)]),
    "zv_gemm_selftest": (_I, [_I, _I, _I, _I, _I, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]),
    "zv_profile_report": (_I, [ctypes.c_char_p, _I]),
    "zv_host_block_count": (ctypes.c_int64, []),
    "zv_attn_fallbacks": (_I, [_P, _I, _P]),
    "zv_attn2_check": (_I, [_I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _I, _P, _P]),
    "zv_attn_plan": (_I, [_I, _I, _I, _I, _I, _P, _P, _P, _P]),
    "zv_mx8_quantize": (_I, [_P, _I, _I, _P, _P]),
    "zv_mx8_gemm_check": (_I, [_I, _I, _I, _P, _P, _P, _P, _P]),
    "zv_fm_decoder": (_I, [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _P, _P]),
    "zv_velocity": (_I, [_P, _F, _F, _P, _P, _P, _P, _I, _I, _P, _P]),
    "zv_euler_sample": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _F, _F, _F, _F, _P]),
    "zv_velocity_rows": (_I, [_P, _F, _P, _P, _P, _P, _P, _I, _I, _P, _P]),
    "zv_euler_sample_rows": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _P, _F, _F, _F, _P]),
    "zv_text_encode": (_I, [_P, _P, _P, _P, _I, _I, _P, _P]),
    "zv_text_condition": (_I, [_P, _P, _I, _I, _P, _P, _I, _P, _P]),
    "zv_speech_condition": (_I, [_P, _P, _I, _I, _I, _P, _I, _P, _P]),
    # vocoder (zipvoice_amd/vocoder.py)
    "zv_vocoder_create": (_P, [_P]),
    "zv_vocoder_destroy": (None, [_P]),
    "zv_vocoder_set_weight": (_I, [_P, ctypes.c_char_p, _P, ctypes.c_int64]),
    "zv_vocoder_finalize": (_I, [_P]),
    "zv_vocoder_decode": (_I, [_P, _P, _I, _F, _F, _P, _I, _I, _P, _I, _P]),
    "zv_vocoder_device_bytes": (ctypes.c_int64, [_P]),
    "zv_bigvgan_create": (_P, [_P]),
    "zv_bigvgan_destroy": (None, [_P]),
    "zv_bigvgan_set_weight": (_I, [_P, ctypes.c_char_p, _P, ctypes.c_int64]),
    "zv_bigvgan_finalize": (_I, [_P]),
    "zv_bigvgan_decode": (_I, [_P, _P, _I, _F, _F, _P, _I, _I, _P, _P]),
    "zv_bigvgan_device_bytes": (ctypes.c_int64, [_P]),
    # prompt feature extractor (zipvoice_amd/feature.py)
    "zv_fbank_create": (_P, [_I, _I, _I, _P, _P]),
    "zv_fbank_destroy": (None, [_P]),
    "zv_fbank_extract": (_I, [_P, _P, ctypes.c_int64, _P, _I, _I, _P, ctypes.c_int64, _P]),
    "zv_fbank_configure": (_I, [_P, _I, _F, _F]),
}

_libs: Dict[str, ctypes.CDLL] = {}
_lib = None            # the main (bf16-operand) library


def load_library(path: Optional[str] = None, operand: str = "bf16"):
    """dlopen the engine (fails loudly when it has not been built).  operand "f16" loads the
    fp16-operand build.  ZV_LIB_PATH selects an alternative build of the main library (A/B
    measurements), ZV_LIB_F16_PATH one of the fp16-operand library.  Both are loaded RTLD_LOCAL (and linked -Bsymbolic): the two libraries
    export the same entry points and each binds its own."""
    global _lib
    if path is None:
        path = ((os.environ.get("ZV_LIB_F16_PATH") or LIB_F16_PATH) if operand == "f16"
                else (os.environ.get("ZV_LIB_PATH") or LIB_PATH))
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        raise RuntimeError(
            f"{os.path.basename(path)} not found at {path}: build it with "
            "`python zipvoice_amd/csrc/build.py` (or __graft_entry__.build()). "
            "There is no CPU fallback for the ZipVoice hot path.")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    for name, (res, args) in SIGNATURES.items():
        if path not in (LIB_PATH, LIB_F16_PATH) and not hasattr(lib, name):
            continue        # an older A/B build without this entry point
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _libs[path] = lib
    if operand != "f16" and _lib is None:
        _lib = lib
    return lib


def _check(rc: int, lib=None):
    if rc != 0:
        msg = (lib or _lib).zv_last_error().decode()
        if "missing weight" in msg or "expected" in msg or "unexpected" in msg:
            raise KeyError(msg)
        raise RuntimeError(f"zipvoice_hip: {msg}")


def make_zv_config(cfg: ModelConfig, precision: str) -> ZvConfig:
    c = ZvConfig()
    c.variant = VARIANT_ID[cfg.variant]
    c.precision = MODES[precision][1]
    c.feat_dim = cfg.feat_dim
    n = len(cfg.fm_decoder_downsampling_factor)
    if n > MAX_STACKS:
        raise ValueError(f"at most {MAX_STACKS} decoder stacks supported")
    c.num_stacks = n
    for i in range(n):
        c.downsampling_factor[i] = cfg.fm_decoder_downsampling_factor[i]
        c.num_layers[i] = cfg.fm_decoder_num_layers[i]
        c.cnn_module_kernel[i] = cfg.fm_decoder_cnn_module_kernel[i]
    for f in ("fm_decoder_dim", "fm_decoder_feedforward_dim", "fm_decoder_num_heads",
              "text_encoder_num_layers", "text_encoder_feedforward_dim",
              "text_encoder_cnn_module_kernel", "text_encoder_num_heads", "text_encoder_dim",
              "time_embed_dim", "text_embed_dim", "query_head_dim", "value_head_dim",
              "pos_head_dim", "pos_dim", "vocab_size", "pad_id", "spk_a_id", "spk_b_id"):
        setattr(c, f, int(getattr(cfg, f)))
    return c


def profile(enable: bool, detail: bool = False):
    """Enable/disable (and clear) the engine's per-launch event profiler (in every loaded
    engine library); ``detail`` keys the GEMM records by shape."""
    load_library()
    for lib in list(_libs.values()):
        _check(lib.zv_profile((2 if detail else 1) if enable else 0), lib)


def host_block_count() -> int:
    """Host-blocking HIP runtime calls issued so far, summed over the loaded engine libraries
    (zv_host_block_count: allocations, synchronous copies, synchronisations, ...)."""
    load_library()
    return sum(int(lib.zv_host_block_count()) for lib in list(_libs.values()))


def profile_report() -> dict:
    """{tag: {launches, flops, bytes, ms}} merged over the loaded engine libraries."""
    import json
    load_library()
    rep: dict = {}
    for lib in list(_libs.values()):
        buf = ctypes.create_string_buffer(1 << 20)
        _check(lib.zv_profile_report(buf, len(buf)), lib)
        for k, v in json.loads(buf.value.decode()).items():
            if k in rep:
                for f in ("launches", "flops", "bytes", "ms"):
                    rep[k][f] += v[f]
            else:
                rep[k] = v
    return rep


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


class HipEngine:
    """One engine per GPU per process: device weights + workspace."""

    def __init__(self, cfg: ModelConfig, state_dict: Dict[str, np.ndarray],
                 precision: str = "fp32", device: Optional[torch.device] = None):
        if precision not in MODES:
            raise ValueError(f"precision must be one of {list(MODES)}")
        if not torch.cuda.is_available():
            raise RuntimeError("zipvoice_amd needs a ROCm GPU (MI355X); no CPU fallback exists")
        operand, self.mode_id = MODES[precision]
        load_library()                       # the main library (error strings, profiler)
        self.lib = load_library(operand=operand)
        self.cfg = cfg
        self.precision = precision
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        check_state_dict(cfg, state_dict)
        with torch.cuda.device(self.device):
            zc = make_zv_config(cfg, precision)
            self.h = self.lib.zv_create(ctypes.byref(zc))
            if not self.h:
                raise RuntimeError(self.lib.zv_last_error().decode())
            for k, v in state_dict.items():
                a = np.ascontiguousarray(np.asarray(v, dtype=np.float32))
                self._check(self.lib.zv_set_weight(self.h, k.encode(), a.ctypes.data_as(ctypes.c_void_p),
                                              a.size))
            self._check(self.lib.zv_finalize(self.h))

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            try:
                torch.cuda.synchronize(self.device)
            except Exception:
                pass
            self.lib.zv_destroy(h)
            self.h = None

    def _check(self, rc: int):
        _check(rc, self.lib)

    # ------------------------------------------------------------------ checks
    def _f32(self, t: torch.Tensor, name: str, shape=None) -> torch.Tensor:
        if not isinstance(t, torch.Tensor):
            raise TypeError(f"{name} must be a torch.Tensor")
        if t.device != self.device:
            t = t.to(self.device)
        t = t.to(torch.float32).contiguous()
        if shape is not None and tuple(t.shape) != tuple(shape):
            raise ValueError(f"{name}: expected shape {tuple(shape)}, got {tuple(t.shape)}")
        return t

    def _mask(self, m: Optional[torch.Tensor], shape) -> Optional[torch.Tensor]:
        if m is None:
            return None
        m = m.to(self.device)
        if tuple(m.shape) != tuple(shape):
            raise ValueError(f"padding_mask: expected shape {tuple(shape)}, got {tuple(m.shape)}")
        return m.to(torch.uint8).contiguous()

    def device_bytes(self) -> int:
        return int(self.lib.zv_device_bytes(self.h))

    def attn_fallbacks(self, reset: bool = False) -> tuple:
        """(low, high, total) exact-path runs of the second-generation attention consumers since
        the last reset (zv_attn_fallbacks; synchronises the device)."""
        c = (ctypes.c_int64 * 3)()
        with torch.cuda.device(self.device):
            self._check(self.lib.zv_attn_fallbacks(self.h, int(reset), ctypes.cast(c, ctypes.c_void_p)))
        return int(c[0]), int(c[1]), int(c[2])

    # ------------------------------------------------------------------ ops
    def fm_decoder(self, t: torch.Tensor, xt, text_c, speech_c, padding_mask=None,
                   guidance: Optional[torch.Tensor] = None) -> torch.Tensor:
        N, T, Fx = xt.shape
        xt = self._f32(xt, "xt")
        text_c = self._f32(text_c, "text_condition", (N, T, self.cfg.feat_dim))
        speech_c = self._f32(speech_c, "speech_condition", (N, T, Fx))
        t = self._f32(t.reshape(-1).expand(N) if t.numel() == 1 else t.reshape(N), "t")
        g = None
        if guidance is not None:
            g = self._f32(guidance.reshape(-1).expand(N) if guidance.numel() == 1
                          else guidance.reshape(N), "guidance_scale")
        pm = self._mask(padding_mask, (N, T))
        if self.cfg.stereo:
            out_w = self.cfg.decoder_out_dims()[0 if 2 * Fx + self.cfg.feat_dim ==
                                                self.cfg.decoder_in_dims()[0] else 1]
        else:
            out_w = self.cfg.feat_dim
        v = torch.empty((N, T, out_w), dtype=torch.float32, device=self.device)
        self._check(self.lib.zv_fm_decoder(self.h, _ptr(t), _ptr(g), _ptr(xt), _ptr(text_c),
                                      _ptr(speech_c), _ptr(pm), N, T, Fx, _ptr(v), _stream()))
        return v

    def _guidance_rows(self, guidance_scale, B: int) -> Optional[torch.Tensor]:
        """None for a scalar guidance scale; else the (B,) fp32 device vector of a
        per-utterance guidance tensor ((batch, 1, 1) in the reference, solver.py:61-62)."""
        if not torch.is_tensor(guidance_scale) or guidance_scale.numel() == 1:
            return None
        if guidance_scale.numel() != B:
            raise ValueError(f"guidance_scale: expected 1 or {B} values (shape (batch, 1, 1)), "
                             f"got shape {tuple(guidance_scale.shape)}")
        return guidance_scale.reshape(B).to(self.device, torch.float32).contiguous()

    def velocity(self, t: float, guidance_scale, x, text_c, speech_c,
                 padding_mask=None) -> torch.Tensor:
        B, T, Fx = x.shape
        x = self._f32(x, "x")
        text_c = self._f32(text_c, "text_condition", (B, T, self.cfg.feat_dim))
        speech_c = self._f32(speech_c, "speech_condition", (B, T, Fx))
        pm = self._mask(padding_mask, (B, T))
        v = torch.empty_like(x)
        gr = self._guidance_rows(guidance_scale, B)
        if gr is not None:
            self._check(self.lib.zv_velocity_rows(self.h, float(t), _ptr(gr), _ptr(x), _ptr(text_c),
                                             _ptr(speech_c), _ptr(pm), B, T, _ptr(v), _stream()))
        else:
            self._check(self.lib.zv_velocity(self.h, float(t), float(guidance_scale), _ptr(x),
                                        _ptr(text_c), _ptr(speech_c), _ptr(pm), B, T, _ptr(v),
                                        _stream()))
        return v

    def euler_sample(self, x0, text_c, speech_c, padding_mask, num_step: int,
                     guidance_scale, t_start=0.0, t_end=1.0, t_shift=1.0) -> torch.Tensor:
        B, T, Fx = x0.shape
        x = self._f32(x0, "x").clone()
        text_c = self._f32(text_c, "text_condition", (B, T, self.cfg.feat_dim))
        speech_c = self._f32(speech_c, "speech_condition", (B, T, Fx))
        pm = self._mask(padding_mask, (B, T))
        gr = self._guidance_rows(guidance_scale, B)
        if gr is not None:
            self._check(self.lib.zv_euler_sample_rows(self.h, _ptr(x), _ptr(text_c), _ptr(speech_c),
                                                 _ptr(pm), B, T, int(num_step), _ptr(gr),
                                                 float(t_start), float(t_end), float(t_shift),
                                                 _stream()))
        else:
            self._check(self.lib.zv_euler_sample(self.h, _ptr(x), _ptr(text_c), _ptr(speech_c),
                                            _ptr(pm), B, T, int(num_step), float(guidance_scale),
                                            float(t_start), float(t_end), float(t_shift),
                                            _stream()))
        return x

    def reserve(self, max_batch: int, max_frames: int) -> None:
        """Pre-size the decoder workspace (zv_reserve)."""
        self._check(self.lib.zv_reserve(self.h, int(max_batch), int(max_frames)))

    def text_encode(self, tokens: torch.Tensor, padding_mask: torch.Tensor,
                    spk: Optional[torch.Tensor] = None) -> torch.Tensor:
        B, S = tokens.shape
        tokens = tokens.to(self.device, torch.int64).contiguous()
        pm = self._mask(padding_mask, (B, S))
        if spk is not None:
            spk = spk.to(self.device, torch.int8).contiguous()
        out = torch.empty((B, S, self.cfg.feat_dim), dtype=torch.float32, device=self.device)
        self._check(self.lib.zv_text_encode(self.h, _ptr(tokens), _ptr(pm), _ptr(spk), B, S, _ptr(out),
                                       _stream()))
        return out

    def text_condition(self, embed, tokens_lens, features_lens, num_frames: int):
        B, S, C = embed.shape
        embed = self._f32(embed, "embed")
        tl = tokens_lens.to(self.device, torch.int32).contiguous()
        fl = features_lens.to(self.device, torch.int32).contiguous()
        out = torch.empty((B, num_frames, C), dtype=torch.float32, device=self.device)
        self._check(self.lib.zv_text_condition(self.h, _ptr(embed), B, S, _ptr(tl), _ptr(fl),
                                          int(num_frames), _ptr(out), _stream()))
        return out

    def speech_condition(self, prompt_features, prompt_lens, num_frames: int):
        B, Tp, F = prompt_features.shape
        pf = self._f32(prompt_features, "prompt_features")
        pl = prompt_lens.to(self.device, torch.int32).contiguous()
        out = torch.empty((B, num_frames, F), dtype=torch.float32, device=self.device)
        self._check(self.lib.zv_speech_condition(self.h, _ptr(pf), B, Tp, F, _ptr(pl), int(num_frames),
                                            _ptr(out), _stream()))
        return out

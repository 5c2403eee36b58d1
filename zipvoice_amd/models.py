"""Drop-in mirrors of the reference's inference model classes.

Same class names, constructor keywords, method names, argument meanings and
return tuples as ``zipvoice/models/zipvoice.py`` (ZipVoice),
``zipvoice_distill.py`` (ZipVoiceDistill) and ``zipvoice_dialog.py``
(ZipVoiceDialog, ZipVoiceDialogStereo), restricted to inference.  The compute
of every method runs in the HIP engine (``engine.HipEngine``); this module only
does host-side integer glue (token lists -> padded ids / lengths / masks),
exactly where the reference does it on the host.

Usage (mirrors ``infer_zipvoice.py:549-577``)::

    model = ZipVoice(**model_json["model"], vocab_size=V, pad_id=0)
    model.load_state_dict(state_dict)        # reference key names, strict
    model = model.to("cuda:0").eval()
    pred, pred_lens, prompt, prompt_lens = model.sample(tokens=..., ...)
"""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np
import torch

from .common import make_pad_mask, pad_labels, predict_features_lens, speaker_turn_indices
from .config import ModelConfig
from .engine import HipEngine
from .solver import DistillEulerSolver, EulerSolver
from .weights import check_state_dict, load_checkpoint_state_dict, synthetic_state_dict


class ZipVoice:
    """The ZipVoice model (inference), zipvoice.py:35-486."""

    variant = "zipvoice"
    solver_cls = EulerSolver

    def __init__(self, fm_decoder_downsampling_factor: List[int] = [1, 2, 4, 2, 1],
                 fm_decoder_num_layers: List[int] = [2, 2, 4, 4, 4],
                 fm_decoder_cnn_module_kernel: List[int] = [31, 15, 7, 15, 31],
                 fm_decoder_feedforward_dim: int = 1536, fm_decoder_num_heads: int = 4,
                 fm_decoder_dim: int = 512, text_encoder_num_layers: int = 4,
                 text_encoder_feedforward_dim: int = 512, text_encoder_cnn_module_kernel: int = 9,
                 text_encoder_num_heads: int = 4, text_encoder_dim: int = 192,
                 time_embed_dim: int = 192, text_embed_dim: int = 192, query_head_dim: int = 32,
                 value_head_dim: int = 12, pos_head_dim: int = 4, pos_dim: int = 48,
                 feat_dim: int = 100, vocab_size: int = 26, pad_id: int = 0,
                 precision: str = "fp32", **extra):
        self.cfg = ModelConfig(
            fm_decoder_downsampling_factor=list(fm_decoder_downsampling_factor),
            fm_decoder_num_layers=list(fm_decoder_num_layers),
            fm_decoder_cnn_module_kernel=list(fm_decoder_cnn_module_kernel),
            fm_decoder_feedforward_dim=fm_decoder_feedforward_dim,
            fm_decoder_num_heads=fm_decoder_num_heads, fm_decoder_dim=fm_decoder_dim,
            text_encoder_num_layers=text_encoder_num_layers,
            text_encoder_feedforward_dim=text_encoder_feedforward_dim,
            text_encoder_cnn_module_kernel=text_encoder_cnn_module_kernel,
            text_encoder_num_heads=text_encoder_num_heads, text_encoder_dim=text_encoder_dim,
            time_embed_dim=time_embed_dim, text_embed_dim=text_embed_dim,
            query_head_dim=query_head_dim, value_head_dim=value_head_dim,
            pos_head_dim=pos_head_dim, pos_dim=pos_dim, feat_dim=feat_dim,
            vocab_size=vocab_size, pad_id=pad_id, variant=self.variant,
            **{k: v for k, v in extra.items() if k in ("spk_a_id", "spk_b_id")})
        unknown = set(extra) - {"spk_a_id", "spk_b_id"}
        if unknown:
            raise TypeError(f"unexpected keyword arguments {sorted(unknown)}")
        self.feat_dim = feat_dim
        self.text_embed_dim = text_embed_dim
        self.pad_id = pad_id
        self.precision = precision
        self._state: Optional[Dict[str, np.ndarray]] = None
        self.engine: Optional[HipEngine] = None
        self.device = torch.device("cpu")
        self.solver = self.solver_cls(self, func_name="forward_fm_decoder")

    # ------------------------------------------------------------------ weights
    def load_state_dict(self, state_dict, strict: bool = True):
        sd = {}
        for k, v in state_dict.items():
            if k.startswith("module."):
                k = k[len("module."):]
            if isinstance(v, torch.Tensor):
                v = v.detach().to("cpu", torch.float32).numpy()
            sd[k] = np.asarray(v, np.float32)
        if not strict:
            raise NotImplementedError("only strict=True loading is supported")
        check_state_dict(self.cfg, sd)
        self._state = sd
        if self.engine is not None:
            self._build_engine(self.engine.device)
        return self

    def load_checkpoint(self, path: str):
        """checkpoint.py:108-146 / infer_zipvoice.py:561-566 (.pt or .safetensors)."""
        return self.load_state_dict(load_checkpoint_state_dict(path))

    def load_synthetic(self, seed: int = 0):
        """Deterministic synthetic weights (no pretrained weights offline)."""
        return self.load_state_dict(synthetic_state_dict(self.cfg, seed))

    def _build_engine(self, device):
        if self._state is None:
            raise RuntimeError("load_state_dict() must be called before moving to a GPU")
        self.engine = HipEngine(self.cfg, self._state, precision=self.precision, device=device)
        self.device = self.engine.device

    def to(self, device):
        device = torch.device(device)
        if device.type != "cuda":
            raise RuntimeError("zipvoice_amd runs on ROCm GPUs only (no CPU fallback)")
        self._build_engine(device)
        self._state = self._state  # keep host copy for re-targeting
        return self

    def cuda(self, index: int = 0):
        return self.to(torch.device("cuda", index))

    def eval(self):
        return self

    def parameters_count(self) -> int:
        return int(sum(v.size for v in self._state.values())) if self._state else 0

    def _need_engine(self):
        if self.engine is None:
            raise RuntimeError("model is not on a GPU: call .to('cuda')")
        return self.engine

    # ------------------------------------------------------------------ decoder
    def forward_fm_decoder(self, t: torch.Tensor, xt: torch.Tensor, text_condition: torch.Tensor,
                           speech_condition: torch.Tensor,
                           padding_mask: Optional[torch.Tensor] = None,
                           guidance_scale: Optional[torch.Tensor] = None) -> torch.Tensor:
        """zipvoice.py:135-185: velocity of the raw decoder (no CFG)."""
        eng = self._need_engine()
        if not torch.is_tensor(t):
            t = torch.tensor(float(t))
        assert t.dim() in (0, 1, 3)
        if guidance_scale is not None and not torch.is_tensor(guidance_scale):
            guidance_scale = torch.tensor(float(guidance_scale))
        if self.cfg.distill and guidance_scale is None:
            raise ValueError("ZipVoiceDistill.forward_fm_decoder needs guidance_scale")
        return eng.fm_decoder(t.reshape(-1), xt, text_condition, speech_condition, padding_mask,
                              guidance_scale.reshape(-1) if (guidance_scale is not None
                                                            and self.cfg.distill) else None)

    # ------------------------------------------------------------------ text side
    def forward_text_embed(self, tokens: List[List[int]]):
        """zipvoice.py:187-212 (dialog: + speaker-turn embeddings, zipvoice_dialog.py:127-159)."""
        eng = self._need_engine()
        tokens_padded = pad_labels(tokens, pad_id=self.pad_id, device=self.device)
        tokens_lens = torch.tensor([len(t) for t in tokens], dtype=torch.int64,
                                   device=self.device)
        pm = make_pad_mask(tokens_lens, tokens_padded.shape[1])
        spk = None
        if self.cfg.dialog:
            spk = speaker_turn_indices(tokens_padded, self.cfg.spk_a_id, self.cfg.spk_b_id,
                                       self.pad_id)
        embed = eng.text_encode(tokens_padded, pm, spk)
        return embed, tokens_lens

    def forward_text_condition(self, embed: torch.Tensor, tokens_lens: torch.Tensor,
                               features_lens: torch.Tensor):
        """zipvoice.py:214-251."""
        eng = self._need_engine()
        num_frames = int(features_lens.max())
        padding_mask = make_pad_mask(features_lens.to(self.device), max_len=num_frames)
        tc = eng.text_condition(embed, tokens_lens, features_lens, num_frames)
        return tc, padding_mask

    def forward_text_inference_gt_duration(self, tokens, features_lens, prompt_tokens,
                                           prompt_features_lens):
        """zipvoice.py:270-288."""
        tokens = [p + t for p, t in zip(prompt_tokens, tokens)]
        features_lens = prompt_features_lens.to(self.device) + features_lens.to(self.device)
        embed, tokens_lens = self.forward_text_embed(tokens)
        return self.forward_text_condition(embed, tokens_lens, features_lens)

    def forward_text_inference_ratio_duration(self, tokens, prompt_tokens, prompt_features_lens,
                                              speed: float):
        """zipvoice.py:290-330."""
        cat_tokens = [p + t for p, t in zip(prompt_tokens, tokens)]
        ptl = torch.tensor([len(t) for t in prompt_tokens], dtype=torch.int64, device=self.device)
        tl = torch.tensor([len(t) for t in tokens], dtype=torch.int64, device=self.device)
        cat_embed, cat_tokens_lens = self.forward_text_embed(cat_tokens)
        features_lens = predict_features_lens(prompt_features_lens.to(self.device), ptl, tl, speed)
        return self.forward_text_condition(cat_embed, cat_tokens_lens, features_lens)

    # ------------------------------------------------------------------ sampling
    def sample(self, tokens: List[List[int]], prompt_tokens: List[List[int]],
               prompt_features: torch.Tensor, prompt_features_lens: torch.Tensor,
               features_lens: Optional[torch.Tensor] = None, speed: float = 1.0,
               t_shift: float = 1.0, duration: str = "predict", num_step: int = 5,
               guidance_scale: float = 0.5, x0: Optional[torch.Tensor] = None):
        """zipvoice.py:388-486.  ``x0`` (extra, optional) supplies the initial noise
        explicitly; otherwise it is drawn with torch.randn on the device as the
        reference does (:453-458)."""
        eng = self._need_engine()
        assert duration in ["real", "predict"]
        prompt_features_lens = prompt_features_lens.to(self.device)
        if duration == "predict":
            text_condition, padding_mask = self.forward_text_inference_ratio_duration(
                tokens=tokens, prompt_tokens=prompt_tokens,
                prompt_features_lens=prompt_features_lens, speed=speed)
        else:
            assert features_lens is not None
            text_condition, padding_mask = self.forward_text_inference_gt_duration(
                tokens=tokens, features_lens=features_lens, prompt_tokens=prompt_tokens,
                prompt_features_lens=prompt_features_lens)
        batch_size, num_frames, _ = text_condition.shape
        speech_condition = eng.speech_condition(prompt_features, prompt_features_lens, num_frames)
        F = prompt_features.size(-1)
        if x0 is None:
            x0 = torch.randn(batch_size, num_frames, F, device=self.device)
        elif tuple(x0.shape) != (batch_size, num_frames, F):
            raise ValueError(f"x0 must have shape {(batch_size, num_frames, F)}, got "
                             f"{tuple(x0.shape)}")
        # the output shapes are known before sampling: reading them here (the text path has
        # already synchronised for num_frames) keeps the host from waiting on the Euler loop,
        # so the prompt split and the vocoder are queued behind it without an idle gap
        x1_wo_prompt_lens = (~padding_mask).sum(-1) - prompt_features_lens
        Tg, Tp = (int(v) for v in torch.stack([x1_wo_prompt_lens.max(),
                                                prompt_features_lens.max()]).tolist())
        x1 = self.solver.sample(x=x0, text_condition=text_condition,
                                speech_condition=speech_condition, padding_mask=padding_mask,
                                num_step=num_step, guidance_scale=guidance_scale, t_shift=t_shift)
        return split_prompt(x1, prompt_features_lens, x1_wo_prompt_lens, Tg, Tp) + (
            prompt_features_lens,)


def split_prompt(x1: torch.Tensor, prompt_lens: torch.Tensor, gen_lens: torch.Tensor,
                 Tg: Optional[int] = None, Tp: Optional[int] = None):
    """zipvoice.py:469-486 without the per-item python slicing loop: one gather.  Tg / Tp
    (the longest generated / prompt part) are read from the lengths when not given."""
    B, T, F = x1.shape
    dev = x1.device
    Tg = int(gen_lens.max()) if Tg is None else Tg
    Tp = int(prompt_lens.max()) if Tp is None else Tp
    ar_g = torch.arange(Tg, device=dev)[None]
    idx = (prompt_lens[:, None] + ar_g).clamp(max=T - 1)
    gen = torch.gather(x1, 1, idx[..., None].expand(B, Tg, F))
    gen = gen * (ar_g < gen_lens[:, None])[..., None]
    ar_p = torch.arange(Tp, device=dev)[None]
    prm = x1[:, :Tp] * (ar_p < prompt_lens[:, None])[..., None]
    return gen, gen_lens, prm


class ZipVoiceDistill(ZipVoice):
    """zipvoice_distill.py:27-94: guidance-scale embedding, no CFG doubling."""

    variant = "zipvoice_distill"
    solver_cls = DistillEulerSolver


class ZipVoiceDialog(ZipVoice):
    """zipvoice_dialog.py:28-215 (speaker-turn embeddings on the text encoder)."""

    variant = "zipvoice_dialog"

    def __init__(self, *args, spk_a_id: int = 360, spk_b_id: int = 361, **kw):
        super().__init__(*args, spk_a_id=spk_a_id, spk_b_id=spk_b_id, **kw)
        self.spk_a_id, self.spk_b_id = spk_a_id, spk_b_id


class ZipVoiceDialogStereo(ZipVoiceDialog):
    """zipvoice_dialog.py:218-256: two-stream decoder (500->512 / 512->200)."""

    variant = "zipvoice_dialog_stereo"


MODEL_CLASSES = {"zipvoice": ZipVoice, "zipvoice_distill": ZipVoiceDistill,
                 "zipvoice_dialog": ZipVoiceDialog,
                 "zipvoice_dialog_stereo": ZipVoiceDialogStereo}


def build_model(cfg: ModelConfig, precision: str = "fp32"):
    cls = MODEL_CLASSES[cfg.variant]
    kw = cfg.model_kwargs()
    return cls(**kw, precision=precision)

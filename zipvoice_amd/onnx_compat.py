"""ONNX-contract adapter: the engine behind the reference's ONNX operator API.

The reference exports two graphs (``zipvoice/bin/onnx_export.py``):
``text_encoder.onnx(tokens (1,S_t), prompt_tokens (1,S_p), prompt_features_len
(), speed ()) -> text_condition (1,T,F)`` (``OnnxTextModel``, :112-154) and
``fm_decoder.onnx(t (), x (N,T,F), text_condition, speech_condition,
guidance_scale ()) -> v`` with classifier-free guidance folded in
(``OnnxFlowMatchingModel``, :157-204; metadata ``feat_dim``), and drives them
from ``infer_zipvoice_onnx.py`` through ``OnnxModel.run_text_encoder`` /
``run_fm_decoder`` (:243-314) and ``sample`` (:317-381).

:class:`OnnxModel` here has the same methods, argument order, shapes and
return types, but runs on the MI355X engine (``zv_text_encode`` +
``zv_text_condition``, ``zv_velocity``); an ``infer_zipvoice_onnx``-style driver
swaps ``OnnxModel(text_encoder_path, fm_decoder_path)`` for
``OnnxModel.from_model(model)`` and keeps its own loop.  Tensors may be CPU
(returned on CPU, as onnxruntime does) or CUDA (stay on the device).
"""
from __future__ import annotations

from typing import List

import torch

from .solver import get_time_steps


class OnnxModel:
    def __init__(self, model):
        self.model = model
        self.feat_dim = model.feat_dim
        self.distill = model.cfg.distill

    @classmethod
    def from_model(cls, model) -> "OnnxModel":
        return cls(model)

    def run_text_encoder(self, tokens: torch.Tensor, prompt_tokens: torch.Tensor,
                         prompt_features_len: torch.Tensor, speed: torch.Tensor) -> torch.Tensor:
        """OnnxTextModel.forward (onnx_export.py:121-154), batch 1."""
        m = self.model
        on_cpu = not tokens.is_cuda
        cat = torch.cat([prompt_tokens.cpu(), tokens.cpu()], dim=1)
        assert cat.shape[0] == 1, "the ONNX text encoder contract is batch 1"
        tokens_len = cat.shape[1]
        # float32 duration arithmetic exactly as the exported graph: ceil(P / S_p * S / speed)
        features_len = torch.ceil(prompt_features_len.cpu() / prompt_tokens.shape[1]
                                  * tokens_len / speed.cpu()).to(torch.int64).reshape(1)
        embed, tl = m.forward_text_embed([cat[0].tolist()])
        tc, _ = m.forward_text_condition(embed, tl, features_len.to(m.device))
        return tc.cpu() if on_cpu else tc

    def run_fm_decoder(self, t: torch.Tensor, x: torch.Tensor, text_condition: torch.Tensor,
                       speech_condition: torch.Tensor, guidance_scale: torch.Tensor) -> torch.Tensor:
        """OnnxFlowMatchingModel.forward (onnx_export.py:166-204): CFG folded in
        (t > 0.5 drops the uncond speech condition, else doubles the scale); the
        distill graph feeds the scale to the guidance embedding."""
        m = self.model
        on_cpu = not x.is_cuda
        v = m.engine.velocity(float(t), float(guidance_scale), x.to(m.device),
                              text_condition.to(m.device), speech_condition.to(m.device))
        return v.cpu() if on_cpu else v


def sample(model: OnnxModel, tokens: List[List[int]], prompt_tokens: List[List[int]],
           prompt_features: torch.Tensor, speed: float = 1.0, t_shift: float = 0.5,
           guidance_scale: float = 1.0, num_step: int = 16, x0: torch.Tensor = None
           ) -> torch.Tensor:
    """infer_zipvoice_onnx.sample (:317-381) on the adapter (``x0`` optional)."""
    assert len(tokens) == len(prompt_tokens) == 1
    tokens_t = torch.tensor(tokens, dtype=torch.int64)
    prompt_tokens_t = torch.tensor(prompt_tokens, dtype=torch.int64)
    prompt_features_len = torch.tensor(prompt_features.size(1), dtype=torch.int64)
    text_condition = model.run_text_encoder(tokens_t, prompt_tokens_t, prompt_features_len,
                                            torch.tensor(speed, dtype=torch.float32))
    batch_size, num_frames, _ = text_condition.shape
    timesteps = get_time_steps(t_start=0.0, t_end=1.0, num_step=num_step, t_shift=t_shift)
    x = torch.randn(batch_size, num_frames, model.feat_dim) if x0 is None else x0.cpu()
    speech_condition = torch.nn.functional.pad(
        prompt_features.cpu(), (0, 0, 0, num_frames - prompt_features.shape[1]))
    g = torch.tensor(guidance_scale, dtype=torch.float32)
    for step in range(num_step):
        v = model.run_fm_decoder(t=timesteps[step], x=x, text_condition=text_condition,
                                 speech_condition=speech_condition, guidance_scale=g)
        x = x + v * (timesteps[step + 1] - timesteps[step])
    return x[:, prompt_features_len.item():, :]

"""End-to-end generation on the engine: the reference's ``generate_sentence``
(``zipvoice/bin/infer_zipvoice.py:276-403``) from token ids to waveform, and a
batched form for serving.

Steps, as the reference: prompt RMS normalisation to ``target_rms`` (:340-342)
-> VocosFbank / BigVGANFbank prompt features (:345-347, :583-590) -> ``(feat + feat_bias) * feat_scale``
(:349) -> ``model.sample(duration="predict")`` (:355-371) -> ``pred /
feat_scale - feat_bias`` -> vocoder decode -> ``clamp(-1, 1)`` (:374-378) ->
RTF metrics (:381-396) -> RMS restore (:399-400).  Text normalisation /
tokenisation (jieba, pypinyin, piper) and audio file I/O + resampling
(torchaudio) are outside the ported path: callers pass token ids and 24 kHz
samples.
"""
from __future__ import annotations

import datetime as dt
from typing import Dict, List, Sequence, Tuple

import numpy as np
import torch


def get_feature_extractor(feature_type: str, num_channels: int = 1):
    """The reference's feature-extractor choice by ``model_config["feature"]["type"]``
    (infer_zipvoice.py:583-590): "vocos" -> VocosFbank, "bigvgan_v2" -> BigVGANFbank."""
    from .feature import BigVGANFbank, VocosFbank
    if feature_type == "vocos":
        return VocosFbank(num_channels=num_channels)
    if feature_type == "bigvgan_v2":
        return BigVGANFbank(num_channels=num_channels)
    raise NotImplementedError(f"Unsupported feature type: {feature_type}")


def _prompt_rms_normalise(wav: torch.Tensor, target_rms: float) -> Tuple[torch.Tensor, float]:
    rms = float(torch.sqrt(torch.mean(torch.square(wav))))
    if rms < target_rms:
        wav = wav * target_rms / rms
    return wav, rms


@torch.inference_mode()
def generate_sentence(tokens: List[int], prompt_tokens: List[int], prompt_wav, model, vocoder,
                      feature_extractor, num_step: int = 16, guidance_scale: float = 1.0,
                      speed: float = 1.0, t_shift: float = 0.5, target_rms: float = 0.1,
                      feat_scale: float = 0.1, feat_bias: float = 0.0,
                      sampling_rate: int = 24000, prompt_sampling_rate: int = 24000
                      ) -> Tuple[torch.Tensor, Dict[str, float]]:
    """One sentence (infer_zipvoice.py:276-403).  Returns (wav (1, N) on the
    device, metrics with the reference's keys)."""
    if prompt_sampling_rate != sampling_rate:
        raise NotImplementedError("resample the prompt to 24 kHz before calling (torchaudio "
                                  "Resample is outside the ported path)")
    dev = model.device
    w = torch.as_tensor(np.asarray(prompt_wav) if not torch.is_tensor(prompt_wav) else prompt_wav,
                        dtype=torch.float32)
    if w.dim() == 1:
        w = w.unsqueeze(0)
    w, prompt_rms = _prompt_rms_normalise(w, target_rms)
    feats = feature_extractor.extract(w.to(dev), sampling_rate=sampling_rate)
    prompt_features = ((feats.unsqueeze(0) + feat_bias) * feat_scale).to(dev)
    prompt_features_lens = torch.tensor([prompt_features.size(1)], device=dev)
    torch.cuda.synchronize(dev)
    start_t = dt.datetime.now()
    pred, pred_lens, _, _ = model.sample(
        tokens=[tokens], prompt_tokens=[prompt_tokens], prompt_features=prompt_features,
        prompt_features_lens=prompt_features_lens, speed=speed, t_shift=t_shift,
        duration="predict", num_step=num_step, guidance_scale=guidance_scale)
    torch.cuda.synchronize(dev)
    start_vocoder_t = dt.datetime.now()
    wav = vocoder.decode_features(pred, pred_lens, feat_scale=feat_scale, feat_bias=feat_bias,
                                  clamp=True)
    torch.cuda.synchronize(dev)
    t = (dt.datetime.now() - start_t).total_seconds()
    t_no_vocoder = (start_vocoder_t - start_t).total_seconds()
    t_vocoder = (dt.datetime.now() - start_vocoder_t).total_seconds()
    wav_seconds = wav.shape[-1] / sampling_rate
    metrics = {"t": t, "t_no_vocoder": t_no_vocoder, "t_vocoder": t_vocoder,
               "wav_seconds": wav_seconds, "rtf": t / wav_seconds,
               "rtf_no_vocoder": t_no_vocoder / wav_seconds, "rtf_vocoder": t_vocoder / wav_seconds}
    if prompt_rms < target_rms:
        wav = wav * prompt_rms / target_rms
    return wav, metrics


@torch.inference_mode()
def generate_batch(items: Sequence[Tuple[List[int], List[int], np.ndarray]], model, vocoder,
                   feature_extractor, num_step: int = 16, guidance_scale: float = 1.0,
                   speed: float = 1.0, t_shift: float = 0.5, target_rms: float = 0.1,
                   feat_scale: float = 0.1, feat_bias: float = 0.0, x0=None
                   ) -> Tuple[List[torch.Tensor], Dict[str, float]]:
    """Batched serving form: items = [(tokens, prompt_tokens, prompt_wav_24k), ...].
    Each output equals what ``generate_sentence`` would produce for that item with
    the same initial noise (per-utterance lengths and masks throughout)."""
    dev = model.device
    B = len(items)
    wavs, rms = [], []
    for _, _, pw in items:
        w = torch.as_tensor(np.asarray(pw), dtype=torch.float32).reshape(-1)
        w, r = _prompt_rms_normalise(w, target_rms)
        wavs.append(w)
        rms.append(r)
    n = max(len(w) for w in wavs)
    wb = torch.zeros((B, n), dtype=torch.float32)
    for i, w in enumerate(wavs):
        wb[i, :len(w)] = w
    lens = torch.tensor([len(w) for w in wavs])
    feats, nfr = feature_extractor.extract_batch(wb.to(dev), lens)
    prompt_features = (feats + feat_bias) * feat_scale
    torch.cuda.synchronize(dev)
    t0 = dt.datetime.now()
    pred, pred_lens, _, _ = model.sample(
        tokens=[it[0] for it in items], prompt_tokens=[it[1] for it in items],
        prompt_features=prompt_features, prompt_features_lens=nfr, speed=speed,
        t_shift=t_shift, duration="predict", num_step=num_step, guidance_scale=guidance_scale,
        x0=x0)
    out = vocoder.decode_features(pred, pred_lens, feat_scale=feat_scale, feat_bias=feat_bias,
                                  clamp=True)
    torch.cuda.synchronize(dev)
    t = (dt.datetime.now() - t0).total_seconds()
    hop = vocoder.cfg.hop_length
    res = []
    for i in range(B):
        w = out[i, :int(pred_lens[i]) * hop]
        if rms[i] < target_rms:
            w = w * rms[i] / target_rms
        res.append(w.unsqueeze(0))
    secs = float(pred_lens.sum()) * hop / 24000
    return res, {"t": t, "wav_seconds": secs, "rtf": t / secs}

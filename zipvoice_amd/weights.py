"""State-dict layout and weight sources for the engine.

The engine is keyed by the reference's own state-dict names so that a trained
checkpoint loads unchanged (``zipvoice/utils/checkpoint.py:108-146`` loads
``checkpoint["model"]`` strictly; ``infer_zipvoice.py:561-566`` also accepts
``.safetensors``).  Pretrained weights cannot be fetched here (no network), so
tests and the benchmark use :func:`synthetic_state_dict`, a deterministic
generator (numpy PCG64, per-tensor stream keyed by the tensor name) that builds
the same tensors in this container and on the GPU box.

Key enumeration follows the module tree of
``zipvoice/models/modules/zipformer.py`` (``TTSZipformer.__init__`` :179-240,
``Zipformer2EncoderLayer.__init__`` :350-404, ``Zipformer2Encoder`` :673-687,
``DownsampledZipformer2Encoder`` :814-821) and the model wrappers
(``zipvoice.py:98-133``, ``zipvoice_distill.py:52-68``,
``zipvoice_dialog.py:115-116``, ``zipformer_two_stream.py:160-167``).
"""
from __future__ import annotations

import zlib
from collections import OrderedDict
from typing import Dict, Tuple

import numpy as np

from .config import ModelConfig

Shape = Tuple[int, ...]


def _layer_keys(prefix: str, dim: int, ff: int, heads: int, qdim: int, pdim: int,
                vdim: int, pos_dim: int, kernel: int) -> "OrderedDict[str, Shape]":
    d: "OrderedDict[str, Shape]" = OrderedDict()
    d[prefix + "bypass.bypass_scale"] = (dim,)
    d[prefix + "bypass_mid.bypass_scale"] = (dim,)
    in_proj_dim = (2 * qdim + pdim) * heads
    d[prefix + "self_attn_weights.in_proj.weight"] = (in_proj_dim, dim)
    d[prefix + "self_attn_weights.in_proj.bias"] = (in_proj_dim,)
    d[prefix + "self_attn_weights.linear_pos.weight"] = (heads * pdim, pos_dim)
    for sa in ("self_attn1", "self_attn2"):
        d[prefix + f"{sa}.in_proj.weight"] = (heads * vdim, dim)
        d[prefix + f"{sa}.in_proj.bias"] = (heads * vdim,)
        d[prefix + f"{sa}.out_proj.weight"] = (dim, heads * vdim)
        d[prefix + f"{sa}.out_proj.bias"] = (dim,)
    for name, h in (("feed_forward1", ff * 3 // 4), ("feed_forward2", ff),
                    ("feed_forward3", ff * 5 // 4)):
        d[prefix + f"{name}.in_proj.weight"] = (h, dim)
        d[prefix + f"{name}.in_proj.bias"] = (h,)
        d[prefix + f"{name}.out_proj.weight"] = (dim, h)
        d[prefix + f"{name}.out_proj.bias"] = (dim,)
    hid = 3 * dim // 4
    d[prefix + "nonlin_attention.in_proj.weight"] = (3 * hid, dim)
    d[prefix + "nonlin_attention.in_proj.bias"] = (3 * hid,)
    d[prefix + "nonlin_attention.out_proj.weight"] = (dim, hid)
    d[prefix + "nonlin_attention.out_proj.bias"] = (dim,)
    for cm in ("conv_module1", "conv_module2"):
        d[prefix + f"{cm}.in_proj.weight"] = (2 * dim, dim)
        d[prefix + f"{cm}.in_proj.bias"] = (2 * dim,)
        d[prefix + f"{cm}.depthwise_conv.weight"] = (dim, 1, kernel)
        d[prefix + f"{cm}.depthwise_conv.bias"] = (dim,)
        d[prefix + f"{cm}.out_proj.weight"] = (dim, dim)
        d[prefix + f"{cm}.out_proj.bias"] = (dim,)
    d[prefix + "norm.log_scale"] = ()
    d[prefix + "norm.bias"] = (dim,)
    return d


def zipformer_keys(prefix: str, *, in_dims, out_dims, factors, layers, kernels, dim, ff,
                   heads, qdim, pdim, vdim, pos_dim, time_embed_dim, guidance_embed,
                   two_stream=False) -> "OrderedDict[str, Shape]":
    d: "OrderedDict[str, Shape]" = OrderedDict()
    if two_stream:
        for i, (ind, outd) in enumerate(zip(in_dims, out_dims)):
            d[prefix + f"in_proj.{i}.weight"] = (dim, ind)
            d[prefix + f"in_proj.{i}.bias"] = (dim,)
        for i, outd in enumerate(out_dims):
            d[prefix + f"out_proj.{i}.weight"] = (outd, dim)
            d[prefix + f"out_proj.{i}.bias"] = (outd,)
    else:
        d[prefix + "in_proj.weight"] = (dim, in_dims[0])
        d[prefix + "in_proj.bias"] = (dim,)
        d[prefix + "out_proj.weight"] = (out_dims[0], dim)
        d[prefix + "out_proj.bias"] = (out_dims[0],)
    for s, ds in enumerate(factors):
        sp = prefix + f"encoders.{s}."
        if ds != 1:
            d[sp + "downsample.bias"] = (ds,)
            ep = sp + "encoder."
        else:
            ep = sp
        if time_embed_dim > 0:
            d[ep + "time_emb.1.weight"] = (dim, time_embed_dim)
            d[ep + "time_emb.1.bias"] = (dim,)
        for li in range(layers[s]):
            d.update(_layer_keys(ep + f"layers.{li}.", dim, ff, heads, qdim, pdim, vdim,
                                 pos_dim, kernels[s]))
        if ds != 1:
            d[sp + "out_combiner.bypass_scale"] = (dim,)
    if time_embed_dim > 0:
        d[prefix + "time_embed.0.weight"] = (2 * time_embed_dim, time_embed_dim)
        d[prefix + "time_embed.0.bias"] = (2 * time_embed_dim,)
        d[prefix + "time_embed.2.weight"] = (time_embed_dim, 2 * time_embed_dim)
        d[prefix + "time_embed.2.bias"] = (time_embed_dim,)
    if guidance_embed:
        d[prefix + "guidance_scale_embed.weight"] = (time_embed_dim, time_embed_dim)
    return d


def state_dict_shapes(cfg: ModelConfig) -> "OrderedDict[str, Shape]":
    """Every tensor of the reference model's state dict, with its shape."""
    d: "OrderedDict[str, Shape]" = OrderedDict()
    d.update(zipformer_keys(
        "fm_decoder.", in_dims=cfg.decoder_in_dims(), out_dims=cfg.decoder_out_dims(),
        factors=cfg.fm_decoder_downsampling_factor, layers=cfg.fm_decoder_num_layers,
        kernels=cfg.fm_decoder_cnn_module_kernel, dim=cfg.fm_decoder_dim,
        ff=cfg.fm_decoder_feedforward_dim, heads=cfg.fm_decoder_num_heads,
        qdim=cfg.query_head_dim, pdim=cfg.pos_head_dim, vdim=cfg.value_head_dim,
        pos_dim=cfg.pos_dim, time_embed_dim=cfg.time_embed_dim,
        guidance_embed=cfg.distill, two_stream=cfg.stereo))
    d.update(zipformer_keys(
        "text_encoder.", in_dims=(cfg.text_embed_dim,), out_dims=(cfg.feat_dim,),
        factors=[1], layers=[cfg.text_encoder_num_layers],
        kernels=[cfg.text_encoder_cnn_module_kernel], dim=cfg.text_encoder_dim,
        ff=cfg.text_encoder_feedforward_dim, heads=cfg.text_encoder_num_heads,
        qdim=cfg.query_head_dim, pdim=cfg.pos_head_dim, vdim=cfg.value_head_dim,
        pos_dim=cfg.pos_dim, time_embed_dim=-1, guidance_embed=False))
    d["embed.weight"] = (cfg.vocab_size, cfg.text_embed_dim)
    if cfg.dialog:
        d["spk_embed.weight"] = (2, cfg.feat_dim)
    return d


# ---------------------------------------------------------------------------
# deterministic synthetic weights
# ---------------------------------------------------------------------------

def _gain(key: str) -> float:
    """Output-scale of each linear layer.  Chosen so that every sub-module
    contributes visibly to the residual stream (parity tests then see every
    kernel) while softmax scores stay in a realistic range (std ~2)."""
    if "self_attn_weights.in_proj" in key:
        return 0.6
    if "linear_pos" in key:
        return 1.0
    if key.endswith("out_proj.weight") and ("self_attn" in key or "nonlin" in key
                                            or "conv_module" in key or "feed_forward" in key):
        return 0.5
    return 1.0


def synthetic_tensor(key: str, shape: Shape, seed: int = 0) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64([seed, zlib.crc32(key.encode())]))
    n = int(np.prod(shape)) if len(shape) else 1

    def uni(lo, hi):
        return (lo + (hi - lo) * rng.random(n, dtype=np.float32)).astype(np.float32)

    if key.endswith("bypass_scale"):
        v = uni(0.25, 0.75)
    elif key.endswith("norm.log_scale"):
        v = uni(-0.2, 0.6)
    elif key.endswith("norm.bias"):
        v = uni(-0.5, 0.5)
    elif key.endswith("downsample.bias"):
        v = uni(-1.0, 1.0)
    elif key.endswith("depthwise_conv.weight"):
        k = shape[-1]
        a = float(np.sqrt(3.0 / k))
        v = uni(-a, a)
    elif key == "embed.weight":
        v = rng.standard_normal(n, dtype=np.float32)
    elif key == "spk_embed.weight":
        v = 0.5 * rng.standard_normal(n, dtype=np.float32)
    elif key.endswith(".bias"):
        v = uni(-0.1, 0.1)
    elif key.endswith(".weight") and len(shape) == 2:
        a = float(np.sqrt(3.0 / shape[1])) * _gain(key)
        v = uni(-a, a)
    else:
        raise KeyError(f"no synthetic rule for {key} {shape}")
    return v.reshape(shape)


def synthetic_state_dict(cfg: ModelConfig, seed: int = 0) -> "OrderedDict[str, np.ndarray]":
    return OrderedDict((k, synthetic_tensor(k, s, seed))
                       for k, s in state_dict_shapes(cfg).items())


# ---------------------------------------------------------------------------
# checkpoint ingestion (safe loaders only)
# ---------------------------------------------------------------------------

def load_checkpoint_state_dict(path: str) -> Dict[str, np.ndarray]:
    """Read a reference checkpoint without executing code from the file.

    ``model.pt`` (``checkpoint.py:87-105``: a dict whose ``"model"`` entry is the
    state dict, possibly with DDP ``module.`` prefixes, stripped as in
    ``checkpoint.py:121-131``) is read with ``torch.load(weights_only=True)``;
    ``.safetensors`` with safetensors.
    """
    if path.endswith(".safetensors"):
        from safetensors.numpy import load_file
        sd = load_file(path)
    elif path.endswith(".pt"):
        import torch
        blob = torch.load(path, map_location="cpu", weights_only=True)
        sd = blob["model"] if isinstance(blob, dict) and "model" in blob else blob
        sd = {k: v.float().numpy() for k, v in sd.items()}
    else:
        raise NotImplementedError(f"Unsupported model checkpoint format: {path}")
    out = {}
    for k, v in sd.items():
        if k.startswith("module."):
            k = k[len("module."):]
        out[k] = np.asarray(v, dtype=np.float32)
    return out


def check_state_dict(cfg: ModelConfig, sd: Dict[str, np.ndarray]) -> None:
    """strict=True semantics of ``nn.Module.load_state_dict``."""
    want = state_dict_shapes(cfg)
    missing = [k for k in want if k not in sd]
    unexpected = [k for k in sd if k not in want]
    if missing or unexpected:
        raise KeyError(f"state dict mismatch: missing={missing[:5]} (+{max(0, len(missing)-5)}), "
                       f"unexpected={unexpected[:5]} (+{max(0, len(unexpected)-5)})")
    for k, s in want.items():
        if tuple(sd[k].shape) != tuple(s):
            raise ValueError(f"shape mismatch for {k}: {sd[k].shape} vs {s}")

"""Model configuration for the ZipVoice hot path.

Mirrors the ``"model"`` block of the reference's ``model.json``
(``egs/zipvoice/conf/zipvoice_base.json:2-25``) and the constructor keywords of
``ZipVoice.__init__`` (``zipvoice/models/zipvoice.py:38-60``), plus the variant
selector for the four model classes the reference inference CLIs build
(``zipvoice/bin/infer_zipvoice.py:549-559``,
``zipvoice/bin/infer_zipvoice_dialog.py:679-689``).
"""
from __future__ import annotations

import dataclasses
import json
from typing import List, Tuple

VARIANTS = ("zipvoice", "zipvoice_distill", "zipvoice_dialog", "zipvoice_dialog_stereo")


@dataclasses.dataclass
class ModelConfig:
    fm_decoder_downsampling_factor: List[int] = dataclasses.field(
        default_factory=lambda: [1, 2, 4, 2, 1])
    fm_decoder_num_layers: List[int] = dataclasses.field(
        default_factory=lambda: [2, 2, 4, 4, 4])
    fm_decoder_cnn_module_kernel: List[int] = dataclasses.field(
        default_factory=lambda: [31, 15, 7, 15, 31])
    fm_decoder_feedforward_dim: int = 1536
    fm_decoder_num_heads: int = 4
    fm_decoder_dim: int = 512
    text_encoder_num_layers: int = 4
    text_encoder_feedforward_dim: int = 512
    text_encoder_cnn_module_kernel: int = 9
    text_encoder_num_heads: int = 4
    text_encoder_dim: int = 192
    time_embed_dim: int = 192
    text_embed_dim: int = 192
    query_head_dim: int = 32
    value_head_dim: int = 12
    pos_head_dim: int = 4
    pos_dim: int = 48
    feat_dim: int = 100
    vocab_size: int = 360
    pad_id: int = 0
    # dialog only (zipvoice/models/zipvoice_dialog.py:58-59)
    spk_a_id: int = 360
    spk_b_id: int = 361
    variant: str = "zipvoice"

    def __post_init__(self):
        if self.variant not in VARIANTS:
            raise ValueError(f"unknown variant {self.variant!r}; expected one of {VARIANTS}")
        for name in ("fm_decoder_downsampling_factor", "fm_decoder_num_layers",
                     "fm_decoder_cnn_module_kernel"):
            v = getattr(self, name)
            if isinstance(v, int):
                v = [v]
            setattr(self, name, list(v))
        n = len(self.fm_decoder_downsampling_factor)
        if len(self.fm_decoder_num_layers) == 1:
            self.fm_decoder_num_layers = self.fm_decoder_num_layers * n
        if len(self.fm_decoder_cnn_module_kernel) == 1:
            self.fm_decoder_cnn_module_kernel = self.fm_decoder_cnn_module_kernel * n
        _check_unet(self.fm_decoder_downsampling_factor)

    # ---- derived quantities -------------------------------------------------
    @property
    def stereo(self) -> bool:
        return self.variant == "zipvoice_dialog_stereo"

    @property
    def distill(self) -> bool:
        return self.variant == "zipvoice_distill"

    @property
    def dialog(self) -> bool:
        return self.variant in ("zipvoice_dialog", "zipvoice_dialog_stereo")

    @property
    def io_feat_dim(self) -> int:
        """Width of x / speech condition: 2*feat_dim for the stereo model."""
        return 2 * self.feat_dim if self.stereo else self.feat_dim

    def decoder_in_dims(self) -> Tuple[int, ...]:
        # zipvoice.py:100 (feat*3); zipvoice_dialog.py:241-243 ((feat*5, feat*3))
        if self.stereo:
            return (self.feat_dim * 5, self.feat_dim * 3)
        return (self.feat_dim * 3,)

    def decoder_out_dims(self) -> Tuple[int, ...]:
        if self.stereo:
            return (self.feat_dim * 2, self.feat_dim)
        return (self.feat_dim,)

    @classmethod
    def from_json(cls, path: str, variant: str = "zipvoice", **overrides) -> "ModelConfig":
        with open(path) as f:
            blob = json.load(f)
        model = dict(blob.get("model", blob))
        model.update(overrides)
        model["variant"] = variant
        return cls(**model)

    def model_kwargs(self) -> dict:
        """Keyword arguments accepted by the reference model constructors."""
        d = dataclasses.asdict(self)
        d.pop("variant")
        if not self.dialog:
            d.pop("spk_a_id")
            d.pop("spk_b_id")
        return d


def _check_unet(factors):
    """zipformer.py:149-157: U-Net style factor list."""
    if factors[0] != 1 or factors[-1] != 1:
        raise ValueError(f"downsampling factors must start and end with 1: {factors}")
    for i in range(1, len(factors) // 2 + 1):
        if factors[i] != factors[i - 1] * 2:
            raise ValueError(f"bad U-Net downsampling factors {factors}")
    for i in range(len(factors) // 2 + 1, len(factors)):
        if factors[i] * 2 != factors[i - 1]:
            raise ValueError(f"bad U-Net downsampling factors {factors}")


def default_config(variant: str = "zipvoice", **kw) -> ModelConfig:
    """The published base architecture (zipvoice_base.json)."""
    if variant in ("zipvoice_dialog", "zipvoice_dialog_stereo"):
        kw.setdefault("vocab_size", 362)
    return ModelConfig(variant=variant, **kw)


# Per-variant inference defaults (infer_zipvoice.py:479-488,
# infer_zipvoice_dialog.py:132-144).
INFER_DEFAULTS = {
    "zipvoice": dict(num_step=16, guidance_scale=1.0, t_shift=0.5),
    "zipvoice_distill": dict(num_step=8, guidance_scale=3.0, t_shift=0.5),
    "zipvoice_dialog": dict(num_step=16, guidance_scale=1.5, t_shift=0.5),
    "zipvoice_dialog_stereo": dict(num_step=16, guidance_scale=1.5, t_shift=0.5),
}

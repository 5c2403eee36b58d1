#!/usr/bin/env python3
"""Generate golden fixtures by running the REFERENCE PyTorch code on CPU.

Container-only tool (needs /root/reference, which never travels to the GPU
box).  It imports the reference model classes read-only (tensorboard stubbed:
``zipvoice/utils/common.py:21`` imports it but inference never uses it), loads
the engine's deterministic synthetic weights
(``zipvoice_amd.weights.synthetic_state_dict``) with ``strict=True``, feeds
explicit inputs (x0 is injected in place of ``torch.randn`` at
``zipvoice/models/zipvoice.py:453-458``), and writes inputs + outputs as small
``.npz`` files next to this script.  Only the fixtures are committed.

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
"""
import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("ZIPVOICE_REFERENCE", "/root/reference")
sys.dont_write_bytecode = True
sys.path.insert(0, REPO)

tb = types.ModuleType("torch.utils.tensorboard")
tb.SummaryWriter = object
sys.modules["torch.utils.tensorboard"] = tb
sys.path.insert(0, REF)

import torch  # noqa: E402

from zipvoice.models.zipvoice import ZipVoice  # noqa: E402
from zipvoice.models.zipvoice_dialog import ZipVoiceDialog, ZipVoiceDialogStereo  # noqa: E402
from zipvoice.models.zipvoice_distill import ZipVoiceDistill  # noqa: E402

from zipvoice_amd.config import default_config  # noqa: E402
from zipvoice_amd.weights import state_dict_shapes, synthetic_state_dict  # noqa: E402

CLASSES = {"zipvoice": ZipVoice, "zipvoice_distill": ZipVoiceDistill,
           "zipvoice_dialog": ZipVoiceDialog, "zipvoice_dialog_stereo": ZipVoiceDialogStereo}
SEED = 0


def build(variant):
    cfg = default_config(variant)
    model = CLASSES[variant](**cfg.model_kwargs())
    ref_shapes = {k: tuple(v.shape) for k, v in model.state_dict().items()}
    mine = dict(state_dict_shapes(cfg))
    assert ref_shapes == mine, "state-dict layout mismatch vs reference"
    sd = synthetic_state_dict(cfg, SEED)
    model.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in sd.items()}, strict=True)
    model.eval()
    return cfg, model


class InjectRandn:
    """Replace torch.randn for one call so sample() uses our explicit x0."""

    def __init__(self, x0):
        self.x0 = torch.from_numpy(x0)
        self.orig = torch.randn

    def __enter__(self):
        def fake(*size, **kw):
            shp = tuple(size[0]) if len(size) == 1 and isinstance(size[0], (tuple, list)) \
                else tuple(size)
            assert shp == tuple(self.x0.shape), (shp, self.x0.shape)
            return self.x0.clone()
        torch.randn = fake
        return self

    def __exit__(self, *a):
        torch.randn = self.orig


def rand_tokens(rng, n, lo=1, hi=359):
    return [int(v) for v in rng.integers(lo, hi + 1, size=n)]


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print("wrote", path, sum(a.nbytes for a in map(np.asarray, arrays.values())), "bytes")


def ragged_tokens_array(tok_lists):
    n = max(len(t) for t in tok_lists)
    arr = np.full((len(tok_lists), n), -1, np.int64)
    for i, t in enumerate(tok_lists):
        arr[i, :len(t)] = t
    return arr


@torch.inference_mode()
def decoder_fixture(variant, name, guidance=None):
    cfg, model = build(variant)
    rng = np.random.default_rng(11)
    B, T, F = 2, 70, cfg.io_feat_dim
    lens = np.array([70, 53], np.int64)
    x = rng.standard_normal((B, T, F), dtype=np.float32)
    tc = rng.standard_normal((B, T, cfg.feat_dim), dtype=np.float32)
    sc = (0.3 * rng.standard_normal((B, T, F)) - 0.5).astype(np.float32)
    pm = np.arange(T)[None] >= lens[:, None]
    t = np.float32(0.37)
    kw = {}
    if guidance is not None:
        kw["guidance_scale"] = torch.tensor(guidance, dtype=torch.float32)
    v = model.forward_fm_decoder(t=torch.tensor(t), xt=torch.from_numpy(x),
                                 text_condition=torch.from_numpy(tc),
                                 speech_condition=torch.from_numpy(sc),
                                 padding_mask=torch.from_numpy(pm), **kw)
    save(name, t=t, x=x, text_condition=tc, speech_condition=sc, padding_mask=pm,
         guidance_scale=np.float32(guidance if guidance is not None else np.nan),
         v=v.numpy(), variant=np.array(variant), seed=np.int64(SEED))


@torch.inference_mode()
def text_embed_fixture():
    cfg, model = build("zipvoice")
    rng = np.random.default_rng(12)
    toks = [rand_tokens(rng, n) for n in (7, 12, 4)]
    emb, lens = model.forward_text_embed(toks)
    save("text_embed.npz", tokens=ragged_tokens_array(toks), embed=emb.numpy(),
         tokens_lens=lens.numpy(), variant=np.array("zipvoice"), seed=np.int64(SEED))


@torch.inference_mode()
def sample_fixture(variant, name, B, T_p, S_p, S_t, num_step, guidance, t_shift=0.5,
                   speed=1.0, duration="predict", gen_frames=None, rng_seed=13,
                   dialog_turns=False):
    cfg, model = build(variant)
    rng = np.random.default_rng(rng_seed)
    F = cfg.io_feat_dim
    prompt_tokens = [rand_tokens(rng, n) for n in S_p]
    tokens = [rand_tokens(rng, n) for n in S_t]
    if dialog_turns:
        for tl in (prompt_tokens, tokens):
            for row in tl:
                row[0] = cfg.spk_a_id
                row[len(row) // 2] = cfg.spk_b_id
    T_p = np.asarray(T_p, np.int64)
    pf = (0.3 * rng.standard_normal((B, int(T_p.max()), F)) - 0.5).astype(np.float32)
    for i in range(B):
        pf[i, T_p[i]:] = 0.0
    features_lens = None
    if duration == "predict":
        tl = np.array([len(t) for t in tokens], np.float32)
        ptl = np.array([len(t) for t in prompt_tokens], np.float32)
        T_all = T_p + np.ceil(T_p.astype(np.float32) / ptl * tl / np.float32(speed)).astype(
            np.int64)
    else:
        features_lens = np.asarray(gen_frames, np.int64)
        T_all = T_p + features_lens
    T = int(T_all.max())
    x0 = np.random.default_rng(666).standard_normal((B, T, F), dtype=np.float32)
    with InjectRandn(x0):
        out = model.sample(tokens=tokens, prompt_tokens=prompt_tokens,
                           prompt_features=torch.from_numpy(pf),
                           prompt_features_lens=torch.from_numpy(T_p),
                           features_lens=None if features_lens is None
                           else torch.from_numpy(features_lens),
                           speed=speed, t_shift=t_shift, duration=duration,
                           num_step=num_step, guidance_scale=guidance)
    gen, gen_lens, prm, plens = (o.numpy() for o in out)
    save(name, tokens=ragged_tokens_array(tokens),
         prompt_tokens=ragged_tokens_array(prompt_tokens), prompt_features=pf,
         prompt_features_lens=T_p, features_lens=(features_lens if features_lens is not None
                                                  else np.zeros(0, np.int64)),
         x0=x0, speed=np.float32(speed), t_shift=np.float32(t_shift),
         duration=np.array(duration), num_step=np.int64(num_step),
         guidance_scale=np.float32(guidance), gen=gen, gen_lens=gen_lens, prompt=prm,
         prompt_lens=plens, variant=np.array(variant), seed=np.int64(SEED))


def main():
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    decoder_fixture("zipvoice", "decoder_fwd.npz")
    decoder_fixture("zipvoice_distill", "decoder_fwd_distill.npz", guidance=3.0)
    decoder_fixture("zipvoice_dialog_stereo", "decoder_fwd_stereo.npz")
    text_embed_fixture()
    # config C1 of BASELINE.json: B=1, 3 s prompt (281 frames), 40 prompt tokens,
    # 20 text tokens, N=4, guidance 1.0, t_shift 0.5 -> T = 422.
    sample_fixture("zipvoice", "sample_c1.npz", 1, [281], [40], [20], 4, 1.0)
    sample_fixture("zipvoice", "sample_batch.npz", 3, [40, 55, 31], [6, 9, 5], [5, 3, 8],
                   4, 1.0, rng_seed=14)
    sample_fixture("zipvoice", "sample_real_duration.npz", 2, [33, 20], [5, 4], [4, 6], 4,
                   0.7, duration="real", gen_frames=[30, 41], rng_seed=15)
    sample_fixture("zipvoice_distill", "sample_distill.npz", 2, [30, 44], [5, 7], [6, 4], 2,
                   3.0, rng_seed=16)
    sample_fixture("zipvoice_dialog", "sample_dialog.npz", 2, [36, 28], [6, 5], [8, 7], 4,
                   1.5, rng_seed=17, dialog_turns=True)
    sample_fixture("zipvoice_dialog_stereo", "sample_stereo.npz", 1, [40], [7], [9], 4, 1.5,
                   rng_seed=18, dialog_turns=True)
    with open(os.path.join(HERE, "MANIFEST.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "weights_seed": SEED,
                   "reference": "winlaic/ZipVoice @ 2025-08-24 (read-only, CPU fp32)",
                   "torch": torch.__version__}, f, indent=1)


if __name__ == "__main__":
    main()

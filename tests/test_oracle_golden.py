"""Pin the CPU oracle (oracle/zipvoice_np.py) against the golden fixtures that
tests/golden/make_golden.py produced by running the reference's own PyTorch code.

fp32 vs fp32: the only differences are summation order inside matmuls, so the
bar is 5e-5 absolute on O(1) outputs (observed ~1e-5).
"""
import numpy as np
import pytest

from golden_io import load, tokens_list
from oracle.zipvoice_np import ZipVoiceOracle, get_time_steps, linspace_f32
from zipvoice_amd.config import default_config
from zipvoice_amd.weights import synthetic_state_dict

TOL = 5e-5
_cache = {}


def oracle(variant):
    if variant not in _cache:
        cfg = default_config(variant)
        _cache[variant] = ZipVoiceOracle(cfg, synthetic_state_dict(cfg, 0))
    return _cache[variant]


@pytest.mark.parametrize("name,g", [("decoder_fwd.npz", None),
                                    ("decoder_fwd_distill.npz", 3.0),
                                    ("decoder_fwd_stereo.npz", None)])
def test_decoder_forward(name, g):
    d = load(name)
    o = oracle(str(d["variant"]))
    v = o.forward_fm_decoder(d["t"], d["x"], d["text_condition"], d["speech_condition"],
                             d["padding_mask"], guidance_scale=g)
    assert np.abs(v - d["v"]).max() < TOL


def test_text_embed():
    d = load("text_embed.npz")
    e, lens = oracle("zipvoice").forward_text_embed(tokens_list(d["tokens"]))
    assert (lens == d["tokens_lens"]).all()
    assert np.abs(e - d["embed"]).max() < TOL


SAMPLES = ["sample_c1.npz", "sample_batch.npz", "sample_real_duration.npz",
           "sample_distill.npz", "sample_dialog.npz", "sample_stereo.npz"]


def run_sample(o, d):
    fl = d["features_lens"]
    return o.sample(tokens_list(d["tokens"]), tokens_list(d["prompt_tokens"]),
                    d["prompt_features"], d["prompt_features_lens"], x0=d["x0"],
                    features_lens=fl if fl.size else None, speed=float(d["speed"]),
                    t_shift=float(d["t_shift"]), duration=str(d["duration"]),
                    num_step=int(d["num_step"]), guidance_scale=float(d["guidance_scale"]))


@pytest.mark.parametrize("name", SAMPLES)
def test_sample(name):
    d = load(name)
    gen, gl, prm, pl = run_sample(oracle(str(d["variant"])), d)
    assert gen.shape == d["gen"].shape
    assert (gl == d["gen_lens"]).all() and (pl == d["prompt_lens"]).all()
    assert np.abs(gen - d["gen"]).mean() < 1e-5
    assert np.abs(gen - d["gen"]).max() < TOL
    assert np.abs(prm - d["prompt"]).max() < TOL


def test_linspace_matches_torch():
    torch = pytest.importorskip("torch")
    for n in (2, 3, 5, 9, 17, 33):
        a = torch.linspace(0.0, 1.0, n).numpy()
        assert (linspace_f32(0.0, 1.0, n) == a).all()
    ts = get_time_steps(0.0, 1.0, 16, 0.5)
    ref = torch.linspace(0.0, 1.0, 17)
    ref = 0.5 * ref / (1 + (0.5 - 1) * ref)
    assert (ts == ref.numpy()).all()

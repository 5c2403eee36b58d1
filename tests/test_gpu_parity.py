"""GPU parity: the HIP engine (through the C ABI) vs the golden fixtures produced
by the reference, and vs the CPU oracle on the same seeded inputs.

Tolerances (written here, per north_star "within 1e-3 mel L1"):
  * precision="fp32" (bf16x3 split-product GEMMs, fp32 elsewhere): mean |err|
    < 1e-3 against the reference outputs, max |err| < 3e-2.
  * precision="fp16" (the parity-grade fast mode: fp16 MFMA operands in the decoder
    layers, split products for the decoder's in/out projections, the attention-score
    projections and the text encoder):
    mean |err| < 1e-3 (the north-star bar), max |err| < 2e-2.
  * precision="bf16" (bf16 MFMA operands, fp32 accumulate/residual/softmax):
    production mode; the reference's own bf16-autocast drift is 1.4e-2 mean
    (SURVEY.md §0), so the bar here is mean |err| < 5e-2.
"""
import numpy as np
import pytest

from golden_io import load, tokens_list

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

TOL = {"fp32": (1e-3, 3e-2), "fp16": (1e-3, 2e-2), "bf16": (5e-2, 0.25)}
_models = {}


def model(variant, precision):
    key = (variant, precision)
    if key not in _models:
        from zipvoice_amd.config import default_config
        from zipvoice_amd.models import build_model
        from zipvoice_amd.weights import synthetic_state_dict
        cfg = default_config(variant)
        m = build_model(cfg, precision=precision)
        m.load_state_dict(synthetic_state_dict(cfg, 0))
        _models[key] = m.to("cuda:0")
    return _models[key]


def cuda(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0")


def check(out, ref, precision, what):
    out = out.detach().float().cpu().numpy() if torch.is_tensor(out) else out
    assert out.shape == ref.shape, (what, out.shape, ref.shape)
    assert np.isfinite(out).all(), what
    err = np.abs(out - ref)
    mean_tol, max_tol = TOL[precision]
    print(f"{what} [{precision}] mean={err.mean():.3e} max={err.max():.3e}")
    assert err.mean() < mean_tol, (what, err.mean())
    assert err.max() < max_tol, (what, err.max())


@pytest.mark.parametrize("precision", ["fp32", "fp16", "bf16"])
@pytest.mark.parametrize("name,g", [("decoder_fwd.npz", None),
                                    ("decoder_fwd_distill.npz", 3.0),
                                    ("decoder_fwd_stereo.npz", None)])
def test_decoder_forward_golden(name, g, precision):
    d = load(name)
    m = model(str(d["variant"]), precision)
    v = m.forward_fm_decoder(t=torch.tensor(float(d["t"])), xt=cuda(d["x"]),
                             text_condition=cuda(d["text_condition"]),
                             speech_condition=cuda(d["speech_condition"]),
                             padding_mask=cuda(d["padding_mask"]),
                             guidance_scale=None if g is None else torch.tensor(g))
    # padded frames carry reference values too (they are computed, not masked)
    check(v, d["v"], precision, name)


@pytest.mark.parametrize("precision", ["fp32", "fp16", "bf16"])
def test_text_embed_golden(precision):
    d = load("text_embed.npz")
    emb, lens = model("zipvoice", precision).forward_text_embed(tokens_list(d["tokens"]))
    assert (lens.cpu().numpy() == d["tokens_lens"]).all()
    check(emb, d["embed"], precision, "text_embed")


SAMPLES = ["sample_c1.npz", "sample_batch.npz", "sample_real_duration.npz",
           "sample_distill.npz", "sample_dialog.npz", "sample_stereo.npz"]


def run_sample(m, d):
    fl = d["features_lens"]
    return m.sample(tokens=tokens_list(d["tokens"]), prompt_tokens=tokens_list(d["prompt_tokens"]),
                    prompt_features=cuda(d["prompt_features"]),
                    prompt_features_lens=cuda(d["prompt_features_lens"]),
                    features_lens=cuda(fl) if fl.size else None, speed=float(d["speed"]),
                    t_shift=float(d["t_shift"]), duration=str(d["duration"]),
                    num_step=int(d["num_step"]), guidance_scale=float(d["guidance_scale"]),
                    x0=cuda(d["x0"]))


@pytest.mark.parametrize("precision", ["fp32", "fp16", "bf16"])
@pytest.mark.parametrize("name", SAMPLES)
def test_sample_golden(name, precision):
    d = load(name)
    gen, gl, prm, pl = run_sample(model(str(d["variant"]), precision), d)
    assert (gl.cpu().numpy() == d["gen_lens"]).all()
    assert (pl.cpu().numpy() == d["prompt_lens"]).all()
    check(gen, d["gen"], precision, name + ":gen")
    check(prm, d["prompt"], precision, name + ":prompt")


def test_velocity_matches_oracle_both_cfg_branches():
    """DiffusionModel.forward at t <= 0.5 (speech kept, g doubled) and t > 0.5."""
    from oracle.zipvoice_np import ZipVoiceOracle
    from zipvoice_amd.weights import synthetic_state_dict
    m = model("zipvoice", "fp32")
    o = ZipVoiceOracle(m.cfg, synthetic_state_dict(m.cfg, 0))
    rng = np.random.default_rng(3)
    B, T = 2, 33
    x = rng.standard_normal((B, T, 100), dtype=np.float32)
    tc = rng.standard_normal((B, T, 100), dtype=np.float32)
    sc = rng.standard_normal((B, T, 100), dtype=np.float32)
    pm = np.arange(T)[None] >= np.array([33, 20])[:, None]
    for t in (0.25, 0.75):
        v = m.engine.velocity(t, 1.3, cuda(x), cuda(tc), cuda(sc), cuda(pm))
        ref = o.velocity(np.float32(t), x, tc, sc, pm, 1.3)
        check(v, ref, "fp32", f"velocity t={t}")


def test_long_sequence_properties():
    """Full-size (config C2 length) decoder pass: finite, padding-invariant for the
    valid frames of an item whose padding is changed (keys are masked; only the
    SimpleDownsample repeat-pad and conv zeroing see padded frames, and those only
    touch frames near the end of the *batch* tensor)."""
    m = model("zipvoice", "bf16")
    rng = np.random.default_rng(5)
    T = 1219
    x = cuda(rng.standard_normal((1, T, 100), dtype=np.float32))
    tc = cuda(rng.standard_normal((1, T, 100), dtype=np.float32))
    sc = cuda(rng.standard_normal((1, T, 100), dtype=np.float32))
    v1 = m.forward_fm_decoder(torch.tensor(0.4), x, tc, sc, None)
    v2 = m.forward_fm_decoder(torch.tensor(0.4), x, tc, sc,
                              torch.zeros(1, T, dtype=torch.bool, device="cuda:0"))
    assert torch.isfinite(v1).all()
    # an all-false mask is identical to no mask
    assert torch.equal(v1, v2)
    # batch invariance: item 0 of a batch of 2 equals the batch of 1
    v3 = m.forward_fm_decoder(torch.tensor(0.4), torch.cat([x, x.flip(1)]),
                              torch.cat([tc, tc]), torch.cat([sc, sc]), None)
    assert (v3[:1] - v1).abs().max().item() < 1e-5


def test_materialized_attention_path_matches(monkeypatch):
    """A/B: the W-materialising attention path (ZV_ATTN_MATERIALIZE=1) and the fused
    flash-style consumers give the same decoder output (fp32 mode)."""
    from zipvoice_amd.config import default_config
    from zipvoice_amd.models import build_model
    from zipvoice_amd.weights import synthetic_state_dict
    d = load("decoder_fwd.npz")
    cfg = default_config("zipvoice")
    monkeypatch.setenv("ZV_ATTN_MATERIALIZE", "1")
    m = build_model(cfg, precision="fp32")
    m.load_state_dict(synthetic_state_dict(cfg, 0))
    m = m.to("cuda:0")
    args = dict(t=torch.tensor(float(d["t"])), xt=cuda(d["x"]),
                text_condition=cuda(d["text_condition"]),
                speech_condition=cuda(d["speech_condition"]), padding_mask=cuda(d["padding_mask"]))
    v_mat = m.forward_fm_decoder(**args)
    check(v_mat, d["v"], "fp32", "decoder_fwd (materialised W)")
    v_fused = model("zipvoice", "fp32").forward_fm_decoder(**args)
    assert (v_mat - v_fused).abs().max().item() < 1e-4


def test_dialog_long_sequence_fused_vs_materialized():
    """Config C4 length (30 s dialogue: T = 3376 frames, the longest attention the
    benchmark configs reach) on a ragged batch of two with a padded second item:
    the production bf16 path (fused flash-style attention consumers) against the
    fp32-accurate mode, whose fused images do not fit LDS at this length and which
    therefore runs the W-materialising attention (an independent implementation of
    the same softmax).  Bar: the bf16 tolerance of this file."""
    rng = np.random.default_rng(11)
    B, T = 2, 3376
    x = cuda(rng.standard_normal((B, T, 100), dtype=np.float32))
    tc = cuda(rng.standard_normal((B, T, 100), dtype=np.float32))
    sc = cuda((0.3 * rng.standard_normal((B, T, 100)) - 0.5).astype(np.float32))
    pm = cuda(np.arange(T)[None] >= np.array([T, 2901])[:, None])
    args = dict(t=torch.tensor(0.6), xt=x, text_condition=tc, speech_condition=sc, padding_mask=pm)
    fused = model("zipvoice_dialog", "bf16").forward_fm_decoder(**args)
    ref = model("zipvoice_dialog", "fp32").forward_fm_decoder(**args)
    valid = (~pm).cpu().numpy()
    f = fused.float().cpu().numpy()[valid]
    r = ref.float().cpu().numpy()[valid]
    check(f, r, "bf16", f"dialog T={T} bf16 fused vs fp32 materialised")


@pytest.mark.parametrize("T,lens", [(1, [1]), (2, [2, 1]), (5, [5, 3]), (9, [9, 1])])
def test_velocity_tiny_lengths(T, lens):
    """Edge lengths below the stacks' downsampling factors (1..4): single frames, a
    one-frame item padded inside a longer batch, odd lengths, against the oracle."""
    from oracle.zipvoice_np import ZipVoiceOracle
    from zipvoice_amd.weights import synthetic_state_dict
    m = model("zipvoice", "fp32")
    o = ZipVoiceOracle(m.cfg, synthetic_state_dict(m.cfg, 0))
    rng = np.random.default_rng(T)
    B = len(lens)
    x = rng.standard_normal((B, T, 100), dtype=np.float32)
    tc = rng.standard_normal((B, T, 100), dtype=np.float32)
    sc = rng.standard_normal((B, T, 100), dtype=np.float32)
    pm = np.arange(T)[None] >= np.array(lens)[:, None]
    v = m.engine.velocity(0.6, 1.0, cuda(x), cuda(tc), cuda(sc), cuda(pm))
    ref = o.velocity(np.float32(0.6), x, tc, sc, pm, 1.0)
    check(v, ref, "fp32", f"velocity T={T} lens={lens}")


def test_empty_batch_rejected():
    """B = 0 / T = 0 are refused by the C ABI with an error (no launch)."""
    m = model("zipvoice", "fp32")
    z = torch.zeros(0, 4, 100, device="cuda:0")
    with pytest.raises(RuntimeError):
        m.engine.velocity(0.5, 1.0, z, z, z, torch.zeros(0, 4, dtype=torch.bool, device="cuda:0"))
    z = torch.zeros(1, 0, 100, device="cuda:0")
    with pytest.raises(RuntimeError):
        m.engine.velocity(0.5, 1.0, z, z, z, torch.zeros(1, 0, dtype=torch.bool, device="cuda:0"))

"""Fused FeedForward (zv_ffn.inc: in_proj -> SwooshL -> out_proj -> residual in one kernel,
ZV_FFN=1; + the layer's BiasNorm and bypass in FF3's epilogue, ZV_FFN=2) and the pipelined
depthwise conv (ZV_DWCONV_PIPE) through the C ABI.

The fused FF differs from the unfused pair only in the out-projection's K summation order (the
hidden tile is consumed in the 32x32 accumulator's register order) and, with the norm epilogue,
in BiasNorm's sum-of-squares order: each arm is held to its precision mode's parity bar against
the fp32 oracle (reference zipformer.py:1433-1439, :610-618; scaling.py:330-355).  Through the
16-bit model those orders flip roundings, so the arms differ by about one mode error from each
other (the kernel itself matches the unfused pair to 2e-7: tools/lab/ffn_lab,
profiles/r03_ffn_lab.txt).  The pipelined depthwise conv keeps the register-window kernel's FMA
order per output: bitwise equal velocities.  ZV_FFN_MIN_ROWS=0 puts every launch on the fused
kernel (by default launches under 15000 rows keep the unfused pair)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

BAR = {"bf16": 5e-2, "fp16": 1e-3}


def _run(monkeypatch, env, precision, variant="zipvoice", B=2, T=203, lens=(203, 150), t=0.4, seed=11):
    from zipvoice_amd.config import default_config
    from zipvoice_amd.models import build_model
    from zipvoice_amd.weights import synthetic_state_dict
    cfg = default_config(variant)
    sd = synthetic_state_dict(cfg, 0)
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((B, T, cfg.feat_dim), dtype=np.float32)
    tc = rng.standard_normal(x.shape, dtype=np.float32)
    sc = rng.standard_normal(x.shape, dtype=np.float32)
    pm = np.arange(T)[None] >= np.array(lens)[:, None]
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    m = build_model(cfg, precision=precision)
    m.load_state_dict(sd)
    m = m.to("cuda:0")
    cu = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0")
    out = m.engine.velocity(t, 1.0, cu(x), cu(tc), cu(sc), cu(pm)).cpu().numpy()
    del m
    return out, (cfg, sd, x, tc, sc, pm, t)


@pytest.mark.parametrize("precision", ["bf16", "fp16"])
def test_fused_ffn_vs_unfused_and_oracle(monkeypatch, precision):
    from oracle.zipvoice_np import ZipVoiceOracle
    outs = {}
    for ffn in ("0", "1", "2"):
        outs[ffn], inp = _run(monkeypatch, {"ZV_FFN": ffn, "ZV_FFN_MIN_ROWS": "0"}, precision)
    cfg, sd, x, tc, sc, pm, t = inp
    ref = ZipVoiceOracle(cfg, sd).velocity(np.float32(t), x, tc, sc, pm, 1.0)
    valid = ~pm
    e0 = np.abs(outs["0"] - ref)[valid].mean()
    for ffn, o in outs.items():
        e = np.abs(o - ref)[valid]
        d = np.abs(o - outs["0"])[valid].mean()
        print(f"{precision} ZV_FFN={ffn}: vs oracle mean {e.mean():.3e} max {e.max():.3e}; vs unfused mean {d:.3e}")
        assert np.isfinite(o).all()
        # the mode's bar, fixed (north_star's 1e-3 for the fp16 parity mode; this random input sat
        # at 1.07e-3 before round 4's split SelfAttention products, ZV_MIXED_SA)
        bar = BAR[precision]
        assert e.mean() < bar
        # two arms whose own rounding errors are independent: their difference is bounded by
        # the sum of the two bars
        assert d < 2 * bar


def test_fused_ffn_long_ragged(monkeypatch):
    """A length whose row counts are not multiples of the 128-row block at any stack's rate
    (2 CFG rows x 1001 frames; every downsampling factor's FF widths), fp16 parity mode."""
    from oracle.zipvoice_np import ZipVoiceOracle
    o, inp = _run(monkeypatch, {"ZV_FFN": "2", "ZV_FFN_MIN_ROWS": "0"}, "fp16", B=1, T=1001, lens=(1001,), t=0.6)
    cfg, sd, x, tc, sc, pm, t = inp
    ref = ZipVoiceOracle(cfg, sd).velocity(np.float32(t), x, tc, sc, pm, 1.0)
    e = np.abs(o - ref)[~pm]
    o0, _ = _run(monkeypatch, {"ZV_FFN": "0"}, "fp16", B=1, T=1001, lens=(1001,), t=0.6)
    e0 = np.abs(o0 - ref)[~pm].mean()
    print(f"T=1001 fp16 ZV_FFN=2: mean {e.mean():.3e} max {e.max():.3e} (unfused {e0:.3e})")
    assert e.mean() < BAR["fp16"] and e0 < BAR["fp16"]


def test_dwconv_pipe_bitwise(monkeypatch):
    outs = []
    for flag in ("0", "1", "2"):      # register-window / pipelined (auto chunk) / pipelined, 2-tile chunks
        o, _ = _run(monkeypatch, {"ZV_DWCONV_PIPE": flag, "ZV_DWCONV_LDS": "0"}, "bf16", B=2, T=1219,
                    lens=(1219, 1000))
        outs.append(o)
    for o in outs[1:]:
        assert np.array_equal(o, outs[0]), np.abs(o - outs[0]).max()


def test_fused_ffn_short_utterances(monkeypatch):
    """Utterances shorter than a wave's 32 rows at the downsampled stacks (T = 40: 20 / 10 frames at
    ds 2 / 4): the row-vector epilogues whose groups are shorter than a wave take their per-lane
    forms (the transposed FF1 epilogue's TP = false instantiation, the FF3 + BiasNorm epilogue's
    global row-vector loads instead of the staged LDS rows).  Fused vs the oracle at the bf16 bar and
    vs the unfused pair."""
    from oracle.zipvoice_np import ZipVoiceOracle
    outs = {}
    for ffn in ("0", "2"):
        outs[ffn], inp = _run(monkeypatch, {"ZV_FFN": ffn, "ZV_FFN_MIN_ROWS": "0"}, "bf16", B=8, T=40,
                              lens=(40, 33, 40, 17, 25, 40, 9, 31), t=0.6, seed=5)
    cfg, sd, x, tc, sc, pm, t = inp
    ref = ZipVoiceOracle(cfg, sd).velocity(np.float32(t), x, tc, sc, pm, 1.0)
    valid = ~pm
    for ffn, o in outs.items():
        e = np.abs(o - ref)[valid]
        print(f"short utterances ZV_FFN={ffn}: vs oracle mean {e.mean():.3e} max {e.max():.3e}; "
              f"vs unfused {np.abs(o - outs['0'])[valid].mean():.3e}")
        assert np.isfinite(o).all()
        assert e.mean() < BAR["bf16"], (ffn, e.mean())

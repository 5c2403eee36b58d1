"""GPU parity of the BigVGAN-v2 vocoder (zv_bigvgan_* through the C ABI) against the
CPU oracle (oracle/bigvgan_np.py, itself pinned to torch's conv / conv_transpose /
replicate-pad ops in tests/test_bigvgan_oracle.py; the bigvgan package composition is
"parity unpinned").

Tolerance: precision="fp32" (split bf16x3 GEMMs, fp32 activation kernels) wav
RMS(err) < 1e-4 and max |err| < 2e-3 — the same bar as the Vocos vocoder;
precision="bf16" RMS(err) < 5e-3 (18 residual conv pairs per stage in bf16).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

from oracle.bigvgan_np import bigvgan_forward  # noqa: E402
from zipvoice_amd.bigvgan import BigVGAN, BigVGANConfig, synthetic_bigvgan_state_dict  # noqa: E402
from oracle.bigvgan_np import anti_alias_filter  # noqa: E402

RMS_TOL = {"fp32": 1e-4, "bf16": 5e-3}
SMALL = BigVGANConfig(upsample_initial_channel=128, upsample_rates=(4, 2, 2),
                      upsample_kernel_sizes=(8, 4, 4))
_voc = {}


def ocfg(cfg):
    return dict(upsample_rates=cfg.upsample_rates, upsample_kernel_sizes=cfg.upsample_kernel_sizes,
                resblock_kernel_sizes=cfg.resblock_kernel_sizes,
                resblock_dilation_sizes=cfg.resblock_dilation_sizes, use_tanh_at_final=False)


def vocoder(precision, cfg=BigVGANConfig()):
    key = (precision, cfg.upsample_initial_channel, cfg.upsample_rates)
    if key not in _voc:
        v = BigVGAN(cfg, precision=precision)
        v.load_state_dict(synthetic_bigvgan_state_dict(cfg, 0))
        _voc[key] = v.to("cuda:0")
    return _voc[key]


def rms(a):
    return float(np.sqrt(np.mean(np.square(a))))


def check(out, ref, precision, what):
    assert out.shape == ref.shape, (out.shape, ref.shape)
    assert np.isfinite(out).all()
    e = out - ref
    print(f"{what} [{precision}] wav rms={rms(ref):.3e} err rms={rms(e):.3e} max={np.abs(e).max():.3e}")
    assert rms(e) < RMS_TOL[precision], rms(e)
    if precision == "fp32":
        assert np.abs(e).max() < 2e-3


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_full_config_matches_oracle(precision):
    """bigvgan_v2_24khz_100band_256x shapes (112M params), 12 frames -> 3072 samples."""
    rng = np.random.default_rng(0)
    mel = (1.5 * rng.standard_normal((1, 100, 12)) - 4.0).astype(np.float32)
    v = vocoder(precision)
    out = v.decode(torch.from_numpy(mel).cuda())
    assert out.shape == (1, 1, 12 * 256)
    ref = bigvgan_forward(mel[0], synthetic_bigvgan_state_dict(BigVGANConfig(), 0))
    check(out[0, 0].cpu().numpy(), ref, precision, "full")


@pytest.mark.parametrize("T", [1, 2, 7, 40])
def test_small_config_lengths(T):
    """Edge lengths: a single frame (every halo replicated / zero-padded), short and
    longer sequences, against the oracle."""
    rng = np.random.default_rng(T)
    mel = (1.5 * rng.standard_normal((1, 100, T)) - 4.0).astype(np.float32)
    out = vocoder("fp32", SMALL).decode(torch.from_numpy(mel).cuda())[0, 0].cpu().numpy()
    ref = bigvgan_forward(mel[0], synthetic_bigvgan_state_dict(SMALL, 0), ocfg(SMALL))
    check(out, ref, "fp32", f"small T={T}")


def test_ragged_batch_postprocess_equals_separate_calls():
    """decode_features: (B, T, C) model output / feat_scale - feat_bias with per-utterance
    lengths == separate single-utterance forwards; samples past len*hop are 0."""
    rng = np.random.default_rng(5)
    B, T, hop = 3, 21, SMALL.hop_length
    lens = np.array([21, 9, 1])
    pred = (0.1 * (1.5 * rng.standard_normal((B, T, 100)) - 4.0)).astype(np.float32)
    v = vocoder("fp32", SMALL)
    out = v.decode_features(torch.from_numpy(pred).cuda(), torch.from_numpy(lens).cuda(),
                            feat_scale=0.1, feat_bias=0.0).cpu().numpy()
    assert out.shape == (B, T * hop)
    sd = synthetic_bigvgan_state_dict(SMALL, 0)
    for b in range(B):
        mel = pred[b, :lens[b]].T / 0.1
        ref = bigvgan_forward(mel, sd, ocfg(SMALL))
        check(out[b, :lens[b] * hop], ref, "fp32", f"ragged b={b}")
        assert np.all(out[b, lens[b] * hop:] == 0)


def test_filter_buffers_accepted_and_checked():
    sd = dict(synthetic_bigvgan_state_dict(SMALL, 0))
    f = anti_alias_filter(2).astype(np.float32).reshape(1, 1, 12)
    sd["resblocks.0.activations.0.upsample.filter"] = f
    sd["resblocks.0.activations.0.downsample.lowpass.filter"] = f
    v = BigVGAN(SMALL).load_state_dict(sd).to("cuda:0")
    mel = torch.full((1, 100, 3), -4.0, device="cuda:0")
    assert torch.isfinite(v.decode(mel)).all()
    sd["activation_post.downsample.lowpass.filter"] = f[..., ::-1] * 1.1
    with pytest.raises(RuntimeError, match="alias-free filter"):
        BigVGAN(SMALL).load_state_dict(sd).to("cuda:0")


def test_unexpected_key_rejected():
    sd = dict(synthetic_bigvgan_state_dict(SMALL, 0))
    sd["conv_post.bias"] = np.zeros(1, np.float32)
    with pytest.raises(KeyError):
        BigVGAN(SMALL).load_state_dict(sd)


@pytest.mark.parametrize("precision", ["bf16", "fp32"])
def test_full_size_batch_equals_separate_calls(precision):
    """Size-independent property at production lengths (oracle too slow there): a ragged
    batch of 7 s and 4 s utterances decodes bit-identically to separate single-utterance
    calls (the zero halos isolate utterances; per-row GEMM arithmetic does not depend on
    the batch), and every sample is finite and inside the final clamp."""
    rng = np.random.default_rng(11)
    T, lens = 656, [656, 375]
    pred = (0.1 * (1.5 * rng.standard_normal((2, T, 100)) - 4.0)).astype(np.float32)
    v = vocoder(precision)
    x = torch.from_numpy(pred).cuda()
    out = v.decode_features(x, torch.tensor(lens, device="cuda"))
    for b, n in enumerate(lens):
        one = v.decode_features(x[b:b + 1, :n].contiguous())
        assert torch.isfinite(one).all() and float(one.abs().max()) <= 1.0
        assert torch.equal(out[b, :n * 256], one[0]), (b, float((out[b, :n * 256] - one[0]).abs().max()))
        assert torch.all(out[b, n * 256:] == 0)

"""GPU parity of the prompt feature extractor (zv_fbank_* via zipvoice_amd.feature)
against the numpy oracle (oracle/fbank_np.py), fp32 throughout.

Tolerance: |log-mel error| < 1e-4 where mel > 1e-3 (quiet bins: both sides are
fp32 sums whose absolute error ~1e-7 * ||frame|| dominates the log), and every
row count follows lhotse compute_num_frames."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

from oracle.fbank_np import vocos_fbank  # noqa: E402
from zipvoice_amd.feature import VocosFbank  # noqa: E402


def speechlike(n, seed):
    rng = np.random.default_rng(seed)
    t = np.arange(n) / 24000.0
    x = 0.2 * np.sin(2 * np.pi * 180 * t) * (1 + 0.5 * np.sin(2 * np.pi * 3 * t))
    x += 0.05 * rng.standard_normal(n)
    return x.astype(np.float32)


def compare(got, ref):
    assert got.shape == ref.shape, (got.shape, ref.shape)
    mask = ref > np.log(1e-3)
    err = np.abs(got - ref)[mask]
    print(f"fbank: max err {err.max():.3e} (of {mask.sum()} bins)")
    assert err.max() < 1e-4


def test_extract_matches_oracle_mono():
    fx = VocosFbank()
    x = speechlike(24000 * 3 + 100, 0)
    got = fx.extract(x, sampling_rate=24000)
    ref = vocos_fbank(x, fx.window.numpy(), fx.fb.numpy())
    compare(got, ref)


def test_extract_batch_ragged_equals_single():
    fx = VocosFbank()
    lens = [24000 * 2 + 7, 24000, 5000]
    N = max(lens)
    wav = np.zeros((3, N), np.float32)
    for i, n in enumerate(lens):
        wav[i, :n] = speechlike(n, i + 1)
    feats, nfr = fx.extract_batch(torch.from_numpy(wav).cuda(), torch.tensor(lens))
    feats = feats.cpu().numpy()
    for i, n in enumerate(lens):
        ref = vocos_fbank(wav[i, :n], fx.window.numpy(), fx.fb.numpy())
        assert int(nfr[i]) == ref.shape[0]
        compare(feats[i, :ref.shape[0]], ref)
        assert np.all(feats[i, ref.shape[0]:] == 0)


def test_extract_stereo_concatenates_channels():
    fx = VocosFbank(num_channels=2)
    x = np.stack([speechlike(30000, 5), speechlike(30000, 6)])
    got = fx.extract(torch.from_numpy(x), sampling_rate=24000)
    assert got.shape == (compute := (30000 + 128) // 256, 200)
    for c in range(2):
        ref = vocos_fbank(x[c], fx.window.numpy(), fx.fb.numpy())
        compare(got[:, c * 100:(c + 1) * 100].numpy(), ref)


# ---- BigVGANFbank (feature.py:133-204): same kernel, BigVGAN framing / eps / floor

def test_bigvgan_extract_matches_oracle_mono_and_replicate_tail():
    from oracle.fbank_np import bigvgan_fbank
    from zipvoice_amd.feature import BigVGANFbank
    fx = BigVGANFbank()
    for n, seed in ((24000 * 3 + 100, 3), (1000, 4)):   # 1000: last frame replicated
        x = speechlike(n, seed)
        got = fx.extract(x, 24000)
        ref = bigvgan_fbank(x, fx.window.numpy(), fx.fb)
        compare(got, ref)


def test_bigvgan_batch_ragged_and_stereo():
    from oracle.fbank_np import bigvgan_fbank
    from zipvoice_amd.feature import BigVGANFbank
    fx = BigVGANFbank()
    lens = [24000 + 7, 24000 * 2 - 300, 5000]
    wavs = np.zeros((3, max(lens)), np.float32)
    for i, n in enumerate(lens):
        wavs[i, :n] = speechlike(n, 10 + i)
    feats, nfr = fx.extract_batch(torch.from_numpy(wavs).cuda(), torch.tensor(lens))
    for i, n in enumerate(lens):
        ref = bigvgan_fbank(wavs[i, :n], fx.window.numpy(), fx.fb)
        assert int(nfr[i]) == ref.shape[0]
        compare(feats[i, :ref.shape[0]].cpu().numpy(), ref)
    st = BigVGANFbank(num_channels=2)
    x2 = np.stack([speechlike(24000, 20), speechlike(24000, 21)])
    got = st.extract(x2, 24000)
    ref = np.concatenate([bigvgan_fbank(x2[0], st.window.numpy(), st.fb),
                          bigvgan_fbank(x2[1], st.window.numpy(), st.fb)], axis=1)
    compare(got, ref)

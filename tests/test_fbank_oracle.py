"""Pin the VocosFbank oracle (oracle/fbank_np.py): its STFT magnitude against
torch.stft(center=True, reflect) — the op torchaudio's Spectrogram(power=1)
calls — and the mel filterbank against the torchaudio formula's properties.
torchaudio / lhotse are absent, so the filterbank itself is "parity unpinned"
beyond the formula (zipvoice_amd/feature.py:melscale_fbanks)."""
import numpy as np
import torch

from oracle.fbank_np import vocos_fbank
from zipvoice_amd.feature import compute_num_frames, melscale_fbanks


def test_stft_magnitude_matches_torch_stft():
    rng = np.random.default_rng(0)
    x = (0.1 * rng.standard_normal(24000 // 2 + 77)).astype(np.float32)
    win = torch.hann_window(1024)
    fb = torch.eye(513)[:, :513]            # identity "filterbank": raw magnitudes
    got = vocos_fbank(x, win.numpy(), fb.numpy())
    S = torch.stft(torch.from_numpy(x), 1024, 256, 1024, win, center=True, pad_mode="reflect",
                   return_complex=True).abs()
    want = torch.log(torch.clamp(S, min=1e-7)).T.numpy()[:got.shape[0]]
    assert got.shape[0] == compute_num_frames(len(x), 256)
    big = want > np.log(1e-3)
    np.testing.assert_allclose(got[big], want[big], atol=2e-5)


def test_melscale_fbanks_shape_and_triangles():
    fb = melscale_fbanks(513, 0.0, 12000.0, 100, 24000).numpy()
    assert fb.shape == (513, 100)
    assert (fb >= 0).all() and fb.max() <= 1.0 + 1e-6
    peaks = fb.argmax(0)
    assert (np.diff(peaks) >= 0).all()          # filters ordered by centre frequency
    assert (fb.sum(0) > 0).all()


def test_num_frames_rule():
    # lhotse compute_num_frames: (n + hop // 2) // hop; the centred STFT has 1 + n // hop
    for n in (513, 1000, 24000, 24000 * 3 + 129):
        assert compute_num_frames(n, 256) == (n + 128) // 256 <= 1 + n // 256


# ---- BigVGANFbank (zipvoice/utils/feature.py:133-204, _bigvgan_mel_feature.py:42-111)

def _bigvgan_mel_torch(x: np.ndarray, fb: np.ndarray) -> np.ndarray:
    """The reference's mel_spectrogram restated with the same torch ops (reflect
    F.pad by (n_fft - hop) // 2, torch.stft center=False, sqrt(|X|^2 + 1e-9),
    matmul with the mel basis, log(clamp(1e-5))) -> (frames, n_mels)."""
    y = torch.from_numpy(x)[None]
    p = (1024 - 256) // 2
    y = torch.nn.functional.pad(y.unsqueeze(1), (p, p), mode="reflect").squeeze(1)
    spec = torch.stft(y, 1024, hop_length=256, win_length=1024, window=torch.hann_window(1024),
                      center=False, pad_mode="reflect", normalized=False, onesided=True,
                      return_complex=True)
    spec = torch.sqrt(torch.view_as_real(spec).pow(2).sum(-1) + 1e-9)
    mel = torch.matmul(torch.from_numpy(fb).T, spec)
    return torch.log(torch.clamp(mel, min=1e-5))[0].T.numpy()


def test_bigvgan_oracle_matches_torch_restatement():
    from oracle.fbank_np import bigvgan_fbank
    from zipvoice_amd.feature import slaney_mel_fbanks
    rng = np.random.default_rng(1)
    fb = slaney_mel_fbanks(24000, 1024, 100)
    for n in (24000 + 333, 1000):              # 1000: fewer STFT frames than the lhotse count
        x = (0.2 * rng.standard_normal(n)).astype(np.float32)
        got = bigvgan_fbank(x, torch.hann_window(1024).numpy(), fb)
        want = _bigvgan_mel_torch(x, fb)
        keep = compute_num_frames(n, 256)
        assert got.shape == (keep, 100)
        m = min(keep, want.shape[0])
        np.testing.assert_allclose(got[:m], want[:m], atol=2e-4)
        if want.shape[0] < keep:               # feature.py:197-201 replicate pad of the last frame
            assert np.array_equal(got[m:], np.repeat(got[m - 1:m], keep - m, axis=0))


def test_slaney_filterbank_formula():
    """librosa.filters.mel(htk=False, norm='slaney') properties (librosa is absent:
    parity of the exact matrix is unpinned beyond the published formula)."""
    from zipvoice_amd.feature import _hz_to_mel_slaney, _mel_to_hz_slaney, slaney_mel_fbanks
    assert abs(float(_hz_to_mel_slaney(1000.0)) - 15.0) < 1e-12          # linear part: 3 f / 200
    assert abs(float(_hz_to_mel_slaney(6400.0)) - 42.0) < 1e-9           # 27 mels per factor 6.4
    f = np.array([0.0, 300.0, 999.0, 1000.0, 4321.0, 12000.0])
    np.testing.assert_allclose(_mel_to_hz_slaney(_hz_to_mel_slaney(f)), f, rtol=1e-12, atol=1e-9)
    fb = slaney_mel_fbanks(24000, 1024, 100)
    assert fb.shape == (513, 100) and fb.dtype == np.float32 and (fb >= 0).all()
    assert (np.diff(fb.argmax(0)) >= 0).all()
    # Slaney normalisation: each triangle integrates to ~1 over Hz (bins 23.4 Hz apart;
    # the widest filters are resolved well enough to check)
    area = fb.sum(0) * (24000 / 1024)
    np.testing.assert_allclose(area[50:], 1.0, rtol=0.05)

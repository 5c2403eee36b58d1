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

"""Pin the vocoder oracle (oracle/vocos_np.py) against the torch primitives the
vocos package calls (the package itself is not installed and no reference
fixture exists, so the network composition is "parity unpinned"; each
primitive is pinned here):

* ISTFT(padding="same") == irfft * window -> F.fold overlap-add -> trim ->
  / folded squared window (vocos/spectral_ops.py), and its interior equals
  torch.istft(center=True) shifted by (n_fft/2 - (n_fft-hop)/2) samples;
* the backbone/head composition == the same graph built from F.conv1d,
  F.layer_norm, F.gelu, F.linear, torch.exp/clip/cos/sin.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle.vocos_np import VocosOracle, istft_same, postprocess_features
from zipvoice_amd.vocoder import VocosConfig, synthetic_vocos_state_dict

SMALL = VocosConfig(n_mels=100, dim=64, intermediate_dim=192, num_layers=2)


def torch_istft_same(spec: torch.Tensor, window: torch.Tensor, hop: int) -> torch.Tensor:
    """vocos ISTFT.forward, padding='same', written with the torch ops it uses."""
    n_fft = window.shape[0]
    pad = (n_fft - hop) // 2
    B, N, T = spec.shape
    ifft = torch.fft.irfft(spec, n_fft, dim=1, norm="backward") * window[None, :, None]
    out_size = (T - 1) * hop + n_fft
    y = F.fold(ifft, output_size=(1, out_size), kernel_size=(1, n_fft), stride=(1, hop))[:, 0, 0, pad:-pad]
    wsq = window.square().expand(1, T, -1).transpose(1, 2)
    env = F.fold(wsq, output_size=(1, out_size), kernel_size=(1, n_fft), stride=(1, hop)).squeeze()[pad:-pad]
    assert (env > 1e-11).all()
    return y / env


def torch_vocos_decode(sd, mel: torch.Tensor, num_layers: int) -> torch.Tensor:
    t = {k: torch.from_numpy(v) for k, v in sd.items()}
    x = F.conv1d(mel, t["backbone.embed.weight"], t["backbone.embed.bias"], padding=3)
    C = x.shape[1]
    x = F.layer_norm(x.transpose(1, 2), (C,), t["backbone.norm.weight"], t["backbone.norm.bias"],
                     eps=1e-6).transpose(1, 2)
    for i in range(num_layers):
        p = f"backbone.convnext.{i}."
        r = x
        h = F.conv1d(x, t[p + "dwconv.weight"], t[p + "dwconv.bias"], padding=3, groups=C)
        h = F.layer_norm(h.transpose(1, 2), (C,), t[p + "norm.weight"], t[p + "norm.bias"], eps=1e-6)
        h = F.linear(h, t[p + "pwconv1.weight"], t[p + "pwconv1.bias"])
        h = F.gelu(h)
        h = F.linear(h, t[p + "pwconv2.weight"], t[p + "pwconv2.bias"])
        x = r + (t[p + "gamma"] * h).transpose(1, 2)
    x = F.layer_norm(x.transpose(1, 2), (C,), t["backbone.final_layer_norm.weight"],
                     t["backbone.final_layer_norm.bias"], eps=1e-6)
    o = F.linear(x, t["head.out.weight"], t["head.out.bias"]).transpose(1, 2)
    mag, ph = o.chunk(2, dim=1)
    mag = torch.clip(torch.exp(mag), max=1e2)
    S = mag * (torch.cos(ph) + 1j * torch.sin(ph))
    return torch_istft_same(S, t["head.istft.window"], 256)


def test_istft_same_matches_fold_and_torch_istft():
    rng = np.random.default_rng(0)
    T, n_fft, hop = 23, 1024, 256
    re = rng.standard_normal((T, n_fft // 2 + 1)).astype(np.float32)
    im = rng.standard_normal((T, n_fft // 2 + 1)).astype(np.float32)
    win = torch.hann_window(n_fft).numpy()
    y = istft_same(re, im, win, hop)
    assert y.shape == (T * hop,)
    spec = torch.from_numpy(re.T + 1j * im.T)[None]
    y_fold = torch_istft_same(spec, torch.from_numpy(win), hop)[0].numpy()
    np.testing.assert_allclose(y, y_fold, atol=2e-5, rtol=1e-4)
    # interior vs torch.istft(center=True): trim differs by n_fft/2 - (n_fft-hop)/2
    y_t = torch.istft(spec, n_fft, hop, n_fft, torch.from_numpy(win), center=True).numpy()[0]
    sh = n_fft // 2 - (n_fft - hop) // 2
    n = min(len(y_t), len(y) - sh) - n_fft      # stay clear of the envelope edges
    np.testing.assert_allclose(y[sh:sh + n], y_t[:n], atol=2e-5, rtol=1e-4)


def test_vocos_oracle_matches_torch_composition():
    sd = synthetic_vocos_state_dict(SMALL, seed=3)
    rng = np.random.default_rng(1)
    mel = (rng.standard_normal((2, 100, 37)) - 3.0).astype(np.float32)
    got = VocosOracle(sd, num_layers=SMALL.num_layers).decode(mel)
    want = torch_vocos_decode(sd, torch.from_numpy(mel), SMALL.num_layers).numpy()
    assert got.shape == want.shape == (2, 37 * 256)
    err = np.sqrt(np.mean((got - want) ** 2))
    assert err < 1e-5 * max(1.0, float(np.sqrt(np.mean(want ** 2)))), err


def test_vocos_oracle_ragged_equals_separate_calls():
    sd = synthetic_vocos_state_dict(SMALL, seed=4)
    o = VocosOracle(sd, num_layers=SMALL.num_layers)
    rng = np.random.default_rng(2)
    mel = rng.standard_normal((2, 100, 30)).astype(np.float32)
    out = o.decode(mel, lens=[30, 17])
    np.testing.assert_array_equal(out[1, 17 * 256:], 0)
    np.testing.assert_allclose(out[1, :17 * 256], o.decode(mel[1:, :, :17])[0], atol=1e-6)


def test_postprocess_matches_reference_expression():
    rng = np.random.default_rng(5)
    pred = rng.standard_normal((2, 11, 100)).astype(np.float32)
    want = (torch.from_numpy(pred).permute(0, 2, 1) / 0.1 - 0.0).numpy()
    np.testing.assert_array_equal(postprocess_features(pred, 0.1, 0.0), want)


def test_synthetic_vocos_weights_have_reference_shapes():
    sd = synthetic_vocos_state_dict()
    assert sd["head.out.weight"].shape == (1026, 512)
    assert sd["backbone.embed.weight"].shape == (512, 100, 7)
    np.testing.assert_array_equal(sd["head.istft.window"], torch.hann_window(1024).numpy())
    assert len(sd) == 6 + 9 * 8 + 3

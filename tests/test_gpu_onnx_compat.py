"""The ONNX-contract adapter (zipvoice_amd/onnx_compat.py) on the engine:
run_fm_decoder == the CFG-folded velocity of the oracle, run_text_encoder ==
the oracle text encoder + the exported graph's duration rule, and the
infer_zipvoice_onnx-style sample loop == the oracle Euler solve."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

from oracle.zipvoice_np import ZipVoiceOracle  # noqa: E402
from zipvoice_amd.config import default_config  # noqa: E402
from zipvoice_amd.models import build_model  # noqa: E402
from zipvoice_amd.onnx_compat import OnnxModel, sample  # noqa: E402
from zipvoice_amd.weights import synthetic_state_dict  # noqa: E402

_m = {}


def setup(variant="zipvoice"):
    if variant not in _m:
        cfg = default_config(variant)
        sd = synthetic_state_dict(cfg, 0)
        m = build_model(cfg, precision="fp32")
        m.load_state_dict(sd)
        _m[variant] = (OnnxModel.from_model(m.to("cuda:0")), ZipVoiceOracle(cfg, sd))
    return _m[variant]


@pytest.mark.parametrize("variant,g,t", [("zipvoice", 1.0, 0.3), ("zipvoice", 1.0, 0.7),
                                         ("zipvoice_distill", 3.0, 0.4)])
def test_run_fm_decoder_matches_oracle(variant, g, t):
    om, orc = setup(variant)
    rng = np.random.default_rng(0)
    T = 57
    x = rng.standard_normal((1, T, 100), dtype=np.float32)
    tc = rng.standard_normal((1, T, 100), dtype=np.float32)
    sc = (0.3 * rng.standard_normal((1, T, 100)) - 0.5).astype(np.float32)
    v = om.run_fm_decoder(torch.tensor(t), torch.from_numpy(x), torch.from_numpy(tc),
                          torch.from_numpy(sc), torch.tensor(g)).numpy()
    ref = orc.velocity(np.float32(t), x, tc, sc, np.zeros((1, T), bool), g)
    err = np.abs(v - ref).mean()
    print(variant, t, "mean err", err)
    assert err < 1e-3


def test_run_text_encoder_duration_rule_and_values():
    om, orc = setup()
    rng = np.random.default_rng(1)
    toks = [[int(v) for v in rng.integers(1, 360, 23)]]
    ptoks = [[int(v) for v in rng.integers(1, 360, 9)]]
    P = 77
    tc = om.run_text_encoder(torch.tensor(toks), torch.tensor(ptoks), torch.tensor(P),
                             torch.tensor(1.3, dtype=torch.float32))
    S = 9 + 23
    want_T = int(torch.ceil(torch.tensor(P) / 9 * S / torch.tensor(1.3, dtype=torch.float32)))
    assert tc.shape == (1, want_T, 100)
    emb, _ = orc.forward_text_embed([ptoks[0] + toks[0]])   # (1, S+1, 100) incl. the pad slot
    d = want_T // S
    idx = np.minimum(np.arange(want_T) // d, S)
    np.testing.assert_allclose(tc.numpy()[0], emb[0][idx], atol=1e-3)


def test_onnx_style_sample_matches_oracle_euler():
    om, orc = setup()
    rng = np.random.default_rng(2)
    toks = [[int(v) for v in rng.integers(1, 360, 12)]]
    ptoks = [[int(v) for v in rng.integers(1, 360, 8)]]
    pf = (0.3 * rng.standard_normal((1, 40, 100)) - 0.5).astype(np.float32)
    tc = om.run_text_encoder(torch.tensor(toks), torch.tensor(ptoks), torch.tensor(40),
                             torch.tensor(1.0))
    T = tc.shape[1]
    x0 = torch.from_numpy(rng.standard_normal((1, T, 100), dtype=np.float32))
    out = sample(om, toks, ptoks, torch.from_numpy(pf), num_step=3, t_shift=0.5,
                 guidance_scale=1.0, x0=x0)
    sc = np.zeros((1, T, 100), np.float32)
    sc[:, :40] = pf
    ref = orc.euler(x0.numpy(), tc.numpy(), sc, np.zeros((1, T), bool), 3, 1.0, t_shift=0.5)
    err = np.abs(out.numpy() - ref[:, 40:]).mean()
    print("onnx-style sample mean err", err)
    assert err < 1e-3

"""End-to-end generation on the engine (zipvoice_amd/infer.py), the reference's
generate_sentence flow: prompt RMS normalisation -> VocosFbank -> sample ->
vocoder -> clamp -> RMS restore; batched serving form with ragged prompts."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

from zipvoice_amd.config import default_config  # noqa: E402
from zipvoice_amd.feature import VocosFbank  # noqa: E402
from zipvoice_amd.infer import generate_batch, generate_sentence  # noqa: E402
from zipvoice_amd.models import build_model  # noqa: E402
from zipvoice_amd.vocoder import Vocos  # noqa: E402
from zipvoice_amd.weights import synthetic_state_dict  # noqa: E402


@pytest.fixture(scope="module")
def stack():
    cfg = default_config("zipvoice")
    m = build_model(cfg, precision="bf16")
    m.load_state_dict(synthetic_state_dict(cfg, 0))
    m = m.to("cuda:0")
    voc = Vocos().load_synthetic(0).to("cuda:0")
    return m, voc, VocosFbank()


def prompt(n, seed):
    rng = np.random.default_rng(seed)
    return (0.05 * rng.standard_normal(n)).astype(np.float32)   # quiet: RMS < target


def test_generate_sentence_runs_and_reports(stack):
    m, voc, fx = stack
    wav, met = generate_sentence(list(range(1, 30)), list(range(40, 52)), prompt(24000, 0), m,
                                 voc, fx, num_step=4)
    assert wav.shape[0] == 1 and wav.shape[1] % 256 == 0 and wav.shape[1] > 0
    assert torch.isfinite(wav).all()
    assert float(wav.abs().max()) <= 1.0 * 0.05 / 0.1 + 1e-6     # clamp then RMS restore
    for k in ("t", "t_no_vocoder", "t_vocoder", "wav_seconds", "rtf", "rtf_no_vocoder",
              "rtf_vocoder"):
        assert k in met


def test_generate_batch_ragged(stack):
    m, voc, fx = stack
    items = [(list(range(1, 20)), list(range(30, 40)), prompt(24000, 1)),
             (list(range(5, 50)), list(range(60, 66)), prompt(36000, 2))]
    outs, met = generate_batch(items, m, voc, fx, num_step=4)
    assert len(outs) == 2 and met["rtf"] > 0
    for o in outs:
        assert o.dim() == 2 and o.shape[1] > 0 and torch.isfinite(o).all()


def test_generate_sentence_bigvgan_stack(stack):
    """feature.type "bigvgan_v2" (egs/zipvoice/conf/zipvoice_base_bigvgan_v2.json):
    BigVGANFbank prompt features + the BigVGAN-v2 vocoder, through the same flow."""
    from zipvoice_amd.bigvgan import BigVGAN
    from zipvoice_amd.infer import get_feature_extractor
    m, _, _ = stack
    voc = BigVGAN(precision="bf16").load_synthetic(0).to("cuda:0")
    fx = get_feature_extractor("bigvgan_v2")
    wav, met = generate_sentence(list(range(1, 30)), list(range(40, 52)), prompt(24000, 3), m,
                                 voc, fx, num_step=4)
    assert wav.shape[0] == 1 and wav.shape[1] % 256 == 0 and wav.shape[1] > 0
    assert torch.isfinite(wav).all()
    assert float(wav.abs().max()) <= 1.0 * 0.05 / 0.1 + 1e-6
    assert met["rtf_vocoder"] > 0

"""The convolution module's GLU linear + depthwise conv + SwooshR as one launch (ZV_GLU_DW=1, the
16-bit engines' default; csrc/zv_gemm256.inc g256_epi_glu_dw) against the unfused pair (the GLU
linear's bf16 output in HBM, then zv_dwconv_pipe_kernel): bitwise equal velocities -- the fused
kernel rounds the GLU values to the same 16-bit numbers and runs the conv in the same tap-major
FMA order.  Reference: zipformer.py:1638-1680 (ConvolutionModule), scaling.py:1185-1191.

Shapes: ragged batches whose 256-row tiles cross utterance boundaries (the conv's zero padding
at every utterance edge), padded frames (masked_fill before the conv), every kernel size of the
decoder (31 / 15 / 7 at the full / half / quarter-rate stacks), C2's and C4's lengths."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def engine(monkeypatch, precision, fused, variant="zipvoice"):
    from zipvoice_amd.config import default_config
    from zipvoice_amd.models import build_model
    from zipvoice_amd.weights import synthetic_state_dict
    monkeypatch.setenv("ZV_GLU_DW", "1" if fused else "0")
    cfg = default_config(variant)
    m = build_model(cfg, precision=precision)
    m.load_state_dict(synthetic_state_dict(cfg, 0))
    m = m.to("cuda:0")
    monkeypatch.delenv("ZV_GLU_DW")
    return m


def inputs(lens, T, Fx=100, seed=0):
    rng = np.random.default_rng(seed)
    B = len(lens)
    x = rng.standard_normal((B, T, Fx), dtype=np.float32)
    tc = rng.standard_normal((B, T, 100), dtype=np.float32)
    sc = (0.3 * rng.standard_normal((B, T, Fx)) - 0.5).astype(np.float32)
    pm = np.arange(T)[None] >= np.array(lens)[:, None]
    return [torch.from_numpy(a).to("cuda:0") for a in (x, tc, sc, pm)]


CASES = {"short-ragged": ([97, 60, 33], 97), "C2": ([1219, 1004], 1219),
         "C2-batch8": ([1219] * 8, 1219), "C4": ([3376, 2900], 3376)}


@pytest.mark.parametrize("precision", ["bf16", "fp16"])
def test_glu_dwconv_fused_bitwise(monkeypatch, precision):
    mu = engine(monkeypatch, precision, fused=False)
    mf = engine(monkeypatch, precision, fused=True)
    from zipvoice_amd import engine as eng
    for name, (lens, T) in CASES.items():
        x, tc, sc, pm = inputs(lens, T, seed=T)
        eng.profile(True)
        vf = mf.engine.velocity(0.3, 1.0, x, tc, sc, pm)
        torch.cuda.synchronize()
        rep = eng.profile_report()
        eng.profile(False)
        vu = mu.engine.velocity(0.3, 1.0, x, tc, sc, pm)
        torch.cuda.synchronize()
        fused = rep.get("gemm_bf16_glu_dw", {}).get("launches", 0)
        print(f"{name} [{precision}]: fused launches {fused}, max |fused - unfused| = "
              f"{(vf - vu).abs().max().item():.3e}")
        assert fused > 0 and "dwconv_bf16" not in rep, (name, sorted(rep))
        assert torch.equal(vf, vu), (name, (vf - vu).abs().max().item())


def test_glu_dwconv_fused_stereo_bitwise(monkeypatch):
    """Dialog-Stereo (C5's model, 200-dim features) at the C5 length."""
    mu = engine(monkeypatch, "bf16", fused=False, variant="zipvoice_dialog_stereo")
    mf = engine(monkeypatch, "bf16", fused=True, variant="zipvoice_dialog_stereo")
    x, tc, sc, pm = inputs([3376, 3100], 3376, Fx=200, seed=5)
    vf = mf.engine.velocity(0.4, 1.5, x, tc, sc, pm)
    vu = mu.engine.velocity(0.4, 1.5, x, tc, sc, pm)
    torch.cuda.synchronize()
    assert torch.equal(vf, vu), (vf - vu).abs().max().item()

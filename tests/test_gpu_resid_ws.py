"""The wave-specialised residual-stream GEMM (zv_gemm_ws.inc, default in the bf16
mode for K <= 64, forced on every residual linear here with ZV_RESID_WS=2)
against the plain residual GEMM (zv_gemm_kernel ROLE = 1, ZV_RESID_WS=0): same K order, same MFMA sequence, same epilogue arithmetic, so
the decoder velocity must agree to fp32 rounding (bitwise in practice).  Shapes
cover a ragged batch (M not a multiple of the 128-row tile, padded frames) and
one with more tiles than CUs (each block walks several tiles, so the epilogue
of one tile runs under the next tile's K steps).  Parity with the reference is
covered by test_gpu_parity.py, which runs this kernel in its bf16 cases."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, scope="module")
def _needs_ab_build():
    """A/B arm: its kernel is compiled only into the A/B build (build.py --out PATH
    -DZV_AB_KERNELS, loaded with ZV_LIB_PATH=PATH); the product library skips this file."""
    from zipvoice_amd import engine
    if "ab_kernels" not in engine.load_library().zv_version().decode():
        pytest.skip("A/B kernel not in the product build (build.py -DZV_AB_KERNELS)")

torch = pytest.importorskip("torch")


def _model(ws: int):
    from zipvoice_amd.config import default_config
    from zipvoice_amd.models import build_model
    from zipvoice_amd.weights import synthetic_state_dict
    old = os.environ.get("ZV_RESID_WS")
    os.environ["ZV_RESID_WS"] = str(ws)
    try:
        cfg = default_config("zipvoice")
        m = build_model(cfg, precision="bf16")
        m.load_state_dict(synthetic_state_dict(cfg, 0))
        return m.to("cuda:0")
    finally:
        if old is None:
            del os.environ["ZV_RESID_WS"]
        else:
            os.environ["ZV_RESID_WS"] = old


@pytest.fixture(scope="module")
def models():
    return _model(2), _model(0)     # 2: every residual linear on the ws kernel


@pytest.mark.parametrize("B,T,lens", [(3, 203, [203, 150, 77]), (16, 1219, None)])
def test_resid_ws_matches_plain_kernel(models, B, T, lens):
    rng = np.random.default_rng(5)
    dev = torch.device("cuda:0")
    f = lambda a: torch.from_numpy(a.astype(np.float32)).to(dev)  # noqa: E731
    x = f(rng.standard_normal((B, T, 100)))
    tc = f(rng.standard_normal((B, T, 100)))
    sc = f(0.3 * rng.standard_normal((B, T, 100)) - 0.5)
    pm = None
    if lens is not None:
        pm = torch.from_numpy(np.arange(T)[None] >= np.array(lens)[:, None]).to(dev)
    outs = [m.forward_fm_decoder(t=torch.tensor(0.37), xt=x, text_condition=tc, speech_condition=sc,
                                 padding_mask=pm) for m in models]
    torch.cuda.synchronize()
    a, b = (o.float().cpu() for o in outs)
    assert torch.isfinite(a).all()
    diff = (a - b).abs().max().item()
    scale = b.abs().max().item()
    print(f"B={B} T={T}: max |ws - plain| = {diff:.3e} (max |v| {scale:.3e}), bitwise={torch.equal(a, b)}")
    assert diff <= 1e-5 * max(scale, 1.0), diff

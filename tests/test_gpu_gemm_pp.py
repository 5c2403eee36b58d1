"""The ping-pong GEMM (zv_gemm_pp.inc) against the 128x128 kernel it replaces for the
bf16 linears: same MFMA order per output element, same epilogue arithmetic, so the
results must be bitwise equal — per launch on random operands (plain, SwooshL,
residual read-modify-write) and for the whole decoder forward (every linear, the GLU and
NonlinAttention in-projections included), ZV_GEMM_PP=0 vs the default."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _needs_ab_build():
    """A/B arm: its kernel is compiled only into the A/B build (build.py --out PATH
    -DZV_AB_KERNELS, loaded with ZV_LIB_PATH=PATH); the product library skips this file."""
    from zipvoice_amd import engine
    if "ab_kernels" not in engine.load_library().zv_version().decode():
        pytest.skip("A/B kernel not in the product build (build.py -DZV_AB_KERNELS)")

torch = pytest.importorskip("torch")

SHAPES = [(1000, 384, 200), (78016, 1536, 512), (4096, 512, 1920), (777, 1024, 48),
          (256, 256, 64), (19520, 512, 1152), (129, 128, 600)]


@pytest.mark.parametrize("variant", [50])
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_pp_launch_bitwise(M, N, K, variant):
    from zipvoice_amd import engine
    lib = engine.load_library()
    for mode in (0, 1, 2):
        d, r = ctypes.c_float(), ctypes.c_float()
        rc = lib.zv_gemm_selftest(M, N, K, variant, mode, ctypes.byref(d), ctypes.byref(r))
        assert rc == 0, lib.zv_last_error().decode()
        print(f"M={M} N={N} K={K} v={variant} mode={mode}: maxdiff {d.value:.3e} (|ref| {r.value:.3e})")
        assert d.value == 0.0, (M, N, K, variant, mode, d.value)


def test_pp_decoder_forward_bitwise(monkeypatch):
    from zipvoice_amd.config import default_config
    from zipvoice_amd.models import build_model
    from zipvoice_amd.weights import synthetic_state_dict
    cfg = default_config("zipvoice")
    sd = synthetic_state_dict(cfg, 0)
    rng = np.random.default_rng(2)
    B, T = 3, 333
    dev = "cuda:0"
    x = torch.from_numpy(rng.standard_normal((B, T, 100), dtype=np.float32)).to(dev)
    tc = torch.from_numpy(rng.standard_normal((B, T, 100), dtype=np.float32)).to(dev)
    sc = torch.from_numpy(rng.standard_normal((B, T, 100), dtype=np.float32)).to(dev)
    pm = torch.from_numpy(np.arange(T)[None] >= np.array([T, 250, 97])[:, None]).to(dev)
    outs = []
    for flag in ("0", "1"):
        monkeypatch.setenv("ZV_GEMM_PP", flag)
        m = build_model(cfg, precision="bf16")
        m.load_state_dict(sd)
        m = m.to(dev)
        outs.append(m.engine.velocity(0.4, 1.0, x, tc, sc, pm).cpu())
        del m
    d = (outs[0] - outs[1]).abs().max().item()
    print(f"decoder velocity ZV_GEMM_PP=0 vs 1: max |diff| = {d:.3e}")
    assert torch.equal(outs[0], outs[1])

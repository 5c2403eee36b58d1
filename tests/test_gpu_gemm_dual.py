"""The dual-group residual GEMM (zv_gemm_dual.inc: two phase-offset 4-wave tile groups
per CU, hand-counted vmcnt) against the 128x128 kernel it replaces for the residual
linears: same MFMA order per accumulator and the same epilogue arithmetic, so bitwise
equal -- per launch on random operands (bias + fp32 residual read-modify-write, variant
60; + bypass original / scale, variant 61; ragged M, K = 64 .. 1920) and for the whole
decoder forward with every eligible residual linear on it (ZV_GEMM_DUAL=1 vs 0)."""
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

SHAPES = [(1000, 512, 1536), (78016, 512, 512), (4096, 512, 1920), (777, 256, 64),
          (19520, 512, 1152), (129, 128, 384), (25599, 512, 384)]


@pytest.mark.parametrize("variant", [60, 61])
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_dual_launch_bitwise(M, N, K, variant):
    from zipvoice_amd import engine
    lib = engine.load_library()
    d, r = ctypes.c_float(), ctypes.c_float()
    rc = lib.zv_gemm_selftest(M, N, K, variant, 2, ctypes.byref(d), ctypes.byref(r))
    assert rc == 0, lib.zv_last_error().decode()
    print(f"M={M} N={N} K={K} v={variant}: maxdiff {d.value:.3e} (|ref| {r.value:.3e})")
    assert d.value == 0.0, (M, N, K, variant, d.value)


def test_dual_decoder_forward_bitwise(monkeypatch):
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
        monkeypatch.setenv("ZV_GEMM_DUAL", flag)
        m = build_model(cfg, precision="bf16")
        m.load_state_dict(sd)
        m = m.to(dev)
        outs.append(m.engine.velocity(0.4, 1.0, x, tc, sc, pm).cpu())
        del m
    d = (outs[0] - outs[1]).abs().max().item()
    print(f"decoder velocity ZV_GEMM_DUAL=0 vs 1: max |diff| = {d:.3e}")
    assert torch.equal(outs[0], outs[1])

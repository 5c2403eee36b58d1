"""The counted GEMM epilogue (zv_gemm.inc gemm_epilogue_res: the residual-stream linears'
ROLE 1 / 2 kernels and the plain linears' ROLE 3; every epilogue load and store
unconditional, stores outside the output to a sink) against the general epilogue it
replaces: same arithmetic in the same order, so bitwise equal -- per launch on random
operands (bias + fp32 residual read-modify-write, variant 70; + bypass original / scale,
variant 71; bias (+ SwooshL) -> bf16, variant 72; ragged M and N, K = 64 .. 1920) and for
the decoder forward in the bf16 and fp32 modes and the Distill variant
(ZV_RES_COUNTED=1 vs 0)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

SHAPES = [(1000, 512, 1536), (78016, 512, 512), (4096, 512, 1920), (777, 256, 64),
          (19520, 512, 1152), (129, 128, 384), (25599, 512, 384), (3001, 192, 768),
          (517, 200, 256)]


@pytest.mark.parametrize("variant", [70, 71])
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_counted_epilogue_launch_bitwise(M, N, K, variant):
    from zipvoice_amd import engine
    lib = engine.load_library()
    d, r = ctypes.c_float(), ctypes.c_float()
    rc = lib.zv_gemm_selftest(M, N, K, variant, 2, ctypes.byref(d), ctypes.byref(r))
    assert rc == 0, lib.zv_last_error().decode()
    print(f"M={M} N={N} K={K} v={variant}: maxdiff {d.value:.3e} (|ref| {r.value:.3e})")
    assert d.value == 0.0, (M, N, K, variant, d.value)


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("M,N,K", SHAPES[:4] + [(78016, 1536, 512), (3001, 272, 512)])
def test_counted_plain_epilogue_launch_bitwise(M, N, K, mode):
    from zipvoice_amd import engine
    lib = engine.load_library()
    d, r = ctypes.c_float(), ctypes.c_float()
    rc = lib.zv_gemm_selftest(M, N, K, 72, mode, ctypes.byref(d), ctypes.byref(r))
    assert rc == 0, lib.zv_last_error().decode()
    print(f"M={M} N={N} K={K} v=72 mode={mode}: maxdiff {d.value:.3e} (|ref| {r.value:.3e})")
    assert d.value == 0.0, (M, N, K, mode, d.value)


@pytest.mark.parametrize("variant,precision", [("zipvoice", "bf16"), ("zipvoice", "fp32"),
                                               ("zipvoice_distill", "bf16")])
def test_counted_epilogue_decoder_bitwise(monkeypatch, variant, precision):
    from zipvoice_amd.config import default_config
    from zipvoice_amd.models import build_model
    from zipvoice_amd.weights import synthetic_state_dict
    cfg = default_config(variant)
    sd = synthetic_state_dict(cfg, 0)
    rng = np.random.default_rng(2)
    B, T = 3, 333
    dev = "cuda:0"
    f = lambda: torch.from_numpy(rng.standard_normal((B, T, 100), dtype=np.float32)).to(dev)
    x, tc, sc = f(), f(), f()
    pm = torch.from_numpy(np.arange(T)[None] >= np.array([T, 250, 97])[:, None]).to(dev)
    outs = []
    for flag in ("0", "1"):
        monkeypatch.setenv("ZV_RES_COUNTED", flag)
        m = build_model(cfg, precision=precision)
        m.load_state_dict(sd)
        m = m.to(dev)
        outs.append(m.engine.velocity(0.4, 1.0, x, tc, sc, pm).cpu())
        del m
    d = (outs[0] - outs[1]).abs().max().item()
    print(f"{variant} {precision} decoder velocity ZV_RES_COUNTED=0 vs 1: max |diff| = {d:.3e}")
    assert torch.equal(outs[0], outs[1])
